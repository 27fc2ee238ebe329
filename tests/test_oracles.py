"""Independent oracles for the engine's device paths.

Every test runs the engine op on the CPU engine and (gpu-marked) on cuda, and
compares BOTH with a result computed outside the engine: published lookup3
test vectors and a pure-Python hashlittle, Python dict/Counter group-by,
Python `sorted`, numpy per-group reductions, scipy.sparse.csgraph
(connected_components, dijkstra), a numpy independence/maximality check of
the Luby set, and a numpy Lloyd step. A logic error shared by the HIP kernel
and its CPU twin fails here (test_kernels_gpu.py only compares the two).
"""
import collections

import numpy as np
import pytest
import torch

import gpu_mapreduce_amd as g
from gpu_mapreduce_amd import C

DEVS = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]
M32 = 0xFFFFFFFF


# ---------------------------------------------------------------- lookup3 (Bob Jenkins, public domain)
def _rot(x, k):
    return ((x << k) | (x >> (32 - k))) & M32


def hashlittle_py(key: bytes, initval: int) -> int:
    """byte-at-a-time lookup3 hashlittle (little-endian word reads)"""
    n = len(key)
    a = b = c = (0xDEADBEEF + n + initval) & M32
    i = 0
    while n > 12:
        a = (a + int.from_bytes(key[i:i + 4], "little")) & M32
        b = (b + int.from_bytes(key[i + 4:i + 8], "little")) & M32
        c = (c + int.from_bytes(key[i + 8:i + 12], "little")) & M32
        a = (a - c) & M32; a ^= _rot(c, 4); c = (c + b) & M32
        b = (b - a) & M32; b ^= _rot(a, 6); a = (a + c) & M32
        c = (c - b) & M32; c ^= _rot(b, 8); b = (b + a) & M32
        a = (a - c) & M32; a ^= _rot(c, 16); c = (c + b) & M32
        b = (b - a) & M32; b ^= _rot(a, 19); a = (a + c) & M32
        c = (c - b) & M32; c ^= _rot(b, 4); b = (b + a) & M32
        n -= 12
        i += 12
    if n == 0:
        return c
    tail = key[i:i + n] + bytes(12 - n)
    a = (a + int.from_bytes(tail[0:4], "little")) & M32
    b = (b + int.from_bytes(tail[4:8], "little")) & M32
    c = (c + int.from_bytes(tail[8:12], "little")) & M32
    c ^= b; c = (c - _rot(b, 14)) & M32
    a ^= c; a = (a - _rot(c, 11)) & M32
    b ^= a; b = (b - _rot(a, 25)) & M32
    c ^= b; c = (c - _rot(b, 16)) & M32
    a ^= c; a = (a - _rot(c, 4)) & M32
    b ^= a; b = (b - _rot(a, 14)) & M32
    c ^= b; c = (c - _rot(b, 24)) & M32
    return c


def _var_kv(keys, values, dev):
    from gpu_mapreduce_amd.runtime.keyvalue import KeyValue
    kv = KeyValue("cpu")
    for k, v in zip(keys, values):
        kv.add(k, v)
    out = kv.finish()
    return out if dev == "cpu" else out.to(dev)


def _col(data, off, w, n):
    d = bytes(data.cpu().numpy())
    if w >= 0:
        return [d[i * w:(i + 1) * w] for i in range(n)]
    o = off.cpu().tolist()
    return [d[o[i]:o[i + 1]] for i in range(n)]


def _kmv_rows(kmv):
    keys = _col(kmv.keys.kdata, kmv.keys.koff, kmv.keys.kw, kmv.nkey)
    vals = _col(kmv.vdata, kmv.voff, kmv.vw, kmv.nval)
    seg = kmv.seg.cpu().tolist()
    return [(keys[i], vals[seg[i]:seg[i + 1]]) for i in range(kmv.nkey)]


def test_lookup3_published_vectors():
    # lookup3.c driver5: the reference values of hashlittle
    assert hashlittle_py(b"", 0) == 0xDEADBEEF
    assert hashlittle_py(b"", 0xDEADBEEF) == 0xBD5B7DDE
    assert hashlittle_py(b"Four score and seven years ago", 0) == 0x17770551
    assert hashlittle_py(b"Four score and seven years ago", 1) == 0xCD628161


@pytest.mark.parametrize("dev", DEVS)
def test_hash32_keys_vs_python_lookup3(dev):
    rng = np.random.default_rng(11)
    keys = [b"Four score and seven years ago", b"", b"a"] + \
        [bytes(rng.integers(0, 256, int(rng.integers(1, 40))).astype(np.uint8)) for _ in range(3000)]
    for seed in (0, 1, 0xDEADBEEF):
        kv = _var_kv(keys, [b""] * len(keys), dev)
        got = C.hash32_keys(kv, seed).cpu().numpy().astype(np.int64) & M32
        assert [int(x) for x in got] == [hashlittle_py(k, seed) for k in keys]


# ---------------------------------------------------------------- group-by, reductions, sorts
@pytest.mark.parametrize("dev", DEVS)
def test_convert_vs_python_groupby(dev):
    rng = np.random.default_rng(5)
    n = 60_000
    vocab = [b"k%d_" % i * (1 + i % 5) for i in range(2500)]
    keys = [vocab[i] for i in rng.zipf(1.4, n) % len(vocab)]
    vals = [b"%d" % i for i in range(n)]
    kmv, st = C.convert(_var_kv(keys, vals, dev))
    ref = collections.defaultdict(list)
    for k, v in zip(keys, vals):
        ref[k].append(v)
    got = _kmv_rows(kmv)
    assert len(got) == len(ref) == len(set(keys))
    # each group's values are exactly the key's occurrences (multiset)
    for k, vs in got:
        assert sorted(vs) == sorted(ref[k]), k


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("op", ["sum", "min", "max", "count"])
def test_reduce_builtin_vs_numpy(dev, op):
    rng = np.random.default_rng(7)
    n = 80_000
    k = np.concatenate([rng.integers(0, 3000, n - 4000), np.full(4000, 42)]).astype(np.int64)
    v = rng.integers(-10 ** 6, 10 ** 6, n).astype(np.int64)
    kv = C.make_kv(torch.from_numpy(k), None, torch.from_numpy(v), None, n, "cpu")
    kmv, _ = C.convert(kv if dev == "cpu" else kv.to(dev))
    out = C.reduce_builtin(kmv, op, "int64" if op != "count" else "")
    keys = np.frombuffer(bytes(out.kdata.cpu().numpy()), dtype=np.int64)
    vals = np.frombuffer(bytes(out.vdata.cpu().numpy()), dtype=np.int64 if op != "count" else np.int32)
    if op == "count" and len(vals) != len(keys):
        vals = np.frombuffer(bytes(out.vdata.cpu().numpy()), dtype=np.int64)
    uk = np.unique(k)
    assert sorted(keys.tolist()) == uk.tolist()
    fn = {"sum": np.add, "min": np.minimum, "max": np.maximum}
    order = np.argsort(k, kind="stable")
    ks, vs = k[order], v[order]
    starts = np.flatnonzero(np.r_[True, ks[1:] != ks[:-1]])
    if op == "count":
        ref = np.diff(np.r_[starts, len(ks)])
    else:
        ref = fn[op].reduceat(vs, starts)
    refd = dict(zip(ks[starts].tolist(), ref.tolist()))
    assert {int(a): int(b) for a, b in zip(keys, vals)} == refd


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("flag", [1, -1, 2, 5, -5, 6])
def test_sort_keys_vs_python_sorted(dev, flag):
    rng = np.random.default_rng(abs(flag) + 100)
    n = 30_000
    if abs(flag) == 1:
        kk = rng.integers(-10 ** 6, 10 ** 6, n).astype(np.int32)
        kv = C.make_kv(torch.from_numpy(kk), None, torch.arange(n, dtype=torch.int32), None, n, "cpu")
        ref = sorted(kk.tolist(), reverse=flag < 0)
        decode = lambda b: np.frombuffer(b, dtype=np.int32).tolist()  # noqa: E731
    elif flag == 2:
        kk = rng.integers(0, 2 ** 63, n, dtype=np.int64).astype(np.uint64)
        kv = C.make_kv(torch.from_numpy(kk.view(np.int64)), None, torch.arange(n, dtype=torch.int32), None, n, "cpu")
        ref = sorted(kk.tolist())
        decode = lambda b: np.frombuffer(b, dtype=np.uint64).tolist()  # noqa: E731
    else:
        # URLs sharing a long prefix: ties past 8 bytes on the device path
        words = [b"http://www.example.com/%d/%s\0" % (i, b"x" * int(i % 7)) for i in rng.integers(0, 10 ** 7, n)]
        kv = _var_kv(words, [b"v"] * n, "cpu")
        ref = sorted(words, reverse=flag < 0)
        decode = None
    if dev != "cpu":
        kv = kv.to(dev)
    out = C.sort_kv(kv, flag, False)
    if decode is None:
        got = _col(out.kdata, out.koff, out.kw, out.n)
    else:
        got = decode(bytes(out.kdata.cpu().numpy()))
    assert got == ref


# ---------------------------------------------------------------- graph algorithms vs scipy
def _random_graph(n, m, seed):
    rng = np.random.default_rng(seed)
    e = rng.integers(0, n, (m, 2)).astype(np.int64)
    e = e[e[:, 0] != e[:, 1]]
    # a few isolated chains so there are several components
    return e


@pytest.mark.parametrize("dev", DEVS)
def test_connected_components_vs_scipy(dev):
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components as sp_cc
    from gpu_mapreduce_amd.models.graph import EdgePlan, connected_components
    n, m = 20_000, 18_000  # sparse: many components
    e = _random_graph(n, m, 3)
    both = np.concatenate([e, e[:, ::-1]])
    mr = g.MapReduce(g.Comm(device=dev))
    plan = EdgePlan(mr, torch.from_numpy(both).to(mr.device), n, symmetric=True)
    lab, _ = connected_components(plan)
    lab = lab.cpu().numpy()
    ids = plan.local_ids.cpu().numpy()
    A = coo_matrix((np.ones(len(e)), (e[:, 0], e[:, 1])), shape=(n, n))
    ncomp, comp = sp_cc(A, directed=False)
    # label = smallest vertex id of the component
    minid = np.full(ncomp, n)
    np.minimum.at(minid, comp, np.arange(n))
    ref = minid[comp]
    assert np.array_equal(lab, ref[ids])


@pytest.mark.parametrize("dev", DEVS)
def test_sssp_vs_scipy_dijkstra(dev):
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import dijkstra
    from gpu_mapreduce_amd.models.graph import EdgePlan, sssp
    n, m = 5000, 40_000
    rng = np.random.default_rng(9)
    e = _random_graph(n, m, 9)
    w = rng.uniform(0.5, 10.0, len(e))
    # keep the lightest of parallel edges so scipy's duplicate summing does not differ
    key = e[:, 0] * n + e[:, 1]
    order = np.lexsort((w, key))
    first = np.r_[True, key[order][1:] != key[order][:-1]]
    e, w = e[order][first], w[order][first]
    mr = g.MapReduce(g.Comm(device=dev))
    plan = EdgePlan(mr, torch.from_numpy(e).to(mr.device), n, weights=torch.from_numpy(w).to(mr.device))
    dist, _ = sssp(plan, 0)
    dist = dist.cpu().numpy()
    ids = plan.local_ids.cpu().numpy()
    ref = dijkstra(csr_matrix((w, (e[:, 0], e[:, 1])), shape=(n, n)), directed=True, indices=0)
    np.testing.assert_allclose(dist, ref[ids], rtol=1e-12)


@pytest.mark.parametrize("dev", DEVS)
def test_luby_mis_is_maximal_independent(dev):
    from gpu_mapreduce_amd.models.graph import EdgePlan, luby_mis
    n, m = 10_000, 30_000
    e = _random_graph(n, m, 4)
    both = np.concatenate([e, e[:, ::-1]])
    mr = g.MapReduce(g.Comm(device=dev))
    plan = EdgePlan(mr, torch.from_numpy(both).to(mr.device), n, symmetric=True)
    ins, _ = luby_mis(plan, 12345)
    S = np.zeros(n, bool)
    S[plan.local_ids.cpu().numpy()] = ins.cpu().numpy().astype(bool)
    # independent: no edge inside S
    assert not np.any(S[e[:, 0]] & S[e[:, 1]])
    # maximal: every vertex outside S has a neighbour in S (isolated ones are in S)
    covered = S.copy()
    covered[e[:, 0][S[e[:, 1]]]] = True
    covered[e[:, 1][S[e[:, 0]]]] = True
    assert covered.all()


# ---------------------------------------------------------------- K-means vs numpy Lloyd
@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("D,K", [(2, 16), (64, 32)])
def test_kmeans_step_vs_numpy(dev, D, K):
    from gpu_mapreduce_amd.models.kmeans import KMeans, blobs
    pts = blobs(40_000, D, K, seed=D + K, device="cpu")
    cen = pts[:K].clone()
    km = KMeans(g.Comm(device=dev), pts.to(dev), cen.to(dev))
    km.iterate()
    got = km.centroids.cpu().numpy().astype(np.float64)
    P = pts.numpy().astype(np.float64)
    Cc = cen.numpy().astype(np.float64)
    d2 = (P ** 2).sum(1)[:, None] - 2 * P @ Cc.T + (Cc ** 2).sum(1)[None, :]
    a = d2.argmin(1)
    ref = Cc.copy()
    for k in range(K):
        if (a == k).any():
            ref[k] = P[a == k].mean(0)
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4)
