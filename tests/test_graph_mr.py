"""sssp_mr and luby_find_mr: the reference's MapReduce formulations of
single-source shortest paths (oink/sssp.cpp:49-184) and of Luby's maximal
independent set (oink/luby_find.cpp:53-97) as OINK commands, their
callbacks as device kernels (csrc/kernels/graphmr.hip) on cuda and host twins
on cpu.

Oracles: scipy's Dijkstra (distances and, with random real weights, the
unique predecessors) and the greedy MIS in the reference's (drand48 after
srand48(v + seed), v) order, which Luby's rounds with fixed priorities
produce exactly — so the MIS is the set the reference's command prints for
the same seed."""
import io
import re

import numpy as np
import pytest

from gpu_mapreduce_amd.oink.interp import OINK


def run(script, tmp_path, monkeypatch, comm=None):
    monkeypatch.chdir(tmp_path)
    out = io.StringIO()
    o = OINK(comm, screen=out, logfile="log.oink")
    o.file(text=script)
    return out.getvalue()


def comm_for(dev):
    if dev == "cpu":
        return None
    from gpu_mapreduce_amd.parallel.comm import Comm
    return Comm(device=dev)


def weighted_graph(tmp_path, n, m, seed):
    """m distinct directed edges without self loops, random real weights"""
    rng = np.random.default_rng(seed)
    a = rng.integers(1, n, size=4 * m)
    b = rng.integers(1, n, size=4 * m)
    k = a != b
    e = np.unique(np.stack([a[k], b[k]], 1), axis=0)
    e = e[rng.permutation(len(e))[:m]]
    w = rng.uniform(0.25, 4.0, size=len(e))
    with open(tmp_path / "graph.w", "w") as f:
        for (x, y), z in zip(e, w):
            f.write(f"{x} {y} {float(z)!r}\n")
    return e, w


def parse_sources(text):
    return [(int(s), int(i), int(c)) for s, i, c in
            re.findall(r"Source = (\d+); Iterations = (\d+); Num Vtx Labeled = (\d+)", text)]


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_sssp_mr_matches_dijkstra(tmp_path, monkeypatch, dev):
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import dijkstra
    n = 200 if dev == "cpu" else 3000
    e, w = weighted_graph(tmp_path, n, 4 * n, 5)
    s = ("sssp_mr 3 777 -i graph.w -o tmp.ssspmr NULL\n"
         "sssp 3 777 -i graph.w -o tmp.sssp NULL\n")
    text = run(s, tmp_path, monkeypatch, comm_for(dev))
    lines = text.splitlines()
    mr_text = "\n".join(lines[:[i for i, ln in enumerate(lines) if "Total time in SSSP" in ln][0] + 1])
    mr_src, plan_src = parse_sources(mr_text), parse_sources(text)[3:]
    assert len(mr_src) == 3 and [x[0] for x in mr_src] == [x[0] for x in plan_src]
    assert [x[2] for x in mr_src] == [x[2] for x in plan_src]
    assert all(it > 2 for _, it, _ in mr_src)
    G = csr_matrix((w, (e[:, 0], e[:, 1])), shape=(n, n))
    rows = np.loadtxt(tmp_path / "tmp.ssspmr.0", ndmin=2)
    assert sum(c for _, _, c in mr_src) == len(rows)
    start = 0
    for src, _, cnt in mr_src:
        r = rows[start:start + cnt]
        start += cnt
        d, pred = dijkstra(G, indices=src, return_predecessors=True)
        got = {int(v): (dv, int(pv)) for v, dv, pv in r}
        assert set(got) == {i for i in range(n) if np.isfinite(d[i])}
        for v, (dv, pv) in got.items():
            assert dv == pytest.approx(d[v], rel=1e-5)
            assert pv == (0 if v == src else pred[v]), (v, pv, pred[v])


def drand48_after_srand48(v, seed):
    x0 = (((v + seed) & 0xFFFFFFFF) << 16) | 0x330E
    return ((0x5DEECE66D * x0 + 0xB) & ((1 << 48) - 1)) / float(1 << 48)


def greedy_mis(e, seed):
    nb = {}
    for a, b in e:
        if a == b:
            continue
        nb.setdefault(int(a), set()).add(int(b))
        nb.setdefault(int(b), set()).add(int(a))
    order = sorted(nb, key=lambda v: (drand48_after_srand48(v, seed), v))
    mis = set()
    for v in order:
        if not nb[v] & mis:
            mis.add(v)
    return mis, nb


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("upper", [True, False])
def test_luby_find_mr_is_greedy_mis(tmp_path, monkeypatch, dev, upper):
    scale = 8 if dev == "cpu" else 12
    s = (f"rmat {scale} 4 0.25 0.25 0.25 0.25 0.0 12345 -o tmp.rmat mre\n"
         + ("edge_upper -i mre -o NULL mre\n" if upper else "")
         + "luby_find_mr 4321 -i mre -o tmp.mis NULL\n")
    text = run(s, tmp_path, monkeypatch, comm_for(dev))
    e = np.loadtxt(tmp_path / "tmp.rmat.0", dtype=np.int64, ndmin=2)
    want, nb = greedy_mis(e, 4321)
    got = set(np.loadtxt(tmp_path / "tmp.mis.0", dtype=np.int64, ndmin=1).tolist())
    assert got == want
    m = re.search(r"Luby_find: (\d+) MIS vertices in (\d+) iterations", text)
    assert m and int(m.group(1)) == len(want) and int(m.group(2)) >= 1
    for v, ns in nb.items():  # independent and maximal
        assert not (v in got and ns & got)
        assert v in got or ns & got


def test_graph_mr_callbacks_host_twin_edge_cases():
    """the callbacks' semantic corners on hand-built groups (cpu twins)"""
    import torch
    from gpu_mapreduce_amd.runtime.mapreduce import MapReduce
    FLT = 3.4028234663852886e38

    def dist(pred, wt, cur):
        return np.array([pred, np.float64(wt).view(np.int64), cur], dtype=np.int64)

    mr = MapReduce()
    # vertex 5: own record (current, unreached) + two candidates, the later one shorter
    # vertex 6: own record only (unchanged); vertex 7: own record 2.0 + a tie at 2.0
    recs = [(5, dist(0, FLT, 1)), (5, dist(9, 3.0, 0)), (5, dist(8, 1.5, 0)),
            (6, dist(4, 2.5, 1)), (7, dist(3, 2.0, 1)), (7, dist(1, 2.0, 0))]

    def m(itask, kv):
        for k, v in recs:
            kv.add(np.int64(k).tobytes(), v.tobytes())
    mr.map(1, m)
    picked = {}

    def pick(kmv, kv):
        from gpu_mapreduce_amd import C
        p = C.ssspmr_pick(kmv)
        keys = kmv.keys.kdata.view(torch.int64).tolist()
        for k, d in zip(keys, p[0].tolist()):
            picked[k] = d
        picked["changed"] = p[1].tolist()
    mr.compress_batch(pick)
    assert picked[5] == [8, int(np.float64(1.5).view(np.int64)), 1]
    assert picked[6] == [4, int(np.float64(2.5).view(np.int64)), 1]
    assert picked[7] == [3, int(np.float64(2.0).view(np.int64)), 1]  # the own record wins a tie
    assert picked["changed"] == [5]


@pytest.mark.gpu
def test_graph_mr_commands_out_of_core(tmp_path, monkeypatch):
    """sssp_mr and luby_find_mr under a 128 KiB HBM budget (8 pages of 16 KiB):
    their aggregates, appends and compress / reduce groups go through the
    out-of-core paths; the results must not change"""
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import dijkstra
    n = 3000
    e, w = weighted_graph(tmp_path, n, 4 * n, 5)
    s = ("set memsize -16384 maxpage 8\n"
         "sssp_mr 2 777 -i graph.w -o tmp.ssspmr NULL\n"
         "rmat 12 4 0.25 0.25 0.25 0.25 0.0 12345 -o tmp.rmat mre\n"
         "edge_upper -i mre -o NULL mre\n"
         "luby_find_mr 4321 -i mre -o tmp.mis NULL\n")
    text = run(s, tmp_path, monkeypatch, comm_for("cuda"))
    src = parse_sources(text)
    G = csr_matrix((w, (e[:, 0], e[:, 1])), shape=(n, n))
    rows = np.loadtxt(tmp_path / "tmp.ssspmr.0", ndmin=2)
    start = 0
    for s0, _, cnt in src:
        r = rows[start:start + cnt]
        start += cnt
        d = dijkstra(G, indices=s0)
        got = {int(v): dv for v, dv, _ in r}
        assert set(got) == {i for i in range(n) if np.isfinite(d[i])}
        assert all(got[v] == pytest.approx(d[v], rel=1e-5) for v in got)
    ed = np.loadtxt(tmp_path / "tmp.rmat.0", dtype=np.int64, ndmin=2)
    want, _ = greedy_mis(ed, 4321)
    assert set(np.loadtxt(tmp_path / "tmp.mis.0", dtype=np.int64, ndmin=1).tolist()) == want


@pytest.mark.gpu
def test_oink_device_functor_methods(tmp_path, monkeypatch):
    """the OINK MR methods for device functors (map/mr/device, reduce/device,
    compress/device, sort_values/device): out-degrees of an R-MAT graph,
    largest first, against numpy"""
    (tmp_path / "src.hip").write_text(
        "__device__ void mr_map(mrd::Bytes k, mrd::Bytes v, long long i, mrd::Emit& out) {\n"
        "  out.emit(k.as<long long>(0), (int)1);\n}\n")
    (tmp_path / "sum.hip").write_text(
        "struct mr_acc { long long n; };\n"
        "__device__ void mr_init(mrd::Bytes k, mr_acc& a) { a.n = 0; }\n"
        "__device__ void mr_add(mr_acc& a, mrd::Bytes v) { a.n += v.as<int>(); }\n"
        "__device__ void mr_merge(mr_acc& a, const mr_acc& b) { a.n += b.n; }\n"
        "__device__ void mr_finish(mrd::Bytes k, const mr_acc& a, mrd::Emit& out) {"
        " out.emit(k.as<long long>(), a.n); }\n")
    (tmp_path / "desc.hip").write_text(
        "__device__ unsigned long long mr_sortkey(mrd::Bytes v) { return ~(unsigned long long)v.as<long long>(); }\n")
    s = ("rmat 10 8 0.25 0.25 0.25 0.25 0.0 12345 -o tmp.rmat mre\n"
         "mre map/mr/device mre src.hip\n"
         "mre compress/device sum.hip\n"
         "mre collate NULL\n"
         "mre reduce/device sum.hip\n"
         "mre sort_values/device desc.hip\n"
         "mre print tmp.deg 0 0 1 2 2\n")
    run(s, tmp_path, monkeypatch, comm_for("cuda"))
    e = np.loadtxt(tmp_path / "tmp.rmat.0", dtype=np.int64, ndmin=2)
    deg = np.bincount(e[:, 0])
    lines = [ln for ln in (tmp_path / "tmp.deg").read_text().splitlines() if ln.startswith("KV pair")]
    got = [(int(ln.split("key ")[1].split(",")[0]), int(ln.split("value ")[1])) for ln in lines]
    assert dict(got) == {v: int(d) for v, d in enumerate(deg) if d}
    counts = [c for _, c in got]
    assert counts == sorted(counts, reverse=True)
