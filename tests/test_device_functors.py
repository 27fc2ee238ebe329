"""Device functors (csrc/engine/devfn.cpp): user map / reduce HIP device code
compiled at run time (hiprtc, gfx950) into the engine's two-pass emit kernels.
Compilation (and its error reporting) is checked without a GPU; the runs
(map over tasks and over pairs, reduce after collate, compress) are checked
against Python oracles on the GPU."""
import collections
import struct

import numpy as np
import pytest

from gpu_mapreduce_amd import C

SUM_I32 = r"""
__device__ void mr_reduce(mrd::Bytes key, mrd::Values vals, mrd::Emit& out) {
  long long s = 0;
  for (long long i = 0; i < vals.n; ++i) s += vals.get<int>(i);
  out.emit(key.as<long long>(), s);
}
"""

GEN = r"""
// task t -> (t % 97, 1) and, for every 5th task, a second pair (t % 89 + 1000, 2)
__device__ void mr_map(mrd::Bytes key, mrd::Bytes value, long long t, mrd::Emit& out) {
  out.emit((long long)(t % 97), (int)1);
  if (t % 5 == 0) out.emit((long long)(t % 89 + 1000), (int)2);
}
"""

# var-width keys: every word of the value text, with the word's length as value
WORDS = r"""
__device__ void mr_map(mrd::Bytes key, mrd::Bytes value, long long index, mrd::Emit& out) {
  long long i = 0;
  while (i < value.n) {
    while (i < value.n && value.p[i] == ' ') ++i;
    long long j = i;
    while (j < value.n && value.p[j] != ' ') ++j;
    if (j > i) { int len = (int)(j - i); out.emit(value.p + i, j - i, &len, 4); }
    i = j;
  }
}
"""


def test_functor_compiles_and_reports_errors():
    assert C.device_functor_check(SUM_I32, True) > 0
    assert C.device_functor_check(GEN, False) > 0
    src = C.device_functor_source(SUM_I32, True)
    assert "#define MRD_REDUCE 1" in src and "mr_reduce" in src and "mrd_count" in src
    with pytest.raises(RuntimeError, match="does not compile"):
        C.device_functor_check("__device__ void mr_map(int x) { return 1; }", False)
    with pytest.raises(RuntimeError, match="mr_reduce"):  # a map functor where a reduce is expected
        C.device_functor_check(GEN, True)


def test_functor_needs_a_gpu_mapreduce():
    from gpu_mapreduce_amd.parallel.comm import Comm
    from gpu_mapreduce_amd.runtime.mapreduce import MapReduce
    mr = MapReduce(Comm(device="cpu"))
    with pytest.raises(RuntimeError, match="GPU MapReduce"):
        mr.map_device(10, GEN)


def pairs(mr):
    out = []
    mr.scan_kv(lambda k, v: out.append((bytes(k), bytes(v))))
    return out


@pytest.mark.gpu
def test_functor_map_tasks_collate_reduce():
    from gpu_mapreduce_amd.parallel.comm import Comm
    from gpu_mapreduce_amd.runtime.mapreduce import MapReduce
    n = 200_000
    mr = MapReduce(Comm(device="cuda"))
    assert mr.map_device(n, GEN) == n + (n + 4) // 5
    assert mr.kv.kw == 8 and mr.kv.vw == 4  # uniform widths -> fixed-width columns
    mr.collate()
    assert mr.reduce_device(SUM_I32) == 97 + 89
    got = {struct.unpack("<q", k)[0]: struct.unpack("<q", v)[0] for k, v in pairs(mr)}
    t = np.arange(n)
    want = collections.Counter((t % 97).tolist())
    for x in t[t % 5 == 0]:
        want[int(x % 89 + 1000)] += 2
    assert got == dict(want)


@pytest.mark.gpu
def test_functor_map_pairs_var_width_and_compress():
    from gpu_mapreduce_amd.parallel.comm import Comm
    from gpu_mapreduce_amd.runtime.mapreduce import MapReduce
    rng = np.random.default_rng(1)
    vocab = ["a", "bb", "ccc", "dddd", "eeeee", "ff", "g" * 17]
    lines = [" ".join(rng.choice(vocab, size=rng.integers(0, 12))) for _ in range(3000)]
    comm = Comm(device="cuda")
    src = MapReduce(comm)

    def m(itask, kv):
        for i, ln in enumerate(lines):
            kv.add(struct.pack("<q", i), ln.encode())
    src.map(1, m)
    mr = MapReduce(comm)
    nw = mr.map_device(src, WORDS)
    want = collections.Counter(w for ln in lines for w in ln.split())
    assert nw == sum(want.values())
    assert mr.kv.kw == -1 and mr.kv.vw == 4  # words: variable keys, int values
    mr.compress_device(r"""
__device__ void mr_reduce(mrd::Bytes key, mrd::Values vals, mrd::Emit& out) {
  long long s = 0;
  for (long long i = 0; i < vals.n; ++i) s += vals.get<int>(i);
  out.emit(key.p, key.n, &s, 8);
}
""")
    got = {k.decode(): struct.unpack("<q", v)[0] for k, v in pairs(mr)}
    assert got == {w: c * len(w) for w, c in want.items()}


# the fold tier: an accumulator per chunk of values (one thread per chunk),
# merged per key, finished per key — hot keys spread over the whole GPU
FOLD = r"""
struct mr_acc { long long s; long long n; int mn; int mx; };
__device__ void mr_init(mrd::Bytes key, mr_acc& a) { a.s = 0; a.n = 0; a.mn = 2147483647; a.mx = -2147483647 - 1; }
__device__ void mr_add(mr_acc& a, mrd::Bytes v) {
  const int x = v.as<int>();
  a.s += x; a.n += 1; a.mn = x < a.mn ? x : a.mn; a.mx = x > a.mx ? x : a.mx;
}
__device__ void mr_merge(mr_acc& a, const mr_acc& b) {
  a.s += b.s; a.n += b.n; a.mn = b.mn < a.mn ? b.mn : a.mn; a.mx = b.mx > a.mx ? b.mx : a.mx;
}
__device__ void mr_finish(mrd::Bytes key, const mr_acc& a, mrd::Emit& out) {
  long long r[4] = {a.s, a.n, a.mn, a.mx};
  out.emit(key.p, key.n, r, 32);
}
"""

HOT = r"""
// task t -> key (t % 3 == 0 ? 0 : t % 1000), value t % 1009 - 500: key 0 holds a third of all pairs
__device__ void mr_map(mrd::Bytes key, mrd::Bytes value, long long t, mrd::Emit& out) {
  out.emit((long long)(t % 3 == 0 ? 0 : t % 1000), (int)(t % 1009 - 500));
}
"""


def test_fold_functor_compiles():
    assert C.device_functor_check(FOLD, True) > 0
    assert "#define MRD_REDUCE 2" in C.device_functor_source(FOLD, True)


@pytest.mark.gpu
@pytest.mark.parametrize("compress", [False, True])
def test_fold_functor_hot_keys(compress):
    from gpu_mapreduce_amd.parallel.comm import Comm
    from gpu_mapreduce_amd.runtime.mapreduce import MapReduce
    n = 3_000_000
    mr = MapReduce(Comm(device="cuda"))
    mr.map_device(n, HOT)
    if compress:
        mr.compress_device(FOLD)
    else:
        mr.collate()
        mr.reduce_device(FOLD)
    got = {struct.unpack("<q", k)[0]: struct.unpack("<4q", v) for k, v in pairs(mr)}
    t = np.arange(n)
    key = np.where(t % 3 == 0, 0, t % 1000)
    val = t % 1009 - 500
    want = {}
    for k in np.unique(key):
        v = val[key == k]
        want[int(k)] = (int(v.sum()), len(v), int(v.min()), int(v.max()))
    assert got == want


def test_compress_batch_is_a_local_combiner():
    """compress_batch: this rank's groups as one KMV, no shuffle (the engine op
    under sssp_mr's combiners); on the CPU engine too"""
    import torch
    from gpu_mapreduce_amd.parallel.comm import Comm
    from gpu_mapreduce_amd.runtime.mapreduce import MapReduce
    mr = MapReduce(Comm(device="cpu"))

    def m(itask, kv):
        for i in range(1000):
            kv.add(struct.pack("<q", i % 37), struct.pack("<i", i))
    mr.map(1, m)
    seen = {}

    def f(kmv, kv):
        keys = kmv.keys.kdata.view(torch.int64)
        seg = kmv.seg
        vals = kmv.vdata.view(torch.int32)
        sums = torch.stack([vals[seg[i]:seg[i + 1]].sum() for i in range(kmv.nkey)]).to(torch.int64)
        seen["nkey"] = kmv.nkey
        kv.add_tensors(keys, sums)
    assert mr.compress_batch(f) == 37
    assert seen["nkey"] == 37
    got = {}
    mr.scan_kv(lambda k, v: got.__setitem__(struct.unpack("<q", k)[0], struct.unpack("<q", v)[0]))
    assert got == {k: sum(i for i in range(1000) if i % 37 == k) for k in range(37)}


@pytest.mark.gpu
def test_functors_out_of_core(tmp_path):
    """under an HBM budget ~1/20 of the data the map's output spools and the
    collate / compress groups reach the functors in budget-sized pieces; the
    fold totals must still equal the oracle's"""
    from gpu_mapreduce_amd.parallel.comm import Comm
    from gpu_mapreduce_amd.runtime.mapreduce import MapReduce
    n = 4_000_000
    data = n * 12
    for op in ("reduce", "compress"):
        mr = MapReduce(Comm(device="cuda"))
        mr.hbm_budget = data // 20
        mr.host_budget = data // 4
        mr.memsize = -65536
        mr.fpath = str(tmp_path)
        mr.map_device(n, HOT)
        if op == "compress":
            mr.compress_device(FOLD)
        else:
            mr.collate()
            mr.reduce_device(FOLD)
        got = {struct.unpack("<q", k)[0]: struct.unpack("<4q", v) for k, v in pairs(mr)}
        t = np.arange(n)
        key = np.where(t % 3 == 0, 0, t % 1000)
        val = t % 1009 - 500
        assert len(got) == 1000
        for k in (0, 1, 500, 999):
            v = val[key == k]
            assert got[k] == (int(v.sum()), len(v), int(v.min()), int(v.max())), (op, k)


@pytest.mark.gpu
def test_python_example_runs():
    """examples/python/device_functors.py (map + fold functors) end to end"""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "examples", "python", "device_functors.py"), "2000000", "64"],
                       env=dict(os.environ, PYTHONPATH=root), capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "2000000 pairs, 64 buckets, total count 2000000" in p.stdout


# sort-key functor: (b descending, then a ascending) of a pair of int32 keys
SORTKEY = r"""
__device__ unsigned long long mr_sortkey(mrd::Bytes k) {
  const unsigned int a = (unsigned int)k.as<int>(0) ^ 0x80000000u;   // signed -> unsigned order
  const unsigned int b = (unsigned int)k.as<int>(4) ^ 0x80000000u;
  return ((unsigned long long)(~b) << 32) | a;
}
"""


def test_sortkey_functor_compiles():
    assert C.device_sortkey_check(SORTKEY) > 0
    with pytest.raises(RuntimeError, match="does not compile"):
        C.device_sortkey_check("__device__ int mr_sortkey(int) { return x; }")


@pytest.mark.gpu
def test_sort_keys_device_composite_and_stable():
    from gpu_mapreduce_amd.parallel.comm import Comm
    from gpu_mapreduce_amd.runtime.mapreduce import MapReduce
    rng = np.random.default_rng(7)
    n = 200_000
    a = rng.integers(-50, 50, n).astype(np.int32)
    b = rng.integers(-20, 20, n).astype(np.int32)
    mr = MapReduce(Comm(device="cuda"))

    def m(itask, kv):
        kv.add_multi_static([struct.pack("<ii", int(x), int(y)) for x, y in zip(a, b)],
                            [struct.pack("<q", i) for i in range(n)])
    mr.map(1, m)
    assert mr.sort_keys_device(SORTKEY) == n
    got = [(struct.unpack("<ii", k), struct.unpack("<q", v)[0]) for k, v in pairs(mr)]
    want = sorted(((int(x), int(y)), i) for i, (x, y) in enumerate(zip(a, b)))
    want.sort(key=lambda r: (-r[0][1], r[0][0]))  # stable: equal keys keep input order (i ascending)
    assert got == want
    # by value: the int64 row index descending
    mr.sort_values_device("__device__ unsigned long long mr_sortkey(mrd::Bytes v) { return ~(unsigned long long)v.as<long long>(); }")
    got = [struct.unpack("<q", v)[0] for _, v in pairs(mr)]
    assert got == list(range(n - 1, -1, -1))
