"""Device functors vs the engine's built-ins on one GPU: n tasks emit
(t % nkey, 1) through a device map functor; collate; the per-key sum by a
device reduce functor and by reduce_builtin("sum") on a copy of the same
groups (results compared). Times each op (device-synchronised, best of 3).

    python tools/devfn_time.py [log2_n=27] [log2_nkey=20]"""
import os
import struct
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpu_mapreduce_amd.parallel.comm import Comm  # noqa: E402
from gpu_mapreduce_amd.runtime.mapreduce import MapReduce  # noqa: E402

ln = int(sys.argv[1]) if len(sys.argv) > 1 else 27
lk = int(sys.argv[2]) if len(sys.argv) > 2 else 20
n, nkey = 1 << ln, 1 << lk
MAP = f"""
__device__ void mr_map(mrd::Bytes key, mrd::Bytes value, long long t, mrd::Emit& out) {{
  unsigned long long h = (unsigned long long)t * 0x9E3779B97F4A7C15ull;
  out.emit((long long)((h >> 20) & {nkey - 1}ull), (int)1);
}}
"""
RED = """
__device__ void mr_reduce(mrd::Bytes key, mrd::Values vals, mrd::Emit& out) {
  int s = 0;
  for (long long i = 0; i < vals.n; ++i) s += vals.get<int>(i);
  out.emit(key.as<long long>(), s);
}
"""
FOLD = """
struct mr_acc { int s; };
__device__ void mr_init(mrd::Bytes key, mr_acc& a) { a.s = 0; }
__device__ void mr_add(mr_acc& a, mrd::Bytes v) { a.s += v.as<int>(); }
__device__ void mr_merge(mr_acc& a, const mr_acc& b) { a.s += b.s; }
__device__ void mr_finish(mrd::Bytes key, const mr_acc& a, mrd::Emit& out) { out.emit(key.as<long long>(), a.s); }
"""
comm = Comm(device="cuda")


def timed(f):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = f()
    torch.cuda.synchronize()
    return r, (time.perf_counter() - t0) * 1e3


best = {}
for rep in range(4):
    mr = MapReduce(comm)
    _, tm = timed(lambda: mr.map_device(n, MAP))
    _, tc = timed(lambda: mr.collate())
    mr2 = mr.copy()
    mr3 = mr.copy()
    _, tf = timed(lambda: mr3.reduce_device(FOLD))
    _, tr = timed(lambda: mr.reduce_device(RED))
    _, tb = timed(lambda: mr2.reduce_builtin("sum:int32") if False else mr2._m.reduce_builtin("sum", "int32"))
    if rep == 0:  # compile + first-touch warm-up; check the two reduces agree
        a, b = {}, {}
        mr.scan_kv(lambda k, v: a.__setitem__(k, struct.unpack("<i", v)[0]))
        mr2.scan_kv(lambda k, v: b.__setitem__(k, struct.unpack("<i", v)[0]))
        c = {}
        mr3.scan_kv(lambda k, v: c.__setitem__(k, struct.unpack("<i", v)[0]))
        assert a == b == c and sum(a.values()) == n, "device reduce / fold != builtin reduce"
        print(f"n = 2^{ln} pairs, {len(a)} keys; device reduce == device fold == reduce_builtin('sum')", flush=True)
        continue
    for k, v in (("map_device", tm), ("collate", tc), ("reduce_device", tr), ("reduce_device_fold", tf), ("reduce_builtin", tb)):
        best[k] = min(best.get(k, 1e30), v)
for k, v in best.items():
    print(f"{k:16s} {v:8.2f} ms  {n / (v * 1e-3) / 1e9:7.2f} G pairs/s", flush=True)
