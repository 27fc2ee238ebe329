"""Why reduce_builtin on a collated device-functor output (1024 keys) runs
~3 ms when the same shape from C.convert runs 0.25 ms: time C.reduce_builtin
on the MR's own KMV, on a contiguous copy of it, and print its layout.

    python tools/segred_mr_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpu_mapreduce_amd import C  # noqa: E402
from gpu_mapreduce_amd.parallel.comm import Comm  # noqa: E402
from gpu_mapreduce_amd.runtime.mapreduce import MapReduce  # noqa: E402

n, nkey = 1 << 27, 1 << 10
MAP = f"""
__device__ void mr_map(mrd::Bytes key, mrd::Bytes value, long long t, mrd::Emit& out) {{
  unsigned long long h = (unsigned long long)t * 0x9E3779B97F4A7C15ull;
  out.emit((long long)((h >> 20) & {nkey - 1}ull), (int)1);
}}
"""
mr = MapReduce(Comm(device="cuda"))
mr.map_device(n, MAP)
mr.collate()
m = mr.kmv
print("nkey", m.nkey, "nval", m.nval, "vw", m.vw, "vdata", tuple(m.vdata.shape), m.vdata.stride(), m.vdata.dtype,
      "contig", m.vdata.is_contiguous(), "storage_offset", m.vdata.storage_offset(),
      "seg", tuple(m.seg.shape), m.seg.is_contiguous(), flush=True)
seg = m.seg.cpu()
lens = (seg[1:] - seg[:-1])
print("segment lengths min/max", int(lens.min()), int(lens.max()), flush=True)


def t(kmv, label):
    best = 1e30
    for _ in range(6):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        C.reduce_builtin(kmv, "sum", "int32")
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b))
    print(f"{label:24s} {best:7.3f} ms", flush=True)


t(m, "MR kmv")
m2 = C.KMV()
m2.keys, m2.vdata, m2.voff, m2.vw, m2.seg, m2.nkey, m2.nval = m.keys, m.vdata.clone(), m.voff, m.vw, m.seg.clone(), m.nkey, m.nval
t(m2, "cloned vdata + seg")
