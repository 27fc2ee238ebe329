"""TriangleGraph fast build path (nv given, GPU) vs CPU at small scales, with
a stack dump if a step hangs."""
import faulthandler
import sys
import time

import torch

sys.path.insert(0, ".")
import gpu_mapreduce_amd as g  # noqa: E402
from gpu_mapreduce_amd._ext import C  # noqa: E402
from gpu_mapreduce_amd.models.pagerank import GRAPH500  # noqa: E402
from gpu_mapreduce_amd.models.triangles import TriangleGraph  # noqa: E402

faulthandler.dump_traceback_later(60, exit=True)
for scale in (8, 12, 16, 20, 24):
    t0 = time.time()
    kv = C.map_rmat((1 << scale) * 16, scale, *GRAPH500, 0.0, 1, 0, "cuda")
    e = kv.kdata.view(torch.int64).view(-1, 2)
    if scale == 8:
        print("old path (nv=None)", TriangleGraph(g.Comm(device="cuda"), e).count(), flush=True)
    tg = TriangleGraph(g.Comm(device="cuda"), e, 1 << scale)
    torch.cuda.synchronize()
    print("scale", scale, "built", tg.nedge, round(time.time() - t0, 2), flush=True)
    n = tg.count()
    print("scale", scale, "count", n, round(time.time() - t0, 2), flush=True)
    if scale <= 16:
        ref = TriangleGraph(g.Comm(device="cpu"), e.cpu(), 1 << scale).count()
        print("  cpu", ref, "match", ref == n, flush=True)
