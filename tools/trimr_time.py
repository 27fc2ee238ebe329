"""tri_find_mr (the 4-collate MapReduce pipeline) on one R-MAT graph, twice
(the second run is warm); prints the per-stage times of each run."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpu_mapreduce_amd as g  # noqa: E402
from gpu_mapreduce_amd import C  # noqa: E402
from gpu_mapreduce_amd.models.pagerank import GRAPH500  # noqa: E402
from gpu_mapreduce_amd.models.triangles import tri_find_mr  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 20
comm = g.Comm(device=os.environ.get("DEV", "cuda:0"))
kv = C.map_rmat((1 << scale) * 16, scale, *GRAPH500, 0.0, 1, 0, comm.device)
e = kv.kdata.view(torch.int64).view(-1, 2)
for rep in range(2):
    r = tri_find_mr(comm, e)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    tot = sum(s["ms"] for s in r["stages"])
    print(f"rep {rep}: {tot:.1f} ms, {r['triangles']} triangles", flush=True)
    if torch.cuda.is_available():
        from gpu_mapreduce_amd.runtime import hbm_pool
        print("   pool:", hbm_pool.stats(0), flush=True)
    for s in r["stages"]:
        print(f"   {s['op']:<24} {s['ms']:9.2f} ms  in {s['pairs_in']:>12}  out {s['pairs_out']:>12}", flush=True)
