"""PageRank graph replay vs plain steps at growing scales (equality of the
ranks), default XCD ranges; stops at the first mismatch."""
import sys

import torch

sys.path.insert(0, ".")
import gpu_mapreduce_amd as g  # noqa: E402
from gpu_mapreduce_amd.models.pagerank import PageRank, rmat_map  # noqa: E402

for scale in [int(x) for x in sys.argv[1:]] or [22, 24, 26]:
    mr = g.MapReduce(g.Comm(device="cuda"))
    rmat_map(mr, scale, 16, seed=1)
    pr = PageRank(mr, 1 << scale).build()
    del mr
    pr.use_graph = False
    pr.reset()
    pr.run(20)
    _, a = pr.ranks()
    a = a.clone()
    torch.cuda.synchronize()
    print("scale", scale, "plain done, xcd ranges", pr.xcd_ranges, flush=True)
    pr.use_graph = True
    pr.reset()
    pr.run(20)
    torch.cuda.synchronize()
    _, b = pr.ranks()
    print("scale", scale, "graph done, equal", bool(torch.equal(a, b)), "graph iters", pr.graph_iterations, flush=True)
    del pr
    torch.cuda.empty_cache()
