"""Work counts of the tri_find hub sub-problem on RMAT-<scale> (one GPU).

For the oriented hub subgraph (top K ranks): sum_u C(d+(u), 2) (elements a
'stream N+(u) past v, test against a bitmap of N+(v)' kernel reads), sum over
hub edges (u, v) of d+(v) (a 'bitmap of N+(u), stream N+(v)' kernel), the
edge count and the d+ distribution.
usage: python tools/tri_hub_stats.py [scale]"""
import sys

import torch

sys.path.insert(0, ".")
import gpu_mapreduce_amd as g  # noqa: E402
from gpu_mapreduce_amd._ext import C  # noqa: E402
from gpu_mapreduce_amd.models.pagerank import GRAPH500  # noqa: E402
from gpu_mapreduce_amd.models.triangles import TriangleGraph  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
comm = g.Comm(device="cuda")
kv = C.map_rmat((1 << scale) * 16, scale, *GRAPH500, 0.0, 1, 0, "cuda")
edges = kv.kdata.view(torch.int64).view(-1, 2)
tg = TriangleGraph(comm, edges, 1 << scale)
rp, col = tg.rowptr, tg.col.long()
n = rp.numel() - 1
d = (rp[1:] - rp[:-1])
for K in (n // 32, n // 64, n // 128):
    hb = n - K
    dh = d[hb:].double()
    e0 = int(rp[hb])
    hu = torch.repeat_interleave(torch.arange(hb, n, device="cuda"), d[hb:])
    hv = col[e0:]
    pairs = float((dh * (dh - 1) / 2).sum())
    old = float(d[hv].double().sum())
    # elements of N+(u) after v, summed over hub edges == pairs (check)
    print(f"K={K} hub_edges={int(rp[n]) - e0} nonhub_edges={e0} sum_C(d+,2)={pairs:.4g} "
          f"sum_edges_d+(v)={old:.4g} d+ max={int(dh.max())} "
          f"p50/p90/p99={[float(x) for x in torch.quantile(dh[dh > 0][:16000000], torch.tensor([.5, .9, .99], device='cuda', dtype=torch.float64))]}")
    del hu, hv
# the non-hub part with K = n/32: wave-hash work = sum over edges (u,v), u < hb, of d+(v) cut
