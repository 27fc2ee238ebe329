#!/usr/bin/env python3
"""One-rank RCCL loopback check (MRH_FORCE_RCCL=2, csrc/engine/comm.h): the
multi-GPU code paths with every collective going through its nccl* call.

usage: rccl_loopback.py MODE OUT_PREFIX
  MODE: local (no communicator), force1 (send/recv through RCCL, collectives
  the identity), force2 (every collective through RCCL), force2_eager (force2
  with the PageRank iteration kept eager: MRH_PR_DIST_GRAPH=0).
Writes OUT_PREFIX.npz (PageRank ranks, tri_find counts, wordfreq top-10) and
prints one JSON line: transport, counters per nccl* entry point after each
workload, PageRank replayed iterations. Run by tests/test_rccl_loopback_gpu.py
(reference collectives it stands in for: src/mapreduce.cpp:539, 597-605;
src/irregular.cpp:111-178)."""
import json
import os
import sys

MODE, OUT = sys.argv[1], sys.argv[2]
os.environ["MRH_FORCE_RCCL"] = {"local": "0", "force1": "1", "force2": "2", "force2_eager": "2"}[MODE]
if MODE == "force2_eager":
    os.environ["MRH_PR_DIST_GRAPH"] = "0"
os.environ["MRH_PR_L2_BYTES"] = "65536"   # several XCD source ranges at RMAT-18
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gpu_mapreduce_amd as g  # noqa: E402
from gpu_mapreduce_amd import C  # noqa: E402
from gpu_mapreduce_amd.models.pagerank import GRAPH500, PageRank, rmat_map  # noqa: E402
from gpu_mapreduce_amd.models.triangles import TriangleGraph, tri_find_mr  # noqa: E402
from gpu_mapreduce_amd.models.wordfreq import WordFreq  # noqa: E402
from gpu_mapreduce_amd.utils import synth  # noqa: E402

C.rccl_counters_reset()
comm = g.Comm(device="cuda")
rec = {"mode": MODE, "transport": comm.native.transport, "loopback": bool(comm.native.loopback_collectives)}
out = {}


def snap(tag):
    torch.cuda.synchronize()
    rec["counters_" + tag] = dict(C.rccl_counters())


# 1. PageRank RMAT-18: the replicated plan (source pieces, side-stream rounds,
#    stats allreduce) with HIP-graph replay; a 20-run after reset, then a 7-run
mr = g.MapReduce(comm)
rmat_map(mr, 18, 16, seed=7)
pr = PageRank(mr, 1 << 18).build()
for it in (20, 7):
    pr.reset()
    pr.run(it)
ids, r = pr.ranks()
pranks = np.zeros(1 << 18, dtype=np.float32)
pranks[ids.cpu().numpy()] = r.cpu().numpy()
out["pagerank"] = pranks
rec["pr_graph_iters"] = int(pr.graph_iterations)
rec["pr_layout"] = pr.layout
del pr, mr
snap("pagerank")

# 2. tri_find: the split build on a distributed communicator (allreduces of
#    the build, the count's allreduce); RMAT-16
e = C.map_rmat((1 << 16) * 16, 16, *GRAPH500, 0.0, 11, 0, "cuda").kdata.view(torch.int64).view(-1, 2)
tg = TriangleGraph(comm, e, 1 << 16)
out["trifind"] = np.array([tg.count()], dtype=np.int64)
rec["tri_split"] = bool(tg._g.split)
del tg
snap("trifind")

# 3. tri_find_mr RMAT-16 on the generic engine (aggregate rounds, every op's
#    count allreduce)
res = tri_find_mr(comm, e)
out["trifind_mr"] = np.array([int(res["triangles"])], dtype=np.int64)
snap("trifind_mr")

# 4. wordfreq without the combiner: one (word, NULL) pair per occurrence;
#    distributed -> materialised, partitioned, exchanged, grouped as it lands
chunks = [synth.zipf_text(2_000_000, seed=40 + i).pin_memory() for i in range(3)]
app = WordFreq(g.MapReduce(comm), chunks, ntop=10, combiner=False)
out["wf_nwords"] = np.array([app.run()], dtype=np.int64)
out["wf_nunique"] = np.array([app.nunique], dtype=np.int64)
rec["wf_top"] = app.top
rec["wf_route"] = app.route
snap("wordfreq")

# 5. the remaining entry points: broadcast (MR broadcast op, string bcast),
#    allgather of a device block, scalar allreduces
mr = g.MapReduce(comm)
keys = [b"k%04d\0" % i for i in range(300)]
mr.map(1, lambda i, kv: [kv.add(k, k) for k in keys])
rec["mr_broadcast"] = int(mr.broadcast(0))
rec["mr_gather"] = int(mr.gather(1))
rec["bcast"] = comm.native.bcast("hello-rccl", 0).decode()
rec["allreduce"] = comm.native.allreduce([5, -3], 0)
x = torch.arange(4096, dtype=torch.float32, device="cuda")
rec["allgather_var_ok"] = bool(torch.equal(comm.native.allgather_var(x), x))
snap("final")
np.savez(OUT + ".npz", **out)
print(json.dumps(rec), flush=True)
