#!/usr/bin/env python3
"""Per-op wall time of one K-means iteration (device-synced after each op):
where the ~0.35 ms of non-kernel time per Lloyd iteration goes."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpu_mapreduce_amd as g  # noqa: E402
from gpu_mapreduce_amd._ext import C  # noqa: E402
from gpu_mapreduce_amd.models.kmeans import KMeans, blobs  # noqa: E402

comm = g.Comm(device="cuda:0")
p = blobs(32 << 20, 2, 32, seed=1, device="cuda:0")
km = KMeans(comm, p, blobs(32, 2, 32, seed=2, device="cuda:0"))
for _ in range(5):
    km.iterate()
tot = {}
for it in range(20):
    mr = g.MapReduce(comm)
    t = [time.perf_counter()]
    mr.map(mr.nprocs, lambda itask, kv: kv.add_kv(C.kmeans_map(km.points, km.centroids)))
    torch.cuda.synchronize(); t.append(time.perf_counter())
    mr.collate(); torch.cuda.synchronize(); t.append(time.perf_counter())
    mr.reduce("sum:float64"); torch.cuda.synchronize(); t.append(time.perf_counter())
    mr.gather(1); mr.broadcast(0); torch.cuda.synchronize(); t.append(time.perf_counter())
    for name, a, b in zip(("map", "collate", "reduce", "gather+bcast"), t[:-1], t[1:]):
        tot[name] = tot.get(name, 0.0) + (b - a)
t0 = time.perf_counter()
for _ in range(20):
    km.iterate()
torch.cuda.synchronize()
print({k: round(v / 20 * 1e6, 1) for k, v in tot.items()}, "us per iteration; iterate()", round((time.perf_counter() - t0) / 20 * 1e6, 1), "us")
