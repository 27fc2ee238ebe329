#!/usr/bin/env python3
"""PageRank RMAT-26 setup split: R-MAT map vs plan build (device-synced),
run twice in one process (the second run is warm)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpu_mapreduce_amd as g  # noqa: E402
from gpu_mapreduce_amd.models.pagerank import PageRank, rmat_map  # noqa: E402

comm = g.Comm(device="cuda:0")
scale = int(sys.argv[1]) if len(sys.argv) > 1 else 26
for rep in range(2):
    mr = g.MapReduce(comm)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rmat_map(mr, scale, 16, seed=1)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    pr = PageRank(mr, 1 << scale).build()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"rep {rep}: rmat {1e3 * (t1 - t0):.1f} ms, plan build {1e3 * (t2 - t1):.1f} ms", flush=True)
    del pr, mr
