#!/usr/bin/env python3
"""Forced-RCCL single-rank check of large transfers: Comm.alltoallv (grouped
ncclSend/ncclRecv to self) and the engine exchange of fixed 8-byte keys at
1-4 GiB must return their input unchanged."""
import os, sys
os.environ["MRH_FORCE_RCCL"] = "1"
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gpu_mapreduce_amd as g
C = g._ext.C
comm = g.Comm(device="cuda:0")
nc = comm.native
assert nc.transport == "rccl"
for logn in (26, 27, 28, 29):
    n = (1 << logn) + 5
    x = torch.arange(n, dtype=torch.int64, device="cuda").mul_(2654435761)
    y = nc.alltoallv(x, [n], [n])
    ok = torch.equal(x, y)
    bad = (x != y).nonzero()
    print(f"alltoallv n=2^{logn}+5 bytes={8*n} equal={ok} first_bad={bad[0].item() if bad.numel() else -1}", flush=True)
    del y
    kv = C.make_kv(x.view(torch.uint8), None, torch.empty(0, dtype=torch.uint8, device="cuda"), None, n, "cuda:0")
    out, st = C.exchange(kv, torch.zeros(n, dtype=torch.int32, device="cuda"), nc)
    z = out.kdata.view(torch.int64)
    ok2 = torch.equal(x, z)
    bad = (x != z).nonzero()
    print(f"exchange  n=2^{logn}+5 equal={ok2} first_bad={bad[0].item() if bad.numel() else -1}", flush=True)
    del kv, out, z, x
    torch.cuda.empty_cache()
