"""reduce_builtin('sum', int32) over 2^27 values grouped into 2^k keys of
equal size (k = 0, 5, 10, 15, 20): device time of the segmented reduce alone
(best of 5), to see how it behaves from one hot key to a million small ones.

    python tools/segred_keys_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpu_mapreduce_amd import C  # noqa: E402

if os.environ.get("POOL") == "1":  # the engine's HBM pool as the allocator (a Comm installs it)
    from gpu_mapreduce_amd.parallel.comm import Comm
    Comm(device="cuda")
    from gpu_mapreduce_amd.runtime import hbm_pool
    print("hbm pool installed:", hbm_pool.installed(), flush=True)
n = 1 << 27
for lk, unaligned in ((0, 0), (5, 0), (10, 0), (15, 0), (20, 0), (5, 1), (10, 1), (15, 1)):
    nk = (1 << lk) - unaligned  # unaligned: segment ends fall inside the 4096-value tiles
    keys = (torch.arange(n, device="cuda", dtype=torch.int64) * nk) // n
    vals = torch.ones(n, device="cuda", dtype=torch.int32)
    kv = C.make_kv(keys, None, vals, None, n, "cuda")
    kg, _ = C.convert(kv)
    best = 1e30
    for _ in range(6):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        r = C.reduce_builtin(kg, "sum", "int32")
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b))
    tot = int(torch.frombuffer(bytearray(r.vdata.cpu().numpy().tobytes()), dtype=torch.int32).sum())
    assert tot == n and r.n == nk
    print(f"{nk:8d} keys{' (unaligned)' if unaligned else ''}: {best:7.3f} ms  {n * 4 / (best * 1e-3) / 1e9:7.1f} GB/s", flush=True)
