"""Radix sort throughput on the device: C.radix_sort_pairs (one-sweep
passes) vs torch.sort(stable) at several sizes; prints one line per size."""
import sys
import time

import torch

sys.path.insert(0, ".")
from gpu_mapreduce_amd import C  # noqa: E402


def t_ms(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for n in [600_000, 5_400_000, 50_000_000, 200_000_000]:
    for bits in (64, 24):
        k = torch.randint(0, 2 ** 62, (n,), dtype=torch.int64, device="cuda") & ((1 << bits) - 1)
        v = torch.arange(n, dtype=torch.int32, device="cuda")
        ours = t_ms(lambda: C.radix_sort_pairs(k, v, 0, bits, False))
        tor = t_ms(lambda: torch.sort(k, stable=True))
        passes = (bits + 7) // 8
        print(f"n={n:>11,} bits={bits}: ours {ours:8.3f} ms ({ours * 1e3 / passes:7.1f} us/pass, "
              f"{n * 24 * passes / ours / 1e6:7.0f} GB/s pass traffic)  torch.sort {tor:8.3f} ms", flush=True)
