"""Keys-only radix sort throughput at PageRank scale (1.07 G u64 keys, 29
sorted bits = 4 passes) for the tile size chosen by MRH_RX_KIT; one line."""
import os
import sys

import torch

sys.path.insert(0, ".")
from gpu_mapreduce_amd import C  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1 << 30
bits = int(sys.argv[2]) if len(sys.argv) > 2 else 29
k = torch.randint(0, 1 << 62, (n,), dtype=torch.int64, device="cuda")
k = (k & ((1 << bits) - 1)) << 32 | (k >> 40)  # sorted bits above a payload word
C.radix_sort_keys(k, 32, 32 + bits, False)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(3):
    out = C.radix_sort_keys(k, 32, 32 + bits, False)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / 3
ok = bool((out[1:] >> 32 >= out[:-1] >> 32).all())
passes = (bits + 7) // 8
print(f"KIT={os.environ.get('MRH_RX_KIT', 'default')} n={n} bits={bits}: {ms:.2f} ms ({ms / passes:.2f} ms/pass, "
      f"{n * 16 * passes / ms / 1e6:.0f} GB/s), sorted={ok}", flush=True)
