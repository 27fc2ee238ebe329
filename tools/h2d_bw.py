"""Measure host(pinned)->HBM and HBM->host copy bandwidth on this box (the
floor for an end-to-end InvertedIndex step whose input starts in host RAM)."""
import time
import torch

n = 1 << 30
h = torch.empty(n, dtype=torch.uint8).pin_memory()
d = torch.empty(n, dtype=torch.uint8, device="cuda")
for _ in range(2):
    d.copy_(h, non_blocking=True)
torch.cuda.synchronize()
for chunk in (n, 128 << 20, 32 << 20):
    t = time.perf_counter()
    for r in range(3):
        for o in range(0, n, chunk):
            d[o:o + chunk].copy_(h[o:o + chunk], non_blocking=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 3
    print(f"H2D chunk {chunk >> 20} MiB: {n / dt / 1e9:.1f} GB/s ({dt * 1e3:.2f} ms per GiB)")
t = time.perf_counter()
for r in range(3):
    h.copy_(d, non_blocking=True)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / 3
print(f"D2H: {n / dt / 1e9:.1f} GB/s")
