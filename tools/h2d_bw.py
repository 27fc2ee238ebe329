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
# the same GiB split over several copy streams (several SDMA engines in flight)
for ns in (2, 4):
    streams = [torch.cuda.Stream() for _ in range(ns)]
    part = n // ns
    torch.cuda.synchronize()
    t = time.perf_counter()
    for r in range(3):
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                d[i * part:(i + 1) * part].copy_(h[i * part:(i + 1) * part], non_blocking=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 3
    print(f"H2D {ns} streams: {n / dt / 1e9:.1f} GB/s ({dt * 1e3:.2f} ms per GiB)")
