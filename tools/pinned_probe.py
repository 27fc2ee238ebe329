"""Pinned host buffers as the benchmarks make them (device tensor ->
.cpu().pin_memory()): H2D time of each 128 MiB buffer and the NUMA node of
its first page (get_mempolicy MPOL_F_NODE | MPOL_F_ADDR), with and without
the NUMA bind of parallel.comm.init()."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, ".")
import gpu_mapreduce_amd as g  # noqa: E402,F401
from gpu_mapreduce_amd.parallel import comm as pcomm  # noqa: E402

libc = ctypes.CDLL("libc.so.6", use_errno=True)
MPOL_F_NODE, MPOL_F_ADDR = 1, 2


def node_of(addr):
    mode = ctypes.c_int(-1)
    r = libc.syscall(239, ctypes.byref(mode), None, ctypes.c_ulong(0), ctypes.c_void_p(addr),
                     ctypes.c_ulong(MPOL_F_NODE | MPOL_F_ADDR))  # SYS_get_mempolicy
    return mode.value if r == 0 else f"err{ctypes.get_errno()}"


print("affinity before", len(os.sched_getaffinity(0)), "cpus", flush=True)
comm = pcomm.init()
print("affinity after", len(os.sched_getaffinity(0)), "cpus; bound to", pcomm.bind_numa_local(0) and "gpu-local node",
      flush=True)
dev = torch.empty(128 << 20, dtype=torch.uint8, device="cuda")
for mode in ("cpu().pin_memory()", "empty(pin_memory=True)"):
    bufs = []
    for i in range(10):
        t = torch.randint(0, 255, (128 << 20,), dtype=torch.uint8, device="cuda")
        if mode.startswith("cpu"):
            h = t.cpu().pin_memory()
        else:
            h = torch.empty(128 << 20, dtype=torch.uint8, pin_memory=True)
            h.copy_(t)
        bufs.append(h)
    torch.cuda.synchronize()
    for i, h in enumerate(bufs):
        dev.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            dev.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 3 * 1e3
        print(f"{mode:24s} buf {i}: {ms:6.2f} ms  node {node_of(h.data_ptr())}  addr {h.data_ptr():#x}", flush=True)
