"""The wordfreq bench's input chunks (bench_wordfreq's generation): H2D time
and NUMA node of every chunk, to find why one chunk copies at half speed."""
import ctypes
import sys
import time

import torch

sys.path.insert(0, ".")
import gpu_mapreduce_amd as g  # noqa: E402,F401
from gpu_mapreduce_amd.parallel import comm as pcomm  # noqa: E402
from gpu_mapreduce_amd.utils import synth  # noqa: E402

libc = ctypes.CDLL("libc.so.6", use_errno=True)


def nodes(t, samples=16):
    out = []
    step = max(1, t.numel() // samples)
    for off in range(0, t.numel(), step):
        mode = ctypes.c_int(-1)
        r = libc.syscall(239, ctypes.byref(mode), None, ctypes.c_ulong(0), ctypes.c_void_p(t.data_ptr() + off),
                         ctypes.c_ulong(3))
        out.append(mode.value if r == 0 else -9)
    return "".join(str(x) for x in out)


comm = pcomm.init()
chunks = []
for i in range(8):
    t = synth.zipf_text(128 << 20, seed=7919 + i, device="cuda")
    chunks.append(t.cpu().pin_memory())
torch.cuda.empty_cache()
dev = torch.empty(130 << 20, dtype=torch.uint8, device="cuda")
for i, h in enumerate(chunks):
    dev[: h.numel()].copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        dev[: h.numel()].copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 3 * 1e3
    print(f"chunk {i}: {ms:6.2f} ms  nodes {nodes(h)}  addr {h.data_ptr():#x} size {h.numel()}", flush=True)
