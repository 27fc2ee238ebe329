"""Pinned host memory reserved up front for the out-of-core host tier.

The spool's host tier, the drained pieces on their way to disk and the
staging of uploads are pinned host memory from PyTorch's caching host
allocator. Its first allocations pin fresh pages (~5-15 GB/s) inside the job
that first spools — the out-of-core job's "cold" run paid ~0.8 s of it at
RMAT-18 (profiles/r6_ooc_prepin.txt). A reserve segment
(`pinned_reserve_segment_size_mb`) is pinned once, at the moment the process
chooses (`prepin()`, e.g. at start-up next to the HBM pool), and every later
pinned allocation that fits is carved from it.

`MRH_PIN_RESERVE_MB=N` asks for an N MiB reserve. The allocator reads its
configuration from `PYTORCH_HIP_ALLOC_CONF` once, so `configure()` must run
before torch is imported — `import gpu_mapreduce_amd` does it when it comes
first; otherwise set `PYTORCH_HIP_ALLOC_CONF=pinned_reserve_segment_size_mb:N`
in the environment yourself."""
import os
import sys
import time

_KEY = "pinned_reserve_segment_size_mb"


def configure(mb=None):
    """put the reserve size into PYTORCH_HIP_ALLOC_CONF (before torch is
    imported); returns the MiB in effect (0: none)"""
    mb = int(mb if mb is not None else os.environ.get("MRH_PIN_RESERVE_MB", "0") or 0)
    conf = os.environ.get("PYTORCH_HIP_ALLOC_CONF", "")
    if _KEY in conf:
        return int(conf.split(_KEY + ":")[1].split(",")[0])
    if mb <= 0 or "torch" in sys.modules:
        return 0
    os.environ["PYTORCH_HIP_ALLOC_CONF"] = (conf + "," if conf else "") + f"{_KEY}:{mb}"
    return mb


def prepin():
    """allocate the reserve now (the first pinned allocation of the process
    pins the whole segment); returns the milliseconds it took"""
    import torch
    if not torch.cuda.is_available():
        return 0.0
    t0 = time.perf_counter()
    torch.empty(1, pin_memory=True)
    return (time.perf_counter() - t0) * 1e3
