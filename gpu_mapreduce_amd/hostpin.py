"""Pinned host memory reserved up front for the out-of-core host tier.

The spool's host tier, drained pieces and host copies of device columns are
pinned host memory. Taken from PyTorch's caching host allocator, the first of
them pin fresh pages inside the job that first spools (~0.8 s at RMAT-18),
and blocks that earlier jobs left cached at other sizes (an 8 GiB text
input) are not reused. The engine's pinned host arena
(csrc/engine/hostarena.cpp) is one segment pinned once, when the process
chooses — `prepin()`, e.g. at start-up next to the HBM pool — and carved
best-fit for those allocations; a request that does not fit falls back to the
caching host allocator.

`MRH_PIN_RESERVE_MB=N` is the default size for `prepin()`."""
import os


def reserve_mb():
    """the arena size asked for by MRH_PIN_RESERVE_MB (0: none)"""
    return int(os.environ.get("MRH_PIN_RESERVE_MB", "0") or 0)


def prepin(mb=None):
    """pin the arena now (once per process); returns the milliseconds it took
    (0: it exists already or none was asked for; -1: the host could not pin
    that much, the job goes on with the caching host allocator)"""
    import torch
    from ._ext import C
    mb = reserve_mb() if mb is None else int(mb)
    if mb <= 0 or not torch.cuda.is_available():
        return 0.0
    return float(C.host_arena_reserve(mb << 20))  # 0 when the arena exists already


def stats():
    """reserved / in_use / peak bytes, hits / misses (fallbacks) of the arena"""
    from ._ext import C
    return dict(C.host_arena_stats())
