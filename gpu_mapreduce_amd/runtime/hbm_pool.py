"""Python face of the HBM page pool (csrc/engine/hbmpool.h).

The pool replaces the ATen caching allocator for the whole process: it is
installed when `gpu_mapreduce_amd` is imported before any device tensor
exists (`MRH_HBM_POOL=0` opts out, `=1` fails loudly if it cannot install),
or by `install()` under the same condition. Every
device allocation then comes from per-device stream-ordered HIP memory pools
with a hard cap; a MapReduce op whose object has a page budget B
(`maxpage` x `memsize`, or `hbm_budget`) may hold at most 2B of new device
memory, and fails with "Cannot allocate page" past it — the reference's
maxpage limit (src/mapreduce.cpp:3397-3466) — unless the op streams out of
core. Stats give the hi-water mark (reference `hiwater`, :3569-3574).
"""
from __future__ import annotations

from .._ext import C


def install() -> bool:
    """make the pool the device allocator; False if device memory was already allocated"""
    return bool(C.hbm_pool_install())


def installed() -> bool:
    return bool(C.hbm_pool_installed())


def stats(device: int = 0) -> dict:
    """{in_use, peak, reserved, reserved_peak, cap, allocs, frees, failures,
    cached, cross_stream_reuse, faulted} in bytes / counts"""
    return dict(C.hbm_pool_stats(int(device)))


def reset_peak(device: int = 0) -> None:
    C.hbm_pool_reset_peak(int(device))


def set_cap(cap_bytes: int, device: int = 0) -> int:
    """hard cap on bytes in use (0 = none); returns the previous cap"""
    return int(C.hbm_pool_set_cap(int(device), int(cap_bytes)))


def trim(keep_bytes: int = 0, device: int = 0) -> None:
    """return cached free memory of the pool to the driver"""
    C.hbm_pool_trim(int(device), int(keep_bytes))
