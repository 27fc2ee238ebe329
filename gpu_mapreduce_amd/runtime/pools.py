"""Persistent staging pools of the runtime (the MI355X analog of MR-MPI's
page pool, reference src/mapreduce.cpp:3318-3547): device staging buffers for
streamed input and pinned host buffers for device->host output are allocated
once per process and reused by every job, so no job pays hipMalloc /
hipHostMalloc on its critical path. Device scratch of the engine itself goes
through the ATen caching allocator (stream-ordered reuse)."""
from __future__ import annotations

import torch

_dev = {}
_host = {}


def device_buffer(device: str, nbytes: int, slot: int = 0) -> torch.Tensor:
    key = (str(device), slot)
    b = _dev.get(key)
    if b is None or b.numel() < nbytes:
        b = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
        _dev[key] = b
    return b


def pinned_buffer(nbytes: int, slot: int = 0) -> torch.Tensor:
    b = _host.get(slot)
    if b is None or b.numel() < nbytes:
        b = torch.empty(max(int(nbytes * 1.25), 1), dtype=torch.uint8, pin_memory=torch.cuda.is_available())
        _host[slot] = b
    return b[:nbytes]


def clear():
    _dev.clear()
    _host.clear()
