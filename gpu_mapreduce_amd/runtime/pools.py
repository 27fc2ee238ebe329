"""Persistent staging pools of the runtime (the MI355X analog of MR-MPI's
page pool, reference src/mapreduce.cpp:3318-3547): device staging buffers for
streamed input and pinned host buffers for device->host output are allocated
once per process and reused by every job, so no job pays hipMalloc /
hipHostMalloc on its critical path. Every other device allocation goes through
the engine's HBM page pool (csrc/engine/hbmpool.h), the process's device
allocator."""
from __future__ import annotations

import torch

_dev = {}
_host = {}
_streams = {}
_events = {}
_ring = {}
_const = {}
_cursor = {}
_prefetch = {}


def device_buffer(device: str, nbytes: int, slot: int = 0) -> torch.Tensor:
    key = (str(device), slot)
    b = _dev.get(key)
    if b is None or b.numel() < nbytes:
        if b is not None and str(device).startswith("cuda"):
            # a copy (e.g. a previous job's prefetch) or a kernel may still use
            # the old buffer: it is freed only after the device is idle, and a
            # prefetch into it is void (take_prefetch also checks the buffer)
            torch.cuda.synchronize(device)
            _prefetch.pop(key, None)
        # MRH_STAGE_MIN_BYTES: allocate staging buffers at least this large
        # (an experiment on H2D copy speed by allocation path)
        import os
        floor = int(os.environ.get("MRH_STAGE_MIN_BYTES", "0") or 0)
        b = torch.empty(max(nbytes, floor, 1), dtype=torch.uint8, device=device)
        _dev[key] = b
    return b


def device_constant(device: str, t: torch.Tensor) -> torch.Tensor:
    """A small host tensor uploaded once per (device, content) and reused:
    job metadata that repeats between jobs (InvertedIndex's file-name table)
    must not cost a pageable H2D copy per job — that copy waits for the
    device queue, i.e. for the previous job's tail, before the next job can
    issue its first input copy."""
    key = (str(device), t.dtype, tuple(t.shape), t.numpy().tobytes())
    d = _const.get(key)
    if d is None:
        if len(_const) > 64:
            _const.clear()
        d = t.to(device)
        _const[key] = d
    return d


def pinned_buffer(nbytes: int, slot: int = 0) -> torch.Tensor:
    b = _host.get(slot)
    if b is None or b.numel() < nbytes:
        b = torch.empty(max(int(nbytes * 1.25), 1), dtype=torch.uint8, pin_memory=torch.cuda.is_available())
        _host[slot] = b
    return b[:nbytes]


def stream(device: str, name: str):
    """A persistent side stream (H2D staging, D2H output drain) per device."""
    key = (str(device), name)
    st = _streams.get(key)
    if st is None:
        st = torch.cuda.Stream(device=device)
        _streams[key] = st
    return st


def last_use(device: str, slot: int):
    """Event recorded after the last kernel that read staging buffer `slot`
    (None before first use): a later job's H2D into the slot waits on it."""
    return _events.get((str(device), slot))


def mark_use(device: str, slot: int, stream) -> None:
    ev = torch.cuda.Event()
    ev.record(stream)
    _events[(str(device), slot)] = ev


def ring_cursor(device: str, name: str, advance: int = 0, n: int = 1) -> int:
    """Persistent position of a staging ring (which slot the next job's first
    input lands in); advance moves it by the job's input count."""
    key = (str(device), name)
    c = _cursor.get(key, 0)
    if advance:
        _cursor[key] = (c + advance) % max(1, n)
    return c


def set_prefetch(device: str, slot: int, src: torch.Tensor, event, dst: torch.Tensor) -> None:
    """Record that `src` (a host tensor) is being copied into staging buffer
    `dst` (slot `slot`), complete at `event` — issued by the previous job of a
    pipeline."""
    _prefetch[(str(device), slot)] = (src.data_ptr(), src.numel(), dst.data_ptr(), dst.numel(), event)


def take_prefetch(device: str, slot: int, src: torch.Tensor, dst: torch.Tensor):
    """The copy event if `src` was prefetched into `dst`, the current buffer of
    `slot` (consumed), else None — also None when the slot's buffer was
    reallocated since (the copy went to the old one)."""
    rec = _prefetch.pop((str(device), slot), None)
    if rec is not None and rec[:4] == (src.data_ptr(), src.numel(), dst.data_ptr(), dst.numel()):
        return rec[4]
    return None


def next_slot(name: str, n: int = 2) -> int:
    """Round-robin slot index for double-buffered outputs (job k uses slot k % n)."""
    i = _ring.get(name, 0)
    _ring[name] = i + 1
    return i % n


def generation(name: str) -> int:
    """How many slots of ring `name` have been handed out so far."""
    return _ring.get(name, 0)


def clear():
    _dev.clear()
    _host.clear()
    _streams.clear()
    _events.clear()
    _ring.clear()
    _const.clear()
    _cursor.clear()
    _prefetch.clear()
