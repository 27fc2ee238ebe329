"""Communicator: one process per MI355X, torch.distributed over RCCL/xGMI.

Replaces MR-MPI's MPI_Comm plumbing (reference src/mapreduce.cpp:93-161) and
the serial `mpistubs/` fake MPI (mpistubs/mpi.cpp:57-67): with no process
group (world size 1) every collective is the identity.

Backend choice is not a dispatch layer: device tensors go through the "nccl"
backend (which IS RCCL on ROCm); the CPU engine path (tests, no GPU) uses
"gloo". The native shuffle calls the c10d ProcessGroup directly from C++.
"""
from __future__ import annotations

import datetime
import os
import time

import torch
import torch.distributed as dist

_WORLD = None


class Comm:
    """Thin host-side view of a c10d process group plus the engine device."""

    def __init__(self, group=None, device=None):
        if group is None and dist.is_available() and dist.is_initialized():
            group = dist.group.WORLD
        self.group = group
        if group is not None:
            self.rank = dist.get_rank(group)
            self.size = dist.get_world_size(group)
            backend = dist.get_backend(group)
        else:
            self.rank, self.size, backend = 0, 1, None
        self.backend = backend
        if device is None:
            if backend == "gloo" or not torch.cuda.is_available():
                device = "cpu"
            else:
                device = f"cuda:{torch.cuda.current_device()}"
        self.device = str(device)
        self.is_cuda = self.device.startswith("cuda")
        # the c10d ProcessGroup handed to the native shuffle (None when P == 1)
        self.pg = group if (group is not None and self.size > 1) else None
        self._native = None

    @property
    def native(self):
        """The C++ communicator (csrc/engine/comm.h) the native MapReduce uses:
        same process group, plus the rendezvous store for mapstyle 2."""
        if self._native is None:
            from .._ext import C
            store = None
            if self.size > 1:
                try:
                    store = dist.distributed_c10d._get_default_store()
                except Exception:
                    store = None
            # RCCL (native communicator over xGMI) for device engines whose
            # group is the nccl backend or that run alone; a gloo group (CPU
            # engine, or the MRH_DIST_BACKEND=gloo rehearsal of several ranks
            # on one GPU) keeps its process group as the transport
            transport = "pg" if self.backend == "gloo" else ""
            self._native = C.NativeComm(self.pg, self.device, store, transport)
        return self._native

    # ---- scalar collectives (every MR op returns a global count) ----------
    def _t(self, vals, dtype):
        return torch.tensor(vals, dtype=dtype, device=self.device)

    def allreduce(self, vals, op="sum", dtype=torch.int64):
        scalar = not isinstance(vals, (list, tuple))
        v = [vals] if scalar else list(vals)
        if self.size == 1:
            return v[0] if scalar else v
        t = self._t(v, dtype)
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        dist.all_reduce(t, op=rop, group=self.group)
        out = t.cpu().tolist()
        return out[0] if scalar else out

    def allgather(self, val, dtype=torch.float64):
        if self.size == 1:
            return [val]
        t = self._t([val], dtype)
        out = [torch.empty_like(t) for _ in range(self.size)]
        dist.all_gather(out, t, group=self.group)
        return [x.item() for x in out]

    def allgather_object(self, obj):
        if self.size == 1:
            return [obj]
        out = [None] * self.size
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def barrier(self):
        if self.size > 1:
            if self.is_cuda:
                # a 1-element allreduce on the device is the RCCL barrier
                self.allreduce(0)
            else:
                dist.barrier(group=self.group)

    def bcast_object(self, obj, root=0):
        if self.size == 1:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=root, group=self.group,
                                   device=torch.device(self.device) if self.is_cuda else None)
        return lst[0]

    def wtime(self):
        if self.is_cuda:
            torch.cuda.synchronize()
        return time.perf_counter()

    def split(self, color, key=0):
        """MPI_Comm_split analog (OINK -partition worlds): new group per color."""
        if self.size == 1:
            return self
        colors = self.allgather(float(color))
        members = sorted(r for r, c in enumerate(colors) if c == float(color))
        groups = {}
        for c in sorted(set(colors)):
            ranks = [r for r, cc in enumerate(colors) if cc == c]
            groups[c] = dist.new_group(ranks, backend=self.backend)
        return Comm(groups[float(color)], device=self.device) if members else None


def init(backend=None, timeout_s=None):
    """Initialise the process group from torchrun-style env vars
    (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR/MASTER_PORT), bind this process to
    GPU LOCAL_RANK, and return a Comm. World size 1 needs no env at all.
    Collectives are bounded by timeout_s (default MRH_COMM_TIMEOUT or 600 s):
    a dead peer becomes an error on the other ranks, not a hang."""
    global _WORLD
    if timeout_s is None:
        timeout_s = int(os.environ.get("MRH_COMM_TIMEOUT", "600"))
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    # MRH_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share a
    # device, LOCAL_RANK modulo the device count); production is "nccl" = RCCL
    backend = backend or os.environ.get("MRH_DIST_BACKEND") or None
    if ws > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if torch.cuda.is_available():
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device(f"cuda:{torch.cuda.current_device()}")
        dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    elif torch.cuda.is_available() and ws == 1:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    if torch.cuda.is_available():
        bind_numa_local(torch.cuda.current_device())
    dev = f"cuda:{torch.cuda.current_device()}" if torch.cuda.is_available() else "cpu"
    _WORLD = Comm(device=dev)
    return _WORLD


def bind_numa_local(dev: int) -> list | None:
    """Pin this process to the CPUs of its GPU's NUMA node (sysfs local_cpulist
    of the GPU's PCI function), so the pinned host buffers it allocates next —
    input files staged for H2D, spill buffers — land in socket-local DRAM and
    the 8 ranks' PCIe streams do not cross the socket interconnect. Disable
    with MRH_NUMA_BIND=0."""
    if os.environ.get("MRH_NUMA_BIND", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return None
    try:
        from .._ext import C
        bus = C.gpu_pci_bus_id(dev).lower()
        if not bus:
            return None
        with open(f"/sys/bus/pci/devices/{bus}/local_cpulist") as f:
            spec = f.read().strip()
        cpus = set()
        for part in spec.split(","):
            if "-" in part:
                a, b = part.split("-")
                cpus.update(range(int(a), int(b) + 1))
            elif part:
                cpus.add(int(part))
        cpus &= os.sched_getaffinity(0)   # stay inside the launcher's cgroup/cpuset
        if cpus:
            os.sched_setaffinity(0, cpus)
            return sorted(cpus)
    except (OSError, ValueError, RuntimeError):
        return None
    return None


def world():
    global _WORLD
    if _WORLD is None:
        _WORLD = Comm()
    return _WORLD
