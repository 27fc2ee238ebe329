"""Communicator: one process per MI355X; RCCL over xGMI for the data plane.

Replaces MR-MPI's MPI_Comm plumbing (reference src/mapreduce.cpp:93-161) and
the serial `mpistubs/` fake MPI (mpistubs/mpi.cpp:57-67): with no process
group (world size 1) every collective is the identity.

Exactly ONE RCCL communicator per process (per member set): the native
engine's (csrc/engine/rccl.h), created by `Comm.native` and shared by every
Comm over the same ranks. torch.distributed runs the **gloo** backend and only
carries host objects and host scalars (the global pair counts every op returns,
file lists, pickled objects) — so an op's return value never forces a device
round trip, and no second (c10d) RCCL communicator competes for the xGMI links.
The engine's device data (shuffle rounds, allgathers, PageRank/graph
exchanges) goes through the native RCCL communicator.

Engine transport "pg" (several ranks sharing one GPU, where RCCL cannot run —
the multi-rank rehearsal on a 1-GPU box — or MRH_TRANSPORT=pg) keeps the
engine's collectives on the gloo group instead.
"""
from __future__ import annotations

import atexit
import datetime
import os
import sys
import time

import torch
import torch.distributed as dist

_WORLD = None
_NATIVE = {}          # (group key, device, transport) -> NativeComm: one per member set
_HOOKS = [False]


def _shares_devices(size: int) -> bool:
    """True when more local ranks than visible GPUs: ranks share a device,
    which RCCL refuses (two ranks of one communicator on one GPU). Without
    LOCAL_WORLD_SIZE (a single-node launcher) every rank is local."""
    try:
        lws = int(os.environ.get("LOCAL_WORLD_SIZE", str(size)))
        return torch.cuda.is_available() and lws > torch.cuda.device_count()
    except (ValueError, RuntimeError):
        return False


def _engine_transport(device: str, size: int) -> str:
    if not device.startswith("cuda"):
        return "pg"
    if os.environ.get("MRH_TRANSPORT") == "pg" or _shares_devices(size):
        return "pg"
    return ""


def _install_exit_hooks():
    """A multi-rank job must end one of two ways for its peers: an orderly
    shutdown handshake (atexit, after a clean run), or a poisoned communicator
    (an exception escaped: peers fail within seconds instead of waiting on a
    rank that is gone). Teardown alone never counts as a clean exit."""
    if _HOOKS[0]:
        return
    _HOOKS[0] = True
    prev = sys.excepthook

    def hook(tp, val, tb):
        for n in list(_NATIVE.values()):
            try:
                if n.size > 1:
                    n.poison(f"uncaught {tp.__name__} on rank {dist.get_rank() if dist.is_initialized() else '?'}: {val}")
            except Exception:  # noqa: BLE001
                pass
        prev(tp, val, tb)

    sys.excepthook = hook

    def retire():
        done = set()
        for n in list(_NATIVE.values()):
            try:
                key = tuple(n.members)
                if n.size > 1 and not n.failed and key not in done and \
                        (not dist.is_initialized() or n.size == dist.get_world_size()):
                    done.add(key)
                    n.shutdown()
            except Exception:  # noqa: BLE001
                pass

    atexit.register(retire)


class Comm:
    """Host-side view of a process group (gloo), the engine device and the
    engine's native communicator (RCCL for device engines)."""

    def __init__(self, group=None, device=None, transport=None):
        if group is None and dist.is_available() and dist.is_initialized():
            group = dist.group.WORLD
        self.group = group
        if group is not None:
            self.rank = dist.get_rank(group)
            self.size = dist.get_world_size(group)
            backend = dist.get_backend(group)
            self.members = list(dist.get_process_group_ranks(group))
        else:
            self.rank, self.size, backend = 0, 1, None
            self.members = [0]
        self.backend = backend
        if device is None:
            device = f"cuda:{torch.cuda.current_device()}" if torch.cuda.is_available() else "cpu"
        self.device = str(device)
        self.is_cuda = self.device.startswith("cuda")
        # engine transport: "" = native RCCL for device engines, "pg" = the group
        self.transport = _engine_transport(self.device, self.size) if transport is None else transport
        # the c10d ProcessGroup handed to the native engine (None when P == 1)
        self.pg = group if (group is not None and self.size > 1) else None
        # host scalars on the host group; device tensors only if the group is
        # an explicit (non-default) nccl group
        self._sdev = self.device if (backend == "nccl") else "cpu"

    @property
    def native(self):
        """The C++ communicator (csrc/engine/comm.h) the native engine uses:
        this group for host scalars, the root store for the RCCL id
        rendezvous and mapstyle 2, and the process's RCCL communicator over
        these members (shared with every other Comm over them)."""
        if self.size == 1 and "_native1" in self.__dict__:
            return self.__dict__["_native1"]
        key = (tuple(self.members), self.device, self.transport)
        n = _NATIVE.get(key) if self.size > 1 else None
        if n is None:
            from .._ext import C
            store = None
            wr, ws = -1, -1
            if self.size > 1:
                store = dist.distributed_c10d._get_default_store()
                wr, ws = dist.get_rank(), dist.get_world_size()
            n = C.NativeComm(self.pg, self.device, store, self.transport,
                             self.members if self.size > 1 else [], wr, ws)
            if self.size > 1:
                _NATIVE[key] = n
                _install_exit_hooks()
            else:
                self.__dict__["_native1"] = n
        return n if self.size > 1 else self.__dict__["_native1"]

    def rccl_info(self):
        """What RCCL itself reports for this communicator (ncclCommCount,
        ncclCommCuDevice, ncclCommUserRank) plus the number of RCCL
        communicators this process holds."""
        return dict(self.native.rccl_info())

    # ---- scalar collectives (every MR op returns a global count) ----------
    def _t(self, vals, dtype):
        return torch.tensor(vals, dtype=dtype, device=self._sdev)

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
        """Host barrier (MPI_Barrier): every rank has reached this point; it
        does not wait for queued device work (torch.cuda.synchronize does)."""
        if self.size > 1:
            if self.backend == "nccl":
                self.allreduce(0)
            else:
                dist.barrier(group=self.group)

    def bcast_object(self, obj, root=0):
        if self.size == 1:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=root, group=self.group,
                                   device=torch.device(self.device) if self.backend == "nccl" else None)
        return lst[0]

    def wtime(self):
        if self.is_cuda:
            torch.cuda.synchronize()
        return time.perf_counter()

    def split(self, color, key=0):
        """MPI_Comm_split analog (OINK -partition worlds): new group per color.
        Its native communicator gets its own RCCL id key (tag + member list +
        sequence), so colours never read each other's id."""
        if self.size == 1:
            return self
        colors = self.allgather(float(color))
        members = sorted(r for r, c in enumerate(colors) if c == float(color))
        groups = {}
        for c in sorted(set(colors)):
            ranks = [self.members[r] for r, cc in enumerate(colors) if cc == c]
            groups[c] = dist.new_group(ranks, backend=self.backend)
        return Comm(groups[float(color)], device=self.device, transport=self.transport) if members else None


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
    # torch.distributed is the HOST group (gloo): host objects and scalars.
    # The device data plane is the engine's own RCCL communicator (one per
    # process). MRH_DIST_BACKEND=nccl is honoured but adds a second RCCL
    # communicator per process; ranks may share GPUs (LOCAL_RANK modulo the
    # device count: the rehearsal on a 1-GPU box, engine transport "pg").
    backend = backend or os.environ.get("MRH_DIST_BACKEND") or "gloo"
    if ws > 1 and not dist.is_initialized():
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
