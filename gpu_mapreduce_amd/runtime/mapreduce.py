"""MapReduce object: the user API of the framework.

Same method names, settings, defaults and return values (global pair counts)
as MR-MPI's `class MapReduce` (reference src/mapreduce.h:28-126,
src/mapreduce.cpp:93-3574), re-designed for MI355X:

* the MR owns one KV **or** one KMV (reference src/mapreduce.h:43-44), but
  they are device-resident SoA tensors (csrc/engine/kv.h), not paged byte
  buffers; every data-plane op (hash/partition, shuffle, group-by, sort,
  segmented reduce, gathers) runs in the native engine;
* the shuffle (`aggregate`/`collate`/`gather`) is an RCCL all-to-all over
  xGMI issued from C++ on the c10d process group; `broadcast` an RCCL bcast;
* callbacks come in two tiers: host callbacks with MR-MPI semantics
  (per-pair / per-key Python functions) and device batch callbacks
  (`*_batch`, `reduce("sum:float32")` built-ins) that keep data in HBM.

Settings that configured the paged memory model (memsize, minpage, maxpage,
freepage, zeropage, keyalign, valuealign, outofcore) are accepted and kept;
`memsize`/`outofcore` drive the host spill tier (`spill()`/`unspill()`), the
alignment settings only affect the byte layout handed to C-ABI callbacks.
"""
from __future__ import annotations

import functools
import inspect
import os
import struct
import sys
import time

import torch

from .._ext import C
from ..parallel.comm import Comm, world
from . import stats as _stats
from .keyvalue import KeyValue, to_bytes

MRMPI_VERSION = "gpu_mapreduce_amd 0.1 (MR-MPI 11 Mar 2013 API)"


def _arity(fn):
    try:
        sig = inspect.signature(fn)
    except (TypeError, ValueError):
        return None
    params = [p for p in sig.parameters.values()
              if p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD)]
    if any(p.kind == p.VAR_POSITIONAL for p in sig.parameters.values()):
        return None
    return len(params)


def _call(fn, nargs_without_ptr, args, ptr):
    """MR-MPI callbacks take an optional trailing `ptr`; pass it only if the
    callback accepts it (the reference Python wrapper does the same,
    python/mrmpi.py:185-188)."""
    n = _arity(fn)
    if n is None or n > nargs_without_ptr:
        return fn(*args, ptr)
    return fn(*args)


class MultiValue(list):
    """The values of one KMV key as a list of bytes objects. Long value lists
    can also be walked in blocks (MR-MPI multivalue_blocks/multivalue_block,
    reference src/mapreduce.cpp:1874-1925)."""

    block_size = 1 << 20

    def nblocks(self):
        return max(1, (len(self) + self.block_size - 1) // self.block_size)

    def block(self, i):
        return self[i * self.block_size:(i + 1) * self.block_size]


class MapReduce:
    # static counters across all MR objects (reference src/mapreduce.h:46-57)
    instances_now = 0
    instances_ever = 0
    msize = 0
    msizemax = 0
    rsize = 0
    wsize = 0
    cssize = 0
    crsize = 0
    commtime = 0.0

    def __init__(self, comm: Comm | None = None, device: str | None = None):
        self.comm = comm if comm is not None else world()
        self.device = str(device) if device is not None else self.comm.device
        self.me = self.comm.rank
        self.nprocs = self.comm.size
        # settings (reference defaults: src/mapreduce.cpp:201-229)
        self.mapstyle = 0
        self.all2all = 1
        self.verbosity = 0
        self.timer = 0
        self.memsize = 64
        self.minpage = 0
        self.maxpage = 0
        self.freepage = 1
        self.outofcore = 0
        self.zeropage = 0
        self.keyalign = 4
        self.valuealign = 4
        self.fpath = os.environ.get("MRMPI_FPATH", ".")
        self.mapfilecount = 0
        self.kv = None      # native KV (device)
        self.kmv = None     # native KMV (device)
        self._open = None   # KeyValue being filled by another MR's callbacks
        self._open_add = 0
        self._time_start = 0.0
        self._cs_one = self._cr_one = 0
        self._mv_block = 0
        self.last_convert = None
        MapReduce.instances_now += 1
        MapReduce.instances_ever += 1
        self.instance_me = MapReduce.instances_ever

    # ------------------------------------------------------------------ helpers
    def _new_kv(self):
        return KeyValue(self.device)

    def _count(self, n):
        return int(self.comm.allreduce(int(n), "sum"))

    def _start(self):
        if self.timer:
            if self.timer == 1:
                self.comm.barrier()
            self._time_start = self.comm.wtime()
        self._cs_one, self._cr_one = MapReduce.cssize, MapReduce.crsize

    def _track_mem(self):
        b = 0
        if self.kv is not None:
            b += self.kv.nbytes()
        if self.kmv is not None:
            b += self.kmv.nbytes()
        MapReduce.msize = b
        MapReduce.msizemax = max(MapReduce.msizemax, b)

    def _stats(self, heading, which):
        self._track_mem()
        if self.timer:
            if self.timer == 1:
                self.comm.barrier()
                if self.me == 0:
                    print(f"{heading} time (secs) = {self.comm.wtime() - self._time_start:g}")
            elif self.timer == 2:
                _stats.write_histo(self.comm, self.comm.wtime() - self._time_start, f"{heading} time (secs) =")
        if self.verbosity == 0:
            return
        if which == 0:
            if self.me == 0:
                print(f"{heading} KV = ", end="")
            self.kv_stats(self.verbosity)
        else:
            if self.me == 0:
                print(f"{heading} KMV = ", end="")
            self.kmv_stats(self.verbosity)
        s_one = MapReduce.cssize - self._cs_one
        r_one = MapReduce.crsize - self._cr_one
        sall, rall = self.comm.allreduce([s_one, r_one], "sum")
        if sall or rall:
            mb = 1024.0 * 1024.0
            if self.me == 0:
                print(f"{heading} Comm = {sall / mb:.3g} Mb send, {rall / mb:.3g} Mb recv")
            if self.verbosity == 2:
                _stats.write_histo(self.comm, s_one / mb, "  Send (Mb):")
                _stats.write_histo(self.comm, r_one / mb, "  Recv (Mb):")

    def _need_kv(self, what):
        if self.kv is None:
            raise RuntimeError(f"Cannot {what} without KeyValue")

    def _need_kmv(self, what):
        if self.kmv is None:
            raise RuntimeError(f"Cannot {what} without KeyMultiValue")

    def _note_shuffle(self, st):
        MapReduce.cssize += st.send_bytes
        MapReduce.crsize += st.recv_bytes
        MapReduce.commtime += st.seconds

    def _empty(self):
        return C.empty_kv(self.device, 0, 0)

    # ------------------------------------------------------------------ lifecycle
    def copy(self):
        """Deep copy of settings and KV/KMV (reference src/mapreduce.cpp:269-316)."""
        mr = MapReduce(self.comm, self.device)
        for k in ("mapstyle", "all2all", "verbosity", "timer", "memsize", "minpage", "maxpage",
                  "freepage", "outofcore", "zeropage", "keyalign", "valuealign", "fpath"):
            setattr(mr, k, getattr(self, k))
        if self.kv is not None:
            mr.kv = _clone_kv(self.kv)
        if self.kmv is not None:
            mr.kmv = _clone_kmv(self.kmv)
        return mr

    def destroy(self):
        self.kv = self.kmv = None
        MapReduce.instances_now = max(0, MapReduce.instances_now - 1)

    def __del__(self):
        try:
            MapReduce.instances_now = max(0, MapReduce.instances_now - 1)
        except Exception:
            pass

    def set_fpath(self, path):
        self.fpath = str(path)

    def communicator(self):
        return self.comm

    def num_procs(self):
        return self.nprocs

    def my_proc(self):
        return self.me

    # ------------------------------------------------------------------ add / open / close
    def add(self, mr: "MapReduce"):
        """Append another MR's KV pairs to this KV (reference :348-374)."""
        self._start()
        self._need_kv("add")
        if mr.kv is None:
            raise RuntimeError("MapReduce passed to add() does not have KeyValue pairs")
        self.kv = C.concat([self.kv, mr.kv], self.device)
        self._stats("Add", 0)
        return self._count(self.kv.n)

    def open(self, addflag=0):
        """Let other MRs' callbacks add pairs into this MR via `mr.kv_open`
        (reference :1648-1664; used by luby_find / sssp)."""
        self._open = self._new_kv()
        self._open_add = addflag
        self.kmv = None
        return self._open

    @property
    def kv_open(self):
        if self._open is None:
            raise RuntimeError("MapReduce is not open")
        return self._open

    def close(self):
        if self._open is None:
            raise RuntimeError("Cannot close MapReduce that is not open")
        new = self._open.finish()
        self._open = None
        if self._open_add and self.kv is not None:
            self.kv = C.concat([self.kv, new], self.device)
        else:
            self.kv = new
        self._stats("Close", 0)
        return self._count(self.kv.n)

    # ------------------------------------------------------------------ map variants
    def _my_tasks(self, nmap):
        P, me = self.nprocs, self.me
        if self.mapstyle == 0 or P == 1:
            lo, hi = me * nmap // P, (me + 1) * nmap // P
            return range(lo, hi)
        if self.mapstyle == 1:
            return range(me, nmap, P)
        return _dynamic_tasks(self, nmap)

    def _finish_map(self, kvb, addflag, heading="Map"):
        new = kvb.finish()
        if addflag and self.kv is not None:
            self.kv = C.concat([self.kv, new], self.device)
        else:
            self.kv = new
        self.kmv = None
        self._stats(heading, 0)
        return self._count(self.kv.n)

    def map(self, nmap, fn, ptr=None, addflag=0):
        """nmap tasks; fn(itask, kv[, ptr]) (reference :1044-1051, map_tasks :1102-1225)."""
        if isinstance(nmap, MapReduce):  # map(mr, fn, ptr, addflag) overload
            return self.map_mr(nmap, fn, ptr, addflag)
        self._start()
        kvb = self._new_kv()
        for t in self._my_tasks(int(nmap)):
            _call(fn, 2, (t, kvb), ptr)
        return self._finish_map(kvb, addflag)

    def map_batch(self, nmap, fn, ptr=None, addflag=0):
        """Device-tier map: same task partitioning, but fn(itask, kv, ptr) is
        expected to emit whole tensors via kv.add_tensors()/kv.add_kv()."""
        return self.map(nmap, fn, ptr, addflag)

    def map_file(self, files, selfflag, recurse, readflag, fn, ptr=None, addflag=0):
        """One task per file; fn(itask, filename, kv[, ptr]) (reference :1060-1092)."""
        self._start()
        flist = _stats.find_files(self.comm, files, selfflag, recurse, readflag)
        self.mapfilecount = len(flist)
        kvb = self._new_kv()
        if selfflag:
            tasks = range(len(flist))
        else:
            tasks = self._my_tasks(len(flist))
        for t in tasks:
            _call(fn, 3, (t, flist[t], kvb), ptr)
        return self._finish_map(kvb, addflag)

    def map_file_char(self, nmap, files, selfflag, recurse, readflag, sepchar, delta, fn, ptr=None,
                      addflag=0):
        """Split files into nmap chunks at a separator char; fn(itask, chunk_bytes, kv[, ptr])
        (reference map_chunks/map_file_wrapper :1232-1262, :1312-1552)."""
        sep = sepchar.encode() if isinstance(sepchar, str) else bytes([sepchar]) if isinstance(sepchar, int) else sepchar
        return self._map_chunks(nmap, files, selfflag, recurse, readflag, sep, True, delta, fn, ptr, addflag)

    def map_file_str(self, nmap, files, selfflag, recurse, readflag, sepstr, delta, fn, ptr=None,
                     addflag=0):
        sep = sepstr.encode() if isinstance(sepstr, str) else bytes(sepstr)
        return self._map_chunks(nmap, files, selfflag, recurse, readflag, sep, False, delta, fn, ptr, addflag)

    def _map_chunks(self, nmap, files, selfflag, recurse, readflag, sep, is_char, delta, fn, ptr, addflag):
        self._start()
        flist = _stats.find_files(self.comm, files, selfflag, recurse, readflag)
        self.mapfilecount = len(flist)
        plan = _stats.plan_chunks(self.comm, flist, nmap, delta)
        kvb = self._new_kv()
        verbosity, timer = self.verbosity, self.timer
        for t in self._my_tasks(len(plan)):
            ifile, itask, ntask, fsize = plan[t]
            chunk = _stats.read_chunk(flist[ifile], fsize, itask, ntask, delta, sep, is_char)
            MapReduce.rsize += len(chunk)
            _call(fn, 3, (t, chunk, kvb), ptr)
        self.verbosity, self.timer = verbosity, timer
        return self._finish_map(kvb, addflag)

    def map_mr(self, mr, fn, ptr=None, addflag=0):
        """fn(itask, key, value, kv[, ptr]) for each pair of mr's KV (reference :1560-1642)."""
        self._start()
        if mr.kv is None:
            raise RuntimeError("MapReduce passed to map() does not have KeyValue pairs")
        src = mr.kv
        kvb = self._new_kv()
        C.kv_iter(src, lambda i, k, v: _call(fn, 4, (i, k, v, kvb), ptr))
        if mr is self and addflag:
            new = kvb.finish()
            self.kv = C.concat([src, new], self.device)
            self.kmv = None
            self._stats("Map", 0)
            return self._count(self.kv.n)
        return self._finish_map(kvb, addflag)

    def map_mr_batch(self, mr, fn, ptr=None, addflag=0):
        """Device-tier map over another MR: fn(src_kv, kv[, ptr]) receives the
        whole native KV (device tensors) once and emits tensors."""
        self._start()
        if mr.kv is None:
            raise RuntimeError("MapReduce passed to map() does not have KeyValue pairs")
        src = mr.kv
        kvb = self._new_kv()
        _call(fn, 2, (src, kvb), ptr)
        if mr is self and addflag:
            new = kvb.finish()
            self.kv = C.concat([src, new], self.device)
            self.kmv = None
            self._stats("Map", 0)
            return self._count(self.kv.n)
        return self._finish_map(kvb, addflag)

    # ------------------------------------------------------------------ shuffle
    def aggregate(self, hash=None):
        """Send each KV pair to the rank owning its key (reference :385-563).
        hash=None: hashlittle(key, kb, P) % P computed on the GPU.
        hash=callable(key_bytes) -> int: user hash (evaluated on the host)."""
        self._start()
        self._need_kv("aggregate")
        if self.nprocs > 1:
            if hash is None:
                kv, st = C.aggregate(self.kv, self.comm.pg)
            else:
                dest = []
                C.kv_iter(self.kv, lambda i, k, v: dest.append(int(hash(k)) % self.nprocs))
                d = torch.tensor(dest, dtype=torch.int32, device=self.device)
                kv, st = C.exchange(self.kv, d, self.comm.pg)
            self.kv = kv
            self._note_shuffle(st)
        self._stats("Aggregate", 0)
        return self._count(self.kv.n)

    def aggregate_dest(self, dest: torch.Tensor):
        """Shuffle with an explicit int32 destination rank per pair (device)."""
        self._start()
        self._need_kv("aggregate")
        if self.nprocs > 1:
            kv, st = C.exchange(self.kv, dest.to(device=self.device, dtype=torch.int32), self.comm.pg)
            self.kv = kv
            self._note_shuffle(st)
        self._stats("Aggregate", 0)
        return self._count(self.kv.n)

    def broadcast(self, root):
        """Root's KV replicated to all ranks (reference :569-623)."""
        self._start()
        self._need_kv("broadcast")
        if self.nprocs > 1:
            self.kv = C.broadcast(self.kv, int(root), self.comm.pg)
        self._stats("Broadcast", 0)
        return self._count(self.kv.n)

    def gather(self, nprocs):
        """Move all pairs onto ranks 0..nprocs-1 (reference :893-1036)."""
        self._start()
        self._need_kv("gather")
        if nprocs < 1 or nprocs > self.nprocs:
            raise RuntimeError("Invalid proc count for gather")
        if self.nprocs > 1 and nprocs < self.nprocs:
            kv, st = C.gather_to(self.kv, int(nprocs), self.comm.pg)
            self.kv = kv
            self._note_shuffle(st)
        self._stats("Gather", 0)
        return self._count(self.kv.n)

    # ------------------------------------------------------------------ group-by
    def convert(self):
        """Local group-by KV -> KMV (reference :861-886)."""
        self._start()
        self._need_kv("convert")
        self.kmv, self.last_convert = C.convert(self.kv)
        self.kv = None
        self._stats("Convert", 1)
        return self._count(self.kmv.nkey)

    def collate(self, hash=None):
        """aggregate + convert (reference :710-738)."""
        self._start()
        self._need_kv("collate")
        v, t = self.verbosity, self.timer
        self.verbosity = self.timer = 0
        self.aggregate(hash)
        self.convert()
        self.verbosity, self.timer = v, t
        self._stats("Collate", 1)
        return self._count(self.kmv.nkey)

    def clone(self):
        """KV -> KMV with one value per key (reference :631-652)."""
        self._start()
        self._need_kv("clone")
        self.kmv = C.clone(self.kv)
        self.kv = None
        self._stats("Clone", 1)
        return self._count(self.kmv.nkey)

    def collapse(self, key):
        """Local KV -> one KMV pair key -> [k0,v0,k1,v1,...] (reference :681-702)."""
        self._start()
        self._need_kv("collapse")
        self.kmv = C.collapse(self.kv, to_bytes(key))
        self.kv = None
        self._stats("Collapse", 1)
        return self._count(self.kmv.nkey)

    def scrunch(self, nprocs, key):
        """gather(nprocs) + collapse(key) (reference :2075-2095)."""
        self._start()
        v, t = self.verbosity, self.timer
        self.verbosity = self.timer = 0
        self.gather(nprocs)
        self.collapse(key)
        self.verbosity, self.timer = v, t
        self._stats("Scrunch", 1)
        return self._count(self.kmv.nkey)

    # ------------------------------------------------------------------ reduce family
    def _reduce_impl(self, fn, ptr, heading):
        kmv = self.kmv
        if isinstance(fn, str):
            op, _, dtype = fn.partition(":")
            self.kv = C.reduce_builtin(kmv, op, dtype or "int32")
        else:
            kvb = self._new_kv()
            self._cur_kmv = kmv

            def one(key, values):
                mv = MultiValue(values)
                _call(fn, 3, (key, mv, kvb), ptr)

            C.kmv_iter(kmv, one)
            self.kv = kvb.finish()
        self.kmv = None
        self._stats(heading, 0)
        return self._count(self.kv.n)

    def reduce(self, fn, ptr=None):
        """KMV -> KV. fn(key, values, kv[, ptr]) per unique key (reference :1769-1867).
        fn may also be a built-in device reducer name: "count", "first", "last",
        "sum:<dtype>", "min:<dtype>", "max:<dtype>" (dtype int32|int64|float32|float64)."""
        self._start()
        self._need_kmv("reduce")
        return self._reduce_impl(fn, ptr, "Reduce")

    def reduce_batch(self, fn, ptr=None):
        """Device-tier reduce: fn(kmv, kv[, ptr]) gets the whole native KMV
        (unique keys, values, CSR seg offsets in HBM) and emits tensors."""
        self._start()
        self._need_kmv("reduce")
        kvb = self._new_kv()
        _call(fn, 2, (self.kmv, kvb), ptr)
        self.kv = kvb.finish()
        self.kmv = None
        self._stats("Reduce", 0)
        return self._count(self.kv.n)

    def compress(self, fn, ptr=None):
        """Local convert + reduce: a combiner before the shuffle (reference :749-851)."""
        self._start()
        self._need_kv("compress")
        self.kmv, self.last_convert = C.convert(self.kv)
        self.kv = None
        return self._reduce_impl(fn, ptr, "Compress")

    def scan_kv(self, fn, ptr=None):
        """Read-only fn(key, value[, ptr]) over the KV (reference :1933-1976)."""
        self._start()
        self._need_kv("scan")
        C.kv_iter(self.kv, lambda i, k, v: _call(fn, 2, (k, v), ptr))
        self._stats("Scan", 0)
        return self._count(self.kv.n)

    def scan_kmv(self, fn, ptr=None):
        """Read-only fn(key, values[, ptr]) over the KMV (reference :1984-2065)."""
        self._start()
        self._need_kmv("scan")
        C.kmv_iter(self.kmv, lambda k, vals: _call(fn, 2, (k, MultiValue(vals)), ptr))
        self._stats("Scan", 1)
        return self._count(self.kmv.nkey)

    def scan(self, fn, ptr=None):
        return self.scan_kv(fn, ptr) if self.kv is not None else self.scan_kmv(fn, ptr)

    # multi-block KMV iteration (reference :1874-1925): values are lists, so a
    # "block" is a slice of MultiValue.block_size values
    def multivalue_blocks(self, mv: MultiValue):
        return len(mv), mv.nblocks()

    def multivalue_block_select(self, which):
        self._mv_block = which

    def multivalue_block(self, mv: MultiValue, iblock):
        return mv.block(iblock)

    # ------------------------------------------------------------------ sorting
    def _sort(self, what, flag_or_fn, heading):
        self._start()
        if what == "multi":
            self._need_kmv("sort_multivalues")
            if callable(flag_or_fn):
                self.kmv = _host_sort_multivalues(self.kmv, flag_or_fn, self.device)
            else:
                self.kmv = C.sort_multivalues(self.kmv, int(flag_or_fn))
            self._stats(heading, 1)
            return self._count(self.kmv.nkey)
        self._need_kv(heading.lower())
        by_value = what == "values"
        if callable(flag_or_fn):
            self.kv = _host_sort_kv(self.kv, flag_or_fn, by_value, self.device)
        else:
            self.kv = C.sort_kv(self.kv, int(flag_or_fn), by_value)
        self._stats(heading, 0)
        return self._count(self.kv.n)

    def sort_keys(self, flag):
        """Local sort by key: flag 1 int,2 uint64,3 float,4 double,5 str,6 strn (negative =
        descending) or a compare(a_bytes, b_bytes) -> int callable (reference :2102-2149)."""
        return self._sort("keys", flag, "Sort_keys")

    def sort_values(self, flag):
        return self._sort("values", flag, "Sort_values")

    def sort_multivalues(self, flag):
        return self._sort("multi", flag, "Sort_multivalues")

    # reference python wrapper names
    sort_keys_flag = sort_keys
    sort_values_flag = sort_values
    sort_multivalues_flag = sort_multivalues

    # ------------------------------------------------------------------ printing
    def print(self, proc=-1, nstride=1, kflag=5, vflag=5, file=None, fflag=0):
        """Print KV/KMV pairs (reference :1671-1761). proc=-1: every rank in order."""
        if self.kv is None and self.kmv is None:
            raise RuntimeError("Cannot print without KeyValue or KeyMultiValue")
        if not (0 <= kflag <= 7 and 0 <= vflag <= 7):
            raise RuntimeError("Invalid print args")
        lines = _stats.format_pairs(self, nstride, kflag, vflag)
        if proc == self.me:
            _emit(lines, file, "w")
        if proc >= 0:
            return
        if file is not None and fflag == 1:
            _emit(lines, f"{file}.{self.me}", "w")
            return
        for r in range(self.nprocs):
            self.comm.barrier()
            if r == self.me:
                _emit(lines, file, "a" if file else "w")
        self.comm.barrier()

    def print_screen(self, proc, nstride, kflag, vflag):
        return self.print(proc, nstride, kflag, vflag)

    def print_file(self, file, fflag, proc, nstride, kflag, vflag):
        return self.print(proc, nstride, kflag, vflag, file=file, fflag=fflag)

    # ------------------------------------------------------------------ stats
    def kv_stats(self, level=0):
        self._need_kv("print stats")
        kv = self.kv
        n, kb, vb, eb = self.comm.allreduce([kv.n, kv.key_bytes(), kv.value_bytes(), kv.nbytes()], "sum")
        mb = 1024.0 * 1024.0
        if level == 1 and self.me == 0:
            print(f"{n} pairs, {kb / mb:.3g} Mb keys, {vb / mb:.3g} Mb values, {eb / mb:.3g} Mb, 1 pages")
        if level == 2:
            _stats.write_histo(self.comm, float(kv.n), "  KV pairs:")
            _stats.write_histo(self.comm, kv.key_bytes() / mb, "  Kdata (Mb):")
            _stats.write_histo(self.comm, kv.value_bytes() / mb, "  Vdata (Mb):")
        return n

    def kmv_stats(self, level=0):
        self._need_kmv("print stats")
        kmv = self.kmv
        vbytes = kmv.nval * kmv.vw if kmv.vw >= 0 else int(kmv.voff[kmv.nval].item()) if kmv.nval else 0
        n, kb, vb, eb = self.comm.allreduce([kmv.nkey, kmv.keys.key_bytes(), vbytes, kmv.nbytes()], "sum")
        mb = 1024.0 * 1024.0
        if level == 1 and self.me == 0:
            print(f"{n} pairs, {kb / mb:.3g} Mb keys, {vb / mb:.3g} Mb values, {eb / mb:.3g} Mb, 1 pages")
        if level == 2:
            _stats.write_histo(self.comm, float(kmv.nkey), "  KMV pairs:")
            _stats.write_histo(self.comm, kmv.keys.key_bytes() / mb, "  Kdata (Mb):")
            _stats.write_histo(self.comm, vbytes / mb, "  Vdata (Mb):")
        return n

    def cummulative_stats(self, level=1, reset=0):
        mb, gb = 1024.0 * 1024.0, 1024.0 ** 3
        if self.me == 0:
            print(f"MapReduce-MPI ({MRMPI_VERSION})")
        mx = self.comm.allreduce(MapReduce.msizemax, "max")
        sm = self.comm.allreduce(MapReduce.msizemax, "sum")
        if self.me == 0:
            print(f"Cummulative hi-water mem = {mx / mb:.3g} Mb any proc, {sm / gb:.3g} Gb all procs")
        cs, cr = self.comm.allreduce([MapReduce.cssize, MapReduce.crsize], "sum")
        ct = self.comm.allreduce(MapReduce.commtime, "sum", dtype=torch.float64)
        if cs or cr:
            if self.me == 0:
                print(f"Cummulative comm = {cs / mb:.3g} Mb send, {cr / mb:.3g} Mb recv, {ct / self.nprocs:.3g} secs")
            if level == 2:
                _stats.write_histo(self.comm, MapReduce.cssize / mb, "  Send (Mb):")
                _stats.write_histo(self.comm, MapReduce.crsize / mb, "  Recv (Mb):")
        rs, ws = self.comm.allreduce([MapReduce.rsize, MapReduce.wsize], "sum")
        if rs or ws:
            if self.me == 0:
                print(f"Cummulative I/O = {rs / mb:.3g} Mb read, {ws / mb:.3g} Mb write")
        if reset:
            MapReduce.rsize = MapReduce.wsize = MapReduce.cssize = MapReduce.crsize = 0

    # ------------------------------------------------------------------ host spill tier
    def spill(self):
        """Move this MR's data to pinned host DRAM (the out-of-core tier)."""
        if self.kv is not None:
            self.kv = _kv_to_host(self.kv)
        if self.kmv is not None:
            self.kmv = _kmv_to(self.kmv, "cpu", pin=True)

    def unspill(self):
        if self.kv is not None:
            self.kv = self.kv.to(self.device)
        if self.kmv is not None:
            self.kmv = _kmv_to(self.kmv, self.device)

    # ------------------------------------------------------------------ python convenience
    def kv_pairs(self):
        """Local KV pairs as a list of (key_bytes, value_bytes) (host)."""
        out = []
        if self.kv is not None:
            C.kv_iter(self.kv, lambda i, k, v: out.append((k, v)))
        return out

    def kmv_pairs(self):
        out = []
        if self.kmv is not None:
            C.kmv_iter(self.kmv, lambda k, vals: out.append((k, list(vals))))
        return out


# ---------------------------------------------------------------------- module helpers

def _emit(lines, file, mode):
    if file is None:
        sys.stdout.write("".join(lines))
        sys.stdout.flush()
    else:
        with open(file, mode) as f:
            f.write("".join(lines))


def _clone_t(t):
    return t.clone() if t is not None and isinstance(t, torch.Tensor) and t.numel() >= 0 else t


def _clone_kv(kv):
    o = C.KV()
    o.n, o.kw, o.vw = kv.n, kv.kw, kv.vw
    o.kdata, o.vdata = kv.kdata.clone(), kv.vdata.clone()
    if kv.kw < 0:
        o.koff = kv.koff.clone()
    if kv.vw < 0:
        o.voff = kv.voff.clone()
    return o


def _clone_kmv(kmv):
    o = C.KMV()
    o.keys = _clone_kv(kmv.keys)
    o.vdata = kmv.vdata.clone()
    if kmv.vw < 0:
        o.voff = kmv.voff.clone()
    o.vw, o.seg, o.nkey, o.nval = kmv.vw, kmv.seg.clone(), kmv.nkey, kmv.nval
    return o


def _kv_to_host(kv):
    o = C.KV()
    o.n, o.kw, o.vw = kv.n, kv.kw, kv.vw

    def pin(t):
        h = torch.empty(t.shape, dtype=t.dtype, pin_memory=torch.cuda.is_available())
        h.copy_(t, non_blocking=False)
        return h
    o.kdata, o.vdata = pin(kv.kdata), pin(kv.vdata)
    if kv.kw < 0:
        o.koff = pin(kv.koff)
    if kv.vw < 0:
        o.voff = pin(kv.voff)
    return o


def _kmv_to(kmv, dev, pin=False):
    o = C.KMV()
    o.keys = _kv_to_host(kmv.keys) if pin else kmv.keys.to(dev)
    o.vdata = kmv.vdata.to(dev)
    if kmv.vw < 0:
        o.voff = kmv.voff.to(dev)
    o.vw, o.seg, o.nkey, o.nval = kmv.vw, kmv.seg.to(dev), kmv.nkey, kmv.nval
    return o


def _dynamic_tasks(mr, nmap):
    """mapstyle 2: dynamic load balancing. The reference uses rank 0 as a
    master handing out tasks over MPI (src/mapreduce.cpp:1164-1211); here
    every rank (including 0) pulls the next task id from an atomic counter in
    the c10d TCPStore, so no rank idles as a pure master."""
    import torch.distributed as dist
    store = dist.distributed_c10d._get_default_store()
    key = f"mrhip_map_{mr.instance_me}_{_dynamic_tasks.seq}"
    _dynamic_tasks.seq += 1
    mr.comm.barrier()
    while True:
        t = store.add(key, 1) - 1
        if t >= nmap:
            break
        yield t
    mr.comm.barrier()


_dynamic_tasks.seq = 0


def _host_sort_kv(kv, cmp, by_value, device):
    pairs = []
    C.kv_iter(kv, lambda i, k, v: pairs.append((v if by_value else k)))
    order = sorted(range(len(pairs)), key=functools.cmp_to_key(lambda a, b: cmp(pairs[a], pairs[b])))
    perm = torch.tensor(order, dtype=torch.int32, device=device)
    return C.gather(kv, perm)


def _host_sort_multivalues(kmv, cmp, device):
    groups = []
    C.kmv_iter(kmv, lambda k, vals: groups.append(list(vals)))
    perm = []
    base = 0
    for vals in groups:
        order = sorted(range(len(vals)), key=functools.cmp_to_key(lambda a, b: cmp(vals[a], vals[b])))
        perm.extend(base + o for o in order)
        base += len(vals)
    p = torch.tensor(perm, dtype=torch.int32, device=device)
    vkv = C.KV()
    vkv.n, vkv.kw, vkv.vw = kmv.nval, 0, kmv.vw
    vkv.kdata = torch.empty(0, dtype=torch.uint8, device=device)
    vkv.vdata = kmv.vdata
    if kmv.vw < 0:
        vkv.voff = kmv.voff
    g = C.gather(vkv, p)
    o = C.KMV()
    o.keys, o.vw, o.seg, o.nkey, o.nval = kmv.keys, kmv.vw, kmv.seg, kmv.nkey, kmv.nval
    o.vdata = g.vdata
    if kmv.vw < 0:
        o.voff = g.voff
    return o
