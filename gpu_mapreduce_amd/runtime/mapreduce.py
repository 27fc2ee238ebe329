"""MapReduce object: the Python face of the native MapReduce
(csrc/engine/mapreduce.h, the same object the MR_* C API drives).

Same method names, settings, defaults and return values (global pair counts)
as MR-MPI's `class MapReduce` (reference src/mapreduce.h:28-126,
src/mapreduce.cpp:93-3574). Everything below the callbacks is native:
the MR's KV/KMV live in HBM as SoA tensors, the shuffle is an RCCL
all-to-all over xGMI issued from C++, group-by / sort / segmented reduce are
HIP kernels. This layer only adapts Python callables:

* host callbacks keep MR-MPI shapes, with bytes instead of (char*, int):
  map(itask, kv), map_file(itask, fname, kv), map_file_char/str(itask, chunk, kv),
  map_mr(itask, key, value, kv), reduce/compress(key, values, kv) where
  `values` is a MultiValue list (multi-block keys arrive whole; the block
  API is still available), scan(key, value) / scan(key, values), hash(key),
  compare(a, b); each may take a trailing `ptr` (MR-MPI's void* APPptr);
* batch callbacks (`map_batch`, `map_mr_batch`, `reduce_batch`) receive the
  device KV / KMV and emit tensors, keeping data in HBM;
* built-in device reducers: reduce("count"), reduce("sum:float32"), ...
"""
from __future__ import annotations

import inspect
import os
import sys

from .._ext import C
from ..parallel.comm import Comm, world
from .keyvalue import KeyValue, to_bytes

MRMPI_VERSION = "gpu_mapreduce_amd 0.1 (MR-MPI 11 Mar 2013 API)"

_SETTINGS = ("mapstyle", "all2all", "verbosity", "timer", "memsize", "minpage", "maxpage", "freepage",
             "outofcore", "zeropage", "keyalign", "valuealign", "fpath",
             # MI355X-native settings (mapreduce.h): shuffle receive cap, HBM /
             # pinned-host budgets of the out-of-core tiers, pipelined streams
             "chunk_bytes", "hbm_budget", "host_budget", "streams", "pipeline")


def _arity(fn):
    try:
        sig = inspect.signature(fn)
    except (TypeError, ValueError):
        return None
    if any(p.kind == p.VAR_POSITIONAL for p in sig.parameters.values()):
        return None
    return len([p for p in sig.parameters.values() if p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD)])


def _bind(fn, nargs, ptr):
    """MR-MPI callbacks take an optional trailing `ptr`; pass it only if the
    callback accepts it (the reference Python wrapper does the same,
    python/mrmpi.py:185-188)."""
    n = _arity(fn)
    if n is None or n > nargs:
        return lambda *a: fn(*a, ptr)
    return fn


class MultiValue(list):
    """The values of one KMV key as a list of bytes objects. Long value lists
    can also be walked in blocks (MR-MPI multivalue_blocks/multivalue_block,
    reference src/mapreduce.cpp:1874-1925)."""

    block_size = 1 << 20

    def nblocks(self):
        return max(1, (len(self) + self.block_size - 1) // self.block_size)

    def block(self, i):
        return self[i * self.block_size:(i + 1) * self.block_size]

    @staticmethod
    def of(vals):
        """a callback's values: a list, or the engine's multi-block cursor"""
        return BlockMultiValue(vals) if isinstance(vals, C.ValueBlocks) else MultiValue(vals)


class BlockMultiValue:
    """The values of a key that spans several pages (the engine's multi-block
    KMV, reference src/mapreduce.cpp:1828-1848): never one list — block(i)
    materialises one page of values (bytes objects) through the engine's
    multivalue_block; iteration walks the blocks in order. Valid only inside
    the reduce / compress callback it was passed to."""

    block_size = None  # set by the engine (the page size), not by the caller

    def __init__(self, blocks):
        self._b = blocks

    def __len__(self):
        return int(self._b.nvalues)

    def nblocks(self):
        return int(self._b.nblocks)

    def block(self, i):
        return self._b.block(int(i))

    def __iter__(self):
        for i in range(self.nblocks()):
            yield from self._b.block(i)


class _Counters(type):
    """MapReduce.cssize etc. read the native static counters
    (reference src/mapreduce.h:46-57)."""

    def __getattr__(cls, name):
        d = C.mr_counters()
        if name in d:
            return d[name]
        raise AttributeError(name)


class MapReduce(metaclass=_Counters):
    def __init__(self, comm: Comm | None = None, device: str | None = None, _native=None):
        self.comm = comm if comm is not None else world()
        if device is not None and str(device) != self.comm.device:
            self.comm = Comm(self.comm.group, device=str(device))
        self.device = self.comm.device
        self.me = self.comm.rank
        self.nprocs = self.comm.size
        self._m = _native if _native is not None else C.NativeMapReduce(self.comm.native)
        _route_screen()

    # ------------------------------------------------------------------ settings / data
    def __getattr__(self, name):
        if name in _SETTINGS or name in ("mapfilecount", "kv", "kmv", "last_convert", "spool_stats", "kv_parts", "kmv_parts"):
            return getattr(self.__dict__["_m"], name)
        raise AttributeError(name)

    def __setattr__(self, name, value):
        if name in _SETTINGS or name in ("mapfilecount", "kv", "kmv"):
            setattr(self._m, name, value)
        else:
            object.__setattr__(self, name, value)

    @staticmethod
    def count_io(read=0, write=0):
        C.mr_count_io(int(read), int(write))

    @property
    def native(self):
        return self._m

    # ------------------------------------------------------------------ lifecycle
    def copy(self):
        """Deep copy of settings and KV/KMV (reference src/mapreduce.cpp:269-316)."""
        return MapReduce(self.comm, _native=self._m.copy())

    def destroy(self):
        self._m.kv = None
        self._m.kmv = None

    def set_fpath(self, path):
        self._m.fpath = str(path)

    def communicator(self):
        return self.comm

    def num_procs(self):
        return self.nprocs

    def my_proc(self):
        return self.me

    # ------------------------------------------------------------------ add / open / close
    def add(self, mr: "MapReduce"):
        return self._m.add(mr._m)

    def open(self, addflag=0):
        """Let other MRs' callbacks add pairs into this MR via `mr.kv_open`
        (reference :1648-1664; used by luby_find / sssp)."""
        self._m.open(int(addflag))
        return self.kv_open

    @property
    def kv_open(self):
        return KeyValue.wrap(self._m.kv_open())

    def close(self):
        return self._m.close()

    # ------------------------------------------------------------------ map variants
    def map(self, nmap, fn, ptr=None, addflag=0):
        """nmap tasks; fn(itask, kv[, ptr]) (reference :1044-1051, tasks :1102-1225)."""
        if isinstance(nmap, MapReduce):  # map(mr, fn, ptr, addflag) overload
            return self.map_mr(nmap, fn, ptr, addflag)
        f = _bind(fn, 2, ptr)
        return self._m.map(int(nmap), lambda t, h: f(t, KeyValue.wrap(h)), int(addflag))

    map_batch = map

    def map_file(self, files, selfflag, recurse, readflag, fn, ptr=None, addflag=0):
        """One task per file; fn(itask, filename, kv[, ptr]) (reference :1060-1092)."""
        f = _bind(fn, 3, ptr)
        return self._m.map_file(_files(files), int(selfflag), int(recurse), int(readflag),
                                lambda t, name, h: f(t, name, KeyValue.wrap(h)), int(addflag))

    def map_file_char(self, nmap, files, selfflag, recurse, readflag, sepchar, delta, fn, ptr=None, addflag=0):
        """Split files into nmap chunks at a separator char; fn(itask, chunk_bytes, kv[, ptr])
        (reference map_chunks/map_file_wrapper :1232-1262, :1312-1552)."""
        sep = chr(sepchar) if isinstance(sepchar, int) else sepchar.decode() if isinstance(sepchar, bytes) else sepchar
        return self._chunks(nmap, files, selfflag, recurse, readflag, sep, True, delta, fn, ptr, addflag)

    def map_file_str(self, nmap, files, selfflag, recurse, readflag, sepstr, delta, fn, ptr=None, addflag=0):
        sep = sepstr.decode() if isinstance(sepstr, bytes) else sepstr
        return self._chunks(nmap, files, selfflag, recurse, readflag, sep, False, delta, fn, ptr, addflag)

    def _chunks(self, nmap, files, selfflag, recurse, readflag, sep, is_char, delta, fn, ptr, addflag):
        f = _bind(fn, 3, ptr)
        return self._m.map_file_chunks(int(nmap), _files(files), int(selfflag), int(recurse), int(readflag), sep,
                                       is_char, int(delta), lambda t, chunk, h: f(t, chunk, KeyValue.wrap(h)),
                                       int(addflag))

    def map_mr(self, mr, fn, ptr=None, addflag=0):
        """fn(itask, key, value, kv[, ptr]) for each pair of mr's KV (reference :1560-1642)."""
        f = _bind(fn, 4, ptr)
        return self._m.map_mr(mr._m, lambda i, k, v, h: f(i, k, v, KeyValue.wrap(h)), int(addflag))

    def map_mr_batch(self, mr, fn, ptr=None, addflag=0):
        """Device-tier map over another MR: fn(src_kv, kv[, ptr]) receives the
        whole native KV (device tensors) once and emits tensors."""
        f = _bind(fn, 2, ptr)
        return self._m.map_mr_batch(mr._m, lambda src, h: f(src, KeyValue.wrap(h)), int(addflag))

    # ------------------------------------------------------------------ shuffle
    def aggregate(self, hash=None):
        """Send each KV pair to the rank owning its key (reference :385-563).
        hash=None: hashlittle(key, kb, P) % P on the GPU; else hash(key) -> int on the host."""
        return self._m.aggregate(hash)

    def aggregate_dest(self, dest):
        """Shuffle with an explicit int32 destination rank per pair (device tensor)."""
        return self._m.aggregate_dest(dest)

    def broadcast(self, root):
        return self._m.broadcast(int(root))

    def gather(self, nprocs):
        return self._m.gather(int(nprocs))

    # ------------------------------------------------------------------ group-by
    def convert(self):
        return self._m.convert()

    def convert_prehashed(self, hashes):
        """convert with hash64_keys(kv) already computed by the producer (int64 [n])"""
        return self._m.convert_prehashed(hashes)

    def collate(self, hash=None):
        return self._m.collate(hash)

    def clone(self):
        return self._m.clone()

    def collapse(self, key):
        return self._m.collapse(to_bytes(key))

    def scrunch(self, nprocs, key):
        return self._m.scrunch(int(nprocs), to_bytes(key))

    # ------------------------------------------------------------------ reduce family
    def reduce(self, fn, ptr=None):
        """KMV -> KV. fn(key, values, kv[, ptr]) per unique key (reference :1769-1867),
        or a built-in device reducer name: "count", "first", "last",
        "sum:<dtype>", "min:<dtype>", "max:<dtype>" (dtype int32|int64|float32|float64)."""
        if isinstance(fn, str):
            op, _, dtype = fn.partition(":")
            return self._m.reduce_builtin(op, dtype or "int32")
        f = _bind(fn, 3, ptr)
        return self._m.reduce(lambda k, vals, h: f(k, MultiValue.of(vals), KeyValue.wrap(h)))

    def reduce_batch(self, fn, ptr=None):
        """Device-tier reduce: fn(kmv, kv[, ptr]) gets the whole native KMV
        (unique keys, values, CSR seg offsets in HBM) and emits tensors."""
        f = _bind(fn, 2, ptr)
        return self._m.reduce_batch(lambda kmv, h: f(kmv, KeyValue.wrap(h)))

    def compress(self, fn, ptr=None):
        """Local convert + reduce: a combiner before the shuffle (reference :749-851)."""
        if isinstance(fn, str):
            op, _, dtype = fn.partition(":")
            return self._m.compress_builtin(op, dtype or "int32")
        f = _bind(fn, 3, ptr)
        return self._m.compress(lambda k, vals, h: f(k, MultiValue.of(vals), KeyValue.wrap(h)))

    def compress_batch(self, fn, ptr=None):
        """Device-tier compress: fn(kmv, kv[, ptr]) gets this rank's local
        groups as one native KMV (no shuffle) and emits tensors."""
        f = _bind(fn, 2, ptr)
        return self._m.compress_batch(lambda kmv, h: f(kmv, KeyValue.wrap(h)))

    # ---- device functors (csrc/engine/devfn.h): HIP device code compiled at run time
    def map_device(self, src, code, addflag=0):
        """map with a device functor: `src` a MapReduce (every pair through
        `__device__ void mr_map(mrd::Bytes key, mrd::Bytes value, long long
        index, mrd::Emit& out)`) or a task count (key / value empty, index =
        the task). One GPU thread per pair / task; no host round trip."""
        if isinstance(src, int):
            return self._m.map_device_tasks(int(src), code, addflag)
        return self._m.map_device(src._m, code, addflag)

    def reduce_device(self, code):
        """reduce with a device functor: every key through `__device__ void
        mr_reduce(mrd::Bytes key, mrd::Values values, mrd::Emit& out)`."""
        return self._m.reduce_device(code)

    def sort_keys_device(self, code, bits=64):
        """stable sort by a device sort-key functor: `__device__ unsigned long
        long mr_sortkey(mrd::Bytes key)` maps each key to a 64-bit key whose
        unsigned order is the wanted one (a comparator as a key extraction;
        `bits` low bits are sorted on)."""
        return self._m.sort_keys_device(code, bits)

    def sort_values_device(self, code, bits=64):
        """sort_keys_device over the values."""
        return self._m.sort_values_device(code, bits)

    def compress_device(self, code):
        """compress (local groups, no shuffle) with a device reduce functor."""
        return self._m.compress_device(code)

    def scan_kv(self, fn, ptr=None):
        """Read-only fn(key, value[, ptr]) over the KV (reference :1933-1976)."""
        return self._m.scan_kv(_bind(fn, 2, ptr))

    def scan_kmv(self, fn, ptr=None):
        """Read-only fn(key, values[, ptr]) over the KMV (reference :1984-2065)."""
        f = _bind(fn, 2, ptr)
        return self._m.scan_kmv(lambda k, vals: f(k, MultiValue(vals)))

    def scan(self, fn, ptr=None):
        return self.scan_kv(fn, ptr) if self.kv is not None else self.scan_kmv(fn, ptr)

    # multi-block KMV iteration for Python callbacks: values arrive as a whole
    # list; these give the reference's block view of it
    def multivalue_blocks(self, mv):
        return len(mv), mv.nblocks()

    def multivalue_block_select(self, which):
        pass

    def multivalue_block(self, mv, iblock):
        return mv.block(iblock)

    # ------------------------------------------------------------------ sorting
    def sort_keys(self, flag):
        """Local sort by key: flag 1 int,2 uint64,3 float,4 double,5 str,6 strn (negative =
        descending) or a compare(a_bytes, b_bytes) -> int callable (reference :2102-2149)."""
        return self._m.sort_keys_fn(flag) if callable(flag) else self._m.sort_keys(int(flag))

    def sort_values(self, flag):
        return self._m.sort_values_fn(flag) if callable(flag) else self._m.sort_values(int(flag))

    def sort_multivalues(self, flag):
        return self._m.sort_multivalues_fn(flag) if callable(flag) else self._m.sort_multivalues(int(flag))

    sort_keys_flag = sort_keys
    sort_values_flag = sort_values
    sort_multivalues_flag = sort_multivalues

    # ------------------------------------------------------------------ printing / stats
    def print(self, proc=-1, nstride=1, kflag=5, vflag=5, file=None, fflag=0):
        """Print KV/KMV pairs (reference :1671-1761). proc=-1: every rank in order."""
        _route_screen()
        self._m.print(int(proc), int(nstride), int(kflag), int(vflag), None if file is None else str(file), int(fflag))

    def print_screen(self, proc, nstride, kflag, vflag):
        return self.print(proc, nstride, kflag, vflag)

    def print_file(self, file, fflag, proc, nstride, kflag, vflag):
        return self.print(proc, nstride, kflag, vflag, file=file, fflag=fflag)

    def kv_stats(self, level=0):
        _route_screen()
        return self._m.kv_stats(int(level))

    def kmv_stats(self, level=0):
        _route_screen()
        return self._m.kmv_stats(int(level))

    def cummulative_stats(self, level=1, reset=0):
        _route_screen()
        self._m.cummulative_stats(int(level), int(reset))

    # ------------------------------------------------------------------ host spill tier
    def spill(self):
        """Move this MR's data to pinned host DRAM (the out-of-core tier)."""
        self._m.spill()

    def unspill(self):
        self._m.unspill()

    def spill_disk(self):
        """Write the data to fpath/mrmpi.<kv|kmv>.<instance>.<n>.<rank> and free
        it (disk tier); the next op reads it back."""
        self._m.spill_disk()

    @property
    def on_disk(self):
        return self._m.on_disk

    # ------------------------------------------------------------------ checkpoint / restart
    def save(self, path):
        """Write this rank's KV/KMV to `path` (".<rank>" appended when nprocs > 1)."""
        self._m.save(os.fspath(path))

    def load(self, path):
        """Replace this MR's data with a checkpoint written by save(); returns the global count."""
        return self._m.load(os.fspath(path))

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


def _files(files):
    if isinstance(files, (str, bytes, os.PathLike)):
        files = [files]
    return [os.fsdecode(f) for f in files]


_screen_target = [None]


def _route_screen():
    """Native stats/print output goes through the current sys.stdout so that
    redirected or captured Python stdout sees it."""
    if _screen_target[0] is not sys.stdout:
        _screen_target[0] = sys.stdout
        out = sys.stdout
        C.set_screen(lambda s: (out.write(s), out.flush()))
