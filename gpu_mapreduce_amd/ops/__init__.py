"""Typed Python entry points to the hand-written HIP/CDNA4 kernels
(csrc/kernels/*.hip) behind the engine. Every function dispatches on the
tensor device: cuda tensors run the gfx950 kernels, cpu tensors the engine's
host loops with identical semantics (the test oracle). No fallback exists
for a missing extension: importing this module without the built native
library fails.

Arguments are validated here, on the host, before anything launches: the
kernels take raw device pointers, so a wrong dtype, a tensor on another
device or an out-of-range count would otherwise read out of bounds on the
GPU (a fault that can reset the whole node). Each check raises ValueError /
TypeError naming the argument; the native entry points repeat the checks
that guard memory safety.

    exclusive_scan(x)                      scan.hip   reduce-then-scan, n+1 outputs
    radix_sort_pairs(keys, vals, lo, hi)   radix.hip  LSD 8-bit digits, wave64 multi-split
    hash32(kv, seed) / hash64(kv)          hash.hip   lookup3 hashlittle / hashlittle2, bit-exact
    partition_dest(kv, P)                  hash.hip   MR-MPI owner rank hashlittle(key,kb,P) % P
    group_by(kv)                           kvops/radix/segreduce: the convert() KV -> KMV
    segmented_reduce(kmv, op, dtype)       segreduce.hip  value-balanced, LDS-staged
    sort_kv(kv, flag, by_value)            radix.hip + key transforms (MR-MPI flags 1..6, +/-)
    scan_urls(text, n, doc)                text.hip   `<a href="` scan + URL extract
    tokenize(text, n)                      text.hip   whitespace tokenizer
    rmat_edges(...)                        graph.hip  Philox R-MAT generator
    plan_gather_reduce / plan_combine      graphops.hip  edge-plan propagation
    wedges(seg, nbr, centre)               graphops.hip  tri_find wedge generation
"""
from __future__ import annotations

import torch

from .._ext import C

__all__ = ["exclusive_scan", "radix_sort_pairs", "hash32", "hash64", "partition_dest", "group_by",
           "segmented_reduce", "sort_kv", "scan_urls", "tokenize", "rmat_edges", "plan_gather_reduce",
           "plan_combine", "wedges", "segments_sorted"]


def _tensor(t, name: str, dtypes, device=None) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor, got {type(t).__name__}")
    if dtypes is not None and t.dtype not in dtypes:
        raise TypeError(f"{name}: dtype {t.dtype}, expected one of {', '.join(str(d) for d in dtypes)}")
    if device is not None and t.device != device:
        raise ValueError(f"{name}: on {t.device}, the other operands are on {device}")
    if t.dim() != 1:
        raise ValueError(f"{name}: expected a 1-D tensor, got shape {tuple(t.shape)}")
    return t.contiguous()


def _segments(seg, name: str = "seg") -> torch.Tensor:
    seg = _tensor(seg, name, (torch.int64,))
    if seg.numel() < 1:
        raise ValueError(f"{name}: CSR offsets need ngroups + 1 >= 1 entries")
    return seg


_REDUCE_OPS = ("count", "sum", "min", "max", "first", "last")
_PLAN_OPS = {0: "sum", 1: "min", 2: "max"}


def exclusive_scan(x: torch.Tensor) -> torch.Tensor:
    """n+1 int64 outputs; out[n] is the total (int32/int64 input)."""
    return C.exclusive_scan(_tensor(x, "x", (torch.int32, torch.int64)))


def radix_sort_pairs(keys: torch.Tensor, vals: torch.Tensor, begin_bit: int = 0, end_bit: int = 64):
    """Stable sort of int64 keys (bits [begin_bit, end_bit)) carrying int32 values.
    Returns (sorted_keys, permuted_vals, passes_run)."""
    keys = _tensor(keys, "keys", (torch.int64,))
    vals = _tensor(vals, "vals", (torch.int32,), keys.device)
    if vals.numel() != keys.numel():
        raise ValueError(f"vals: {vals.numel()} values for {keys.numel()} keys")
    if not 0 <= begin_bit <= end_bit <= 64:
        raise ValueError(f"bit range [{begin_bit}, {end_bit}) outside [0, 64)")
    return C.radix_sort_pairs(keys, vals, begin_bit, end_bit)


def hash32(kv, seed: int = 0) -> torch.Tensor:
    """lookup3 hashlittle(key, len, seed) of every key (bit-exact with the reference's hash.cpp)."""
    return C.hash32_keys(kv, seed & 0xFFFFFFFF)


def hash64(kv) -> torch.Tensor:
    return C.hash64_keys(kv)


def partition_dest(kv, nprocs: int):
    """(int32 dest rank per pair, int64 per-rank counts)."""
    if nprocs < 1:
        raise ValueError(f"nprocs must be >= 1, got {nprocs}")
    return C.partition_dest(kv, nprocs)


def group_by(kv):
    """KV -> (KMV, ConvertStats): unique keys + values grouped in CSR segments."""
    return C.convert(kv)


def segmented_reduce(kmv, op: str = "count", dtype: str = "int32"):
    """op in count|sum|min|max|first|last over each key's values."""
    if op not in _REDUCE_OPS:
        raise ValueError(f"op {op!r} not one of {'|'.join(_REDUCE_OPS)}")
    return C.reduce_builtin(kmv, op, dtype)


def sort_kv(kv, flag: int, by_value: bool = False):
    """MR-MPI sort flags: +/-1 int32, +/-2 uint64, +/-3 float, +/-4 double, +/-5 string (NUL), +/-6 bytes."""
    if flag == 0 or abs(flag) > 6:
        raise ValueError(f"sort flag {flag} outside +/-1..6")
    return C.sort_kv(kv, flag, by_value)


def _text(text, n: int, name: str) -> torch.Tensor:
    text = _tensor(text, name, (torch.uint8,))
    if not 0 <= n <= text.numel() - 32:
        raise ValueError(f"n={n}: the {name} buffer holds {text.numel()} bytes and must be padded by >= 32")
    return text


def scan_urls(text: torch.Tensor, n: int, doc_id: int):
    """KV(url + NUL, int32 doc_id) for every `<a href="...` in text[:n] (text padded >= 32 B)."""
    return C.map_urls(_text(text, n, "text"), n, doc_id)


def tokenize(text: torch.Tensor, n: int):
    """KV(word + NUL, NULL) for every whitespace-separated word of text[:n]."""
    return C.map_words(_text(text, n, "text"), n)


def rmat_edges(nedges: int, nlevels: int, a: float, b: float, c: float, d: float, fraction: float, seed: int,
               first_edge: int, device: str):
    """KV(EDGE{u64 vi, u64 vj}, NULL) for edge ids [first_edge, first_edge + nedges)."""
    if nedges < 0 or first_edge < 0:
        raise ValueError("nedges and first_edge must be >= 0")
    if not 1 <= nlevels <= 63:
        raise ValueError(f"nlevels {nlevels} outside 1..63 (2^nlevels vertices)")
    if min(a, b, c, d) < 0 or abs(a + b + c + d - 1.0) > 1e-6:
        raise ValueError(f"R-MAT quadrant probabilities {a}, {b}, {c}, {d} must be >= 0 and sum to 1")
    if not 0.0 <= fraction < 1.0:
        raise ValueError(f"fraction {fraction} outside [0, 1)")
    return C.map_rmat(nedges, nlevels, a, b, c, d, fraction, seed, first_edge, device)


def segments_sorted(sorted_keys: torch.Tensor) -> torch.Tensor:
    """CSR offsets (int64, ngroups + 1) of the runs of equal keys in a sorted int64 column."""
    return C.segments_sorted(_tensor(sorted_keys, "sorted_keys", (torch.int64,)))


def plan_gather_reduce(seg, src, x, w, op: int, out):
    """out[g] = OP over e in segment g of x[src[e]] (+ w[e]); op 0 sum, 1 min, 2 max."""
    seg = _segments(seg)
    src = _tensor(src, "src", (torch.int32,), seg.device)
    x = _tensor(x, "x", None, seg.device)
    if w is not None and w.numel():
        w = _tensor(w, "w", (x.dtype,), seg.device)
        if w.numel() != src.numel():
            raise ValueError(f"w: {w.numel()} weights for {src.numel()} source ids")
    else:
        w = torch.empty(0, dtype=x.dtype, device=x.device)
    if op not in _PLAN_OPS:
        raise ValueError(f"op {op} not one of {_PLAN_OPS}")
    if not (out.is_contiguous() and out.dtype == x.dtype and out.device == x.device and out.numel() >= seg.numel() - 1):
        raise ValueError(f"out: need a contiguous {x.dtype} tensor of >= {seg.numel() - 1} elements on {x.device}")
    C.plan_gather_reduce(seg, src, x, w, op, out)


def plan_combine(seg, perm, recv, vid, op: int, acc):
    """acc[vid[g]] = OP over i in segment g of recv[perm[i]]."""
    seg = _segments(seg)
    perm = _tensor(perm, "perm", (torch.int32,), seg.device)
    vid = _tensor(vid, "vid", (torch.int32,), seg.device)
    recv = _tensor(recv, "recv", None, seg.device)
    if vid.numel() < seg.numel() - 1:
        raise ValueError(f"vid: {vid.numel()} ids for {seg.numel() - 1} groups")
    if op not in _PLAN_OPS:
        raise ValueError(f"op {op} not one of {_PLAN_OPS}")
    if not (acc.is_contiguous() and acc.dtype == recv.dtype and acc.device == recv.device):
        raise ValueError(f"acc: need a contiguous {recv.dtype} tensor on {recv.device}")
    C.plan_combine(seg, perm, recv, vid, op, acc)


def wedges(seg, nbr, centre):
    """All neighbour pairs (min, max) of every group and the group's centre vertex."""
    seg = _segments(seg)
    nbr = _tensor(nbr, "nbr", (torch.int64,), seg.device)
    centre = _tensor(centre, "centre", (torch.int64,), seg.device)
    if centre.numel() < seg.numel() - 1:
        raise ValueError(f"centre: {centre.numel()} vertices for {seg.numel() - 1} groups")
    return C.wedges(seg, nbr, centre)
