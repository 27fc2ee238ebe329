"""Typed Python entry points to the hand-written HIP/CDNA4 kernels
(csrc/kernels/*.hip) behind the engine. Every function dispatches on the
tensor device: cuda tensors run the gfx950 kernels, cpu tensors the engine's
host loops with identical semantics (the test oracle). No fallback exists
for a missing extension: importing this module without the built native
library fails.

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


def exclusive_scan(x: torch.Tensor) -> torch.Tensor:
    """n+1 int64 outputs; out[n] is the total (int32/int64 input)."""
    return C.exclusive_scan(x)


def radix_sort_pairs(keys: torch.Tensor, vals: torch.Tensor, begin_bit: int = 0, end_bit: int = 64):
    """Stable sort of int64 keys (bits [begin_bit, end_bit)) carrying int32 values.
    Returns (sorted_keys, permuted_vals, passes_run)."""
    return C.radix_sort_pairs(keys, vals, begin_bit, end_bit)


def hash32(kv, seed: int = 0) -> torch.Tensor:
    return C.hash32_keys(kv, seed & 0xFFFFFFFF)


def hash64(kv) -> torch.Tensor:
    return C.hash64_keys(kv)


def partition_dest(kv, nprocs: int):
    """(int32 dest rank per pair, int64 per-rank counts)."""
    return C.partition_dest(kv, nprocs)


def group_by(kv):
    """KV -> (KMV, ConvertStats): unique keys + values grouped in CSR segments."""
    return C.convert(kv)


def segmented_reduce(kmv, op: str = "count", dtype: str = "int32"):
    """op in count|sum|min|max|first|last over each key's values."""
    return C.reduce_builtin(kmv, op, dtype)


def sort_kv(kv, flag: int, by_value: bool = False):
    return C.sort_kv(kv, flag, by_value)


def scan_urls(text: torch.Tensor, n: int, doc_id: int):
    """KV(url + NUL, int32 doc_id) for every `<a href="...` in text[:n] (text padded >= 32 B)."""
    return C.map_urls(text, n, doc_id)


def tokenize(text: torch.Tensor, n: int):
    """KV(word + NUL, NULL) for every whitespace-separated word of text[:n]."""
    return C.map_words(text, n)


def rmat_edges(nedges: int, nlevels: int, a: float, b: float, c: float, d: float, fraction: float, seed: int,
               first_edge: int, device: str):
    """KV(EDGE{u64 vi, u64 vj}, NULL) for edge ids [first_edge, first_edge + nedges)."""
    return C.map_rmat(nedges, nlevels, a, b, c, d, fraction, seed, first_edge, device)


def segments_sorted(sorted_keys: torch.Tensor) -> torch.Tensor:
    return C.segments_sorted(sorted_keys)


def plan_gather_reduce(seg, src, x, w, op: int, out):
    C.plan_gather_reduce(seg, src, x, w, op, out)


def plan_combine(seg, perm, recv, vid, op: int, acc):
    C.plan_combine(seg, perm, recv, vid, op, acc)


def wedges(seg, nbr, centre):
    return C.wedges(seg, nbr, centre)
