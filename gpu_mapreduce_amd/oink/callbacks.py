"""OINK named-callback library (reference oink/map_*.cpp, reduce_*.cpp,
scan_*.cpp; types oink/typedefs.h: VERTEX=u64, EDGE={u64 vi,vj}, LABEL=int,
WEIGHT=double).

Every callback exists in the reference's per-pair form (usable with any MR
method from scripts), and the hot ones also in a *batch* form that operates
on the whole device-resident KV at once (torch ops / engine kernels on the
MI355X). The MR dispatcher prefers the batch form.
"""
from __future__ import annotations

import struct

import numpy as np
import torch

from .._ext import C

# ------------------------------------------------------------------ helpers


def edges_of(kv):
    """EDGE keys of a native KV as an [n,2] int64 tensor view (device)."""
    return kv.kdata.view(torch.int64).view(-1, 2)


def col_u64(data):
    return data.view(torch.int64)


def _empty(dev):
    return torch.empty(0, dtype=torch.uint8, device=dev)


# ------------------------------------------------------------------ file maps (host parse -> device)

def _read_cols(fname, dtypes):
    with open(fname, "rb") as f:
        toks = f.read().split()
    k = len(dtypes)
    n = len(toks) // k
    arr = np.array(toks[: n * k]).reshape(n, k) if n else np.zeros((0, k), dtype="S1")
    return [arr[:, i].astype(dt) for i, dt in enumerate(dtypes)]


def read_edge(itask, fname, kv, ptr=None):
    vi, vj = _read_cols(fname, [np.uint64, np.uint64])
    kv.add_tensors(torch.from_numpy(np.stack([vi, vj], 1).view(np.int64)))


def read_edge_label(itask, fname, kv, ptr=None):
    vi, vj, lab = _read_cols(fname, [np.uint64, np.uint64, np.int32])
    kv.add_tensors(torch.from_numpy(np.stack([vi, vj], 1).view(np.int64)), torch.from_numpy(lab))


def read_edge_weight(itask, fname, kv, ptr=None):
    vi, vj, w = _read_cols(fname, [np.uint64, np.uint64, np.float64])
    kv.add_tensors(torch.from_numpy(np.stack([vi, vj], 1).view(np.int64)), torch.from_numpy(w))


def read_vertex_label(itask, fname, kv, ptr=None):
    v, lab = _read_cols(fname, [np.uint64, np.int32])
    kv.add_tensors(torch.from_numpy(v.view(np.int64)), torch.from_numpy(lab))


def read_vertex_weight(itask, fname, kv, ptr=None):
    v, w = _read_cols(fname, [np.uint64, np.float64])
    kv.add_tensors(torch.from_numpy(v.view(np.int64)), torch.from_numpy(w))


def read_vertex_vertex(itask, fname, kv, ptr=None):
    """"vi zi" lines -> (VERTEX, VERTEX) (e.g. cc_find output read by cc_stats)"""
    v, z = _read_cols(fname, [np.uint64, np.uint64])
    kv.add_tensors(torch.from_numpy(v.view(np.int64)), torch.from_numpy(z.view(np.int64)))


def read_words(itask, fname, kv, ptr=None):
    """words of a file (strtok " \\t\\n\\f\\r"), key = word + NUL; tokenised on the
    GPU by the same kernel as wordfreq."""
    from ..utils.synth import pad_text
    with open(fname, "rb") as f:
        data = f.read()
    if isinstance(ptr, list):
        ptr[0] += 1
    t = pad_text(torch.frombuffer(bytearray(data or b" "), dtype=torch.uint8).to(kv.device))
    kv.add_kv(C.map_words(t, len(data)))


FILE_MAPS = dict(read_edge=read_edge, read_edge_label=read_edge_label, read_edge_weight=read_edge_weight,
                 read_vertex_label=read_vertex_label, read_vertex_weight=read_vertex_weight, read_vertex_vertex=read_vertex_vertex,
                 read_words=read_words)


# ------------------------------------------------------------------ map(mr) callbacks: per pair

def edge_to_vertex(i, k, v, kv, ptr=None):
    kv.add(k[:8], None)


def edge_to_vertices(i, k, v, kv, ptr=None):
    kv.add(k[:8], None)
    kv.add(k[8:16], None)


def edge_to_vertex_pair(i, k, v, kv, ptr=None):
    kv.add(k[:8], k[8:16])


def edge_upper(i, k, v, kv, ptr=None):
    a, b = struct.unpack("<QQ", k)
    if a < b:
        kv.add(k, None)
    elif a > b:
        kv.add(struct.pack("<QQ", b, a), None)


def invert(i, k, v, kv, ptr=None):
    kv.add(v, k)


def add_label(i, k, v, kv, ptr=None):
    kv.add(k, struct.pack("<i", 1))


def add_weight(i, k, v, kv, ptr=None):
    kv.add(k, struct.pack("<d", 1.0))


# ------------------------------------------------------------------ map(mr) callbacks: device batch

def b_edge_to_vertex(src, kv, ptr=None):
    e = edges_of(src)
    kv.add_tensors(e[:, 0].contiguous())


def b_edge_to_vertices(src, kv, ptr=None):
    e = edges_of(src)
    kv.add_tensors(torch.cat([e[:, 0], e[:, 1]]))


def b_edge_to_vertex_pair(src, kv, ptr=None):
    e = edges_of(src)
    kv.add_tensors(e[:, 0].contiguous(), e[:, 1].contiguous())


def b_edge_upper(src, kv, ptr=None):
    e = edges_of(src)
    # unsigned compare of u64 ids (ids < 2^63 in practice; use signed view safely)
    keep = e[:, 0] != e[:, 1]
    lo = torch.minimum(e[:, 0], e[:, 1])[keep]
    hi = torch.maximum(e[:, 0], e[:, 1])[keep]
    kv.add_tensors(torch.stack([lo, hi], 1))


def b_invert(src, kv, ptr=None):
    o = C.KV()
    o.n, o.kw, o.vw = src.n, src.vw, src.kw
    o.kdata, o.vdata = src.vdata, src.kdata
    if src.vw < 0:
        o.koff = src.voff
    if src.kw < 0:
        o.voff = src.koff
    kv.add_kv(o)


def b_add_label(src, kv, ptr=None):
    o = C.KV()
    o.n, o.kw, o.vw = src.n, src.kw, 4
    o.kdata = src.kdata
    if src.kw < 0:
        o.koff = src.koff
    o.vdata = torch.ones(src.n, dtype=torch.int32, device=src.kdata.device).view(torch.uint8)
    kv.add_kv(o)


def b_add_weight(src, kv, ptr=None):
    o = C.KV()
    o.n, o.kw, o.vw = src.n, src.kw, 8
    o.kdata = src.kdata
    if src.kw < 0:
        o.koff = src.koff
    o.vdata = torch.ones(src.n, dtype=torch.float64, device=src.kdata.device).view(torch.uint8)
    kv.add_kv(o)


MR_MAPS = dict(edge_to_vertex=(edge_to_vertex, b_edge_to_vertex),
               edge_to_vertices=(edge_to_vertices, b_edge_to_vertices),
               edge_to_vertex_pair=(edge_to_vertex_pair, b_edge_to_vertex_pair),
               edge_upper=(edge_upper, b_edge_upper), invert=(invert, b_invert),
               add_label=(add_label, b_add_label), add_weight=(add_weight, b_add_weight))


# ------------------------------------------------------------------ reduce callbacks

def count(key, mv, kv, ptr=None):
    kv.add(key, struct.pack("<i", len(mv)))


def cull(key, mv, kv, ptr=None):
    kv.add(key, mv[0])


# name -> (host fn, builtin device reducer name)
REDUCES = dict(count=(count, "count"), cull=(cull, "first"))


# ------------------------------------------------------------------ scan / printers

def _fmt_u64(t):
    return t.cpu().numpy().view(np.uint64)


def print_edge(mr, fp, ptr=None):
    e = _fmt_u64(edges_of(mr.kv).reshape(-1)).reshape(-1, 2) if mr.kv.n else np.zeros((0, 2), np.uint64)
    np.savetxt(fp, e, fmt="%d %d")


def print_vertex(mr, fp, ptr=None):
    v = _fmt_u64(mr.kv.kdata) if mr.kv.n else np.zeros(0, np.uint64)
    np.savetxt(fp, v, fmt="%d")


def print_string_int(mr, fp, ptr=None):
    for k, v in mr.kv_pairs():
        fp.write("%s %d\n" % (k.split(b"\0", 1)[0].decode("utf-8", "replace"), struct.unpack("<i", v[:4])[0]))


def print_vertex_int(mr, fp, ptr=None):
    k = _fmt_u64(mr.kv.kdata)
    v = mr.kv.vdata.view(torch.int32).cpu().numpy()
    np.savetxt(fp, np.stack([k.astype(np.int64), v.astype(np.int64)], 1), fmt="%d %d")


def print_vertex_u64(mr, fp, ptr=None):
    k = _fmt_u64(mr.kv.kdata)
    v = _fmt_u64(mr.kv.vdata)
    np.savetxt(fp, np.stack([k, v], 1), fmt="%d %d")


def print_vertex_double(mr, fp, ptr=None):
    k = _fmt_u64(mr.kv.kdata)
    v = mr.kv.vdata.view(torch.float64).cpu().numpy()
    for a, b in zip(k, v):
        fp.write("%d %g\n" % (a, b))


def scan_print_edge(k, v, fp):
    fp.write("%d %d\n" % struct.unpack("<QQ", k))


def scan_print_vertex(k, v, fp):
    fp.write("%d\n" % struct.unpack("<Q", k)[0])


def scan_print_string_int(k, v, fp):
    fp.write("%s %d\n" % (k.split(b"\0", 1)[0].decode(), struct.unpack("<i", v)[0]))


SCANS = dict(print_edge=scan_print_edge, print_vertex=scan_print_vertex, print_string_int=scan_print_string_int)


# ------------------------------------------------------------------ hash / compare callbacks (scripts)

def hash_first_u64(key):
    return struct.unpack_from("<Q", key)[0]


HASHES = dict(hash_vertex=hash_first_u64)


def compare_uint64(a, b):
    x, y = struct.unpack_from("<Q", a)[0], struct.unpack_from("<Q", b)[0]
    return (x > y) - (x < y)


COMPARES = dict(compare_uint64=compare_uint64)
