"""Host-side helpers of the MapReduce object: per-rank histograms
(reference src/mapreduce.cpp:3251-3311), file-list expansion
(findfiles/addfiles/bcastfiles :2812-2931), file chunk planning and reading
with separator fix-up (map_chunks/map_file_wrapper :1312-1552), and the
KV/KMV print formats (src/keyvalue.cpp:773-835, src/keymultivalue.cpp:1646-1774).
"""
from __future__ import annotations

import os
import struct

import torch

from .._ext import C


def write_histo(comm, value, title):
    vals = comm.allgather(float(value))
    ave = sum(vals) / len(vals)
    mx, mn = max(vals), min(vals)
    histo = [0] * 10
    d = mx - mn
    for v in vals:
        m = 0 if d == 0.0 else int((v - mn) / d * 10)
        histo[min(m, 9)] += 1
    if comm.rank == 0:
        print(f"{title:<13s} {ave:g} ave {mx:g} max {mn:g} min")
        print(f"{'  Histogram:':<13s}" + "".join(f" {h}" for h in histo))


# ----------------------------------------------------------------------- files

def _expand(path, recurse, out):
    if os.path.isfile(path):
        out.append(path)
    elif os.path.isdir(path):
        for name in sorted(os.listdir(path)):
            full = os.path.join(path, name)
            if os.path.isfile(full):
                out.append(full)
            elif recurse and os.path.isdir(full):
                _expand(full, recurse, out)
    else:
        raise FileNotFoundError(f"Invalid filename {path}")


def find_files(comm, files, selfflag, recurse, readflag):
    """readflag=1: each named file holds a list of file names (one per line)."""
    if isinstance(files, (str, bytes, os.PathLike)):
        files = [files]
    files = [os.fsdecode(f) for f in files]

    def local():
        out = []
        for f in files:
            if readflag:
                with open(f) as fh:
                    for line in fh:
                        w = line.split()
                        if w:
                            _expand(w[0], recurse, out)
            else:
                _expand(f, recurse, out)
        return out

    if selfflag:
        return local()
    lst = local() if comm.rank == 0 else None
    return comm.bcast_object(lst, 0)


def plan_chunks(comm, flist, nmap, delta):
    """Split files into tasks of ~equal bytes: returns [(ifile, itask, ntask, fsize)]."""
    sizes = [os.path.getsize(f) for f in flist] if comm.rank == 0 else None
    sizes = comm.bcast_object(sizes, 0)
    nfile = len(flist)
    if nfile == 0:
        return []
    nmap = max(nmap, nfile)
    total = sum(sizes)
    ideal = max(1, total // nmap)
    tpf = [max(1, s // ideal) for s in sizes]
    ntasks = sum(tpf)
    while ntasks < nmap:
        progressed = False
        for i in range(nfile):
            if sizes[i] > ideal:
                tpf[i] += 1
                ntasks += 1
                progressed = True
                if ntasks == nmap:
                    break
        if not progressed:
            break
    while ntasks > nmap:
        for i in range(nfile):
            if tpf[i] > 1:
                tpf[i] -= 1
                ntasks -= 1
                if ntasks == nmap:
                    break
    # tasks must be larger than delta, else reads overlap
    for i in range(nfile):
        while tpf[i] > 1 and sizes[i] // tpf[i] <= delta:
            tpf[i] -= 1
    plan = []
    for i in range(nfile):
        for j in range(tpf[i]):
            plan.append((i, j, tpf[i], sizes[i]))
    return plan


def read_chunk(fname, fsize, itask, ntask, delta, sep, is_char):
    start = itask * fsize // ntask
    nxt = (itask + 1) * fsize // ntask
    readsize = min(nxt - start + delta, fsize - start)
    with open(fname, "rb") as f:
        f.seek(start)
        buf = f.read(readsize)
    s0 = 0
    if itask > 0:
        p = buf.find(sep)
        if p < 0 or p > delta:
            raise RuntimeError("Could not find file separator within delta")
        s0 = p + (len(sep) if is_char else 0)
    s1 = len(buf)
    if itask < ntask - 1:
        p = buf.find(sep, nxt - start)
        if p < 0:
            raise RuntimeError("Could not find file separator within delta")
        s1 = p + (1 if is_char else 0)
    return buf[s0:s1]


# ----------------------------------------------------------------------- printing

def _fmt(b: bytes, flag):
    if flag == 0:
        return "NULL"
    if flag == 1:
        return "%d" % struct.unpack_from("<i", b)[0]
    if flag == 2:
        return "%d" % struct.unpack_from("<Q", b)[0]
    if flag == 3:
        return "%g" % struct.unpack_from("<f", b)[0]
    if flag == 4:
        return "%g" % struct.unpack_from("<d", b)[0]
    if flag == 5:
        return b.split(b"\0", 1)[0].decode("utf-8", "replace")
    if flag == 6:
        return "%d %d" % struct.unpack_from("<ii", b)
    if flag == 7:
        return "%d %d" % struct.unpack_from("<QQ", b)
    raise ValueError(flag)


def format_pairs(mr, nstride, kflag, vflag):
    lines = []
    me = mr.me
    if mr.kv is not None:
        cnt = [0]

        def one(i, k, v):
            cnt[0] += 1
            if cnt[0] != nstride:
                return
            cnt[0] = 0
            lines.append(f"KV pair: proc {me}, sizes {len(k)} {len(v)}, key {_fmt(k, kflag)}, "
                         f"value {_fmt(v, vflag)}\n")
        C.kv_iter(mr.kv, one)
    if mr.kmv is not None:
        cnt = [0]

        def onek(k, vals):
            cnt[0] += 1
            if cnt[0] != nstride:
                return
            cnt[0] = 0
            mvb = sum(len(v) for v in vals)
            vs = "".join(_fmt(v, vflag) + " " for v in vals) if vflag else "NULL"
            lines.append(f"KMV pair: proc {me}, nvalues {len(vals)}, sizes {len(k)} {mvb}, "
                         f"key {_fmt(k, kflag)}, values {vs}\n")
        C.kmv_iter(mr.kmv, onek)
    return lines
