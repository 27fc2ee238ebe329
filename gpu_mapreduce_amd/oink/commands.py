"""OINK named commands (reference oink/<name>.cpp, registered by CommandStyle).

Each command keeps the reference's inputs/outputs/params contract and its
MapReduce op sequence; the per-pair C++ callbacks become device-batch
callbacks (whole KV/KMV tensors in HBM), and the iterative graph commands
(cc_find, luby_find, sssp, pagerank) run on a reusable edge plan
(models/graph.py) instead of re-shuffling every edge every iteration.
"""
from __future__ import annotations

import os
import struct

import numpy as np
import torch

from .._ext import C
from ..models import graph as G
from . import callbacks as cb
from .variable import OinkError

COMMANDS = {}


def command(name):
    def deco(cls):
        COMMANDS[name] = cls
        cls.name = name
        return cls
    return deco


class Command:
    ninputs = 0
    noutputs = 0

    def __init__(self, oink):
        self.oink = oink
        self.obj = oink.obj
        self.comm = oink.comm
        self.me = oink.comm.rank
        self.nprocs = oink.comm.size

    def params(self, args):
        if args:
            raise OinkError(f"Illegal {self.name} command")

    def inputs(self, args):
        if len(args) != self.ninputs:
            raise OinkError(f"Illegal {self.name} command: {self.ninputs} inputs required")
        for i, a in enumerate(args):
            self.obj.add_input(i, a)

    def outputs(self, args):
        if len(args) != 2 * self.noutputs:
            raise OinkError(f"Illegal {self.name} command: {self.noutputs} outputs (file mr) required")
        for i in range(self.noutputs):
            self.obj.add_output(i, args[2 * i], args[2 * i + 1])

    def message(self, s):
        self.oink.message(s)

    @property
    def dev(self):
        return self.comm.device


# ---------------------------------------------------------------------- batch helpers

def kmv_lens(kmv):
    return kmv.seg[1:] - kmv.seg[:-1]


def kmv_sid(kmv):
    return torch.repeat_interleave(torch.arange(kmv.nkey, device=kmv.seg.device), kmv_lens(kmv),
                                   output_size=kmv.nval)


def u64(t):
    return t.view(torch.int64)


def kmv_vlens(kmv):
    """per-value byte lengths of a KMV (fixed or variable width values)"""
    if kmv.vw >= 0:
        return torch.full((kmv.nval,), kmv.vw, dtype=torch.int64, device=kmv.seg.device)
    return kmv.voff[1:] - kmv.voff[:-1]


def kmv_vstart(kmv):
    if kmv.vw >= 0:
        return torch.arange(kmv.nval, device=kmv.seg.device, dtype=torch.int64) * kmv.vw
    return kmv.voff[:-1]


def _edges_global_nvert(comm, e):
    mx = int(e.max().item()) if e.numel() else -1
    return int(comm.allreduce(mx, "max")) + 1


def _rmat_params(args, name):
    if len(args) != 8:
        raise OinkError(f"Illegal {name} command")
    nlevels, nnz = int(args[0]), int(args[1])
    a, b, c, d, frac = (float(x) for x in args[2:7])
    seed = int(args[7])
    if abs(a + b + c + d - 1.0) > 1e-12:
        raise OinkError("RMAT a,b,c,d must sum to 1")
    if frac >= 1.0:
        raise OinkError("RMAT fraction must be < 1")
    return dict(nlevels=nlevels, nnonzero=nnz, a=a, b=b, c=c, d=d, fraction=frac, seed=seed,
                order=1 << nlevels)


class _RmatGen:
    """map/task callback: generate this rank's share of new R-MAT edges on the GPU.
    Edge ids continue across iterations so every iteration draws fresh edges."""

    def __init__(self, r, comm):
        self.r, self.comm, self.base = r, comm, 0

    def gen(self, nremain):
        P, me = self.comm.size, self.comm.rank
        lo = self.base + me * (nremain // P) + min(me, nremain % P)
        n = nremain // P + (1 if me < nremain % P else 0)
        self.base += nremain
        r = self.r

        def fn(itask, kv):
            if n:
                kv.add_kv(C.map_rmat(n, r["nlevels"], r["a"], r["b"], r["c"], r["d"], r["fraction"],
                                     r["seed"], lo, self.comm.device))
        return fn


@command("rmat")
class RMAT(Command):
    """rmat N Nz a b c d frac seed -o file mr  (oink/rmat.cpp:37-71)"""
    noutputs = 1

    def params(self, args):
        self.r = _rmat_params(args, "rmat")

    def run(self):
        r = self.r
        mr = self.obj.create_mr()
        ntotal = r["order"] * r["nnonzero"]
        nremain, niter = ntotal, 0
        g = _RmatGen(r, self.comm)
        while nremain:
            niter += 1
            mr.map(self.nprocs, g.gen(nremain), addflag=1)
            nunique = mr.collate()
            mr.reduce("first")                    # cull
            nremain = ntotal - nunique
        self.obj.output(1, mr, cb.print_edge)
        self.message(f"RMAT: {r['order']} rows, {ntotal} non-zeroes, {niter} iterations")
        self.obj.cleanup()


@command("rmat2")
class RMAT2(Command):
    """rmat2: generate into a fresh MR, aggregate, add, convert (oink/rmat2.cpp:37-74)"""
    noutputs = 1

    def params(self, args):
        self.r = _rmat_params(args, "rmat")

    def run(self):
        r = self.r
        mr = self.obj.create_mr()
        mrnew = self.obj.create_mr()
        ntotal = r["order"] * r["nnonzero"]
        nremain, niter = ntotal, 0
        g = _RmatGen(r, self.comm)
        mr.map(self.nprocs, lambda i, kv: None)
        while nremain:
            niter += 1
            mrnew.map(self.nprocs, g.gen(nremain))
            mrnew.aggregate()
            mr.add(mrnew)
            nunique = mr.convert()
            mr.reduce("first")
            nremain = ntotal - nunique
        self.obj.output(1, mr, cb.print_edge)
        self.message(f"RMAT2: {r['order']} rows, {ntotal} non-zeroes, {niter} iterations")
        self.obj.cleanup()


@command("edge_upper")
class EdgeUpper(Command):
    ninputs = noutputs = 1

    def run(self):
        mre = self.obj.input(1, cb.read_edge)
        mr = self.obj.create_mr()
        nedge = mre.kv_stats(0)
        mr.map_mr_batch(mre, cb.b_edge_upper)
        mr.collate()
        unique = mr.reduce("first")
        self.obj.output(1, mr, cb.print_edge)
        self.message(f"EdgeUpper: {nedge} original edges, {unique} final edges")
        self.obj.cleanup()


@command("degree")
class Degree(Command):
    """degree dup: dup=1 count edge (vi) only, else both endpoints (oink/degree.cpp)"""
    ninputs = noutputs = 1

    def params(self, args):
        if len(args) != 1:
            raise OinkError("Illegal degree command")
        self.dup = int(args[0])

    def run(self):
        mre = self.obj.input(1, cb.read_edge)
        mrv = self.obj.create_mr()
        nedge = mre.kv_stats(0)
        mrv.map_mr_batch(mre, cb.b_edge_to_vertex if self.dup == 1 else cb.b_edge_to_vertices)
        mrv.collate()
        nvert = mrv.reduce("count")
        self.obj.output(1, mrv, cb.print_vertex_int)
        self.message(f"Degree: {nvert} vertices, {nedge} edges")
        self.obj.cleanup()


def _print_histo(mr, fmt, out=print):
    for k, v in mr.kv_pairs():
        a = struct.unpack("<i", k[:4])[0]
        b = struct.unpack("<i", v[:4])[0]
        out(fmt % (b, a))


@command("degree_stats")
class DegreeStats(Command):
    ninputs = 1

    def params(self, args):
        if len(args) != 1:
            raise OinkError("Illegal degree_stats command")
        self.dup = int(args[0])

    def run(self):
        mre = self.obj.input(1, cb.read_edge)
        mr = self.obj.create_mr()
        nedge = mre.kv_stats(0)
        mr.map_mr_batch(mre, cb.b_edge_to_vertex if self.dup == 1 else cb.b_edge_to_vertices)
        mr.collate()
        nvert = mr.reduce("count")
        mr.map_mr_batch(mr, cb.b_invert)
        mr.collate()
        mr.reduce("count")
        mr.gather(1)
        mr.sort_keys(-1)
        self.message(f"DegreeStats: {nvert} vertices, {nedge} edges")
        if self.me == 0:
            _print_histo(mr, "  %d vertices with %d edges", self.message)
        self.obj.cleanup()


@command("histo")
class Histo(Command):
    ninputs = noutputs = 1

    def run(self):
        mr = self.obj.input(1)
        ntotal = mr.kv_stats(0)
        if self.obj.permanent(mr):
            mr = self.obj.copy_mr(mr)
        mr.collate()
        nunique = mr.reduce("count")
        self.obj.output(1, mr)
        if self.obj.permanent(mr):
            mr = self.obj.copy_mr(mr)
        mr.map_mr_batch(mr, cb.b_invert)
        mr.collate()
        mr.reduce("count")
        mr.gather(1)
        mr.sort_keys(-1)
        self.message(f"Histo: {ntotal} total keys, {nunique} unique")
        if self.me == 0:
            _print_histo(mr, "  %d keys appear %d times", self.message)
        self.obj.cleanup()


@command("degree_weight")
class DegreeWeight(Command):
    """edges + (vertex, int degree) -> (edge, 1/degree(vi)) (oink/degree_weight.cpp)"""
    ninputs = 2
    noutputs = 1

    def run(self):
        mre = self.obj.input(1, cb.read_edge)
        mrd = self.obj.input(2, cb.read_vertex_label)
        mrewt = self.obj.create_mr()
        nvert = mrd.kv_stats(0)
        mrewt.map_mr_batch(mre, cb.b_edge_to_vertex_pair)
        mrewt.add(mrd)
        mrewt.collate()

        def inverse_degree(kmv, kv):
            vl, vs = kmv_vlens(kmv), kmv_vstart(kmv)
            sid = kmv_sid(kmv)
            is_deg = vl == 4
            deg = torch.zeros(kmv.nkey, dtype=torch.float64, device=kmv.seg.device)
            dval = _gather_bytes(kmv.vdata, vs[is_deg], 4).view(torch.int32).view(-1).to(torch.float64)
            deg[sid[is_deg]] = dval
            is_e = vl == 8
            vj = _gather_bytes(kmv.vdata, vs[is_e], 8).view(torch.int64).view(-1)
            vi = u64(kmv.keys.kdata)[sid[is_e]]
            wts = 1.0 / deg[sid[is_e]]
            kv.add_tensors(torch.stack([vi, vj], 1), wts)
        nedge = mrewt.reduce_batch(inverse_degree)
        self.obj.output(1, mrewt, _print_edge_weight)
        self.message(f"DegreeWeight: {nvert} vertices, {nedge} edges")
        self.obj.cleanup()


def _gather_bytes(vdata, pos, w):
    idx = pos.unsqueeze(1) + torch.arange(w, device=vdata.device)
    return vdata[idx].contiguous()


def _print_edge_weight(mr, fp):
    e = mr.kv.kdata.view(torch.int64).view(-1, 2).cpu().numpy().view(np.uint64)
    w = mr.kv.vdata.view(torch.float64).cpu().numpy()
    for (a, b), x in zip(e, w):
        fp.write("%d %d %g\n" % (a, b, x))


@command("wordfreq")
class WordFreqCmd(Command):
    """wordfreq ntop -i files -o file mr (oink/wordfreq.cpp:40-90)"""
    ninputs = noutputs = 1

    def params(self, args):
        if len(args) != 1:
            raise OinkError("Illegal wordfreq command")
        self.ntop = int(args[0])

    def run(self):
        nfiles = [0]
        mr = self.obj.input(1, cb.read_words, None, nfiles)
        nwords = mr.kv_stats(0)
        nfiles_all = self.comm.allreduce(nfiles[0], "sum")
        if self.obj.permanent(mr):
            mr = self.obj.copy_mr(mr)
        mr.collate()
        nunique = mr.reduce("count")
        self.obj.output(1, mr, cb.print_string_int)
        if self.ntop:
            if self.obj.permanent(mr):
                mr = self.obj.copy_mr(mr)
            mr.sort_values(-1)
            keep = lambda src, kv: _keep_first(src, kv, 10)
            mr.map_mr_batch(mr, keep)
            mr.gather(1)
            mr.sort_values(-1)
            if self.me == 0:
                for k, v in mr.kv_pairs()[: self.ntop]:
                    print("%d %s" % (struct.unpack("<i", v)[0], k.split(b"\0", 1)[0].decode("utf-8", "replace")))
        self.message(f"WordFreq: {nfiles_all} files, {nwords} words, {nunique} unique")
        self.obj.cleanup()


def _keep_first(src, kv, n):
    n = min(n, src.n)
    if n == 0:
        return
    idx = torch.arange(n, dtype=torch.int32, device=src.kdata.device)
    kv.add_kv(C.gather(src, idx))


@command("vertex_extract")
class VertexExtract(Command):
    ninputs = noutputs = 1

    def run(self):
        mre = self.obj.input(1, cb.read_edge_weight)
        mrv = self.obj.create_mr()
        mrv.map_mr_batch(mre, cb.b_edge_to_vertices)
        mrv.collate()
        mrv.reduce("first")
        self.obj.output(1, mrv, cb.print_vertex)
        self.obj.cleanup()


@command("neighbor")
class Neighbor(Command):
    """(v, [neighbours]) adjacency lists (oink/neighbor.cpp)"""
    ninputs = noutputs = 1

    def run(self):
        mre = self.obj.input(1, cb.read_edge)
        mrn = self.obj.create_mr()

        def map1(src, kv):
            e = cb.edges_of(src)
            kv.add_tensors(torch.cat([e[:, 0], e[:, 1]]), torch.cat([e[:, 1], e[:, 0]]))
        mrn.map_mr_batch(mre, map1)
        mrn.collate()

        def reduce1(kmv, kv):
            kv.add_tensors(kmv.keys.kdata.view(torch.int64), kmv.vdata, voff=kmv.seg * 8)
        mrn.reduce_batch(reduce1)
        self.obj.output(1, mrn, _print_neighbors)
        self.obj.cleanup()


def _print_neighbors(mr, fp):
    for k, v in mr.kv_pairs():
        nb = np.frombuffer(v, dtype=np.uint64)
        fp.write("%d" % struct.unpack("<Q", k)[0] + "".join(" %d" % x for x in nb) + "\n")


@command("neigh_tri")
class NeighTri(Command):
    """neigh_tri dir -i neighbors triangles: one file per vertex with its
    neighbour edges and the triangles it belongs to (oink/neigh_tri.cpp)"""
    ninputs = 2
    noutputs = 1

    def params(self, args):
        if len(args) != 1:
            raise OinkError("Illegal neigh_tri command")
        self.dirname = args[0]

    def run(self):
        mrn = self.obj.input(1, _read_neighbors)
        mrt = self.obj.input(2, _read_tri)
        mrnplus = self.obj.create_mr()
        mrnplus.map_mr_batch(mrn, _expand_lists)

        def map1(src, kv):
            t = src.kdata.view(torch.int64).view(-1, 3)
            vi, vj, vk = t[:, 0], t[:, 1], t[:, 2]
            keys = torch.cat([vi, vj, vk])
            vals = torch.cat([torch.stack([vj, vk], 1), torch.stack([vi, vk], 1), torch.stack([vi, vj], 1)])
            kv.add_tensors(keys, vals)
        mrnplus.map_mr_batch(mrt, map1, None, 1)
        mrnplus.collate()
        os.makedirs(self.dirname, exist_ok=True)

        def prt(k, vals):
            vi = struct.unpack("<Q", k)[0]
            with open(os.path.join(self.dirname, str(vi)), "w") as fp:
                for v in vals:
                    if len(v) == 8:
                        fp.write("%d %d\n" % (vi, struct.unpack("<Q", v)[0]))
                    else:
                        fp.write("%d %d\n" % struct.unpack("<QQ", v))
        mrnplus.scan_kmv(prt)
        self.obj.output(1, mrnplus)
        self.obj.cleanup()


def _read_neighbors(itask, fname, kv):
    ks, vs = [], []
    with open(fname) as f:
        for line in f:
            t = line.split()
            if t:
                ks += [int(t[0])] * (len(t) - 1)
                vs += [int(x) for x in t[1:]]
    kv.add_tensors(torch.from_numpy(np.array(ks, dtype=np.uint64).view(np.int64)),
                   torch.from_numpy(np.array(vs, dtype=np.uint64).view(np.int64)))


def _read_tri(itask, fname, kv):
    a = np.loadtxt(fname, dtype=np.uint64, ndmin=2).reshape(-1, 3)
    kv.add_tensors(torch.from_numpy(a.view(np.int64)))


def _expand_lists(src, kv):
    """(v, [vj...] packed) -> one (v, vj) pair per neighbour"""
    if src.vw >= 0 and src.vw != 8:
        if src.n and src.vw % 8:
            raise OinkError("neighbor values must be lists of vertices")
    dev = src.kdata.device
    if src.vw == 8:
        kv.add_kv(src)
        return
    if src.vw >= 0:
        cnt = torch.full((src.n,), src.vw // 8, dtype=torch.int64, device=dev)
    else:
        cnt = (src.voff[1:] - src.voff[:-1]) // 8
    keys = torch.repeat_interleave(src.kdata.view(torch.int64), cnt)
    kv.add_tensors(keys, src.vdata.view(torch.int64))


@command("tri_find")
class TriFind(Command):
    """tri_find -i edges -o file mr: every triangle once, as (vi, vj, vk) with
    vi < vj < vk. Degree-oriented CSR + per-edge sorted-list intersection on
    the GPU (models/triangles.py); same result as the reference's 4-shuffle
    pipeline (oink/tri_find.cpp:43-82), which remains available as tri_find_mr."""
    ninputs = noutputs = 1

    def run(self):
        from ..models.triangles import TriangleGraph
        mre = self.obj.input(1, cb.read_edge)
        g = TriangleGraph(self.comm, _edges_from(mre))
        tri = g.triangles()
        ntri = self.comm.allreduce(int(tri.shape[0]), "sum")
        mrt = self.obj.create_mr()
        mrt.map(self.nprocs, lambda i, kv: kv.add_tensors(tri) if tri.shape[0] else None)
        self.obj.output(1, mrt, _print_tri)
        self.message(f"Tri_find: {ntri} triangles")
        self.ntri = ntri
        self.obj.cleanup()


@command("tri_find_mr")
class TriFindMR(Command):
    """triangle enumeration, 4 shuffles (oink/tri_find.cpp:43-82); the O(d^2)
    wedge generation is the load-balanced k_wedges kernel"""
    ninputs = noutputs = 1

    def run(self):
        mre = self.obj.input(1, cb.read_edge)
        mrt = self.obj.create_mr()

        def map_edge_vert(src, kv):
            e = cb.edges_of(src)
            kv.add_tensors(torch.cat([e[:, 0], e[:, 1]]), torch.cat([e[:, 1], e[:, 0]]))
        mrt.map_mr_batch(mre, map_edge_vert)
        mrt.collate()

        def reduce_first_degree(kmv, kv):
            deg = kmv_lens(kmv).to(torch.int32)
            sid = kmv_sid(kmv)
            vi = u64(kmv.keys.kdata)[sid]
            vj = u64(kmv.vdata)
            d = deg[sid]
            lt = vi < vj
            edge = torch.stack([torch.where(lt, vi, vj), torch.where(lt, vj, vi)], 1)
            dg = torch.stack([torch.where(lt, d, 0), torch.where(lt, 0, d)], 1)
            kv.add_tensors(edge, dg)
        mrt.reduce_batch(reduce_first_degree)
        mrt.collate()

        def reduce_second_degree(kmv, kv):
            v = kmv.vdata.view(torch.int32).view(-1, 2)
            one = v[kmv.seg[:-1]]
            two = v[torch.clamp(kmv.seg[:-1] + 1, max=kmv.nval - 1)]
            use1 = one[:, 0] != 0
            dg = torch.stack([torch.where(use1, one[:, 0], two[:, 0]), torch.where(use1, two[:, 1], one[:, 1])], 1)
            kv.add_tensors(kmv.keys.kdata.view(torch.int64).view(-1, 2), dg)
        mrt.reduce_batch(reduce_second_degree)

        def map_low_degree(src, kv):
            e = cb.edges_of(src)
            dg = src.vdata.view(torch.int32).view(-1, 2)
            vi, vj, di, dj = e[:, 0], e[:, 1], dg[:, 0], dg[:, 1]
            first_i = (di < dj) | ((di == dj) & (vi < vj))
            kv.add_tensors(torch.where(first_i, vi, vj), torch.where(first_i, vj, vi))
        mrt.map_mr_batch(mrt, map_low_degree)
        mrt.collate()

        def reduce_nsq_angles(kmv, kv):
            edges, centre = C.wedges(kmv.seg, u64(kmv.vdata), u64(kmv.keys.kdata))
            kv.add_tensors(edges, centre)
        mrt.reduce_batch(reduce_nsq_angles)
        mrt.add(mre)
        mrt.collate()

        def reduce_emit_triangles(kmv, kv):
            dev = kmv.seg.device
            vl, vs = kmv_vlens(kmv), kmv_vstart(kmv)
            sid = kmv_sid(kmv)
            has_edge = torch.zeros(kmv.nkey, dtype=torch.int32, device=dev)
            has_edge[sid[vl == 0]] = 1
            m = (vl == 8) & (has_edge[sid] > 0)
            if not bool(m.any()):
                return
            centre = _gather_bytes(kmv.vdata, vs[m], 8).view(torch.int64).view(-1)
            e = kmv.keys.kdata.view(torch.int64).view(-1, 2)[sid[m]]
            kv.add_tensors(torch.stack([centre, e[:, 0], e[:, 1]], 1))
        ntri = mrt.reduce_batch(reduce_emit_triangles)
        self.obj.output(1, mrt, _print_tri)
        self.message(f"Tri_find: {ntri} triangles")
        self.ntri = ntri
        self.obj.cleanup()


def _print_tri(mr, fp):
    if mr.kv.n:
        np.savetxt(fp, mr.kv.kdata.view(torch.int64).view(-1, 3).cpu().numpy().view(np.uint64), fmt="%d %d %d")


def _edges_from(mr):
    return mr.kv.kdata.view(torch.int64).view(-1, 2)


def _present(plan):
    """local vertices that appear in any edge"""
    cnt = torch.bincount(plan.src.long(), minlength=plan.nlocal)[: plan.nlocal]
    return cnt > 0


@command("cc_find")
class CCFind(Command):
    """cc_find nthresh -i edges -o file mr: (vertex, component id = min vertex id)
    (oink/cc_find.cpp). nthresh (hot-zone splitting) is accepted; the edge plan
    needs no zone splitting because segments are load-balanced by value count."""
    ninputs = noutputs = 1

    def params(self, args):
        if len(args) != 1:
            raise OinkError("Illegal cc_find command")
        self.nthresh = int(args[0])

    def run(self):
        mre = self.obj.input(1, cb.read_edge)
        e = _edges_from(mre)
        N = _edges_global_nvert(self.comm, e)
        plan = G.EdgePlan(mre, e, N, symmetric=True)
        lab, niter = G.connected_components(plan)
        pres = _present(plan)
        ids = plan.local_ids[pres]
        zl = lab[pres]
        mrv = self.obj.create_mr()
        mrv.map(self.nprocs, lambda i, kv: kv.add_tensors(ids, zl))
        self.obj.output(1, mrv, cb.print_vertex_u64)
        ncc = self.comm.allreduce(int((zl == ids).sum().item()), "sum")
        self.message(f"CC_find: {ncc} components in {niter} iterations")
        self.ncc = ncc
        self.obj.cleanup()


@command("cc_stats")
class CCStats(Command):
    ninputs = 1

    def run(self):
        mrv = self.obj.input(1, cb.read_vertex_vertex)
        mr = self.obj.create_mr()
        nvert = mr.map_mr_batch(mrv, cb.b_invert)
        ncc = mr.collate()
        mr.reduce("count")
        mr.map_mr_batch(mr, cb.b_invert)
        mr.collate()
        mr.reduce("count")
        mr.gather(1)
        mr.sort_keys(-1)
        self.message(f"CCStats: {ncc} components, {nvert} vertices")
        if self.me == 0:
            _print_histo(mr, "  %d CCs with %d vertices", self.message)
        self.obj.cleanup()


@command("luby_find")
class LubyFind(Command):
    """maximal independent set (oink/luby_find.cpp)"""
    ninputs = noutputs = 1

    def params(self, args):
        if len(args) != 1:
            raise OinkError("Illegal luby_find command")
        self.seed = int(args[0])

    def run(self):
        mre = self.obj.input(1, cb.read_edge)
        e = _edges_from(mre)
        e = e[e[:, 0] != e[:, 1]]
        N = _edges_global_nvert(self.comm, e)
        plan = G.EdgePlan(mre, e, N, symmetric=True)
        pres = _present(plan)
        mis, niter = G.luby_mis(plan, self.seed, active=pres)
        ids = plan.local_ids[mis]
        mrv = self.obj.create_mr()
        mrv.open()
        mrv.kv_open.add_tensors(ids)
        nset = mrv.close()
        self.obj.output(1, mrv, cb.print_vertex)
        self.message(f"Luby_find: {nset} MIS vertices in {niter} iterations")
        self.nset = nset
        self.obj.cleanup()


@command("sssp")
class SSSPCmd(Command):
    """sssp ncnt seed -i weighted-edges -o file mr: single-source shortest paths
    from ncnt random sources with out-edges (oink/sssp.cpp). Output lines are
    "v distance source" (the reference's 3rd column is the predecessor)."""
    ninputs = noutputs = 1

    def params(self, args):
        if len(args) != 2:
            raise OinkError("Illegal sssp command")
        self.ncnt, self.seed = int(args[0]), int(args[1])

    def run(self):
        mre = self.obj.input(1, cb.read_edge_weight)
        e = _edges_from(mre)
        w = mre.kv.vdata.view(torch.float64) if mre.kv.vw == 8 else torch.ones(e.shape[0], dtype=torch.float64,
                                                                                 device=e.device)
        N = _edges_global_nvert(self.comm, e)
        plan = G.EdgePlan(mre, e, N, weights=w)
        outdeg = torch.bincount(plan.src.long(), minlength=plan.nlocal)[: plan.nlocal]
        cand = plan.local_ids[outdeg > 0].cpu().tolist()
        allc = sorted(x for lst in self.comm.allgather_object(cand) for x in lst)
        rng = np.random.default_rng(self.seed)
        sources = [allc[i] for i in rng.permutation(len(allc))[: self.ncnt]] if allc else []
        mr = self.obj.create_mr()
        self.results = []
        for cnt, s in enumerate(sources):
            d, niter = G.sssp(plan, s)
            ok = torch.isfinite(d)
            nlab = self.comm.allreduce(int(ok.sum().item()), "sum")
            self.results.append((s, niter, nlab))
            self.message(f"{cnt}:  Source = {s}; Iterations = {niter}; Num Vtx Labeled = {nlab}")
            ids, dd = plan.local_ids[ok], d[ok]
            src_col = torch.full_like(ids, s)
            mr.map(self.nprocs, lambda i, kv: kv.add_tensors(ids, torch.stack([dd.view(torch.int64), src_col], 1)),
                   addflag=1)
        self.obj.output(1, mr, _print_sssp)
        self.obj.cleanup()


def _print_sssp(mr, fp):
    if not mr.kv.n:
        return
    k = mr.kv.kdata.view(torch.int64).cpu().numpy().view(np.uint64)
    v = mr.kv.vdata.view(torch.int64).view(-1, 2).cpu().numpy()
    dist = v[:, 0].view(np.float64)
    for a, b, c in zip(k, dist, v[:, 1]):
        fp.write("%d %g %d\n" % (a, b, c))


@command("pagerank")
class PageRankCmd(Command):
    """pagerank tol maxiter alpha -i edges -o file mr (the reference command is a
    stub, oink/pagerank.cpp:54-56; implemented per oinkdoc/pagerank.txt)"""
    ninputs = noutputs = 1

    def params(self, args):
        if len(args) != 3:
            raise OinkError("Illegal pagerank command")
        self.tol, self.maxiter, self.alpha = float(args[0]), int(args[1]), float(args[2])

    def run(self):
        from ..models.pagerank import PageRank
        mre = self.obj.input(1, cb.read_edge)
        e = _edges_from(mre)
        N = _edges_global_nvert(self.comm, e)
        tmp = self.obj.copy_mr(mre)
        pr = PageRank(tmp, N, alpha=self.alpha).build()
        niter = pr.run(self.maxiter, self.tol)
        ids, r = pr.ranks()
        mrr = self.obj.create_mr()
        rr = r.to(torch.float64)
        mrr.map(self.nprocs, lambda i, kv: kv.add_tensors(ids, rr))
        self.obj.output(1, mrr, cb.print_vertex_double)
        self.message(f"PageRank: {N} vertices, {niter} iterations, L1 delta {pr.delta():g}")
        self.obj.cleanup()
