"""Iterative graph algorithms on a reusable MapReduce "edge plan".

An edge plan is the MapReduce dataflow of one propagation step

    map      edge (i -> j)  ->  (j, f(x_i, w_ij))
    combine  OP per j on the sender (MR-MPI compress)
    shuffle  to owner(j) = j % P           (RCCL all-to-all, xGMI)
    reduce   OP per j on the owner

whose keys never change between iterations, so the sort / group / routing
plan is built once with engine ops (aggregate, radix sort, segments) and every
iteration moves only values: one fused gather+segmented-reduce kernel, one
all-to-all, one combine kernel (csrc/kernels/graphops.hip). OP is sum, min or
max; f is x_i or x_i + w_ij. cc_find (min-label propagation), sssp
(Bellman-Ford relaxation) and luby_find (max-priority rounds) are built on
it; PageRank (pagerank.py) uses a specialised float variant.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .._ext import C
from ..runtime.mapreduce import MapReduce

OPS = {"sum": 0, "min": 1, "max": 2}
VMASK = (1 << 40) - 1


class EdgePlan:
    def __init__(self, mr: MapReduce, edges: torch.Tensor, nvert: int, weights: torch.Tensor | None = None,
                 symmetric=False):
        """edges: this rank's [n,2] int64 (vi, vj) (any distribution);
        weights: optional per-edge values (dtype of the propagated values)."""
        self.mr, self.comm = mr, mr.comm
        self.P, self.me, self.dev = mr.nprocs, mr.me, mr.device
        self.N = int(nvert)
        self.nlocal = max(0, (self.N - self.me + self.P - 1) // self.P)
        P, dev = self.P, self.dev
        e = edges.to(dev)
        w = weights.to(dev) if weights is not None else None
        if symmetric:
            e = torch.cat([e, e.flip(1)])
            if w is not None:
                w = torch.cat([w, w])
        # 1. edges to the owner of their source (engine shuffle)
        if P > 1:
            vb = w.contiguous().view(torch.uint8) if w is not None else torch.empty(0, dtype=torch.uint8, device=dev)
            kv = C.make_kv(e.contiguous().view(torch.uint8), None, vb, None, e.shape[0], dev)
            kv, _ = C.exchange(kv, (e[:, 0] % P).to(torch.int32), self.comm.pg)
            e = kv.kdata.view(torch.int64).view(-1, 2)
            if w is not None:
                w = kv.vdata.view(w.dtype)
        self.nedge = e.shape[0]
        src_local = (e[:, 0] // P).to(torch.int32)
        vj = e[:, 1]
        # 2. plan: sort by (owner(vj), vj)
        key = ((vj % P) << 40) | vj if P > 1 else vj.contiguous()
        ks, perm, _ = C.radix_sort_pairs(key, torch.arange(self.nedge, dtype=torch.int32, device=dev), 0, 64)
        pl = perm.long()
        self.src = src_local[pl].contiguous()
        self.w = w[pl].contiguous() if w is not None else None
        self.seg = C.segments_sorted(ks)
        ujv = ks[self.seg[:-1]] & VMASK
        self.ngrp = self.seg.numel() - 1
        if P > 1:
            scount = torch.bincount(ujv % P, minlength=P)
            rcount = torch.empty_like(scount)
            dist.all_to_all_single(rcount, scount, group=self.comm.group)
            self.send_splits = scount.cpu().tolist()
            self.recv_splits = rcount.cpu().tolist()
            rids = torch.empty(sum(self.recv_splits), dtype=torch.int64, device=dev)
            dist.all_to_all_single(rids, ujv.contiguous(), self.recv_splits, self.send_splits, group=self.comm.group)
            rs, rperm, _ = C.radix_sort_pairs(rids // P, torch.arange(rids.numel(), dtype=torch.int32, device=dev), 0, 64)
            self.rseg = C.segments_sorted(rs)
            self.rperm = rperm
            self.rvid = rs[self.rseg[:-1]].to(torch.int32)
            self.nrecv = rids.numel()
        else:
            self.vid = (ujv // P).to(torch.int32)
        self.local_ids = torch.arange(self.nlocal, device=dev, dtype=torch.int64) * P + self.me

    def propagate(self, x: torch.Tensor, op: str, identity, use_weights=False) -> torch.Tensor:
        """acc[v] = OP over in-edges (i -> v) of x[i] (+ w). Vertices without in-edges get identity."""
        o = OPS[op]
        dev = self.dev
        send = torch.empty(self.ngrp, dtype=x.dtype, device=dev)
        w = self.w if (use_weights and self.w is not None) else torch.empty(0, dtype=x.dtype, device=dev)
        C.plan_gather_reduce(self.seg, self.src, x.contiguous(), w, o, send)
        acc = torch.full((self.nlocal,), identity, dtype=x.dtype, device=dev)
        if self.P > 1:
            recv = torch.empty(self.nrecv, dtype=x.dtype, device=dev)
            dist.all_to_all_single(recv, send, self.recv_splits, self.send_splits, group=self.comm.group)
            C.plan_combine(self.rseg, self.rperm, recv, self.rvid, o, acc)
        else:
            acc[self.vid.long()] = send
        return acc

    def any_global(self, flag_tensor) -> bool:
        n = int(flag_tensor.sum().item()) if flag_tensor.numel() else 0
        return self.comm.allreduce(n, "sum") > 0

    def count_global(self, mask) -> int:
        return int(self.comm.allreduce(int(mask.sum().item()), "sum"))


def connected_components(plan: EdgePlan, max_iter=10_000):
    """min-label propagation: label(v) = min vertex id in v's component.
    Returns (labels_local int64, iterations)."""
    lab = plan.local_ids.clone()
    big = (1 << 62)
    it = 0
    while it < max_iter:
        it += 1
        m = plan.propagate(lab, "min", big)
        new = torch.minimum(lab, m)
        changed = new != lab
        lab = new
        if not plan.any_global(changed):
            break
    return lab, it


def _s64(c):
    c &= (1 << 64) - 1
    return c - (1 << 64) if c >= (1 << 63) else c


def luby_mis(plan: EdgePlan, seed: int, active=None, max_iter=10_000):
    """Luby's maximal independent set: each round every active vertex draws a
    random priority; local maxima among active neighbours join the set and
    their neighbours drop out. Returns (in_set bool local, rounds)."""
    dev = plan.dev
    ids = plan.local_ids
    act = torch.ones(plan.nlocal, dtype=torch.bool, device=dev) if active is None else active.clone()
    mis = torch.zeros(plan.nlocal, dtype=torch.bool, device=dev)
    it = 0
    while it < max_iter and plan.count_global(act) > 0:
        it += 1
        # priority = (23 hashed bits of (vertex, seed, round), vertex id): unique per round
        h = ids * _s64(0x9E3779B97F4A7C15) + _s64((seed + 1) * 0x632BE59BD9B4E019 + it * 0x8CB92BA72F3D8DD7)
        h = (h ^ (h >> 31)) * _s64(0x94D049BB133111EB)
        h = h ^ (h >> 29)
        r = ((h >> 40) & ((1 << 23) - 1)) << 40 | (ids & VMASK)
        pri = torch.where(act, r, torch.full_like(r, -1))
        m = plan.propagate(pri, "max", -1)
        join = act & (pri > m)
        mis |= join
        nb = plan.propagate(join.to(torch.int64), "max", 0)
        act &= ~(join | (nb > 0))
    return mis, it


def sssp(plan: EdgePlan, source: int, max_iter=100_000):
    """Bellman-Ford relaxation from `source` over weighted edges (float64).
    Returns (dist local float64 with inf for unreachable, iterations)."""
    dev = plan.dev
    inf = float("inf")
    d = torch.full((plan.nlocal,), inf, dtype=torch.float64, device=dev)
    if source % plan.P == plan.me:
        d[source // plan.P] = 0.0
    it = 0
    while it < max_iter:
        it += 1
        m = plan.propagate(d, "min", inf, use_weights=True)
        new = torch.minimum(d, m)
        changed = new != d
        d = new
        if not plan.any_global(changed):
            break
    return d, it


def reference_cc(edges: np.ndarray, n: int):
    """union-find oracle"""
    parent = np.arange(n)

    def find(a):
        while parent[a] != a:
            parent[a] = parent[parent[a]]
            a = parent[a]
        return a
    for a, b in edges:
        ra, rb = find(a), find(b)
        if ra != rb:
            parent[max(ra, rb)] = min(ra, rb)
    return np.array([find(i) for i in range(n)])
