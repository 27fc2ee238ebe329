"""PageRank on an R-MAT graph as an iterated MapReduce.

The reference's OINK `pagerank` is a stub (oink/pagerank.cpp:54-56; spec in
oinkdoc/pagerank.txt). We define it as the documented iteration:

    w_ij = 1/outdeg(i)                       (oink degree_weight pipeline)
    r'_j = (1-alpha)/N + alpha * (sum_i w_ij r_i + D/N),  D = dangling mass
    stop after maxiter or when ||r' - r||_1 < tol

Graph construction is MapReduce: R-MAT edges come from a device map
(csrc/kernels/graph.hip), edges are aggregated to the owner of their source
vertex (owner(v) = v % P, RCCL all-to-all), and out-degrees come from a
`convert` (group-by source). One PageRank iteration is then the MapReduce

    map      edge (i -> j)       -> (j, w_ij * r_i)
    combine  sum per j locally   (MR-MPI compress)
    shuffle  to owner(j)         (RCCL all-to-all over xGMI)
    reduce   sum per j, update r (+ allreduce of L1 delta / dangling mass)

Because the keys (j) never change between iterations, the sort/group plan is
built once ("shuffle plan"): every iteration moves only float values through
three kernels (fused gather*w segmented sum, combine, update) and one
all-to-all — no host synchronisation inside the loop unless tol > 0.
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.distributed as dist

from .._ext import C
from ..runtime.mapreduce import MapReduce

GRAPH500 = (0.57, 0.19, 0.19, 0.05)
VMASK = (1 << 40) - 1


def rmat_map(mr: MapReduce, scale, edgefactor, seed=1, abcd=GRAPH500, fraction=0.0, addflag=0):
    """Every rank generates its share of the N*edgefactor R-MAT edges on its GPU
    (map task per rank), KV = EDGE{u64 vi, u64 vj}, NULL value."""
    P = mr.nprocs
    total = (1 << scale) * edgefactor
    a, b, c, d = abcd

    def gen(itask, kv):
        lo = itask * total // P
        hi = (itask + 1) * total // P
        kv.add_kv(C.map_rmat(hi - lo, scale, a, b, c, d, fraction, seed, lo, mr.device))
    return mr.map(P, gen, addflag=addflag)


class PageRank:
    def __init__(self, mr: MapReduce, nvert, alpha=0.85):
        self.mr = mr
        self.comm = mr.comm
        self.N = int(nvert)
        self.alpha = float(alpha)
        self.P = mr.nprocs
        self.me = mr.me
        self.dev = mr.device
        self.nlocal = (self.N - self.me + self.P - 1) // self.P

    # ------------------------------------------------------------------ setup
    def build(self):
        """Requires mr.kv = EDGE KVs (any distribution). Builds the iteration plan."""
        mr, P, dev = self.mr, self.P, self.dev
        # 1. edges to the owner of their source vertex
        e = mr.kv.kdata.view(torch.int64).view(-1, 2)
        if P > 1:
            mr.aggregate_dest((e[:, 0] % P).to(torch.int32))
            e = mr.kv.kdata.view(torch.int64).view(-1, 2)
        self.nedge = e.shape[0]
        # 2. out-degree = group-by source vertex (MR convert on u64 keys)
        kv = C.make_kv(e[:, 0].contiguous(), None, e[:, 1].contiguous(), None, self.nedge, dev)
        kmv, _ = C.convert(kv)
        vi = kmv.keys.kdata.view(torch.int64)            # unique sources, sorted
        seg = kmv.seg
        deg = (seg[1:] - seg[:-1])
        vj = kmv.vdata.view(torch.int64)                 # edge targets, grouped by source
        outdeg = torch.zeros(self.nlocal, dtype=torch.int64, device=dev)
        outdeg[(vi // P)] = deg
        # 3. relabel local vertices by out-degree (descending, stable): R-MAT hubs
        #    are spread over ids with few 1-bits; clustering them makes the hot
        #    part of the per-iteration gather array L2/Infinity-Cache resident
        dkey = (1 << 40) - outdeg
        _, order, _ = C.radix_sort_pairs(dkey, torch.arange(self.nlocal, dtype=torch.int32, device=dev), 0, 48)
        self.order = order.long()
        new_of_old = torch.empty(self.nlocal, dtype=torch.int32, device=dev)
        new_of_old[self.order] = torch.arange(self.nlocal, dtype=torch.int32, device=dev)
        src_local = torch.repeat_interleave(new_of_old[vi // P], deg, output_size=self.nedge)
        del kmv, kv, vi, deg, e, dkey
        # 4. combine/shuffle plan: edges sorted by (owner(vj), vj)
        key = ((vj % P) << 40) | vj if P > 1 else vj.clone()
        iota = torch.arange(self.nedge, dtype=torch.int32, device=dev)
        ks, perm, _ = C.radix_sort_pairs(key, iota, 0, 64)
        self.src = src_local[perm.long()].contiguous()
        self.w = torch.empty(0, dtype=torch.float32, device=dev)   # weights folded into c = r/outdeg
        del src_local, vj, key, iota, perm
        self.seg = C.segments_sorted(ks)
        ngrp = self.seg.numel() - 1
        ujv = (ks[self.seg[:-1]] & VMASK)               # unique destination vertices (global ids)
        del ks
        self.send = torch.empty(ngrp, dtype=torch.float32, device=dev)
        if P > 1:
            scount = torch.bincount((ujv % P), minlength=P)
            rcount = torch.empty_like(scount)
            dist.all_to_all_single(rcount, scount, group=self.comm.group)
            self.send_splits = scount.cpu().tolist()
            self.recv_splits = rcount.cpu().tolist()
            rids = torch.empty(sum(self.recv_splits), dtype=torch.int64, device=dev)
            dist.all_to_all_single(rids, ujv.contiguous(), self.recv_splits, self.send_splits, group=self.comm.group)
            rloc = rids // P
            rs, rperm, _ = C.radix_sort_pairs(rloc, torch.arange(rloc.numel(), dtype=torch.int32, device=dev), 0, 64)
            self.rseg = C.segments_sorted(rs)
            self.rperm = rperm
            self.rvid = new_of_old[rs[self.rseg[:-1]]].contiguous()
            self.recv = torch.empty(rloc.numel(), dtype=torch.float32, device=dev)
        else:
            self.vid = new_of_old[ujv // P].contiguous()
        deg_new = outdeg[self.order]
        self.dangling = (deg_new == 0).to(torch.uint8)
        self.invdeg = torch.where(deg_new > 0, 1.0 / deg_new.clamp(min=1).to(torch.float64), 0.0).to(torch.float32)
        del new_of_old, deg_new, outdeg
        self.ndangling = int(self.comm.allreduce(int(self.dangling.sum().item()), "sum"))
        self.acc = torch.empty(self.nlocal, dtype=torch.float32, device=dev)
        self.reset()
        return self

    def reset(self):
        self.r = torch.full((self.nlocal,), 1.0 / self.N, dtype=torch.float32, device=self.dev)
        self.rn = torch.empty_like(self.r)
        self.c = self.r * self.invdeg      # r_i / outdeg_i, the value every out-edge of i carries
        self.dmass = torch.tensor([self.ndangling / self.N], dtype=torch.float64, device=self.dev)
        self.last_delta = None

    # ------------------------------------------------------------------ iterate
    def step(self):
        C.pr_contrib(self.seg, self.src, self.w, self.c, self.send)
        self.acc.zero_()
        if self.P > 1:
            dist.all_to_all_single(self.recv, self.send, self.recv_splits, self.send_splits, group=self.comm.group)
            C.pr_combine(self.rseg, self.rperm, self.recv, self.rvid, self.acc)
        else:
            C.scatter_f32(self.send, self.vid, self.acc)
        base = (1.0 - self.alpha) / self.N
        st = C.pr_update(self.acc, self.r, self.rn, self.dangling, base, self.alpha, self.dmass, 1.0 / self.N,
                         self.invdeg, self.c)
        if self.P > 1:
            dist.all_reduce(st, group=self.comm.group)
        self.dmass = st[1:2]
        self.stats = st
        self.r, self.rn = self.rn, self.r

    def run(self, maxiter=20, tol=0.0):
        it = 0
        for it in range(1, maxiter + 1):
            self.step()
            if tol > 0:
                d = float(self.stats[0].item())
                self.last_delta = d
                if d < tol:
                    break
        return it

    def delta(self):
        return float(self.stats[0].item())

    def ranks(self):
        """(global vertex ids, ranks) owned by this rank."""
        ids = self.order * self.P + self.me
        return ids, self.r


def reference_pagerank(edges: np.ndarray, N: int, alpha=0.85, iters=20):
    """float64 numpy oracle of the same iteration."""
    vi, vj = edges[:, 0].astype(np.int64), edges[:, 1].astype(np.int64)
    outdeg = np.bincount(vi, minlength=N).astype(np.float64)
    r = np.full(N, 1.0 / N)
    dang = outdeg == 0
    w = 1.0 / outdeg[vi]
    for _ in range(iters):
        contrib = np.bincount(vj, weights=r[vi] * w, minlength=N)
        r = (1 - alpha) / N + alpha * (contrib + r[dang].sum() / N)
    return r


def bench_pagerank(comm, args):
    scale, ef, iters = args.scale, 16, args.iters
    mr = MapReduce(comm)
    t0 = time.perf_counter()
    rmat_map(mr, scale, ef, seed=args.seed)
    pr = PageRank(mr, 1 << scale).build()
    torch.cuda.synchronize() if comm.is_cuda else None
    setup = comm.allreduce(time.perf_counter() - t0, "max", dtype=torch.float64)
    nedge = comm.allreduce(pr.nedge, "sum")
    for _ in range(args.warmup):
        pr.reset()
        pr.run(iters)
    if comm.is_cuda:
        torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pr.reset()
        pr.run(iters)
    if comm.is_cuda:
        torch.cuda.synchronize()
    comm.barrier()
    dt = comm.allreduce((time.perf_counter() - t0) / args.steps, "max", dtype=torch.float64)
    return {
        "metric": "KV-pairs/sec (whole node), PageRank edge contributions (RMAT-2^%d, ef16)" % scale,
        "value": nedge * iters / dt,
        "unit": "KV/s",
        "ms_per_step": dt * 1e3,
        "vs_baseline": None,
        "baseline_note": "reference pagerank is a stub (oink/pagerank.cpp:54-56); no published number",
        "iters_per_step": iters,
        "edges": nedge,
        "setup_s": setup,
        "l1_delta_last": pr.delta(),
        "config": {"model": "PageRank", "global_batch": nedge, "seq_len": iters,
                   "parallelism": f"dp{comm.size}", "scale": scale, "edgefactor": ef, "alpha": 0.85},
    }
