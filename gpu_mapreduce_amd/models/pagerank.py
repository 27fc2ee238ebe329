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
built once (native PageRankPlan, csrc/engine/graphplan.cpp): every iteration
moves only float values through three kernels (fused gather segmented sum,
combine, update) and one all-to-all — no host synchronisation inside the
loop unless tol > 0. Local vertices are relabelled by out-degree so the hot
part of the gathered rank array stays cache-resident.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .._ext import C
from ..runtime.mapreduce import MapReduce

GRAPH500 = (0.57, 0.19, 0.19, 0.05)


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
        self._p = None

    def build(self):
        """Requires mr.kv = EDGE KVs (any distribution). Builds the iteration plan."""
        e = self.mr.kv.kdata.view(torch.int64).view(-1, 2)
        self._p = C.PageRankPlan(self.comm.native, e, self.N, self.alpha)
        self.nedge = self._p.nedge
        self.nlocal = self._p.nlocal
        self.ndangling = self._p.ndangling
        # one GPU: propagation-blocked iteration (csrc/kernels/pbpr.hip)
        self.blocking = self._p.blocking
        # source ranges pinned to XCDs (0 = plain pull gather)
        self.xcd_ranges = self._p.xcd_ranges
        # "local" (one GPU), "replicated" (several GPUs: destination-owned
        # edges + all-gathered c = r / outdeg), "partials" (source-owned edges +
        # all-to-all of partial sums: CPU engine / MRH_PR_DIST=partials)
        self.layout = self._p.layout
        self.c_slice = self._p.c_slice
        # bytes this rank receives per iteration (other ranks' c slices + the
        # 16-byte stats allreduce); overlapped: the ring all-gather of c runs
        # under the gather of the slices already in (several GPUs)
        self.comm_bytes_per_iter = self._p.comm_bytes_per_iter
        self.overlapped = self._p.overlapped
        return self

    def reset(self):
        self._p.reset()

    def step(self):
        self._p.step()

    def run(self, maxiter=20, tol=0.0):
        return self._p.run(int(maxiter), float(tol))

    def delta(self):
        return self._p.delta()

    @property
    def use_graph(self) -> bool:
        """fixed-count run() replays a captured HIP graph of two iterations
        (one GPU, XCD tile-step path; MRH_PR_GRAPH=0 turns it off)"""
        return bool(self._p.use_graph)

    @use_graph.setter
    def use_graph(self, on: bool):
        self._p.use_graph = bool(on)

    @property
    def graph_iterations(self) -> int:
        """iterations run so far by graph replay"""
        return int(self._p.graph_iterations)

    def ranks(self):
        """(global vertex ids, ranks) owned by this rank."""
        return self._p.ids(), self._p.ranks()


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
    scale, ef, iters = args.scale, args.edgefactor, args.iters
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
        "metric": "KV-pairs/sec (whole node), PageRank edge contributions (RMAT-2^%d, ef%d)" % (scale, ef),
        "value": nedge * iters / dt,
        "unit": "KV/s",
        "ms_per_step": dt * 1e3,
        "vs_baseline": None,
        "baseline_note": "reference pagerank is a stub (oink/pagerank.cpp:54-56); no published number",
        "iters_per_step": iters,
        "edges": nedge,
        "setup_s": setup,
        "l1_delta_last": pr.delta(),
        "hip_graph_iterations": pr.graph_iterations,
        "layout": pr.layout,
        "comm_bytes_per_iter": comm.allreduce(pr.comm_bytes_per_iter, "max"),
        "comm_overlapped": bool(pr.overlapped),
        "config": {"model": "PageRank", "global_batch": nedge, "seq_len": iters,
                   "parallelism": f"dp{comm.size}", "scale": scale, "edgefactor": ef, "alpha": 0.85},
        "scaling": "strong",
    }
