"""Iterative graph algorithms on the native "edge plan"
(csrc/engine/graphplan.h): the MapReduce dataflow of one propagation step
(map edge -> (dst, f(x_src, w)), combine per dst on the sender, RCCL
all-to-all to owner(dst), reduce per dst) whose routing is built once, so each
iteration moves only values. cc_find (min-label propagation), sssp
(Bellman-Ford relaxation) and luby_find (max-priority rounds) run on it; the
same C++ code serves the OINK commands.
"""
from __future__ import annotations

import numpy as np
import torch

from .._ext import C
from ..runtime.mapreduce import MapReduce

OPS = {"sum": 0, "min": 1, "max": 2}


class EdgePlan:
    def __init__(self, mr: MapReduce, edges: torch.Tensor, nvert: int, weights: torch.Tensor | None = None,
                 symmetric=False):
        """edges: this rank's [n,2] int64 (vi, vj) (any distribution);
        weights: optional per-edge values (dtype of the propagated values)."""
        self.mr, self.comm = mr, mr.comm
        self.dev = mr.device
        self._p = C.EdgePlan(mr.comm.native, edges, int(nvert), weights, bool(symmetric))
        self.P, self.me, self.N = self._p.P, self._p.me, self._p.N
        self.nlocal, self.nedge, self.ngrp = self._p.nlocal, self._p.nedge, self._p.ngrp
        self.src, self.seg, self.local_ids = self._p.src, self._p.seg, self._p.local_ids
        self.w = self._p.w if weights is not None else None

    def propagate(self, x: torch.Tensor, op: str, identity, use_weights=False) -> torch.Tensor:
        """acc[v] = OP over in-edges (i -> v) of x[i] (+ w). Vertices without in-edges get identity."""
        return self._p.propagate(x, OPS[op], float(identity), bool(use_weights))

    def any_global(self, flag_tensor) -> bool:
        return self._p.count_global(flag_tensor) > 0

    def count_global(self, mask) -> int:
        return int(self._p.count_global(mask))


def connected_components(plan: EdgePlan, max_iter=100_000):
    """min-label propagation: label(v) = min vertex id in v's component.
    Returns (labels_local int64, iterations)."""
    return C.connected_components(plan._p, max_iter)


def luby_mis(plan: EdgePlan, seed: int, active=None, max_iter=100_000):
    """Luby's maximal independent set: each round every active vertex draws a
    random priority; local maxima among active neighbours join the set and
    their neighbours drop out. Returns (in_set bool local, rounds)."""
    return C.luby_mis(plan._p, int(seed), active, max_iter)


def sssp(plan: EdgePlan, source: int, max_iter=1_000_000):
    """Bellman-Ford relaxation from `source` over weighted edges (float64).
    Returns (dist local float64 with inf for unreachable, iterations)."""
    return C.sssp(plan._p, int(source), max_iter)


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
