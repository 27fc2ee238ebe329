"""Triangle finding/counting (the tri_find workload).

Reference: oink/tri_find.cpp:43-82 — 4 MapReduce shuffles, O(sum d^2) wedge
KVs. The MI355X design (csrc/kernels/tri.hip) instead:

  1. packs every local edge as lo<<32|hi (self loops dropped) and, for P > 1,
     all-gathers the packed list over RCCL (the whole deduplicated RMAT-24 x16
     graph is ~2 GB; every GPU has 288 GB of HBM, so replication is the
     cheap option and removes all later communication);
  2. radix-sorts and deduplicates (the edge_upper step), computes degrees,
     orients each edge from the lower to the higher (degree, id) endpoint and
     builds a CSR with sorted rows;
  3. every rank intersects N+(u) ∩ N+(v) for its slice of the oriented edges
     (one thread per edge, merge or galloping intersection) and the counts
     are all-reduced. Each triangle is found exactly once.

The OINK command keeps the reference's MapReduce formulation available as
`tri_find_mr`; `tri_find` uses this path.
"""
from __future__ import annotations

import time

import torch

from .._ext import C


def pack_edges(e: torch.Tensor) -> torch.Tensor:
    """[n,2] int64 (any orientation, duplicates ok) -> packed lo<<32|hi, self loops dropped."""
    lo = torch.minimum(e[:, 0], e[:, 1])
    hi = torch.maximum(e[:, 0], e[:, 1])
    keep = lo != hi
    return (lo[keep] << 32) | hi[keep]


class TriangleGraph:
    """Python face of the native TriangleGraph (csrc/engine/graphplan.cpp)."""

    def __init__(self, comm, edges: torch.Tensor, nvert: int | None = None):
        """edges: this rank's [n,2] int64 edges (any distribution)."""
        self.comm = comm
        self._g = C.TriangleGraph(comm.native, edges, -1 if nvert is None else int(nvert))
        self.nedge, self.nvert = self._g.nedge, self._g.nvert
        self.rowptr, self.col, self.okeys, self.perm = self._g.rowptr, self._g.col, self._g.okeys, self._g.perm

    def count(self) -> int:
        return int(self._g.count())

    def triangles(self) -> torch.Tensor:
        """This rank's share of the triangles, [T,3] int64, each row sorted (a<b<c)."""
        return self._g.triangles()


def brute_force_count(edges) -> int:
    """numpy oracle for small graphs: trace(A^3)/6 of the simple undirected graph."""
    import numpy as np
    e = np.asarray(edges)
    lo, hi = np.minimum(e[:, 0], e[:, 1]), np.maximum(e[:, 0], e[:, 1])
    k = lo != hi
    u = np.unique(np.stack([lo[k], hi[k]], 1), axis=0)
    n = int(u.max()) + 1 if len(u) else 0
    A = np.zeros((n, n), dtype=np.int64)
    A[u[:, 0], u[:, 1]] = 1
    A = A + A.T
    return int(np.trace(A @ A @ A) // 6)


def bench_trifind(comm, args):
    """tri_find on an R-MAT graph (BASELINE config: scale 24). One step =
    dedup + orientation + CSR + count from the raw generated edge list (the
    generation itself is the separate `rmat` command and is not timed)."""
    from .pagerank import GRAPH500
    scale, ef = args.scale, args.edgefactor
    ntotal = (1 << scale) * ef
    P, me = comm.size, comm.rank
    lo, hi = me * ntotal // P, (me + 1) * ntotal // P
    ts = time.perf_counter()
    kv = C.map_rmat(hi - lo, scale, *GRAPH500, 0.0, args.seed, lo, comm.device)
    edges = kv.kdata.view(torch.int64).view(-1, 2)
    del kv
    if comm.is_cuda:
        torch.cuda.synchronize()
    setup = comm.allreduce(time.perf_counter() - ts, "max", dtype=torch.float64)

    def sync():
        if comm.is_cuda:
            torch.cuda.synchronize()
        comm.barrier()

    def step():
        g = TriangleGraph(comm, edges, 1 << scale)
        return g, g.count()

    for _ in range(args.warmup):
        step()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        g, ntri = step()
    sync()
    dt = comm.allreduce((time.perf_counter() - t0) / args.steps, "max", dtype=torch.float64)
    return {
        "metric": f"KV-pairs/sec (whole node), tri_find edges processed (RMAT-2^{scale}, ef{ef})",
        "value": ntotal / dt, "unit": "KV/s", "ms_per_step": dt * 1e3, "vs_baseline": None,
        "baseline_note": "reference publishes no tri_find number",
        "config": {"model": "tri_find", "global_batch": ntotal, "seq_len": 1, "parallelism": f"dp{P}",
                   "scale": scale, "edgefactor": ef, "rmat": "graph500 a=.57 b=c=.19"},
        "triangles": ntri, "unique_edges": g.nedge, "scaling": "strong", "setup_ms": setup * 1e3,
        "hub_vertices": int(C.tri_last_hub_size()),
        "build": "split" if g._g.split else ("halo" if g._g.distributed else "replicated"),
    }


def tri_find_mr(comm, edges: torch.Tensor, hbm_budget=0, host_budget=0, fpath="", memsize=0, upper=True):
    """The reference's MapReduce tri_find (oink/tri_find.cpp:43-82): edge_upper
    (map -> collate -> reduce cull) then 4 collates with the O(d^2) wedge
    reduce, on the generic engine ops (csrc/oink/trifind_mr.cpp), every stage
    device-synchronised and timed. edges: this rank's raw [n,2] int64 edges.
    Returns {"triangles", "stages": [{op, ms, pairs_in, pairs_out}], spool stats}."""
    return dict(C.tri_find_mr(comm.native, edges, int(hbm_budget), int(host_budget), str(fpath), int(memsize),
                              bool(upper)))


def bench_trifind_mr(comm, args):
    """tri_find as the 4-collate MapReduce pipeline on an R-MAT graph: the
    generic engine at large KV counts (RMAT-20: ~16 M edges -> ~1.3 G wedge
    pairs through collate 4). Optional out-of-core run (args.mr_ooc_scale)
    under an HBM budget that forces the spool tiers."""
    import shutil
    import tempfile
    from .pagerank import GRAPH500
    scale, ef = args.scale, args.edgefactor
    ntotal = (1 << scale) * ef
    P, me = comm.size, comm.rank

    def edges_of(sc):
        nt = (1 << sc) * ef
        lo, hi = me * nt // P, (me + 1) * nt // P
        kv = C.map_rmat(hi - lo, sc, *GRAPH500, 0.0, args.seed, lo, comm.device)
        return kv.kdata.view(torch.int64).view(-1, 2)

    def sync():
        if comm.is_cuda:
            torch.cuda.synchronize()
        comm.barrier()

    e = edges_of(scale)
    want = TriangleGraph(comm, e, 1 << scale).count()  # the specialised path's count, for the check
    for _ in range(args.warmup):
        tri_find_mr(comm, e)
    sync()
    runs = []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        r = tri_find_mr(comm, e)
        sync()
        runs.append(time.perf_counter() - t0)
    dt = comm.allreduce(sum(runs) / len(runs), "max", dtype=torch.float64)
    stages = [{"op": s["op"], "ms": round(s["ms"], 3), "pairs_in": s["pairs_in"], "pairs_out": s["pairs_out"],
               "Mkvps_in": round(s["pairs_in"] / max(s["ms"], 1e-9) / 1e3, 1)} for s in r["stages"]]
    out = {
        "metric": f"KV-pairs/sec (whole node), tri_find_mr raw edges through the 4-collate pipeline "
                  f"(RMAT-2^{scale}, ef{ef})",
        "value": ntotal / dt, "unit": "KV/s", "ms_per_step": dt * 1e3, "vs_baseline": None,
        "config": {"model": "tri_find_mr", "global_batch": ntotal, "seq_len": 1, "parallelism": f"dp{P}",
                   "scale": scale, "edgefactor": ef},
        "triangles": int(r["triangles"]), "triangles_check": int(want),
        "stages": stages, "scaling": "strong",
        "wedge_pairs": max((s["pairs_out"] for s in r["stages"] if s["op"] == "reduce nsq_angles"), default=0),
        "compact_vb": int(r.get("compact_vb", 0)),
    }
    bscale = getattr(args, "mr_big_scale", 0) or 0
    if bscale > 0:
        # a larger graph in HBM: R-MAT-22's ~7 G wedge pairs go through collate
        # 4 as 12-byte compact pairs, grouped in hash-balanced buckets
        eb = edges_of(bscale)
        wantb = TriangleGraph(comm, eb, 1 << bscale).count()
        tri_find_mr(comm, eb)  # warm: the pool holds the peak afterwards
        sync()
        t0 = time.perf_counter()
        rb = tri_find_mr(comm, eb)
        sync()
        dtb = comm.allreduce(time.perf_counter() - t0, "max", dtype=torch.float64)
        out["big"] = {"scale": bscale, "ms": dtb * 1e3, "triangles": int(rb["triangles"]),
                      "triangles_check": int(wantb), "compact_vb": int(rb.get("compact_vb", 0)),
                      "edges": (1 << bscale) * ef,
                      "wedge_pairs": max((s["pairs_out"] for s in rb["stages"] if s["op"] == "reduce nsq_angles"),
                                         default=0),
                      "stages": [{"op": s["op"], "ms": round(s["ms"], 3), "pairs_in": s["pairs_in"],
                                  "pairs_out": s["pairs_out"]} for s in rb["stages"]]}
        del eb
    oscale = getattr(args, "mr_ooc_scale", 0) or 0
    if oscale > 0:
        root = tempfile.mkdtemp(prefix=f"mrh_trimr_{me}_")
        try:
            e2 = edges_of(oscale)
            want2 = TriangleGraph(comm, e2, 1 << oscale).count()
            budget = int(getattr(args, "mr_ooc_hbm", 256 << 20))
            host = int(getattr(args, "mr_ooc_host", 2 << 30))
            # pages of the reference's default memsize (64 MB): spool pieces of
            # min(page, budget / 4) = 64 MiB. Run twice: the first (cold) run
            # also pays what the process had not set up yet (pinned host
            # allocations beyond the start-up reserve, gpu_mapreduce_amd/hostpin.py;
            # pool growth); the record's numbers are the second run's
            dts = []
            for _ in range(2):
                sync()
                t0 = time.perf_counter()
                r2 = tri_find_mr(comm, e2, hbm_budget=budget, host_budget=host, fpath=root, memsize=64)
                sync()
                dts.append(comm.allreduce(time.perf_counter() - t0, "max", dtype=torch.float64))
            dt2 = dts[-1]
            out["ooc"] = {"note": "run after the in-HBM big graph (its ~180 GB pool peak)",
                          "scale": oscale, "ms": dt2 * 1e3, "ms_cold": dts[0] * 1e3, "triangles": int(r2["triangles"]),
                          "triangles_check": int(want2), "hbm_budget": budget, "host_budget": host,
                          "spool_files": r2["spool_files"], "spool_host_bytes": r2["spool_host_bytes"],
                          "spool_disk_bytes": r2["spool_disk_bytes"],
                          # per stage: host <-> device bytes of this rank, and
                          # the time at the PCIe floor (50 GB/s) they imply;
                          # disk_bytes: spool / result files written (the disk tier)
                          "stages": [{"op": s["op"], "ms": round(s["ms"], 3), "pairs_in": s["pairs_in"],
                                      "pcie_bytes": s["h2d_bytes"] + s["d2h_bytes"],
                                      "pcie_floor_ms": round((s["h2d_bytes"] + s["d2h_bytes"]) / 50e6, 3),
                                      "x_floor": round(s["ms"] / max((s["h2d_bytes"] + s["d2h_bytes"]) / 50e6, 1e-3), 2),
                                      "disk_bytes": s["disk_bytes"]}
                                     for s in r2["stages"]]}
        finally:
            shutil.rmtree(root, ignore_errors=True)
    return out
