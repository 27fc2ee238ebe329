"""K-means (Lloyd) as a MapReduce job — the GPMR K-means workload of the
fork's chapter (chapter_final.pdf §3.4, Fig. 6a: 32 M 2-D points per GPU,
map ≈ 1.4 s per iteration on a GK104). The reference code has no
K-means; this is the same job on the MR-MPI programming model:

  map       every rank assigns its resident points to the nearest centroid and
            emits (cluster, coordinate sums, count) — combined in the map
            kernel (csrc/kernels/kmeans.hip: centroids in LDS, per-workgroup
            LDS partials, fp64 global atomics), the equivalent of GPMR's
            emit(cluster, point) + combiner;
  collate   partition by cluster over RCCL + group-by;
  reduce    sum:float64 (segmented reduce);
  gather(1) + broadcast(0)  every rank receives all cluster sums and forms the
            new centroids (empty clusters keep their centroid).
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .._ext import C
from ..runtime.mapreduce import MapReduce


class KMeans:
    def __init__(self, comm, points: torch.Tensor, centroids: torch.Tensor):
        """points: this rank's [N, D] float32 points on the engine device;
        centroids: initial [K, D] (identical on every rank)."""
        self.comm = comm
        self.points = points.contiguous()
        self.centroids = centroids.to(points.device, torch.float32).contiguous()
        self.K, self.D = self.centroids.shape

    def iterate(self, sync=True):
        """one Lloyd iteration; returns the global point count (sync=False:
        returns None and leaves the shift / count on the device, read through
        the `shift` / `npoints` properties — no host round trip per
        iteration)"""
        K, D = self.K, self.D
        mr = MapReduce(self.comm)
        mr.map(mr.nprocs, lambda itask, kv: kv.add_kv(C.kmeans_map(self.points, self.centroids)))
        mr.collate()
        mr.reduce("sum:float64")
        mr.gather(1)
        mr.broadcast(0)
        kv = mr.kv
        acc = torch.zeros(K * (D + 1), dtype=torch.float64, device=self.points.device)
        if kv is not None and kv.n:
            keys = kv.kdata.view(torch.int32).long()
            acc[keys] = kv.vdata.view(torch.float64)
        acc = acc.view(K, D + 1)
        cnt = acc[:, D:]
        new = torch.where(cnt > 0, acc[:, :D] / cnt.clamp_min(1), self.centroids.double())
        self._shift = (new - self.centroids.double()).norm(dim=1).max()
        self.centroids = new.float().contiguous()
        self.counts = cnt.squeeze(1).long()
        self._npoints = self.counts.sum()
        return self.npoints if sync else None

    @property
    def shift(self):
        """largest centroid move of the last iteration"""
        return float(self._shift)

    @property
    def npoints(self):
        """points assigned in the last iteration (all ranks)"""
        return int(self._npoints)


def blobs(n, D, K, seed, device, spread=0.05):
    """n points around K random centres in the unit cube (float32 [n, D])"""
    g = torch.Generator(device=device).manual_seed(seed)
    centres = torch.rand(K, D, generator=torch.Generator().manual_seed(1234)).to(device)
    lab = torch.randint(0, K, (n,), generator=g, device=device)
    return centres[lab] + spread * torch.randn(n, D, generator=g, device=device)


def reference_lloyd(points: np.ndarray, cen: np.ndarray, iters: int):
    """NumPy oracle (float64)"""
    c = cen.astype(np.float64).copy()
    p = points.astype(np.float64)
    for _ in range(iters):
        d = ((p[:, None, :] - c[None, :, :]) ** 2).sum(-1)
        lab = d.argmin(1)
        for k in range(c.shape[0]):
            m = lab == k
            if m.any():
                c[k] = p[m].mean(0)
    return c


GPMR_POINTS_PER_GPU_S = 32 * 2 ** 20 / 1.4   # 32 M 2-D points per GPU, map ≈ 1.4 s (Fig. 6a)


def bench_kmeans(comm, args):
    n = int(args.kmeans_points)
    D, K = int(args.kmeans_dim), int(args.kmeans_k)
    pts = blobs(n, D, K, seed=args.seed * 7 + comm.rank, device=comm.device)
    init = blobs(K, D, K, seed=99, device="cpu").to(comm.device)      # same on every rank
    iters = int(args.iters)

    def step():
        km = KMeans(comm, pts, init)
        for _ in range(iters):
            km.iterate(sync=False)
        return km

    for _ in range(args.warmup):
        step()
    if comm.is_cuda:
        torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        km = step()
    if comm.is_cuda:
        torch.cuda.synchronize()
    comm.barrier()
    dt = comm.allreduce((time.perf_counter() - t0) / args.steps, "max", dtype=torch.float64)
    total = comm.allreduce(n, "sum")
    value = total * iters / dt
    return {
        "metric": "KV-pairs/sec (whole node), K-means points assigned per second",
        "value": value,
        "unit": "KV/s",
        "ms_per_step": dt * 1e3,
        "vs_baseline": value / (GPMR_POINTS_PER_GPU_S * comm.size),
        "baseline_note": "GPMR K-means (chapter_final.pdf Fig. 6a): 32M 2-D points per GPU, map ~1.4 s "
                         "per iteration on GK104 = 24.0M points/s per GPU",
        "dtype": "fp32 points/distances, fp64 accumulation",
        "iters_per_step": iters,
        "points_per_gpu": n,
        "final_shift": km.shift,
        "config": {"model": "KMeans", "global_batch": total, "seq_len": iters, "parallelism": f"dp{comm.size}",
                   "dim": D, "k": K},
    }
