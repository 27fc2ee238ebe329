"""K-means as a MapReduce job (models/kmeans.py; GPMR K-means workload of the
fork's chapter) vs a NumPy Lloyd oracle."""
import numpy as np
import pytest
import torch

import gpu_mapreduce_amd as g
from gpu_mapreduce_amd import C
from gpu_mapreduce_amd.models.kmeans import KMeans, blobs, reference_lloyd


def _map_ref(p, c):
    p64, c64 = p.double().cpu().numpy(), c.double().cpu().numpy()
    lab = ((p64[:, None, :] - c64[None]) ** 2).sum(-1).argmin(1)
    K, D = c.shape
    acc = np.zeros((K, D + 1))
    for k in range(K):
        m = lab == k
        acc[k, :D] = p64[m].sum(0)
        acc[k, D] = m.sum()
    return acc.reshape(-1)


def _kv_vals(kv):
    keys = kv.kdata.cpu().view(torch.int32).long().numpy()
    vals = kv.vdata.cpu().view(torch.float64).numpy()
    out = np.zeros(keys.max() + 1)
    out[keys] = vals
    return out


@pytest.mark.parametrize("D", [2, 5])
def test_kmeans_map_cpu(D):
    p = blobs(5000, D, 7, seed=1, device="cpu")
    c = blobs(7, D, 7, seed=2, device="cpu")
    np.testing.assert_allclose(_kv_vals(C.kmeans_map(p, c)), _map_ref(p, c), rtol=1e-9, atol=1e-9)


def test_kmeans_job_matches_lloyd():
    p = blobs(4000, 2, 5, seed=3, device="cpu")
    init = blobs(5, 2, 5, seed=4, device="cpu")
    km = KMeans(g.Comm(device="cpu"), p, init)
    for _ in range(6):
        assert km.iterate() == 4000
    ref = reference_lloyd(p.numpy(), init.numpy(), 6)
    np.testing.assert_allclose(km.centroids.double().numpy(), ref, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("D,K", [(2, 32), (3, 5), (1, 8), (3, 64), (8, 64), (16, 10), (5, 7), (32, 64), (64, 128), (100, 40),
                                 (128, 16), (160, 8)])
def test_kmeans_map_gpu(D, K):
    """lane-private accumulator kernel (D <= 3, K * (D+1) <= 184; (3, 64)
    falls back to the LDS-atomic batched kernel), fused assign + LDS combine
    kernel (D <= 8), the matrix-core kernel
    (D <= 128, any K that fits LDS) and the GEMM fallback (D = 160) against
    the float64 oracle; a point equidistant to two centroids may go either
    way, so compare with a tolerance on the counts too"""
    p = blobs(300_000, D, K, seed=5, device="cuda")
    c = blobs(K, D, K, seed=6, device="cuda")
    got = _kv_vals(C.kmeans_map(p, c))
    ref = _map_ref(p, c)
    assert got.shape == ref.shape
    counts_got, counts_ref = got.reshape(K, D + 1)[:, D], ref.reshape(K, D + 1)[:, D]
    assert counts_got.sum() == 300_000
    assert np.abs(counts_got - counts_ref).max() <= 3
    # each point that went to the other of two (near-)equidistant centroids
    # moves its coordinates (< 1.5 in the unit-cube blobs) between two sums
    moved = max(1.0, np.abs(counts_got - counts_ref).sum() / 2)
    np.testing.assert_allclose(got, ref, rtol=1e-3, atol=1.5 * moved)


@pytest.mark.gpu
def test_kmeans_job_gpu_matches_cpu():
    p = blobs(200_000, 2, 16, seed=7, device="cpu")
    init = blobs(16, 2, 16, seed=8, device="cpu")
    cpu = KMeans(g.Comm(device="cpu"), p, init)
    gpu = KMeans(g.Comm(device="cuda"), p.cuda(), init)
    for _ in range(5):
        cpu.iterate()
        gpu.iterate()
    # the engines score ||c||^2 - 2 x.c in different fp32 orders, so a point
    # within rounding of two centroids may go either way (each such point
    # moves a centroid by ~1e-5 here)
    np.testing.assert_allclose(gpu.centroids.cpu().double().numpy(), cpu.centroids.double().numpy(), atol=5e-4)
