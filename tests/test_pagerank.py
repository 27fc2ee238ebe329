"""PageRank (defined per oinkdoc/pagerank.txt; the reference command is a stub)
vs a float64 numpy oracle, on the CPU engine and (marked) on the GPU."""
import numpy as np
import pytest
import torch

import gpu_mapreduce_amd as g
from gpu_mapreduce_amd import C
from gpu_mapreduce_amd.models.pagerank import PageRank, reference_pagerank, rmat_map


def _run(device, scale=10, ef=8, iters=15):
    comm = g.Comm(device=device)
    mr = g.MapReduce(comm)
    rmat_map(mr, scale, ef, seed=3)
    edges = mr.kv.kdata.view(torch.int64).view(-1, 2).cpu().numpy().copy()
    pr = PageRank(mr, 1 << scale).build()
    pr.run(iters)
    ids, r = pr.ranks()
    out = np.zeros(1 << scale)
    out[ids.cpu().numpy()] = r.cpu().numpy()
    return edges, out


def test_rmat_cpu_shape_and_skew():
    mr = g.MapReduce(g.Comm(device="cpu"))
    n = rmat_map(mr, 12, 4, seed=1)
    assert n == 4 << 12
    e = mr.kv.kdata.view(torch.int64).view(-1, 2)
    assert int(e.max()) < (1 << 12) and int(e.min()) >= 0
    deg = torch.bincount(e[:, 0], minlength=1 << 12)
    assert deg.max() > 20 * deg.float().mean()   # R-MAT hubs


def test_pagerank_cpu_matches_numpy():
    edges, r = _run("cpu")
    ref = reference_pagerank(edges, 1 << 10, iters=15)
    np.testing.assert_allclose(r, ref, rtol=2e-4, atol=1e-9)
    assert abs(r.sum() - 1.0) < 1e-3


@pytest.mark.gpu
def test_pagerank_gpu_matches_numpy():
    edges, r = _run("cuda", scale=14, ef=16)
    ref = reference_pagerank(edges, 1 << 14, iters=15)
    np.testing.assert_allclose(r, ref, rtol=2e-4, atol=1e-9)
