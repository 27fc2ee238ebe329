"""Multi-rank device-engine rehearsal on a one-GPU box: world size 2, both
ranks on cuda:0, process group over gloo (which moves CUDA tensors too). The
MapReduce data path is the device one — partition kernels, per-destination
stable radix pass, count exchange, all-to-all of device buffers, group-by and
reduce kernels — so every multi-rank bug short of RCCL itself shows here. On
an 8-GPU node the same C++ shuffle runs over RCCL (backend "nccl")."""
import collections

import numpy as np
import pytest
import torch

from test_distributed_cpu import run_world

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def test_collate_wordcount_gpu():
    from test_distributed_cpu import WORDS
    out = run_world("case_wordcount", 2, DEV)
    total = {}
    for r, (n, nu, local) in out.items():
        assert n == len(WORDS)
        assert nu == len(set(WORDS))
        assert not (set(total) & set(local))
        total.update(local)
    assert total == collections.Counter(WORDS)


def test_mixed_layouts_gpu():
    import struct
    out = run_world("case_fixed_and_var_mixed", 2, DEV)
    merged = collections.Counter()
    for d in out.values():
        for k, c in d.items():
            merged[k] += c
    assert sum(merged.values()) == 150
    assert merged[struct.pack("<q", 3)] == 10


def test_wordfreq_shuffle_gpu_two_ranks():
    """wordfreq with combiner=False on the device engine, 2 ranks: every
    word's count equals collections.Counter, top-10 too"""
    from test_distributed_cpu import _check_wordfreq_shuffle
    _check_wordfreq_shuffle(run_world("case_wordfreq_shuffle", 2, DEV))


def test_inverted_index_gpu_two_ranks():
    out = run_world("case_inverted_index", 2, DEV)
    got, ref = {}, collections.defaultdict(list)
    for g_r, ref_r in out.values():
        assert not (set(got) & set(g_r))
        got.update(g_r)
        for k, v in ref_r.items():
            ref[k].extend(v)
    assert {k: sorted(v) for k, v in got.items()} == {k: sorted(v) for k, v in ref.items()}


def test_pagerank_gpu_two_ranks():
    from gpu_mapreduce_amd.models.pagerank import reference_pagerank
    out = run_world("case_pagerank", 2, DEV)
    edges = np.concatenate([out[r][0] for r in range(2)])
    ref = reference_pagerank(edges, 1 << 9, iters=12)
    got = np.zeros(1 << 9)
    for r in range(2):
        got[out[r][1]] = out[r][2]
    np.testing.assert_allclose(got, ref, rtol=2e-4, atol=1e-9)


def test_shuffle_is_deterministic_gpu():
    out = run_world("case_shuffle_determinism", 2, DEV)
    assert all(same for same, _, _ in out.values()), out
    assert sum(n for _, n, _ in out.values()) == 2 * 3000
    assert sum(u for _, _, u in out.values()) == 211


@pytest.mark.parametrize("overlap", ["1", "0"])
@pytest.mark.parametrize("world", [2, 3])
def test_pagerank_replicated_plan_gpu(world, overlap, monkeypatch):
    """the multi-GPU PageRank plan (destination-owned edges, all-gathered c,
    sigma-mixed vertex owners) against the float64 oracle; R-MAT in-edges
    spread evenly over the ranks. overlap 1 (the default): edges cut by source
    rank into pieces with their own XCD ranges, the c slices go round a ring
    on a side stream while the pieces already in are gathered; 0: XCD ranges
    on the interleaved order, one all-gather after the tile step"""
    from gpu_mapreduce_amd.models.pagerank import reference_pagerank
    monkeypatch.setenv("MRH_PR_OVERLAP", overlap)
    out = run_world("case_pagerank_ranges", world, DEV)
    edges = np.concatenate([out[r][0] for r in range(world)])
    ref = reference_pagerank(edges, 1 << 14, iters=15)
    got = np.full(1 << 14, np.nan)
    for r in range(world):
        _, ids, rk, layout, nranges, _, overlapped, cbytes, S = out[r]
        assert layout == "replicated"
        assert nranges > 9  # several layers of 8 ranges + the cold range
        assert overlapped == (overlap == "1")
        assert cbytes == (world - 1) * S * 4 + 16
        got[ids] = rk
    assert not np.isnan(got).any()  # every vertex owned exactly once
    np.testing.assert_allclose(got, ref, rtol=2e-4, atol=1e-9)
    ne = [out[r][5] for r in range(world)]
    assert sum(ne) == len(edges)
    assert max(ne) < 1.25 * sum(ne) / world, ne  # v % P would give rank 0 0.76^k of them
