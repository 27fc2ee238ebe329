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


PB_CHILD = r"""
import sys, numpy as np, torch
import gpu_mapreduce_amd as g
from gpu_mapreduce_amd.models.pagerank import PageRank, rmat_map
comm = g.Comm(device="cuda")
mr = g.MapReduce(comm)
rmat_map(mr, 20, 16, seed=3)
edges = mr.kv.kdata.view(torch.int64).view(-1, 2).cpu().numpy().copy()
pr = PageRank(mr, 1 << 20).build()
pr.run(15)
ids, r = pr.ranks()
out = np.zeros(1 << 20)
out[ids.cpu().numpy()] = r.cpu().numpy()
np.save(sys.argv[1], out)
if sys.argv[2] == "1":
    from gpu_mapreduce_amd.models.pagerank import reference_pagerank
    np.testing.assert_allclose(out, reference_pagerank(edges, 1 << 20, iters=15), rtol=2e-4, atol=1e-9)
print(int(pr.blocking))
"""


@pytest.mark.gpu
def test_pagerank_blocking_matches_pull_and_numpy(tmp_path):
    """RMAT-20 (64 destination bins, hub bins split over several slices):
    the propagation-blocked iteration and the pull iteration
    (MRH_PR_BLOCKING=0, the default) agree with each other and with the
    float64 oracle"""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for flag in ("1", "0"):
        env = dict(os.environ, MRH_PR_BLOCKING=flag, PYTHONPATH=root)  # "0" = the default pull path
        path = str(tmp_path / f"r{flag}.npy")
        p = subprocess.run([sys.executable, "-c", PB_CHILD, path, flag], env=env, cwd=root, capture_output=True,
                           text=True, timeout=240)
        assert p.returncode == 0, p.stderr[-2000:]
        assert p.stdout.strip() == flag
        res[flag] = np.load(path)
    np.testing.assert_allclose(res["1"], res["0"], rtol=1e-4, atol=1e-10)


XCD_CHILD = r"""
import sys, numpy as np, torch
import gpu_mapreduce_amd as g
from gpu_mapreduce_amd.models.pagerank import PageRank, rmat_map, reference_pagerank
comm = g.Comm(device="cuda")
mr = g.MapReduce(comm)
rmat_map(mr, 18, 16, seed=7)
edges = mr.kv.kdata.view(torch.int64).view(-1, 2).cpu().numpy().copy()
pr = PageRank(mr, 1 << 18).build()
pr.run(15)
ids, r = pr.ranks()
out = np.zeros(1 << 18)
out[ids.cpu().numpy()] = r.cpu().numpy()
np.save(sys.argv[1], out)
np.testing.assert_allclose(out, reference_pagerank(edges, 1 << 18, iters=15), rtol=2e-4, atol=1e-9)
print(int(pr.xcd_ranges))
"""


@pytest.mark.gpu
def test_pagerank_xcd_ranges_match_pull_and_numpy(tmp_path):
    """XCD source ranges (graphplan.cpp xcd_ranges): with the L2 size
    lowered so RMAT-18 needs several layers of ranges, the ranged gather +
    tiled combine equals the plain pull iteration (MRH_PR_XCD=0) and the
    float64 oracle"""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for name, extra in (("xcd", {"MRH_PR_L2_BYTES": "65536"}), ("layer1", {"MRH_PR_L2_BYTES": "65536",
                                                                          "MRH_PR_XCD_LAYERS": "1"}),
                        ("pull", {"MRH_PR_XCD": "0"})):
        env = dict(os.environ, PYTHONPATH=root, **extra)
        path = str(tmp_path / f"{name}.npy")
        p = subprocess.run([sys.executable, "-c", XCD_CHILD, path], env=env, cwd=root, capture_output=True,
                           text=True, timeout=240)
        assert p.returncode == 0, p.stderr[-2000:]
        nr = int(p.stdout.strip().splitlines()[-1])
        if name == "pull":
            assert nr == 0
        elif name == "layer1":
            assert nr == 9
        else:
            assert nr > 9  # several layers of 8 ranges + the cold range
        res[name] = np.load(path)
    np.testing.assert_allclose(res["xcd"], res["pull"], rtol=1e-4, atol=1e-10)
    np.testing.assert_allclose(res["layer1"], res["pull"], rtol=1e-4, atol=1e-10)


@pytest.mark.gpu
def test_pagerank_hip_graph_replay_matches_plain_steps():
    """a fixed-count run replays a captured HIP graph of two iterations; the
    ranks must be bitwise those of the plain per-step launches (even and odd
    counts, and again after reset(), which reuses the captured buffers)"""
    import gpu_mapreduce_amd as g
    from gpu_mapreduce_amd.models.pagerank import PageRank, rmat_map
    import os
    mr = g.MapReduce(g.Comm(device="cuda"))
    rmat_map(mr, 18, 16, seed=3)
    os.environ["MRH_PR_L2_BYTES"] = "65536"  # small ranges: RMAT-18 takes the XCD tile-step path
    try:
        pr = PageRank(mr, 1 << 18).build()
    finally:
        os.environ.pop("MRH_PR_L2_BYTES")
    assert pr.xcd_ranges > 0
    for iters in (20, 7):
        pr.use_graph = False
        pr.reset()
        pr.run(iters)
        _, plain = pr.ranks()
        plain = plain.clone()
        before = pr.graph_iterations
        pr.use_graph = True
        for _ in range(2):
            pr.reset()
            pr.run(iters)
            _, got = pr.ranks()
            assert torch.equal(got, plain), iters
        assert pr.graph_iterations - before == 2 * 2 * (iters // 2)


FORCED_CHILD = r"""
import os, sys, numpy as np, torch
import gpu_mapreduce_amd as g
from gpu_mapreduce_amd.models.pagerank import PageRank, rmat_map
os.environ["MRH_PR_L2_BYTES"] = "65536"
comm = g.Comm(device="cuda")
mr = g.MapReduce(comm)
rmat_map(mr, 18, 16, seed=7)
pr = PageRank(mr, 1 << 18).build()
for it in (20, 7):
    pr.reset()
    pr.run(it)
ids, r = pr.ranks()
out = np.zeros(1 << 18, dtype=np.float32)
out[ids.cpu().numpy()] = r.cpu().numpy()
np.save(sys.argv[1], out)
print(pr.graph_iterations)
print(pr.layout, pr.xcd_ranges, comm.native.transport)
"""


@pytest.mark.gpu
def test_pagerank_forced_rccl_replicated_plan_is_bitwise_local(tmp_path):
    """MRH_FORCE_RCCL=1: one rank runs the multi-GPU plan (edges through two
    RCCL exchanges, c refreshed by an in-place all-gather, stats by an
    allreduce every iteration); with sigma = identity at one rank its ranks
    equal the local plan's (HIP-graph replay) bit for bit"""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res, info = {}, {}
    for flag in ("0", "1"):
        env = dict(os.environ, MRH_FORCE_RCCL=flag, PYTHONPATH=root)
        for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
            env.pop(k, None)
        path = str(tmp_path / f"f{flag}.npy")
        p = subprocess.run([sys.executable, "-c", FORCED_CHILD, path], env=env, cwd=root, capture_output=True,
                           text=True, timeout=240)
        assert p.returncode == 0, p.stderr[-3000:]
        info[flag] = p.stdout.split()[-3:]
        res[flag] = np.load(path)
    assert info["0"][0] == "local" and info["0"][2] == "local", info
    assert info["1"][0] == "replicated" and info["1"][2] == "rccl", info
    assert info["0"][1] == info["1"][1] and int(info["1"][1]) > 9, info  # the same XCD ranges
    assert np.array_equal(res["0"], res["1"])


HOT_CHILD = r"""
import sys, numpy as np, torch
import gpu_mapreduce_amd as g
from gpu_mapreduce_amd.models.pagerank import PageRank, rmat_map, reference_pagerank
comm = g.Comm(device="cuda")
mr = g.MapReduce(comm)
rmat_map(mr, 20, 16, seed=5)
edges = mr.kv.kdata.view(torch.int64).view(-1, 2).cpu().numpy().copy()
pr = PageRank(mr, 1 << 20).build()
pr.run(20)
ids, r = pr.ranks()
out = np.zeros(1 << 20)
out[ids.cpu().numpy()] = r.cpu().numpy()
np.save(sys.argv[1], out)
np.testing.assert_allclose(out, reference_pagerank(edges, 1 << 20, iters=20), rtol=2e-4, atol=1e-9)
print("ok")
"""


@pytest.mark.gpu
def test_pagerank_hot_prefix_gather_matches_global_gather(tmp_path):
    """the persistent gather (wavesegred.h k_ws_gather_reduce_hot) keeps the
    rank contributions of the hottest (lowest relabelled) sources in LDS; on
    RMAT-20 (16 M edges, past its 2^22-edge threshold) its ranks equal the
    all-global gather's (MRH_PR_HOT=0, the default) to L1 <= 1e-6, and the
    float64 oracle (opt-in: MRH_PR_HOT=-1 is the full 32 k-float prefix)"""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for name, hot in (("hot", "-1"), ("small", "2048"), ("off", "0")):
        env = dict(os.environ, PYTHONPATH=root, MRH_PR_HOT=hot)
        path = str(tmp_path / f"{name}.npy")
        p = subprocess.run([sys.executable, "-c", HOT_CHILD, path], env=env, cwd=root, capture_output=True,
                           text=True, timeout=240)
        assert p.returncode == 0, p.stderr[-2000:]
        res[name] = np.load(path)
    assert np.abs(res["hot"] - res["off"]).sum() <= 1e-6
    assert np.abs(res["small"] - res["off"]).sum() <= 1e-6


@pytest.mark.gpu
def test_pagerank_forced_rccl_overlapped_pieces_match_local(tmp_path):
    """MRH_PR_OVERLAP=2 on a forced one-rank RCCL communicator: the multi-GPU
    plan's source chunks (their own XCD ranges, segment indexes and source
    streams), the side-stream exchange rounds (no peers at one rank) and
    their events — the ranks of 27 iterations (a 20-run after reset, then a
    7-run) equal the local plan's to float32 accumulation differences. The
    distributed iteration replays as a HIP graph (side stream, RCCL stream and
    events captured) bit for bit like its eager run (MRH_PR_DIST_GRAPH=0)"""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res, info = {}, {}
    forced = {"MRH_FORCE_RCCL": "1", "MRH_PR_OVERLAP": "2"}
    for name, extra in (("local", {}), ("pieces", forced), ("eager", dict(forced, MRH_PR_DIST_GRAPH="0"))):
        env = dict(os.environ, PYTHONPATH=root, **extra)
        if name == "local":
            env.pop("MRH_FORCE_RCCL", None)
            env.pop("MRH_PR_OVERLAP", None)
        path = str(tmp_path / f"{name}.npy")
        p = subprocess.run([sys.executable, "-c", FORCED_CHILD, path], env=env, cwd=root, capture_output=True,
                           text=True, timeout=240)
        assert p.returncode == 0, p.stderr[-3000:]
        info[name] = p.stdout.split()[-4:]
        res[name] = np.load(path)
    assert info["pieces"][1] == "replicated" and info["pieces"][3] == "rccl", info
    assert int(info["pieces"][2]) > 9, info  # several chunks' ranges
    # 20-run: 2 eager (fresh c, RCCL connections), 18 replayed; 7-run: 1 + 6
    assert int(info["pieces"][0]) == 24 and int(info["eager"][0]) == 0, info
    np.testing.assert_allclose(res["pieces"], res["local"], rtol=1e-4, atol=1e-10)
    assert np.array_equal(res["pieces"], res["eager"])
