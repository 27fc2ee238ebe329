"""Triangle path (models/triangles.py, csrc/kernels/tri.hip) vs brute force,
CPU engine vs HIP kernels, and the OINK tri_find command on it."""
import numpy as np
import pytest
import torch

from gpu_mapreduce_amd import C
from gpu_mapreduce_amd.models.pagerank import GRAPH500
from gpu_mapreduce_amd.models.triangles import TriangleGraph, brute_force_count
from gpu_mapreduce_amd.parallel.comm import Comm


def _rmat(scale, ef, seed, dev="cpu"):
    kv = C.map_rmat((1 << scale) * ef, scale, *GRAPH500, 0.0, seed, 0, dev)
    return kv.kdata.view(torch.int64).view(-1, 2)


def _brute_list(e):
    e = np.asarray(e)
    lo, hi = np.minimum(e[:, 0], e[:, 1]), np.maximum(e[:, 0], e[:, 1])
    k = lo != hi
    adj = {}
    for a, b in zip(lo[k], hi[k]):
        adj.setdefault(a, set()).add(b)
        adj.setdefault(b, set()).add(a)
    out = set()
    for a in adj:
        for b in adj[a]:
            if b > a:
                for c in adj[a] & adj[b]:
                    if c > b:
                        out.add((a, b, c))
    return out


@pytest.mark.parametrize("scale,ef,seed", [(6, 4, 1), (8, 8, 2), (9, 16, 3)])
def test_count_and_list_cpu(scale, ef, seed):
    e = _rmat(scale, ef, seed)
    g = TriangleGraph(Comm(device="cpu"), e)
    want = _brute_list(e.numpy())
    assert g.count() == len(want) == brute_force_count(e.numpy())
    got = {tuple(r) for r in g.triangles().tolist()}
    assert got == want


def test_empty_and_tiny():
    c = Comm(device="cpu")
    assert TriangleGraph(c, torch.zeros((0, 2), dtype=torch.int64)).count() == 0
    k4 = torch.tensor([[0, 1], [1, 2], [2, 0], [3, 0], [3, 1], [3, 2], [2, 2], [1, 0]])
    assert TriangleGraph(c, k4).count() == 4


def _oink_tri(tmp_path, comm=None, scale=9):
    import io
    from gpu_mapreduce_amd.oink.interp import OINK
    out = io.StringIO()
    OINK(comm, screen=out, logfile="none").file(text=(
        f"rmat {scale} 8 0.57 0.19 0.19 0.05 0.0 11 -o NULL mre\n"
        "edge_upper -i mre -o NULL mre\n"     # the MR pipeline needs upper-triangular input (examples/in.tri)
        f"tri_find -i mre -o {tmp_path}/tmp.fast NULL\n"
        f"tri_find_mr -i mre -o {tmp_path}/tmp.mr NULL\n"))
    return [ln for ln in out.getvalue().splitlines() if ln.startswith("Tri_find")]


def _tri_files(tmp_path, stem):
    import glob
    return {tuple(sorted(map(int, ln.split()))) for f in glob.glob(str(tmp_path / f"{stem}.*")) for ln in open(f)}


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_oink_tri_find_matches_mapreduce_pipeline(tmp_path, dev):
    """tri_find_mr (the reference's 4-shuffle pipeline, callbacks as the
    trimr kernels on cuda / their host twins on cpu) lists exactly the
    triangles of tri_find (oriented CSR + LDS-hash kernels)"""
    msgs = _oink_tri(tmp_path, Comm(device=dev), scale=9 if dev == "cpu" else 12)
    assert len(msgs) == 2 and msgs[0] == msgs[1]
    fast, mr = _tri_files(tmp_path, "tmp.fast"), _tri_files(tmp_path, "tmp.mr")
    assert fast == mr and len(fast) == int(msgs[0].split()[1]) > 0


def case_oink_tri_mr(comm):
    import tempfile
    import pathlib
    d = pathlib.Path(tempfile.mkdtemp(prefix=f"trimr{comm.rank}_"))
    msgs = _oink_tri(d, comm)
    return msgs, sorted(_tri_files(d, "tmp.fast")), sorted(_tri_files(d, "tmp.mr"))


def test_oink_tri_find_mr_distributed():
    """3 ranks: every rank's share of the MR pipeline's triangles, unioned,
    equals tri_find's and the single-rank brute force"""
    from test_distributed_cpu import run_world
    out = run_world("test_triangles:case_oink_tri_mr", 3)
    fast, mr = set(), set()
    msgs = out[0][0]  # rank 0 writes the screen
    assert len(msgs) == 2 and msgs[0] == msgs[1]
    for _, f, m in out.values():
        assert not (mr & set(map(tuple, m)))
        fast |= set(map(tuple, f))
        mr |= set(map(tuple, m))
    assert fast == mr and len(mr) == int(msgs[0].split()[1]) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("scale,ef", [(10, 16), (16, 16)])
def test_gpu_matches_cpu(scale, ef):
    e = _rmat(scale, ef, 5)
    cpu = TriangleGraph(Comm(device="cpu"), e)
    gpu = TriangleGraph(Comm(device="cuda"), e.cuda())
    assert gpu.count() == cpu.count()
    assert torch.equal(gpu.okeys.cpu(), cpu.okeys) and torch.equal(gpu.rowptr.cpu(), cpu.rowptr)
    if scale <= 10:
        a = gpu.triangles().cpu()
        b = cpu.triangles()
        a = a[np.lexsort(a.numpy().T[::-1])]
        b = b[np.lexsort(b.numpy().T[::-1])]
        assert torch.equal(a, b)


def case_tri_distributed(comm):
    """each rank holds a slice of the edges; the distributed graph (owned rows
    + halo) must count and list exactly the replicated graph's triangles"""
    import os
    e = _rmat(11, 8, 7)
    mine = e[comm.rank::comm.size]
    g = TriangleGraph(comm, mine)
    os.environ["MRH_TRI_REPLICATED"] = "1"
    r = TriangleGraph(comm, mine)
    os.environ.pop("MRH_TRI_REPLICATED")
    return (g.count(), r.count(), g._g.distributed, g._g.nrows, g.nvert, g._g.okeys.numel(),
            [tuple(t) for t in g.triangles().tolist()])


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_triangles_match_replicated(world):
    from test_distributed_cpu import run_world
    out = run_world("test_triangles:case_tri_distributed", world)
    want = _brute_list(_rmat(11, 8, 7).numpy())
    tris = set()
    owned_edges = 0
    for r, (cnt, rcnt, dist, nrows, nvert, nown, lst) in out.items():
        assert dist and cnt == rcnt == len(want)
        assert nrows < nvert, "a rank must not hold every vertex's row"
        owned_edges += nown
        assert not (tris & set(lst)), "a triangle listed on two ranks"
        tris |= set(lst)
    assert tris == want


def case_tri_split(comm):
    """the split build (sample-sorted dedup, allreduced degrees and d+, rows
    split by work, column arrays all-gathered): the whole CSR on every rank,
    equal to the one-rank build; each rank counts / lists its rows only"""
    import os
    e = _rmat(11, 8, 7)
    mine = e[comm.rank::comm.size]
    os.environ["MRH_TRI_BUILD"] = "split"
    try:
        # on a device engine with nvert given: the one-pass device edge pack
        g = TriangleGraph(comm, mine, (1 << 11) if comm.is_cuda else None)
    finally:
        os.environ.pop("MRH_TRI_BUILD")
    return (g.count(), g._g.split, g._g.u0, g._g.u1, g.rowptr.cpu().numpy().copy(), g.col.cpu().numpy().copy(),
            g.perm.cpu().numpy().copy(), [tuple(t) for t in g.triangles().tolist()])


def _check_split(world, device):
    import numpy as np
    from test_distributed_cpu import run_world
    import gpu_mapreduce_amd as gm
    out = run_world("test_triangles:case_tri_split", world, device)
    e = _rmat(11, 8, 7)
    one = TriangleGraph(gm.Comm(device="cpu"), e, (1 << 11) if device.startswith("cuda") else None)
    want = _brute_list(e.numpy())
    tris, rows = set(), []
    for r in range(world):
        cnt, split, u0, u1, rowptr, col, perm, lst = out[r]
        assert split and cnt == len(want) == one.count()
        np.testing.assert_array_equal(rowptr, one.rowptr.numpy())
        np.testing.assert_array_equal(col, one.col.numpy())
        np.testing.assert_array_equal(perm, one.perm.numpy())
        rows.append((u0, u1))
        assert not (tris & set(lst)), "a triangle listed on two ranks"
        tris |= set(lst)
    assert tris == want
    assert rows[0][0] == 0 and rows[-1][1] == one.nvert
    assert all(rows[i][1] == rows[i + 1][0] for i in range(world - 1))


@pytest.mark.parametrize("world", [2, 3])
def test_split_build_matches_single_rank(world):
    _check_split(world, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_split_build_gpu_matches_single_rank(world):
    """the split build on the device engine (ranks sharing the box's GPU over
    the gloo transport): device pack, exchanges, dedup, degrees, d+, CSR"""
    _check_split(world, "cuda:0")


TRI_HUB_CHILD = r'''
import sys, torch
from gpu_mapreduce_amd import Comm, C
from gpu_mapreduce_amd.models.triangles import TriangleGraph
from tests.test_triangles import _rmat
e = _rmat(17, 16, 3)
gpu = TriangleGraph(Comm(device="cuda"), e.cuda())
print(C.tri_hub_size(gpu.nvert), gpu.count())
'''


@pytest.mark.gpu
def test_gpu_hub_bitmap_split_matches_cpu():
    """the same RMAT-17 count with the hub bitmap path off (hash kernels
    only), on the default (nvert/32 ~ 4096 hubs), 4096 hubs, and 65536 (half
    of the graph in bitmaps), and with the top 1024 / 8192 / all 8192 hubs as
    the dense int8 GEMM core — each must equal the CPU merge count"""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    want = TriangleGraph(Comm(device="cpu"), _rmat(17, 16, 3)).count()
    for hub, K, core, kern in (("0", 0, None, None), (None, 4096, None, None), ("4096", 4096, None, None),
                               ("65536", 65536, None, None), ("4096", 4096, "1024", None),
                               ("65536", 65536, "8192", None), ("8192", 8192, "8192", None),
                               (None, 4096, None, "pull"), ("65536", 65536, None, "pull"),
                               ("65536", 65536, None, "lds")):
        env = dict(os.environ, PYTHONPATH=root)
        env.pop("MRH_TRI_HUB", None)
        env.pop("MRH_TRI_CORE", None)
        env.pop("MRH_TRI_HUB_KERNEL", None)
        if kern is not None:  # hub rows by the v-major pull / LDS-bitmap kernels instead of the bitmap kernel
            env["MRH_TRI_HUB_KERNEL"] = kern
        if hub is not None:
            env["MRH_TRI_HUB"] = hub
        if core is not None:  # the top ranks of the hubs counted by the int8 GEMM
            env["MRH_TRI_CORE"] = core
        r = subprocess.run([sys.executable, "-c", TRI_HUB_CHILD], env=env, cwd=root, capture_output=True, text=True,
                           timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        k, n = map(int, r.stdout.split())
        assert (k == K if hub is not None else 0 < k <= K and k % 64 == 0) and n == want, (hub, core, kern, k, n, want)


@pytest.mark.gpu
def test_gpu_fast_build_with_nvert_matches_cpu():
    """nvert given on one GPU: the one-pass pack (self loops packed as edge
    (0, 0), dropped after the dedup) must build the CPU path's CSR; an id
    outside [0, nvert) is an error, not an out-of-bounds write"""
    e = _rmat(12, 16, 9)
    cpu = TriangleGraph(Comm(device="cpu"), e, 1 << 12)
    gpu = TriangleGraph(Comm(device="cuda"), e.cuda(), 1 << 12)
    assert gpu.count() == cpu.count()
    assert torch.equal(gpu.okeys.cpu(), cpu.okeys) and torch.equal(gpu.rowptr.cpu(), cpu.rowptr)
    with pytest.raises(RuntimeError, match="outside"):
        TriangleGraph(Comm(device="cuda"), e.cuda(), 100)


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_tri_find_mr_pipeline_in_memory_and_out_of_core(dev, tmp_path):
    """the reference's 4-collate pipeline (edge_upper first) on raw R-MAT
    edges: the triangle count equals the brute-force oracle in memory and
    under an HBM budget of ~1/50 of the wedge pairs (spooled collates and
    reduces), with every stage timed"""
    from gpu_mapreduce_amd.models.triangles import tri_find_mr
    import gpu_mapreduce_amd as gm
    e = _rmat(9, 8, 5)
    want = brute_force_count(e.numpy())
    comm = gm.Comm(device=dev)
    r = tri_find_mr(comm, e)
    assert r["triangles"] == want
    ops = [s["op"] for s in r["stages"]]
    assert ops[:3] == ["map edge_upper", "collate 0", "reduce cull"] and ops[-1] == "reduce emit_triangles"
    wedges = next(s["pairs_out"] for s in r["stages"] if s["op"] == "reduce nsq_angles")
    r2 = tri_find_mr(comm, e, hbm_budget=max(4096, wedges * 24 // 50), host_budget=wedges * 24 // 8,
                     fpath=str(tmp_path), memsize=-65536)
    assert r2["triangles"] == want
    assert r2["spool_host_bytes"] > 0


def case_tri_mr_ooc(comm):
    """every rank maps its share of one R-MAT edge list; tri_find_mr in
    memory and under HBM / host budgets (spooled shuffles, collates and
    reduces at every rank, collective out-of-core decisions)"""
    import tempfile
    from gpu_mapreduce_amd.models.triangles import tri_find_mr
    e = _rmat(9, 8, 7)
    P, me = comm.size, comm.rank
    mine = e[me * e.shape[0] // P:(me + 1) * e.shape[0] // P]
    r = tri_find_mr(comm, mine)
    wedges = comm.allreduce(next(s["pairs_out"] for s in r["stages"] if s["op"] == "reduce nsq_angles"), "max")
    d = tempfile.mkdtemp(prefix=f"trimr_ooc{me}_")
    r2 = tri_find_mr(comm, mine, hbm_budget=max(4096, wedges * 24 // 50), host_budget=wedges * 24 // 16, fpath=d,
                     memsize=-65536)
    return r["triangles"], r2["triangles"], r2["spool_host_bytes"] + r2["spool_disk_bytes"], brute_force_count(e.numpy())


def test_tri_find_mr_out_of_core_three_ranks():
    """3 gloo ranks: the 4-collate pipeline gives the brute-force count in
    memory and out of core (no rank waits on a collective another skipped)"""
    from test_distributed_cpu import run_world
    out = run_world("test_triangles:case_tri_mr_ooc", 3)
    for a, b, spooled, want in out.values():
        assert a == b == want
    assert sum(v[2] for v in out.values()) > 0


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_tri_find_mr_leaves_edge_mr_unchanged(dev):
    """advisor r4: the edge MR tri_find_mr reads (a named OINK object) keeps
    its pairs and its NULL values (reference oink/tri_find.cpp:71 adds it
    unchanged); upper edges are marked by their first vertex in a temporary
    MR, non-upper input falls back to empty-value markers with the same count"""
    from gpu_mapreduce_amd.models.triangles import tri_find_mr
    import gpu_mapreduce_amd as gm
    e = _rmat(8, 8, 3)
    want = brute_force_count(e.numpy())
    comm = gm.Comm(device=dev)
    u = torch.unique(torch.sort(e, dim=1).values[e[:, 0] != e[:, 1]], dim=0)  # upper, no self-loops, no dups
    r = tri_find_mr(comm, u, upper=False)
    assert r["triangles"] == want
    assert r["input_value_width_after"] == 0 and r["input_pairs_after"] == u.shape[0]
    # non-upper rows (each edge as (vj, vi), vj > vi): edges carry the empty
    # value marker; wedge keys are (min, max) as in the reference
    # (oink/tri_find.cpp:219-227), so no such edge closes a wedge — the
    # reference counts 0 on this input too (its scripts run edge_upper first)
    r2 = tri_find_mr(comm, torch.flip(u, dims=[1]).contiguous(), upper=False)
    assert r2["input_value_width_after"] == 0 and r2["triangles"] == 0
