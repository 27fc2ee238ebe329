"""GPU numerics of the edge-plan kernels (plan_gather_reduce, plan_combine,
wedges) vs the CPU engine path, and the OINK graph commands run end-to-end on
the HIP engine vs the CPU engine."""
import io

import numpy as np
import pytest
import torch

from gpu_mapreduce_amd import C

pytestmark = pytest.mark.gpu


def _segs(rng, ng, big=True):
    lens = rng.integers(1, 9, ng)
    if big:
        lens[ng // 3] = 200_000        # one hub spanning many value tiles
        lens[ng // 2] = 5_000
    seg = np.zeros(ng + 1, np.int64)
    seg[1:] = np.cumsum(lens)
    return torch.from_numpy(seg)


@pytest.mark.parametrize("dtype", [torch.int64, torch.float32, torch.float64])
@pytest.mark.parametrize("op", [0, 1, 2])
@pytest.mark.parametrize("weighted", [False, True])
def test_plan_gather_reduce(dtype, op, weighted):
    rng = np.random.default_rng(op * 7 + int(weighted))
    ng, nx = 20_000, 50_000
    seg = _segs(rng, ng)
    ne = int(seg[-1])
    src = torch.from_numpy(rng.integers(0, nx, ne).astype(np.int32))
    if dtype == torch.int64:
        x = torch.from_numpy(rng.integers(-1000, 1000, nx))
        w = torch.from_numpy(rng.integers(0, 10, ne)) if weighted else torch.empty(0, dtype=dtype)
    else:
        x = torch.from_numpy(rng.random(nx)).to(dtype)
        w = torch.from_numpy(rng.random(ne)).to(dtype) if weighted else torch.empty(0, dtype=dtype)
    out_c = torch.empty(ng, dtype=dtype)
    C.plan_gather_reduce(seg, src, x, w, op, out_c)
    out_g = torch.empty(ng, dtype=dtype, device="cuda")
    C.plan_gather_reduce(seg.cuda(), src.cuda(), x.cuda(), w.cuda(), op, out_g)
    if dtype == torch.int64 or op != 0:
        assert torch.equal(out_g.cpu(), out_c)
    else:
        ref = torch.zeros(ng, dtype=torch.float64)
        ids = torch.repeat_interleave(torch.arange(ng), seg[1:] - seg[:-1])
        val = x.double()[src.long()] + (w.double() if weighted else 0)
        ref.index_add_(0, ids, val)
        tol = 1e-5 if dtype == torch.float32 else 1e-12
        assert torch.allclose(out_g.cpu().double(), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("dtype", [torch.int64, torch.float64])
@pytest.mark.parametrize("op", [0, 1, 2])
def test_plan_combine(dtype, op):
    rng = np.random.default_rng(11 + op)
    ng = 30_000
    seg = _segs(rng, ng)
    nr = int(seg[-1])
    perm = torch.from_numpy(rng.permutation(nr).astype(np.int32))
    recv = (torch.from_numpy(rng.integers(-50, 50, nr)) if dtype == torch.int64
            else torch.from_numpy(rng.random(nr)))
    vid = torch.from_numpy(rng.permutation(ng).astype(np.int32))
    acc_c = torch.zeros(ng, dtype=dtype)
    C.plan_combine(seg, perm, recv, vid, op, acc_c)
    acc_g = torch.zeros(ng, dtype=dtype, device="cuda")
    C.plan_combine(seg.cuda(), perm.cuda(), recv.cuda(), vid.cuda(), op, acc_g)
    if dtype == torch.int64 or op != 0:
        assert torch.equal(acc_g.cpu(), acc_c)
    else:
        assert torch.allclose(acc_g.cpu(), acc_c, rtol=1e-12, atol=1e-12)


def test_wedges_match_cpu():
    rng = np.random.default_rng(5)
    ng = 3000
    lens = rng.integers(0, 12, ng)
    lens[17] = 700                      # 244,650 wedges from one centre
    seg = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64))
    nb = torch.from_numpy(rng.integers(0, 1 << 40, int(seg[-1])))
    centre = torch.from_numpy(rng.integers(0, 1 << 40, ng))
    ec, cc = C.wedges(seg, nb, centre)
    eg, cg = C.wedges(seg.cuda(), nb.cuda(), centre.cuda())
    assert ec.shape == eg.shape and ec.shape[0] == int((lens * (lens - 1) // 2).sum())
    a = torch.cat([cc[:, None], ec], 1).numpy()
    b = torch.cat([cg[:, None], eg], 1).cpu().numpy()
    assert np.array_equal(a[np.lexsort(a.T[::-1])], b[np.lexsort(b.T[::-1])])


SCRIPT = """rmat 10 8 0.45 0.15 0.15 0.25 0.0 321 -o tmp.rmat mre
edge_upper -i mre -o NULL mre
tri_find -i mre -o tmp.tri NULL
cc_find 0 -i mre -o tmp.cc mrc
cc_stats -i mrc
luby_find 9 -i mre -o tmp.mis NULL
degree 0 -i mre -o tmp.deg NULL
mre map/mr mre add_weight
sssp 2 5 -i mre -o tmp.sssp NULL
"""


def _run(dev, d, monkeypatch):
    from gpu_mapreduce_amd.oink.interp import OINK
    from gpu_mapreduce_amd.parallel.comm import Comm
    monkeypatch.chdir(d)
    out = io.StringIO()
    OINK(Comm(device=dev), screen=out, logfile="none").file(text=SCRIPT)
    files = {}
    for stem in ("tmp.rmat", "tmp.tri", "tmp.cc", "tmp.mis", "tmp.deg", "tmp.sssp"):
        files[stem] = sorted(open(d / f"{stem}.0").read().split("\n"))
    return out.getvalue(), files


def test_oink_graph_gpu_matches_cpu(tmp_path, monkeypatch):
    (tmp_path / "c").mkdir()
    (tmp_path / "g").mkdir()
    tc, fc = _run("cpu", tmp_path / "c", monkeypatch)
    tg, fg = _run("cuda", tmp_path / "g", monkeypatch)
    assert tc == tg
    for k in fc:
        assert fc[k] == fg[k], k
