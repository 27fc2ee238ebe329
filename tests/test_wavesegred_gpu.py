"""Static-segment wave gather-reduce (csrc/kernels/wavesegred.h) vs a plain
PyTorch fp64/int64 reference: segment layouts with long runs crossing many
waves, all-singleton runs, mixed, and sizes that are not a multiple of the
1024-edge wave tile."""
import numpy as np
import pytest
import torch

from gpu_mapreduce_amd._ext import C

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _layout(kind, n, rng):
    if kind == "ones":
        lens = np.ones(n, np.int64)
    elif kind == "hub":
        lens = np.concatenate([[n // 2], np.ones(n - n // 2, np.int64)])
        rng.shuffle(lens)
    elif kind == "long":
        lens = rng.integers(1, 5000, size=max(1, n // 2500))
    else:
        lens = rng.geometric(0.08, size=n // 12 + 1)
    lens = lens[lens > 0]
    seg = np.concatenate([[0], np.cumsum(lens)])
    return seg


def _ref(seg, src, x, w, op):
    v = x[src].astype(np.float64 if x.dtype.kind == "f" else np.int64)
    if w is not None:
        v = v + w
    out = []
    for a, b in zip(seg[:-1], seg[1:]):
        s = v[a:b]
        out.append(s.sum() if op == 0 else s.min() if op == 1 else s.max())
    return np.array(out)


@pytest.mark.parametrize("kind", ["ones", "hub", "long", "mixed"])
@pytest.mark.parametrize("n", [1, 1000, 1024, 70001])
@pytest.mark.parametrize("dtype,op", [(torch.float32, 0), (torch.float64, 1), (torch.int64, 2), (torch.float64, 0)])
def test_ws_gather_reduce(kind, n, dtype, op):
    rng = np.random.default_rng(n + op)
    seg = _layout(kind, n, rng)
    ne = int(seg[-1])
    nx = 5000
    src = rng.integers(0, nx, size=ne).astype(np.int32)
    if dtype == torch.int64:
        x = rng.integers(-10**9, 10**9, size=nx).astype(np.int64)
    else:
        x = rng.standard_normal(nx).astype(np.float32 if dtype == torch.float32 else np.float64)
    w = None
    if op == 1:
        w = rng.standard_normal(ne)
    got = C.seg_gather_reduce(torch.from_numpy(seg).to(DEV), torch.from_numpy(src).to(DEV),
                              torch.from_numpy(x).to(DEV), None if w is None else torch.from_numpy(w).to(DEV), op)
    ref = _ref(seg, src, x, w, op)
    g = got.cpu().numpy()
    if dtype == torch.int64:
        assert np.array_equal(g, ref)
    else:
        tol = 1e-4 if dtype == torch.float32 else 1e-10
        np.testing.assert_allclose(g, ref, rtol=tol, atol=tol * 10)


@pytest.mark.parametrize("kind", ["ones", "hub", "long", "mixed"])
@pytest.mark.parametrize("dtype,op", [(torch.float64, 0), (torch.int64, 2), (torch.int64, 1)])
def test_ws_gather_reduce_two_level_carry(kind, dtype, op):
    """5 M values = 4883 wave tiles: the carry array (2 per tile) is folded in
    two levels (k_carry_fold + k_segred_carry); a hub segment spans half of
    all tiles"""
    n = 5_000_000
    rng = np.random.default_rng(17 + op)
    seg = _layout(kind, n, rng)
    ne = int(seg[-1])
    nx = 100_000
    src = rng.integers(0, nx, size=ne).astype(np.int32)
    if dtype == torch.int64:
        x = rng.integers(-10**9, 10**9, size=nx).astype(np.int64)
    else:
        x = rng.standard_normal(nx)
    got = C.seg_gather_reduce(torch.from_numpy(seg).to(DEV), torch.from_numpy(src).to(DEV),
                              torch.from_numpy(x).to(DEV), None, op).cpu().numpy()
    v = x[src]
    red = {0: np.add, 1: np.minimum, 2: np.maximum}[op]
    ref = red.reduceat(v, seg[:-1])
    if dtype == torch.int64:
        assert np.array_equal(got, ref)
    else:
        np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-9)
