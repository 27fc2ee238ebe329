"""Sort flags +-1..+-4 (int32, uint64, float, double; MR-MPI's sort_keys /
sort_values flags, reference src/mapreduce.cpp:2692-2802) against a numpy
stable-argsort oracle, on the CPU engine and the HIP radix path, with the
awkward values: -0.0 and +0.0 (one key, as the reference's `<` / `>`
comparators see them: ties keep input order), +-inf, NaNs of several payloads
and both signs, denormals, the extremes of each type and many duplicates.

Documented NaN order (the reference's comparators leave it undefined): every
NaN is one key that sorts LAST in both directions, like numpy / pandas; ties
keep input order (the sort is stable)."""

import numpy as np
import pytest
import torch

from gpu_mapreduce_amd import C

SPECIAL_F = [0.0, -0.0, np.inf, -np.inf, np.nan, -np.nan, 1e-45, -1e-45, 1e-40, -1e-40,
             3.4028235e38, -3.4028235e38, 1.0, -1.0, 1.1754944e-38, -1.1754944e-38]
SPECIAL_D = [0.0, -0.0, np.inf, -np.inf, np.nan, -np.nan, 5e-324, -5e-324, 1e-310, -1e-310,
             1.7976931348623157e308, -1.7976931348623157e308, 1.0, -1.0, 2.2250738585072014e-308]


def _values(flag, n, rng):
    f = abs(flag)
    if f == 1:
        base = rng.integers(-50, 50, n).astype(np.int32)
        base[:4] = [np.iinfo(np.int32).min, np.iinfo(np.int32).max, 0, -1]
        return base
    if f == 2:
        base = rng.integers(0, 40, n).astype(np.uint64) * np.uint64(1 << 58)
        base[:4] = [0, np.iinfo(np.uint64).max, 1 << 63, (1 << 63) - 1]
        return base
    dt, spec = (np.float32, SPECIAL_F) if f == 3 else (np.float64, SPECIAL_D)
    v = np.round(rng.standard_normal(n) * 4).astype(dt)  # many duplicates
    pick = rng.integers(0, len(spec), n // 3)
    v[rng.choice(n, n // 3, replace=False)] = np.array(spec, dtype=dt)[pick]
    if f == 3:  # NaNs with other payloads and the sign bit set
        u = v.view(np.uint32)
        u[:3] = [0x7F800001, 0xFFC00123, 0x7FFFFFFF]
    else:
        u = v.view(np.uint64)
        u[:3] = [0x7FF0000000000001, 0xFFF8000000000123, 0x7FFFFFFFFFFFFFFF]
    return v


def _oracle(v, flag):
    idx = np.arange(len(v))
    if v.dtype.kind == "f":
        nan = np.isnan(v)
        nn = idx[~nan]
        key = v[nn] if flag > 0 else -v[nn]    # -(-0.0) == -(+0.0): still one key
        return np.concatenate([nn[np.argsort(key, kind="stable")], idx[nan]])
    if flag > 0:
        return np.argsort(v, kind="stable")
    return np.argsort(~v if v.dtype.kind == "u" else -v.astype(np.int64), kind="stable")


def _sorted_perm(v, flag, dev):
    n = len(v)
    col = torch.from_numpy(np.ascontiguousarray(v).view(np.uint8).copy())
    kv = C.make_kv(col, None, torch.arange(n, dtype=torch.int32).view(torch.uint8), None, n, "cpu")
    out = C.sort_kv(kv.to(dev) if dev != "cpu" else kv, flag, False)
    return out.vdata.cpu().view(torch.int32).numpy().copy()


def _check(flag, dev):
    rng = np.random.default_rng(100 + flag)
    v = _values(flag, 20_000, rng)
    got = _sorted_perm(v, flag, dev)
    want = _oracle(v, flag)
    assert np.array_equal(got, want), (flag, dev, np.flatnonzero(got != want)[:10])


@pytest.mark.parametrize("flag", [1, -1, 2, -2, 3, -3, 4, -4])
def test_sort_flags_numpy_oracle_cpu(flag):
    _check(flag, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("flag", [1, -1, 2, -2, 3, -3, 4, -4])
def test_sort_flags_numpy_oracle_gpu(flag):
    _check(flag, "cuda")


def test_zero_signs_are_one_key():
    """-0.0 and +0.0 group as one key (the reference's comparator sees them
    equal), in input order"""
    v = np.array([0.0, -0.0, 1.0, -0.0, 0.0], dtype=np.float64)
    assert list(_sorted_perm(v, 4, "cpu")) == [0, 1, 3, 4, 2]
    assert list(_sorted_perm(v, -4, "cpu")) == [2, 0, 1, 3, 4]
    f = np.array([np.nan, -np.inf, np.nan, 2.0], dtype=np.float32)
    assert list(_sorted_perm(f, 3, "cpu")) == [1, 3, 0, 2]
    assert list(_sorted_perm(f, -3, "cpu")) == [3, 1, 0, 2]
