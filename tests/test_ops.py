"""gpu_mapreduce_amd.ops: the typed kernel entry points.

Each op runs on the CPU engine and (gpu-marked) on the gfx950 kernels and is
compared with an oracle computed outside the engine (numpy cumsum, Python
stable sort, str.split, a regex URL scan, numpy per-segment reductions,
itertools.combinations). The argument checks are tested too: a wrong dtype,
mixed devices or an out-of-range count must raise on the host instead of
reaching a kernel.
"""
import itertools
import re

import numpy as np
import pytest
import torch

from gpu_mapreduce_amd import C, ops

DEVS = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _col(data, off, w, n):
    d = bytes(data.cpu().numpy())
    if w >= 0:
        return [d[i * w:(i + 1) * w] for i in range(n)]
    o = off.cpu().tolist()
    return [d[o[i]:o[i + 1]] for i in range(n)]


def _padded(text: bytes, dev):
    buf = torch.zeros(len(text) + 64, dtype=torch.uint8)
    buf[:len(text)] = torch.frombuffer(bytearray(text), dtype=torch.uint8)
    return buf.to(dev)


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("dtype", [torch.int32, torch.int64])
def test_exclusive_scan_vs_cumsum(dev, dtype):
    x = torch.randint(0, 1000, (100_003,), dtype=dtype)
    got = ops.exclusive_scan(x.to(dev)).cpu().numpy()
    ref = np.concatenate([[0], np.cumsum(x.numpy().astype(np.int64))])
    assert got.dtype == np.int64 and np.array_equal(got, ref)


@pytest.mark.parametrize("dev", DEVS)
def test_radix_sort_pairs_is_stable(dev):
    g = torch.Generator().manual_seed(3)
    k = torch.randint(0, 1 << 20, (50_000,), generator=g, dtype=torch.int64)
    v = torch.arange(k.numel(), dtype=torch.int32)
    ks, vs, _ = ops.radix_sort_pairs(k.to(dev), v.to(dev), 0, 24)
    order = sorted(range(k.numel()), key=lambda i: int(k[i]))  # Python sort is stable
    assert ks.cpu().tolist() == [int(k[i]) for i in order]
    assert vs.cpu().tolist() == order


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("n", [1, 8191, 8192, 300_001])
def test_radix_sort_keys_vs_sorted(dev, n):
    # keys-only sort (8192-key tiles on the GPU): stable on the sorted bits,
    # the bits below ride along as payload
    g = torch.Generator().manual_seed(n)
    k = torch.randint(0, 1 << 62, (n,), generator=g, dtype=torch.int64)
    k = (k & ((1 << 21) - 1)) << 32 | torch.arange(n, dtype=torch.int64)
    got = C.radix_sort_keys(k.to(dev), 32, 53, False).cpu()
    ref = sorted(k.tolist(), key=lambda x: x >> 32)  # Python sort is stable
    assert got.tolist() == ref


@pytest.mark.parametrize("dev", DEVS)
def test_tokenize_vs_str_split(dev):
    rng = np.random.default_rng(5)
    words = ["w%d" % i for i in rng.integers(0, 500, 4000)]
    seps = [" ", "\n", "\t", "  "]
    text = "".join(w + seps[i % 4] for i, w in enumerate(words)).encode()
    kv = ops.tokenize(_padded(text, dev), len(text))
    got = [k.rstrip(b"\0").decode() for k in _col(kv.kdata, kv.koff, kv.kw, kv.n)]
    assert got == text.decode().split()


@pytest.mark.parametrize("dev", DEVS)
def test_scan_urls_vs_regex(dev):
    parts = []
    for i in range(300):
        parts.append(f'<p>x</p><a href="http://site{i % 17}.example/p{i}">t</a> ')
        if i % 5 == 0:
            parts.append('<a name="z">')
    text = "".join(parts).encode()
    kv = ops.scan_urls(_padded(text, dev), len(text), 42)
    got = [k.rstrip(b"\0") for k in _col(kv.kdata, kv.koff, kv.kw, kv.n)]
    assert got == re.findall(rb'<a href="([^"]*)"', text)
    assert set(np.frombuffer(bytes(kv.vdata.cpu().numpy()), dtype=np.int32).tolist()) == {42}


def _plan_case(dev, dtype=torch.float64):
    g = torch.Generator().manual_seed(9)
    ng, nx = 200, 1000
    deg = torch.randint(1, 12, (ng,), generator=g)
    seg = torch.cat([torch.zeros(1, dtype=torch.int64), deg.cumsum(0)])
    src = torch.randint(0, nx, (int(seg[-1]),), generator=g, dtype=torch.int32)
    x = torch.rand(nx, generator=g, dtype=torch.float64).to(dtype)
    w = torch.rand(src.numel(), generator=g, dtype=torch.float64).to(dtype)
    return seg.to(dev), src.to(dev), x.to(dev), w.to(dev)


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("op", [0, 1, 2])
def test_plan_gather_reduce_vs_numpy(dev, op):
    seg, src, x, w = _plan_case(dev)
    out = torch.empty(seg.numel() - 1, dtype=x.dtype, device=dev)
    ops.plan_gather_reduce(seg, src, x, w, op, out)
    terms = (x.cpu().numpy()[src.cpu().numpy()] + w.cpu().numpy())
    uf = [np.add, np.minimum, np.maximum][op]
    ref = uf.reduceat(terms, seg.cpu().numpy()[:-1])
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-12)


@pytest.mark.parametrize("dev", DEVS)
def test_plan_combine_vs_numpy(dev):
    g = torch.Generator().manual_seed(4)
    ng = 64
    deg = torch.randint(1, 6, (ng,), generator=g)
    seg = torch.cat([torch.zeros(1, dtype=torch.int64), deg.cumsum(0)])
    nr = int(seg[-1])
    perm = torch.randperm(nr, generator=g).to(torch.int32)
    recv = torch.rand(nr, generator=g, dtype=torch.float64)
    vid = torch.randperm(ng + 10, generator=g)[:ng].to(torch.int32)
    acc = torch.full((ng + 10,), -1.0, dtype=torch.float64)
    accd = acc.to(dev)
    ops.plan_combine(seg.to(dev), perm.to(dev), recv.to(dev), vid.to(dev), 2, accd)
    ref = acc.numpy().copy()
    ref[vid.numpy()] = np.maximum.reduceat(recv.numpy()[perm.numpy()], seg.numpy()[:-1])
    np.testing.assert_array_equal(accd.cpu().numpy(), ref)


@pytest.mark.parametrize("dev", DEVS)
def test_wedges_vs_combinations(dev):
    seg = torch.tensor([0, 3, 3, 4, 8], dtype=torch.int64)
    nb = torch.tensor([5, 1, 9, 7, 2, 8, 3, 6], dtype=torch.int64)
    centre = torch.tensor([10, 11, 12, 13], dtype=torch.int64)
    e, c = ops.wedges(seg.to(dev), nb.to(dev), centre.to(dev))
    got = sorted(zip(map(tuple, e.cpu().tolist()), c.cpu().tolist()))
    ref = []
    for gi in range(4):
        for a, b in itertools.combinations(nb[seg[gi]:seg[gi + 1]].tolist(), 2):
            ref.append(((min(a, b), max(a, b)), int(centre[gi])))
    assert got == sorted(ref)


@pytest.mark.parametrize("dev", DEVS)
def test_wedge_chunks_concatenate_to_wedges(dev):
    # bounded emission (tri_find_mr under a page budget): the chunks, in
    # order, are the one-shot wedge set, whatever the chunk size and however
    # many groups have no wedge (degree 0/1)
    g = torch.Generator().manual_seed(11)
    deg = torch.randint(0, 4, (300,), generator=g)
    deg[[5, 120, 299]] = torch.tensor([40, 1, 25])
    seg = torch.cat([torch.zeros(1, dtype=torch.int64), deg.cumsum(0)]).to(dev)
    nb = torch.randint(0, 1 << 40, (int(deg.sum()),), generator=g).to(dev)
    centre = torch.arange(300, dtype=torch.int64).to(dev) + 7
    e, c = C.wedges(seg, nb, centre)
    for step in (1, 7, 64, 1000, 0):
        parts = C.wedge_chunks(seg, nb, centre, step)
        if step:
            assert all(p[1].numel() <= step for p in parts)
        assert torch.equal(torch.cat([p[0] for p in parts]), e)
        assert torch.equal(torch.cat([p[1] for p in parts]), c)


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 70_001])
def test_segments_from_head_bitmap(dev, n):
    # the PageRank plan's unpack emits segment heads as a bitmap (bit i of
    # int32 word i / 32); its segments are the head positions + n
    g = torch.Generator().manual_seed(n)
    heads = torch.rand(n, generator=g) < 0.2
    heads[0] = True
    nw = (n + 63) // 64 * 2 + 3  # padded like the gather's index (words past n zero)
    bits = np.zeros(nw * 32, dtype=np.uint8)
    bits[:n] = heads.numpy()
    words = np.packbits(bits.reshape(-1, 32)[:, ::-1], axis=1).view(">u4").astype(np.uint32).reshape(-1)
    H = torch.from_numpy(words.view(np.int32).copy()).to(dev)
    seg = C.segments_from_bits(H, n).cpu().numpy()
    assert np.array_equal(seg, np.concatenate([np.flatnonzero(heads.numpy()), [n]]))


@pytest.mark.parametrize("dev", DEVS)
def test_segments_sorted_vs_numpy(dev):
    k = torch.sort(torch.randint(0, 50, (3000,), dtype=torch.int64)).values
    seg = ops.segments_sorted(k.to(dev)).cpu().numpy()
    kn = k.numpy()
    starts = np.flatnonzero(np.concatenate([[True], kn[1:] != kn[:-1]]))
    assert np.array_equal(seg, np.concatenate([starts, [kn.size]]))


# ------------------------------------------------------------- argument checks (host-side, before any launch)
def test_checks_reject_bad_operands():
    k = torch.zeros(8, dtype=torch.int64)
    with pytest.raises(TypeError, match="vals"):
        ops.radix_sort_pairs(k, torch.zeros(8, dtype=torch.int64))
    with pytest.raises(ValueError, match="8 keys"):
        ops.radix_sort_pairs(k, torch.zeros(7, dtype=torch.int32))
    with pytest.raises(ValueError, match="bit range"):
        ops.radix_sort_pairs(k, torch.zeros(8, dtype=torch.int32), 0, 65)
    with pytest.raises(TypeError, match="x: dtype"):
        ops.exclusive_scan(torch.zeros(4))
    with pytest.raises(ValueError, match="padded"):
        ops.tokenize(torch.zeros(40, dtype=torch.uint8), 20)
    with pytest.raises(TypeError, match="text"):
        ops.scan_urls(torch.zeros(100, dtype=torch.int32), 10, 0)
    with pytest.raises(ValueError, match="sort flag"):
        ops.sort_kv(None, 7)
    with pytest.raises(ValueError, match="op 'median'"):
        ops.segmented_reduce(None, "median")
    with pytest.raises(ValueError, match="nprocs"):
        ops.partition_dest(None, 0)
    with pytest.raises(ValueError, match="sum to 1"):
        ops.rmat_edges(10, 10, 0.5, 0.5, 0.5, 0.5, 0.0, 1, 0, "cpu")
    seg, src, x, w = _plan_case("cpu")
    out = torch.empty(seg.numel() - 1, dtype=x.dtype)
    with pytest.raises(TypeError, match="src"):
        ops.plan_gather_reduce(seg, src.long(), x, w, 0, out)
    with pytest.raises(ValueError, match="w: "):
        ops.plan_gather_reduce(seg, src, x, w[:-1], 0, out)
    with pytest.raises(ValueError, match="out"):
        ops.plan_gather_reduce(seg, src, x, w, 0, out[:-1])
    with pytest.raises(ValueError, match="centre"):
        ops.wedges(torch.tensor([0, 2, 4]), torch.arange(4), torch.arange(1))


def test_native_entry_points_check_operands():
    """The native layer refuses mismatched operands on its own (the raw C.* calls)."""
    from gpu_mapreduce_amd import C
    k = torch.zeros(8, dtype=torch.int64)
    with pytest.raises(RuntimeError, match="one int32 value per key"):
        C.radix_sort_pairs(k, torch.zeros(4, dtype=torch.int32), 0, 64)
    seg, src, x, w = _plan_case("cpu")
    out = torch.empty(seg.numel() - 1, dtype=x.dtype)
    with pytest.raises(RuntimeError, match="plan_gather_reduce src"):
        C.plan_gather_reduce(seg, src.long(), x, w, 0, out)
    with pytest.raises(RuntimeError, match="plan_gather_reduce seg"):
        C.plan_gather_reduce(seg.int(), src, x, w, 0, out)
    with pytest.raises(RuntimeError, match="wedges neighbours"):
        C.wedges(torch.tensor([0, 2]), torch.arange(2, dtype=torch.int32), torch.arange(1))


@pytest.mark.gpu
def test_checks_reject_mixed_devices():
    k = torch.zeros(8, dtype=torch.int64, device="cuda")
    with pytest.raises(ValueError, match="vals: on cpu"):
        ops.radix_sort_pairs(k, torch.zeros(8, dtype=torch.int32))
    from gpu_mapreduce_amd import C
    with pytest.raises(RuntimeError, match="one int32 value per key"):
        C.radix_sort_pairs(k, torch.zeros(8, dtype=torch.int32), 0, 64)
