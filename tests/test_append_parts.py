"""add / addflag maps are O(appended) (reference
src/keyvalue.cpp:185-209 reopens only the last page, src/mapreduce.cpp:348-374):
the appended pairs stay a separate part of the KV — in HBM, pinned host memory
or a spool file, wherever they were made — and convert / collate on one rank
read every part in place. Every result must equal the flat KV's."""
import collections
import struct

import pytest
import torch

import gpu_mapreduce_amd as g


def _pairs(n, keys, seed, dev):
    gen = torch.Generator().manual_seed(seed)
    k = torch.randint(0, keys, (n, 2), generator=gen, dtype=torch.int64)
    v = torch.randint(0, 1 << 20, (n,), generator=gen, dtype=torch.int64)
    return k.to(dev), v.to(dev)


def _groups(mr):
    out = {}
    for k, vs in mr.kmv_pairs():
        out[struct.unpack("<2q", k)] = sorted(struct.unpack("<q", v)[0] for v in vs)
    return out


def _want(*parts):
    d = collections.defaultdict(list)
    for k, v in parts:
        for (a, b), x in zip(k.cpu().tolist(), v.cpu().tolist()):
            d[(a, b)].append(x)
    return {k: sorted(v) for k, v in d.items()}


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_add_keeps_parts_and_collates_them(dev):
    comm = g.Comm(device=dev)
    a, b = _pairs(30_000, 500, 1, dev), _pairs(7_000, 500, 2, dev)
    mr, other = g.MapReduce(comm), g.MapReduce(comm)
    mr.map(1, lambda i, kv: kv.add_tensors(a[0], a[1]))
    other.map(1, lambda i, kv: kv.add_tensors(b[0], b[1]))
    assert mr.add(other) == 37_000
    assert mr.kv_parts == 2  # nothing concatenated
    assert mr.collate() == len(_want(a, b))
    assert mr.last_convert.exact  # packed pairs read both parts in place
    assert _groups(mr) == _want(a, b)


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_addflag_map_appends_a_part(dev):
    comm = g.Comm(device=dev)
    a, b = _pairs(5_000, 100, 3, dev), _pairs(3_000, 100, 4, dev)
    mr = g.MapReduce(comm)
    mr.map(1, lambda i, kv: kv.add_tensors(a[0], a[1]))
    assert mr.map(1, lambda i, kv: kv.add_tensors(b[0], b[1]), addflag=1) == 8_000
    assert mr.kv_parts == 2
    # an op that does not stream parts sees the flat KV
    kv = mr.kv
    assert kv.n == 8_000 and mr.kv_parts == 1
    assert torch.equal(kv.kdata.view(torch.int64).view(-1, 2).cpu(), torch.cat([a[0], b[0]]).cpu())
    mr.convert()
    assert _groups(mr) == _want(a, b)


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_add_out_of_core_writes_only_the_new_part(dev, tmp_path):
    """under an HBM budget the KV lives on the host / in spool files; add
    writes the appended pairs once (never the pairs already held) and the out
    of core convert reads every part where it lies"""
    comm = g.Comm(device=dev)
    a, b = _pairs(40_000, 2_000, 5, dev), _pairs(10_000, 2_000, 6, dev)
    mr, other = g.MapReduce(comm), g.MapReduce(comm)
    for m in (mr, other):
        m.hbm_budget = 96 << 10
        m.host_budget = 256 << 10
        m.fpath = str(tmp_path)
    mr.map(1, lambda i, kv: kv.add_tensors(a[0], a[1]))
    other.map(1, lambda i, kv: kv.add_tensors(b[0], b[1]))
    before = dict(mr.spool_stats)
    mr.add(other)
    after = dict(mr.spool_stats)
    moved = (after["host_bytes"] - before["host_bytes"]) + (after["disk_bytes"] - before["disk_bytes"])
    assert moved <= 10_000 * 24 + 4096  # at most the appended pairs, once
    assert mr.kv_parts >= 2
    mr.collate()
    assert _groups(mr) == _want(a, b)


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("vbit", [54, 58])
@pytest.mark.parametrize("mixed", [False, True])
def test_packed_pairs_past_64_bits_bucketed(dev, vbit, mixed, monkeypatch):
    """narrow pairs whose key + value bits exceed 64 (R-MAT-22 wedges: 44 +
    22) group in 2^B buckets (B = the excess bits) — exact, every key's values
    in input order, 4- and 8-byte values, given as parts. Up to 2^31 pairs the
    bucket is the top B key bits (keys come out sorted); past that (forced
    here by MRH_PACKED_MIXED=1) the low B bits ^ a mix of the others
    (balanced and invertible)"""
    if mixed:
        monkeypatch.setenv("MRH_PACKED_MIXED", "1")
    else:
        monkeypatch.delenv("MRH_PACKED_MIXED", raising=False)
    gen = torch.Generator().manual_seed(vbit)
    n = 60_000
    k = torch.randint(0, 3000, (n,), generator=gen, dtype=torch.int64)
    k[: n // 3] = 7  # a hot key
    v8 = torch.randint(0, 1 << 20, (n,), generator=gen, dtype=torch.int64) | (1 << (vbit - 1))
    v4 = torch.randint(0, 1 << 31, (n,), generator=gen, dtype=torch.int64).to(torch.int32)
    comm = g.Comm(device=dev)
    for vals, wide in ((v8, 8), (v4, 4)):
        if wide == 4:  # 12 key bits + 31 value bits fit: force a wide key instead
            kk = k | (1 << 40)
        else:
            kk = k
        want = collections.defaultdict(list)
        for a, b in zip(kk.tolist(), vals.tolist()):
            want[a].append(b)
        mr, other = g.MapReduce(comm), g.MapReduce(comm)
        h = n // 2
        mr.map(1, lambda i, kv: kv.add_tensors(kk[:h].to(dev), vals[:h].to(dev)))
        other.map(1, lambda i, kv: kv.add_tensors(kk[h:].to(dev), vals[h:].to(dev)))
        mr.add(other)
        assert mr.convert() == len(want)
        assert mr.last_convert.exact
        fmt = "<q" if wide == 8 else "<i"
        got = {struct.unpack("<q", key)[0]: [struct.unpack(fmt, x)[0] for x in vs] for key, vs in mr.kmv_pairs()}
        assert got == dict(want)
        if not mixed:
            assert list(got) == sorted(got)
