"""Out-of-core hot keys (the reference's extended KMV pair,
src/keymultivalue.cpp:845-846, 974-999, 1219-1350, and its multi-block reduce,
src/mapreduce.cpp:1828-1848, 1874-1925): one key holds 12x the HBM budget of
values — more than the pool's whole op cap (in use + 2 x budget + 16 MiB).
convert groups it on the host without ever moving it to HBM whole
(ooc.cpp ooc_convert_big), builtin reduces cut its values into budget-sized
blocks and carry a partial across them (ooc_for_each_kmv_block), a host
callback walks it block by block (nvalues == 0 protocol), sort_values orders
the results. Everything must equal the in-memory oracle, stay under the
pool's op cap, and leave no spool file behind."""
import gc
import struct

import numpy as np
import pytest
import torch

import gpu_mapreduce_amd as g
from gpu_mapreduce_amd import MapReduce
from gpu_mapreduce_amd.runtime.mapreduce import BlockMultiValue

HOT = 7
BUDGET = 4 << 20          # hot key: 4.5 M x 8 B = 36 MB = 8.6 x the budget, past the op cap of 24 MiB
PAGE = 1 << 20            # a host callback sees the hot key in 1 MB blocks
NMAP = 16


def _data():
    gen = torch.Generator().manual_seed(11)
    nh, no = 4_500_000, 200_000
    keys = torch.cat([torch.full((nh,), HOT, dtype=torch.int64),
                      torch.randint(100, 5100, (no,), generator=gen, dtype=torch.int64)])
    keys = keys[torch.randperm(keys.numel(), generator=gen)]
    vals = torch.randint(0, 1 << 40, (keys.numel(),), generator=gen, dtype=torch.int64)
    return keys, vals


def _oracle(keys, vals):
    k, v = keys.numpy(), vals.numpy()
    out = {}
    order = np.argsort(k, kind="stable")
    ks, vs = k[order], v[order]
    bounds = np.flatnonzero(np.diff(ks)) + 1
    for a, b in zip(np.r_[0, bounds], np.r_[bounds, len(ks)]):
        seg = vs[a:b]
        out[int(ks[a])] = (b - a, int(seg.sum()), int(seg.min()), int(seg.max()), int(seg[0]), int(seg[-1]))
    return out


def _mk(comm, tmp_path):
    mr = MapReduce(comm)
    mr.fpath = str(tmp_path)
    mr.hbm_budget = BUDGET
    mr.host_budget = 24 << 20  # the hot key's values reach the disk tier
    mr.memsize = -PAGE
    return mr


def _map(mr, keys, vals, dev):
    q = (keys.numel() + NMAP - 1) // NMAP
    mr.map(NMAP, lambda i, kv: kv.add_tensors(keys[i * q:(i + 1) * q].to(dev), vals[i * q:(i + 1) * q].to(dev)))


def _pairs(mr, fmt):
    return {struct.unpack("<q", k)[0]: struct.unpack(fmt, v) for k, v in mr.kv_pairs()}


def _run(dev, tmp_path):
    C = g._ext.C
    comm = g.Comm(device=dev)
    keys, vals = _data()
    want = _oracle(keys, vals)
    live0 = C.spool_files_live()
    pool = None
    if dev != "cpu":
        from gpu_mapreduce_amd.runtime import hbm_pool
        pool = hbm_pool if hbm_pool.installed() else None
    if pool:
        torch.cuda.synchronize()
        base = pool.stats(0)["in_use"]
        pool.reset_peak(0)

    # collate -> host-callback reduce over the hot key's blocks
    mr = _mk(comm, tmp_path)
    _map(mr, keys, vals, dev)
    assert mr.kv.nbytes() > 8 * BUDGET
    assert mr.collate() == len(want)
    assert mr.spool_stats["ooc_hot_keys"] >= 1      # grouped on the host, never in HBM whole
    assert mr.kmv_parts > 1                          # one host-resident KMV per partition, not concatenated
    blocks = {}

    def red(k, mv, kv):
        key = struct.unpack("<q", k)[0]
        n, s = 0, 0
        for b in range(mr.multivalue_blocks(mv)[1]):
            blk = mr.multivalue_block(mv, b)
            assert len(blk) * 8 <= PAGE or not isinstance(mv, BlockMultiValue)  # one engine page at a time
            n += len(blk)
            s += int(np.frombuffer(b"".join(blk), dtype=np.int64).sum())
        blocks[key] = (mv.nblocks(), isinstance(mv, BlockMultiValue))
        kv.add(k, struct.pack("<qq", n, s))
    mr.reduce(red)
    assert _pairs(mr, "<qq") == {k: (w[0], w[1]) for k, w in want.items()}
    # the hot key came as the engine's page cursor, never one list
    assert blocks[HOT][0] >= 8 and blocks[HOT][1], blocks[HOT]
    assert not any(isb for k, (nb, isb) in blocks.items() if k != HOT)

    # collate -> builtin reduces: a partial carried across the hot key's blocks
    for op, fmt, pick in (("count", "<i", lambda w: (w[0],)), ("sum:int64", "<q", lambda w: (w[1],)),
                          ("min:int64", "<q", lambda w: (w[2],)), ("max:int64", "<q", lambda w: (w[3],)),
                          ("first", "<q", lambda w: (w[4],)), ("last", "<q", lambda w: (w[5],))):
        m2 = _mk(comm, tmp_path)
        _map(m2, keys, vals, dev)
        m2.collate()
        m2.reduce(op)
        assert m2.spool_stats["ooc_split_keys"] >= 1, op
        assert _pairs(m2, fmt) == {k: pick(w) for k, w in want.items()}, op
        if op == "count":
            m2.sort_values(-1)  # counts, descending: the hot key first
            got = [struct.unpack("<i", v)[0] for _, v in m2.kv_pairs()]
            assert got == sorted((w[0] for w in want.values()), reverse=True)
            assert struct.unpack("<q", next(iter(m2.kv_pairs()))[0])[0] == HOT
        del m2

    # sort_values of the whole KV (out of core, the hot key's values spread
    # over the range buckets)
    m3 = _mk(comm, tmp_path)
    _map(m3, keys, vals, dev)
    m3.sort_values(2)
    got = m3.kv.vdata.view(torch.int64).cpu().numpy().copy()  # (a view would keep the result file)
    assert np.array_equal(got, np.sort(vals.numpy()))
    del m3

    if pool:
        torch.cuda.synchronize()
        # every op ran under its cap: in use at entry + 2 x budget + 16 MiB of scratch
        assert pool.stats(0)["peak"] - base <= 2 * BUDGET + (16 << 20) + (4 << 20), pool.stats(0)
    del mr, red  # (red's closure holds mr)
    gc.collect()
    assert C.spool_files_live() == live0
    assert not [p for p in tmp_path.iterdir() if p.name.startswith("mrmpi.")]


def test_ooc_hot_key_cpu(tmp_path):
    _run("cpu", tmp_path)


@pytest.mark.gpu
def test_ooc_hot_key_gpu(tmp_path):
    _run("cuda:0", tmp_path)


def test_mrmpi_hot_key_blocks(tmp_path):
    """the mrmpi wrapper (pickled keys/values): a hot key out of core reaches
    the reduce as the reference's multi-block protocol (mvalue == []), and
    multivalue_block(i) hands out one engine page of unpickled values at a
    time (reference python/mrmpi.py:335-344, src/mapreduce.cpp:1874-1925)"""
    from gpu_mapreduce_amd.mrmpi import mrmpi
    nhot, page = 60_000, 1 << 16
    m = mrmpi(g.Comm(device="cpu"))
    m.mr.fpath = str(tmp_path)
    m.mr.hbm_budget = 1 << 18
    m.mr.host_budget = 1 << 20
    m.mr.memsize = -page

    def emit(itask, mr):
        for i in range(itask, nhot, 4):
            mr.add("hot", i)
        for i in range(itask, 400, 4):
            mr.add("k%d" % (i % 37), i)
    m.map(4, emit)
    m.collate()
    seen = {}

    def red(key, mvalue, mr):
        nb = mr.multivalue_blocks()
        if mvalue == [] and nb > 1:
            tot, cnt, biggest = 0, 0, 0
            for b in range(nb):
                vals = mr.multivalue_block(b)
                biggest = max(biggest, len(vals))
                cnt += len(vals)
                tot += sum(vals)
            seen[key] = (nb, biggest)
            mr.add(key, (cnt, tot))
        else:
            mr.add(key, (len(mvalue), sum(mvalue)))
    m.reduce(red)
    got = dict(m.pairs())
    assert got["hot"] == (nhot, nhot * (nhot - 1) // 2)
    assert seen["hot"][0] > 4 and seen["hot"][1] < nhot // 4, seen  # pages, not one list
    want = {}
    for i in range(400):
        c, t = want.get("k%d" % (i % 37), (0, 0))
        want["k%d" % (i % 37)] = (c + 1, t + i)
    assert {k: v for k, v in got.items() if k != "hot"} == want
