"""The chunked, bounded exchange (csrc/engine/shuffle.cpp) against its own
one-round result and a multiset oracle, on 3 CPU ranks over gloo.

Cases (SURVEY.md §4 "multi-rank tests", VERDICT r1 "chunked, bounded"):
* a receive cap small enough for >= 10 lock-step rounds must give the
  byte-identical per-rank result of the single-round exchange (the output is
  sender-major / piece-ordered, independent of the cap);
* skewed keys (one hot key carries half the pairs) and an empty rank;
* variable keys + variable values, fixed keys + fixed values, and mixed
  layouts across ranks (one rank's keys fixed-width, the others' variable);
* the reference's ring-ordered custom exchange (all2all = 0) equals the
  grouped all-to-all;
* ownership: every key lives on exactly one rank, and the union of all ranks
  is the input multiset.
The same C++ runs over RCCL on MI355X (tests/test_rccl_gpu.py)."""
import collections
import struct

import pytest
import torch

from test_distributed_cpu import run_world


def _var_kv(C, keys, vals, dev="cpu"):
    kd = torch.tensor(list(b"".join(keys)), dtype=torch.uint8)
    vd = torch.tensor(list(b"".join(vals)), dtype=torch.uint8)
    koff = torch.tensor([0] + list(__import__("itertools").accumulate(len(k) for k in keys)), dtype=torch.int64)
    voff = torch.tensor([0] + list(__import__("itertools").accumulate(len(v) for v in vals)), dtype=torch.int64)
    return C.make_kv(kd, koff, vd, voff, len(keys), dev)


def _fixed_kv(C, keys_u64, vals_u64, dev="cpu"):
    k = torch.tensor(keys_u64, dtype=torch.int64).view(torch.uint8)
    v = torch.tensor(vals_u64, dtype=torch.int64).view(torch.uint8)
    return C.make_kv(k, None, v, None, len(keys_u64), dev)


def _pairs(C, kv):
    out = []
    C.kv_iter(kv, lambda i, k, v: out.append((bytes(k), bytes(v))))
    return out


def _inputs(rank):
    """rank 2 is empty; half of all pairs carry the hot key"""
    if rank == 2:
        return [], []
    keys, vals = [], []
    for j in range(1500):
        k = b"hot-key" if j % 2 == 0 else b"k%d-%d" % (j % 173, rank)
        keys.append(k + b"\0")
        vals.append(b"v" * (1 + (j * 7 + rank) % 23))
    return keys, vals


def case_chunked(comm):
    import gpu_mapreduce_amd as g
    C = g._ext.C
    nc = comm.native
    keys, vals = _inputs(comm.rank)
    res = {}
    base, st0 = C.aggregate(_var_kv(C, keys, vals), nc)
    res["var_one_round"] = _pairs(C, base)
    res["rounds_one"] = st0.rounds
    small, st = C.aggregate(_var_kv(C, keys, vals), nc, chunk_bytes=512)
    res["var_chunked"] = _pairs(C, small)
    res["rounds_chunked"] = st.rounds
    ring, _ = C.aggregate(_var_kv(C, keys, vals), nc, chunk_bytes=2048, all2all=0)
    res["var_ring"] = _pairs(C, ring)
    # fixed 8-byte keys / 8-byte values, skewed
    fk = [] if comm.rank == 2 else [(7 if j % 3 == 0 else j * 31 + comm.rank) for j in range(4000)]
    fv = [x * 10 + comm.rank for x in range(len(fk))]
    f1, _ = C.aggregate(_fixed_kv(C, fk, fv), nc)
    f2, fst = C.aggregate(_fixed_kv(C, fk, fv), nc, chunk_bytes=1024)
    res["fixed_one"] = _pairs(C, f1)
    res["fixed_chunked"] = _pairs(C, f2)
    res["fixed_rounds"] = fst.rounds
    res["fixed_layout"] = (f2.kw, f2.vw)
    # mixed: rank 0 has fixed 8-byte keys, the others variable keys
    if comm.rank == 0:
        mk = _fixed_kv(C, [11, 12, 13, 11], [1, 2, 3, 4])
    else:
        mk = _var_kv(C, [b"ab", b"cde", b"\x0b" + b"\0" * 7], [b"x" * 8, b"y" * 8, b"z" * 8])
    m1, _ = C.aggregate(mk, nc, chunk_bytes=16)
    res["mixed"] = _pairs(C, m1)
    res["mixed_layout"] = (m1.kw, m1.vw)
    res["inputs"] = list(zip(keys, vals))
    res["fixed_inputs"] = [(struct.pack("<q", a), struct.pack("<q", b)) for a, b in zip(fk, fv)]
    return res


def test_chunked_exchange_matches_one_round_and_oracle():
    out = run_world("test_shuffle:case_chunked", 3)
    want = collections.Counter(p for r in out.values() for p in r["inputs"])
    fwant = collections.Counter(p for r in out.values() for p in r["fixed_inputs"])
    owner, fowner = {}, {}
    for r, res in out.items():
        assert res["var_chunked"] == res["var_one_round"], f"rank {r}: chunked result differs"
        assert res["var_ring"] == res["var_one_round"], f"rank {r}: ring-ordered result differs"
        assert res["fixed_chunked"] == res["fixed_one"]
        assert res["fixed_layout"] == (8, 8)
        assert res["rounds_one"] == 1
        for k, _ in res["var_one_round"]:
            assert owner.setdefault(k, r) == r, f"key {k!r} on two ranks"
        for k, _ in res["fixed_one"]:
            assert fowner.setdefault(k, r) == r
    rounds = {res["rounds_chunked"] for res in out.values()}
    assert len(rounds) == 1 and rounds.pop() >= 10, "every rank runs the same >= 10 lock-step rounds"
    assert collections.Counter(p for res in out.values() for p in res["var_one_round"]) == want
    assert collections.Counter(p for res in out.values() for p in res["fixed_one"]) == fwant
    # mixed layouts (rank 0 fixed 8-byte keys and values, the others variable):
    # both columns become variable on every rank, with the same bytes
    layouts = {res["mixed_layout"] for res in out.values()}
    assert layouts == {(-1, -1)}
    got = collections.Counter(p for res in out.values() for p in res["mixed"])
    assert sum(got.values()) == 4 + 3 + 3
    assert got[(struct.pack("<q", 11), struct.pack("<q", 1))] == 1
    assert got[(b"cde", b"y" * 8)] == 2


def case_all_empty(comm):
    import gpu_mapreduce_amd as g
    C = g._ext.C
    # every rank empty, with DIFFERENT local layouts: no column traffic at all
    kv = _var_kv(C, [], []) if comm.rank % 2 else _fixed_kv(C, [], [])
    r, st = C.aggregate(kv, comm.native, chunk_bytes=64)
    return r.n, st.recv_pairs


def test_all_ranks_empty_with_different_layouts():
    out = run_world("test_shuffle:case_all_empty", 3)
    assert all(v == (0, 0) for v in out.values())


def case_mr_chunk_setting(comm):
    """chunk_bytes through the MapReduce settings (collate = aggregate + convert)"""
    import gpu_mapreduce_amd as g
    res = []
    for chunk in (0, 300):
        mr = g.MapReduce(comm)
        mr.chunk_bytes = chunk
        mr.map(2, lambda i, kv: [kv.add(b"w%d\0" % ((i * 5 + j) % 41)) for j in range(2000)])
        mr.collate()
        mr.reduce("count")
        res.append(sorted((k, struct.unpack("<i", v)[0]) for k, v in mr.kv_pairs()))
    return res


def test_chunked_collate_via_settings():
    out = run_world("test_shuffle:case_mr_chunk_setting", 2)
    total = collections.Counter()
    for r, (a, b) in out.items():
        assert a == b
        for k, c in a:
            total[k] += c
    assert sum(total.values()) == 4000


def case_pipelined_collate(comm):
    """collate with the pipelined exchange -> GroupIndex (pipeline=1) vs
    aggregate + convert (pipeline=0): the same keys in the same order, the
    same per-key value multisets; with one round the same value order too.
    Skewed keys (one hot key), rank 2 maps nothing, var and int64 keys."""
    import gpu_mapreduce_amd as g
    out = {}
    for layout in ("var", "i64"):
        for chunk in (0, 200):
            got = []
            for pipe in (1, 0):
                mr = g.MapReduce(comm)
                mr.chunk_bytes = chunk
                mr.pipeline = pipe

                def fn(i, kv):
                    if comm.rank == 2:
                        return
                    for j in range(1500):
                        k = 7 if j % 3 == 0 else (i * 31 + j * 7) % 53
                        key = (b"key%d\0" % k) if layout == "var" else struct.pack("<q", k * 1000003)
                        kv.add(key, struct.pack("<i", comm.rank * 100000 + i * 10000 + j))
                mr.map(6, fn)  # two tasks per rank; rank 2 emits nothing
                nu = mr.collate()
                conv = mr.last_convert.grouped
                pairs = mr.kmv_pairs()
                got.append((nu, conv, [k for k, _ in pairs], [list(v) for _, v in pairs]))
            (n1, g1, k1, v1), (n0, g0, k0, v0) = got
            assert n1 == n0 and k1 == k0, (layout, chunk)
            assert [sorted(a) for a in v1] == [sorted(b) for b in v0], (layout, chunk)
            if chunk == 0:
                assert v1 == v0, (layout, chunk)
            out[(layout, chunk)] = (n1, g1, g0, sum(len(v) for v in v1))
    return out


def test_pipelined_collate_matches_aggregate_convert():
    out = run_world("test_shuffle:case_pipelined_collate", 3)
    for r, res in out.items():
        for (layout, chunk), (nu, g1, g0, nval) in res.items():
            assert g1 == (1 if nval else 0) and g0 == 0, (r, layout, chunk, g1, g0)
    # every pair arrived somewhere: 2 ranks x 2 tasks x 1500 per setting
    for key in out[0]:
        assert sum(out[r][key][3] for r in out) == 6000
