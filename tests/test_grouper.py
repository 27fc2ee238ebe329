"""Incremental group-by (GroupIndex, csrc/engine/grouper.h): a map whose
KeyValue has grouping enabled must convert to exactly the KMV the ordinary
convert produces (same key order = 64-bit hash order, same values in the
same order, same segments; wide fixed keys narrow enough to pack into 64 bits
are grouped exactly by the ordinary convert, so there only the key order
differs), including the exact fallback on forced hash
collisions and the fall back to plain chunks on a layout change.
The CPU engine runs the same algorithm as the HIP kernels (group.hip)."""
import collections
import os
import struct
import random
import subprocess
import sys

import pytest
import torch

import gpu_mapreduce_amd as g
from gpu_mapreduce_amd import C, MapReduce


def _var_part(words, vals, dev):
    kb = [w.encode() + b"\0" for w in words]
    kd = torch.frombuffer(bytearray(b"".join(kb) or b"\0"), dtype=torch.uint8)[: sum(map(len, kb))].clone()
    koff = torch.tensor([0] + [len(x) for x in kb], dtype=torch.int64).cumsum(0)
    vd = torch.tensor(vals, dtype=torch.int32).view(torch.uint8)
    return C.make_kv(kd, koff, vd, None, len(words), dev)


def _fixed_part(keys, vals, dev):
    # 16-byte keys (> 8 bytes: grouped by hash)
    kd = torch.tensor(keys, dtype=torch.int64).reshape(-1, 2).contiguous().view(torch.uint8).reshape(-1)
    vd = torch.tensor(vals, dtype=torch.int64).view(torch.uint8)
    return C.make_kv(kd, None, vd, None, len(vals), dev)


def _run(dev, parts_fn, grouping):
    mr = MapReduce(g.Comm(device=dev))

    def fn(itask, kv):
        if grouping:
            kv.enable_grouping()
        for p in parts_fn(dev):
            kv.add_kv(p)
    n = mr.map(1, fn)
    nu = mr.convert()
    return n, nu, mr.kmv_pairs(), mr.last_convert


def _words(seed, nparts=5, per=300, vocab=120):
    rng = random.Random(seed)
    voc = ["w%d_%s" % (i, "x" * rng.randrange(0, 40)) for i in range(vocab)]
    out = []
    for p in range(nparts):
        ws = [rng.choice(voc) for _ in range(per + rng.randrange(0, 50))]
        out.append((ws, [p * 1000 + i for i in range(len(ws))]))
    return out


@pytest.mark.parametrize("seed", [1, 2])
def test_grouped_convert_matches_convert_var_keys(seed):
    data = _words(seed)
    mk = lambda dev: [_var_part(w, v, dev) for w, v in data]
    a = _run("cpu", mk, False)
    b = _run("cpu", mk, True)
    assert a[0] == b[0] and a[1] == b[1]
    assert a[2] == b[2]
    assert b[3].collisions == 0 and not b[3].exact and b[3].grouped == 1
    assert a[3].grouped == 0


def test_grouped_convert_fixed_wide_keys():
    rng = random.Random(3)
    parts = []
    for p in range(4):
        ks = [rng.randrange(0, 50) for _ in range(400)]
        parts.append(([x for k in ks for x in (k, k * 7)], [p * 10000 + i for i in range(400)]))
    mk = lambda dev: [_fixed_part(k, v, dev) for k, v in parts]
    a = _run("cpu", mk, False)
    b = _run("cpu", mk, True)
    assert a[1] == b[1] == 50
    # the ordinary convert groups these narrow 16-byte keys exactly on packed
    # words (engine.cpp narrow_keys), the incremental index by hash: the same
    # groups with the same values in the same order, keys in another order
    assert a[3].exact and not b[3].exact
    assert sorted(a[2]) == sorted(b[2])


def test_layout_change_falls_back_to_chunks():
    data = _words(4, nparts=2)
    rng = random.Random(5)

    def mk(dev):
        ps = [_var_part(w, v, dev) for w, v in data]
        ks = [rng.randrange(0, 9) for _ in range(50)]
        ps.insert(1, _fixed_part([x for k in ks for x in (k, k)], list(range(50)), dev))
        return ps
    rng.seed(5)
    a = _run("cpu", mk, False)
    rng.seed(5)
    b = _run("cpu", mk, True)
    assert a[2] == b[2]


def _small_parts(dev):
    rng = random.Random(11)
    out = []
    for p in range(4):
        ks = [rng.randrange(0, 300) * (1 if p % 2 else 1 << 33) for _ in range(500)]
        out.append(C.make_kv(torch.tensor(ks, dtype=torch.int64).view(torch.uint8), None,
                             torch.tensor([p * 1000 + i for i in range(500)], dtype=torch.int32).view(torch.uint8),
                             None, 500, dev))
    return out


def test_small_fixed_keys_grouped_in_raw_key_order():
    """int64 keys: convert orders groups by raw key value (exact path); the
    grouped convert must produce the same KMV"""
    a = _run("cpu", _small_parts, False)
    b = _run("cpu", _small_parts, True)
    assert a[1] == b[1] and a[2] == b[2]
    assert b[3].grouped == 1 and a[3].exact


def test_forced_collisions_exact_fallback():
    """MRH_GROUP_HASH_BITS=4: most groups collide in the table; the byte
    check must catch it and convert must still be exact."""
    code = r'''
import random, torch, gpu_mapreduce_amd as g
from gpu_mapreduce_amd import C, MapReduce
from tests.test_grouper import _words, _var_part, _run
data = _words(7)
mk = lambda dev: [_var_part(w, v, dev) for w, v in data]
b = _run("cpu", mk, True)
import collections
want = collections.defaultdict(list)
for ws, vs in data:
    for w, v in zip(ws, vs):
        want[w.encode() + b"\0"].append(v)
got = {k: [int.from_bytes(x, "little", signed=True) for x in vs] for k, vs in b[2]}
assert got == dict(want), "grouping wrong under collisions"
assert b[3].grouped == 2  # the byte check caught the collisions
print("ok")
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MRH_GROUP_HASH_BITS="4", PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_grouped_convert_gpu_matches_cpu(seed):
    data = _words(seed, nparts=6, per=5000, vocab=3000)
    mk = lambda dev: [_var_part(w, v, dev) for w, v in data]
    a = _run("cpu", mk, False)
    b = _run("cuda", mk, True)
    assert a[0] == b[0] and a[1] == b[1]
    assert a[2] == b[2]
    assert b[3].collisions == 0


@pytest.mark.gpu
def test_grouped_convert_gpu_small_fixed():
    a = _run("cpu", _small_parts, False)
    b = _run("cuda", _small_parts, True)
    assert a[2] == b[2] and b[3].grouped == 1


@pytest.mark.gpu
def test_grouped_convert_gpu_fixed_wide():
    rng = random.Random(9)
    parts = []
    for p in range(5):
        ks = [rng.randrange(0, 5000) for _ in range(20000)]
        parts.append(([x for k in ks for x in (k, k ^ 0x5555)], [p * 100000 + i for i in range(20000)]))
    mk = lambda dev: [_fixed_part(k, v, dev) for k, v in parts]
    a = _run("cpu", mk, False)
    b = _run("cuda", mk, True)
    assert a[1] == b[1]
    # packed-word order (ordinary convert) vs hash order (incremental index)
    assert sorted(a[2]) == sorted(b[2])


def _pairs_part(keys, vals, dev, words=1):
    kd = torch.tensor(keys, dtype=torch.int64).reshape(-1, words).contiguous().view(torch.uint8).reshape(-1)
    vd = torch.tensor(vals, dtype=torch.int64).view(torch.uint8)
    return C.make_kv(kd, None, vd, None, len(vals), dev)


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("words", [1, 2])
def test_convert_packed_pairs_vs_dict(dev, words):
    """narrow fixed keys (1 or 2 words) with narrow 8-byte values group as one
    packed u64 per pair: every key's values in input order, against a Python
    dict; with a value too wide to pack the ordinary path gives the same groups"""
    rng = random.Random(11 + words)
    n = 50_000
    keys = [rng.randrange(0, 3000) for _ in range(n * words)]
    vals = [rng.randrange(0, 1 << 20) for _ in range(n)]
    want = collections.defaultdict(list)
    for i in range(n):
        want[tuple(keys[i * words:(i + 1) * words])].append(vals[i])
    for wide in (False, True):
        vv = [v | (1 << 62) for v in vals] if wide else vals  # 63 value bits: not packable
        mr = MapReduce(g.Comm(device=dev))
        mr.map(1, lambda itask, kv: kv.add_kv(_pairs_part(keys, vv, dev, words)))
        assert mr.convert() == len(want)
        got = {}
        for k, mv in mr.kmv_pairs():
            kk = tuple(struct.unpack(f"<{words}q", k))
            got[kk] = [struct.unpack("<q", v)[0] & ((1 << 62) - 1) for v in mv]
        assert got == dict(want)
        assert mr.last_convert.exact
