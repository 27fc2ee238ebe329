"""Hash-dictionary group-by (grouper.h HashDict / convert_dict, kernels in
csrc/kernels/group.hip k_dict_insert): a KV whose keys repeat (words, a hot
key) is grouped in one pass over a device hash table of its distinct keys.
The result must be exactly the sort path's KMV — keys in 64-bit hash order,
every key's values in input order, the same segments — with fixed or zero
width values, a hot key holding half the pairs, and a table that fills up
(MRH_DICT_CAP forces the grow + retry and the regroup-from-scratch paths).
The CPU engine (the oracle) always runs the sort path."""
import collections
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import gpu_mapreduce_amd as g
from gpu_mapreduce_amd import C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def zipf_words(n, vocab, seed, hot=0.0, uniform=False):
    """n word keys (NUL-terminated) drawn Zipf-like (or uniformly) from
    `vocab` words; `hot`: the share of one extra hot word"""
    rng = np.random.default_rng(seed)
    words = [("w%d" % i + "y" * int(rng.integers(0, 30))).encode() + b"\0" for i in range(vocab)]
    p = 1.0 / np.arange(1, vocab + 1)
    idx = rng.integers(0, vocab, size=n) if uniform else rng.choice(vocab, size=n, p=p / p.sum())
    if hot > 0:
        words.append(b"the_hot_key\0")
        idx[rng.random(n) < hot] = vocab
    lens = np.array([len(w) for w in words], dtype=np.int64)[idx]
    koff = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=koff[1:])
    blob = np.frombuffer(b"".join(words), dtype=np.uint8)
    woff = np.zeros(len(words) + 1, dtype=np.int64)
    np.cumsum([len(w) for w in words], out=woff[1:])
    # bytes of every pair: gather each word's bytes by position
    pos = np.arange(koff[-1], dtype=np.int64) - np.repeat(koff[:-1], lens)
    kd = blob[np.repeat(woff[idx], lens) + pos]
    return torch.from_numpy(kd.copy()), torch.from_numpy(koff), idx


def make_kv(kd, koff, n, vw, dev):
    vd = torch.arange(n, dtype=torch.int32).view(torch.uint8) if vw == 4 else torch.empty(0, dtype=torch.uint8)
    return C.make_kv(kd, koff, vd, None, n, dev)


def kmv_tensors(kmv):
    k = kmv.keys
    return (k.kdata.cpu(), k.koff.cpu(), kmv.seg.cpu(), kmv.vdata.cpu(), kmv.nkey, kmv.nval)


def check_same(a, b):
    for x, y in zip(a[:4], b[:4]):
        assert torch.equal(x, y)
    assert a[4:] == b[4:]


@pytest.mark.gpu
@pytest.mark.parametrize("vw", [0, 4])
@pytest.mark.parametrize("hot", [0.0, 0.5])
def test_convert_dict_matches_sort_path(vw, hot):
    n = 1_500_000
    kd, koff, idx = zipf_words(n, 20_000, seed=3 + vw, hot=hot)
    cpu, _ = C.convert(make_kv(kd, koff, n, vw, "cpu"))
    gpu, st = C.convert(make_kv(kd, koff, n, vw, "cuda"))
    assert st.dict == 1 and st.collisions == 0
    check_same(kmv_tensors(cpu), kmv_tensors(gpu))
    assert gpu.nkey == len(set(idx.tolist()))


@pytest.mark.gpu
def test_convert_dict_skips_distinct_keys():
    """mostly distinct keys (a URL list) keep the sort path"""
    n = 1 << 20
    kd, koff, _ = zipf_words(n, 4_000_000, seed=5, uniform=True)
    gpu, st = C.convert(make_kv(kd, koff, n, 4, "cuda"))
    cpu, _ = C.convert(make_kv(kd, koff, n, 4, "cpu"))
    assert st.dict == 0
    check_same(kmv_tensors(cpu), kmv_tensors(gpu))


_FULL_TABLE = r'''
import sys, torch
sys.path.insert(0, "tests")
from test_dict_group import zipf_words, make_kv, kmv_tensors, check_same
from gpu_mapreduce_amd import C
n = 1_200_000
for vw in (0, 4):
    kd, koff, idx = zipf_words(n, 30_000, seed=11 + vw, hot=0.3)
    cpu, _ = C.convert(make_kv(kd, koff, n, vw, "cpu"))
    gpu, st = C.convert(make_kv(kd, koff, n, vw, "cuda"))
    assert st.dict == 1, st.dict
    assert st.dict_cap > 4096, st.dict_cap   # it grew
    check_same(kmv_tensors(cpu), kmv_tensors(gpu))
print("ok")
'''


@pytest.mark.gpu
def test_convert_dict_full_table_grows():
    """a 4096-slot first table (MRH_DICT_CAP) for ~25k distinct keys: with
    values the unassigned rows are retried in a grown table, without values
    the grouping starts again in a table sized from the counts"""
    env = dict(os.environ, MRH_DICT_CAP="4096", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", _FULL_TABLE], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("ok")


_GROUPED_FULL = r'''
import sys, torch
sys.path.insert(0, "tests")
from test_dict_group import zipf_words, make_kv
import gpu_mapreduce_amd as g
from gpu_mapreduce_amd import C, MapReduce
n = 400_000
kd, koff, idx = zipf_words(n, 40_000, seed=17, hot=0.2)
res = []
for dev, grouping in (("cpu", False), ("cuda", True)):
    for vw in (0, 4):
        mr = MapReduce(g.Comm(device=dev))
        def fn(itask, kv):
            if grouping:
                kv.enable_grouping()
            step = n // 4
            for a in range(0, n, step):
                b = min(n, a + step)
                kvp = make_kv(kd[koff[a]:koff[b]].clone(), koff[a:b + 1] - koff[a], b - a, vw, dev)
                if vw:
                    kvp.vdata = (torch.arange(a, b, dtype=torch.int32).view(torch.uint8)).to(dev)
                kv.add_kv(kvp)
        mr.map(1, fn)
        mr.convert()
        if grouping:
            assert mr.last_convert.grouped == 1, mr.last_convert.grouped
        res.append(mr.kmv_pairs())
assert res[0] == res[2] and res[1] == res[3]
print("ok")
'''


@pytest.mark.gpu
def test_grouped_index_full_table_retries_at_finish():
    """the incremental index (GroupIndex) with a 4096-slot table and ~35k
    distinct keys arriving in 4 parts: rows left unassigned are grouped at
    finish() in a grown table; zero-width values take the count segments"""
    env = dict(os.environ, MRH_DICT_CAP="4096", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", _GROUPED_FULL], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("ok")


@pytest.mark.gpu
def test_wordfreq_per_occurrence_gpu_equals_counter():
    """wordfreq without the in-mapper combiner: one (word, NULL) pair per
    occurrence through collate -> reduce(count) -> top-N, grouped on the hash
    dictionary while the map streams the chunks; counts equal
    collections.Counter, top-10 equals the combiner's"""
    from gpu_mapreduce_amd.models.wordfreq import WordFreq
    from gpu_mapreduce_amd.utils import synth
    chunks = [synth.zipf_text(3 << 20, seed=40 + i, device="cuda").cpu() for i in range(3)]
    cnt = collections.Counter()
    for c in chunks:
        cnt.update(bytes(c.numpy()).split())
    comm = g.Comm(device="cuda:0")
    app = WordFreq(g.MapReduce(comm), chunks, ntop=10, combiner=False)
    ph = {}
    assert app.run(ph) == sum(cnt.values())
    assert set(ph) == {"map", "collate", "reduce", "top_n"}
    assert app.mr.last_convert.grouped == 1  # grouped chunk by chunk during the map
    assert app.nunique == len(cnt)
    want = sorted(cnt.items(), key=lambda kv: -kv[1])[:10]
    assert [c for _, c in app.top] == [c for _, c in want]
    assert {w: c for w, c in app.top} == {w.decode(): c for w, c in want if c > want[-1][1]} | \
        {w: c for w, c in app.top if c == want[-1][1]}
    comb = WordFreq(g.MapReduce(comm), chunks, ntop=10, combiner=True)
    comb.run()
    assert comb.top == app.top
