"""Out-of-core convert / sort / builtin reduce under an HBM budget ~10x
smaller than the data (csrc/engine/ooc.cpp).

The reference pages its KV through `memsize` pages and spools partitions and
sort runs to disk when they overflow (src/keymultivalue.cpp:645-789,
src/mapreduce.cpp:2395-2445). Here `memsize` (page size) x `maxpage` (or
`hbm_budget` directly) is the HBM budget: an op over more data than that
streams budget-sized pieces through the device and keeps the result in pinned
host memory. Every result must equal the in-memory op (the oracle), and
kv_stats must report the data spanning more than one page."""
import collections
import struct

import pytest
import torch

import gpu_mapreduce_amd as g
from gpu_mapreduce_amd import MapReduce

WORDS = [b"w%d-%s\0" % (j % 1711, b"x" * (j % 13)) for j in range(60000)]


def _mr(comm, budget):
    mr = MapReduce(comm)
    if budget:
        mr.memsize = -16384           # 16 KB pages (negative = bytes, reference semantics)
        mr.maxpage = budget // 16384  # budget = maxpage x memsize
    return mr


def _wordcount(comm, budget):
    mr = _mr(comm, budget)
    mr.map(3, lambda i, kv: [kv.add(w, struct.pack("<i", j)) for j, w in enumerate(WORDS[i::3])])
    assert mr.kv.nbytes() > 10 * budget if budget else True
    nu = mr.convert()
    mr.reduce("count")
    return nu, dict((k, struct.unpack("<i", v)[0]) for k, v in mr.kv_pairs())


def _sorted(comm, budget, flag, by_value):
    mr = _mr(comm, budget)
    vals = [(j * 2654435761) % 100003 - 50000 for j in range(40000)]
    if by_value:
        mr.map(1, lambda i, kv: [kv.add(WORDS[j], struct.pack("<i", v)) for j, v in enumerate(vals)])
        mr.sort_values(flag)
    else:
        mr.map(1, lambda i, kv: [kv.add(WORDS[j], struct.pack("<i", v)) for j, v in enumerate(vals)])
        mr.sort_keys(flag)
    return list(mr.kv_pairs())


def _run(dev):
    comm = g.Comm(device=dev)
    budget = 64 * 1024
    nu0, c0 = _wordcount(comm, 0)
    nu1, c1 = _wordcount(comm, budget)
    assert nu0 == nu1 == len(set(WORDS))
    assert c0 == c1 == dict(collections.Counter(WORDS))
    for flag, by_value in ((5, False), (-5, False), (1, True), (-1, True)):
        assert _sorted(comm, budget, flag, by_value) == _sorted(comm, 0, flag, by_value), (flag, by_value)
    # stats: a KV ~20x the page spans many pages
    mr = _mr(comm, budget)
    mr.map(1, lambda i, kv: [kv.add(w) for w in WORDS])
    lines = []
    g._ext.C.set_screen(lambda s: lines.append(s))
    try:
        mr.kv_stats(1)
    finally:
        g._ext.C.set_screen(None)
    pages = int("".join(lines).split(" Mb, ")[-1].split()[0])
    assert pages > 10, lines


def test_out_of_core_cpu():
    _run("cpu")


@pytest.mark.gpu
def test_out_of_core_gpu():
    _run("cuda:0")


def _tiered(comm, tmp_path, data_bytes):
    """hbm_budget = 1/20 and host_budget = 1/4 of the data: the map's builder
    spools past both budgets (pinned host, then files under fpath), convert and
    sort partition into spools that also reach the disk tier"""
    mr = MapReduce(comm)
    mr.fpath = str(tmp_path)
    mr.hbm_budget = data_bytes // 20
    mr.host_budget = data_bytes // 4
    mr.memsize = -16384
    return mr


def _tiered_run(dev, tmp_path):
    comm = g.Comm(device=dev)
    C = g._ext.C
    ref = MapReduce(comm)
    ref.map(3, lambda i, kv: [kv.add(w, struct.pack("<i", j)) for j, w in enumerate(WORDS[i::3])])
    data = ref.kv.nbytes()
    ref.convert()
    ref.reduce("count")
    want_counts = dict((k, struct.unpack("<i", v)[0]) for k, v in ref.kv_pairs())
    live0 = C.spool_files_live()
    files_seen = set()

    def peek():
        files_seen.update(p.name for p in tmp_path.iterdir() if p.name.startswith("mrmpi."))

    mr = _tiered(comm, tmp_path, data)
    mr.map(3, lambda i, kv: [kv.add(w, struct.pack("<i", j)) for j, w in enumerate(WORDS[i::3])])
    peek()
    st = mr.spool_stats
    assert st["files"] > 0 and st["disk_bytes"] > 0, st          # the map reached the disk tier
    assert st["host_bytes"] > 0, st                              # ... through the pinned host tier
    assert mr.kv.n == len(WORDS)
    nu = mr.convert()
    peek()
    mr.reduce("count")
    assert nu == len(set(WORDS))
    assert dict((k, struct.unpack("<i", v)[0]) for k, v in mr.kv_pairs()) == want_counts
    assert mr.spool_stats["files"] > st["files"]                 # convert's partition spools went to disk too
    # sort: range-partitioned spools, same order as in memory
    vals = [(j * 2654435761) % 100003 - 50000 for j in range(40000)]
    srt = _tiered(comm, tmp_path, data)
    srt.map(1, lambda i, kv: [kv.add(WORDS[j], struct.pack("<i", v)) for j, v in enumerate(vals)])
    srt.sort_values(-1)
    peek()
    mem = MapReduce(comm)
    mem.map(1, lambda i, kv: [kv.add(WORDS[j], struct.pack("<i", v)) for j, v in enumerate(vals)])
    mem.sort_values(-1)
    assert list(srt.kv_pairs()) == list(mem.kv_pairs())
    assert files_seen, "spool files must appear under fpath"
    assert all(p.startswith("mrmpi.") for p in files_seen)
    del mr, srt
    import gc
    gc.collect()
    # every spool file is removed once nothing views it
    assert C.spool_files_live() == live0
    assert not [p for p in tmp_path.iterdir() if p.name.startswith("mrmpi.")]


def test_tiers_hbm_host_disk_cpu(tmp_path):
    _tiered_run("cpu", tmp_path)


@pytest.mark.gpu
def test_tiers_hbm_host_disk_gpu(tmp_path):
    _tiered_run("cuda:0", tmp_path)


def case_ooc_pipeline(comm):
    """map -> collate -> reduce("count"), -> collate -> host-callback reduce,
    and compress / gather, with hbm_budget = 1/20 and host_budget = 1/4 of the
    data: the shuffle streams budget-sized chunks into host memory
    (ooc_exchange), convert / reduce partition into spools that reach the disk
    tier. Returns what each rank ends with plus the spool evidence."""
    import os
    C = g._ext.C
    d = os.path.join(os.environ["MRH_OOC_TEST_DIR"], f"r{comm.rank}")
    os.makedirs(d, exist_ok=True)
    P = comm.size

    def task(i, kv):  # map task i: WORDS[i::P], whichever rank runs it
        for j, w in enumerate(WORDS[i::P]):
            kv.add(w, struct.pack("<i", j))
    ref = MapReduce(comm)
    ref.map(P, task)
    data = comm.allreduce(ref.kv.nbytes(), "max")
    del ref
    live0 = C.spool_files_live()
    seen = set()

    def peek():
        seen.update(p for p in os.listdir(d) if p.startswith("mrmpi."))

    def tiered():
        mr = MapReduce(comm)
        mr.fpath = d
        mr.hbm_budget = data // 20
        mr.host_budget = data // 4
        mr.memsize = -16384
        mr.map(P, task)
        return mr

    mr = tiered()
    nu = mr.collate()
    peek()
    mr.reduce("count")
    counts = {k: struct.unpack("<i", v)[0] for k, v in mr.kv_pairs()}
    st = dict(mr.spool_stats)
    mr2 = tiered()
    mr2.collate()
    mr2.reduce(lambda k, mv, kv: kv.add(k, struct.pack("<q", sum(struct.unpack("<i", x)[0] for x in mv))))
    sums = {k: struct.unpack("<q", v)[0] for k, v in mr2.kv_pairs()}
    mr3 = tiered()
    mr3.compress("count")              # local groups, out of core
    mr3.gather(1)                      # every rank's pairs to rank 0, chunked into host memory
    gathered = list(mr3.kv_pairs())
    peek()
    del mr, mr2, mr3
    import gc
    gc.collect()
    left = [p for p in os.listdir(d) if p.startswith("mrmpi.")]
    return nu, counts, sums, len(gathered), st, sorted(seen), left, C.spool_files_live() - live0


def _ooc_world(world, device, tmp_path, monkeypatch):
    from test_distributed_cpu import run_world
    monkeypatch.setenv("MRH_OOC_TEST_DIR", str(tmp_path))
    out = run_world("test_outofcore:case_ooc_pipeline", world, device)
    want = collections.Counter(WORDS)
    want_sums = collections.Counter()
    # value sums: map task i numbers WORDS[i::world]
    for i in range(world):
        for j, w in enumerate(WORDS[i::world]):
            want_sums[w] += j
    counts, sums, gathered_total = {}, {}, 0
    for r in range(world):
        nu, c, s, ng, st, seen, left, live = out[r]
        assert nu == len(want)
        assert not (set(counts) & set(c)), "a key owned by two ranks"
        counts.update(c)
        sums.update(s)
        gathered_total += ng
        assert seen, "spool files must appear under fpath"
        assert not left and live == 0, (left, live)      # every spool file removed again
    assert counts == dict(want)
    assert sums == dict(want_sums)
    # compress("count") then gather(1): rank 0 holds every rank's local groups
    assert out[0][3] == gathered_total and gathered_total >= len(want)


def test_ooc_distributed_pipeline_cpu(tmp_path, monkeypatch):
    _ooc_world(2, "cpu", tmp_path, monkeypatch)


@pytest.mark.gpu
def test_ooc_distributed_pipeline_gpu(tmp_path, monkeypatch):
    """two ranks on the box's GPU (gloo transport): the device engine under an
    HBM budget of 1/20 of the data and its pool cap (a chunk too large for
    the cap fails with "Cannot allocate page")"""
    _ooc_world(2, "cuda:0", tmp_path, monkeypatch)


def test_reduce_after_budget_lowered_to_zero(tmp_path):
    """an out-of-core convert leaves several KMV parts; with the budget then
    set to 0 (unlimited) the builtin reduce takes every part whole, not the
    block path with a piece size of budget / 4 = 0"""
    comm = g.Comm(device="cpu")
    mr = _tiered(comm, tmp_path, 1 << 20)
    mr.map(3, lambda i, kv: [kv.add(w, struct.pack("<i", j)) for j, w in enumerate(WORDS[i::3])])
    mr.convert()
    assert mr.kmv_parts > 1
    mr.hbm_budget = 0
    mr.host_budget = 0
    mr.reduce("count")
    got = {k: struct.unpack("<i", v)[0] for k, v in mr.kv_pairs()}
    assert got == dict(collections.Counter(WORDS))
