"""Multi-process correctness of the distributed path (aggregate / collate /
gather / broadcast / scrunch / mapstyle 2 / InvertedIndex) with world size 2
and 3 over gloo on the CPU engine. The same C++ shuffle code runs over RCCL
on MI355X (device tensors); only the c10d backend differs."""
import collections
import os
import socket
import struct
import sys
import traceback

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn_name, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import gpu_mapreduce_amd as g
        dev = os.environ.get("MRH_DIST_DEVICE", "cpu")
        if dev.startswith("cuda"):
            torch.cuda.set_device(0)  # every rank shares the box's one GPU
        comm = g.Comm(device=dev)
        mod, _, name = fn_name.rpartition(":")
        fn = getattr(__import__(mod), name) if mod else globals()[name]
        res = fn(comm)
        q.put((rank, "ok", res))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run_world(fn_name, world, device="cpu"):
    os.environ["MRH_DIST_DEVICE"] = device
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, fn_name, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in range(world):
        r, status, res = q.get(timeout=240)
        assert status == "ok", res
        out[r] = res
    for p in ps:
        p.join(60)
    return out


WORDS = [b"w%03d\0" % (i % 97) for i in range(5000)]


def case_wordcount(comm):
    import gpu_mapreduce_amd as g
    mr = g.MapReduce(comm)
    n = mr.map(7, lambda i, kv: [kv.add(w) for w in WORDS[i::7]])
    nu = mr.collate()
    mr.reduce("count")
    local = {k: struct.unpack("<i", v)[0] for k, v in mr.kv_pairs()}
    return n, nu, local


@pytest.mark.parametrize("world", [2, 3])
def test_collate_wordcount(world):
    out = run_world("case_wordcount", world)
    total = {}
    for r, (n, nu, local) in out.items():
        assert n == len(WORDS)
        assert nu == len(set(WORDS))
        assert not (set(total) & set(local)), "key owned by two ranks"
        total.update(local)
    assert total == collections.Counter(WORDS)


def case_shuffle_determinism(comm):
    """SURVEY.md §5 "deterministic-order checks for the shuffle": the same job
    run twice must give byte-identical KV and KMV sequences, in order, on every
    rank (stable partition, rank-ordered receive, stable sort)."""
    import gpu_mapreduce_amd as g
    rng = [(comm.rank * 7919 + j * 104729) % 613 for j in range(3000)]

    def job():
        mr = g.MapReduce(comm)
        mr.map(comm.size, lambda i, kv: [kv.add(b"key%d" % (x % 211), struct.pack("<ii", i, x)) for x in rng])
        mr.aggregate()
        kv = list(mr.kv_pairs())
        mr.convert()
        kmv = [(k, list(v)) for k, v in mr.kmv_pairs()]
        return kv, kmv

    a, b = job(), job()
    return a == b, len(a[0]), len(a[1])


def test_shuffle_is_deterministic():
    out = run_world("case_shuffle_determinism", 3)
    assert all(same for same, _, _ in out.values()), out
    assert sum(n for _, n, _ in out.values()) == 3 * 3000
    assert sum(u for _, _, u in out.values()) == 211


def case_fixed_and_var_mixed(comm):
    """rank 0 emits fixed-width keys, others variable + one empty rank."""
    import gpu_mapreduce_amd as g
    mr = g.MapReduce(comm)

    def m(i, kv):
        if comm.rank == 0:
            for j in range(100):
                kv.add(struct.pack("<q", j % 10), struct.pack("<i", j))
        elif comm.rank == 1:
            for j in range(50):
                kv.add(b"k" * (1 + j % 4), b"v" * (j % 3))
    mr.map(comm.size, m)
    mr.aggregate()
    mr.convert()
    return {k: len(v) for k, v in mr.kmv_pairs()}


def test_mixed_layouts_and_empty_rank():
    out = run_world("case_fixed_and_var_mixed", 3)
    merged = collections.Counter()
    for r, d in out.items():
        for k, c in d.items():
            merged[k] += c
    assert sum(merged.values()) == 150
    assert merged[struct.pack("<q", 3)] == 10
    assert merged[b"kk"] == 13


def case_gather_bcast(comm):
    import gpu_mapreduce_amd as g
    mr = g.MapReduce(comm)
    mr.map(comm.size, lambda i, kv: [kv.add(struct.pack("<i", i * 100 + j), b"x" * j) for j in range(5)])
    n1 = mr.gather(1)
    local_after_gather = mr.kv.n
    n2 = mr.broadcast(0)
    local_after_bcast = mr.kv.n
    keys = sorted(struct.unpack("<i", k)[0] for k, _ in mr.kv_pairs())
    mr2 = g.MapReduce(comm)
    mr2.map(comm.size, lambda i, kv: kv.add(struct.pack("<i", i), None))
    n3 = mr2.scrunch(1, "all")
    return n1, local_after_gather, n2, local_after_bcast, keys, n3, mr2.kmv.nval


def test_gather_broadcast_scrunch():
    out = run_world("case_gather_bcast", 3)
    for r, (n1, lg, n2, lb, keys, n3, nv) in out.items():
        assert n1 == 15
        assert lg == (15 if r == 0 else 0)
        assert n2 == 45 and lb == 15
        assert keys == sorted(i * 100 + j for i in range(3) for j in range(5))
        assert n3 == 3  # collapse makes one KMV pair per rank, even empty ones (reference semantics)
        assert nv == (6 if r == 0 else 0)


def case_mapstyle2(comm):
    import gpu_mapreduce_amd as g
    mr = g.MapReduce(comm)
    mr.mapstyle = 2
    mine = []
    n = mr.map(40, lambda i, kv: (mine.append(i), kv.add(struct.pack("<i", i), None)))
    return n, mine


def test_mapstyle_dynamic_queue():
    out = run_world("case_mapstyle2", 2)
    allt = sorted(t for _, (n, mine) in out.items() for t in mine)
    assert allt == list(range(40))
    assert all(n == 40 for n, _ in out.values())


def case_inverted_index(comm):
    import gpu_mapreduce_amd as g
    from gpu_mapreduce_amd.models.inverted_index import InvertedIndex, reference_inverted_index
    from gpu_mapreduce_amd.utils import synth
    files = synth.html_corpus(600_000, file_bytes=200_000, seed=11, rank=comm.rank, nurl=3000)
    app = InvertedIndex(g.MapReduce(comm), files)
    app.run()
    got = {}
    for line in app.output_lines():
        url, rest = line.split("\t")
        got[url] = rest.split()
    ref = reference_inverted_index(files)
    return got, {k.decode(): v for k, v in ref.items()}


def case_wordfreq_shuffle(comm):
    """wordfreq without the combiner (a (word, NULL) pair per occurrence
    through the hash-partition exchange and the group-by of each round), and
    the same pairs collated + counted with every count returned"""
    import gpu_mapreduce_amd as g
    from gpu_mapreduce_amd import C
    from gpu_mapreduce_amd.models.wordfreq import WordFreq
    from gpu_mapreduce_amd.utils import synth
    dev = comm.device
    chunks = [synth.zipf_text(700_000, seed=900 + 10 * comm.rank + i, device="cpu") for i in range(2)]
    app = WordFreq(g.MapReduce(comm), chunks, ntop=10, combiner=False)
    nwords = app.run()
    mr = g.MapReduce(comm)

    def fn(itask, kv):
        for c in chunks:
            buf = torch.zeros(c.numel() + 64, dtype=torch.uint8, device=dev)
            buf[: c.numel()].copy_(c)
            kv.add_kv(C.map_words(buf, c.numel()))
    mr.map(comm.size, fn)
    mr.collate()
    mr.reduce("count")
    local = {k.rstrip(b"\0"): struct.unpack("<i", v)[0] for k, v in mr.kv_pairs()}
    text = [bytes(c.numpy()) for c in chunks]
    return nwords, app.nunique, app.top, local, text


def _check_wordfreq_shuffle(out):
    cnt = collections.Counter()
    for _, (_, _, _, _, text) in out.items():
        for t in text:
            cnt.update(t.split())
    total = {}
    for r, (nwords, nunique, top, local, _) in out.items():
        assert nwords == sum(cnt.values()) and nunique == len(cnt)
        assert not (set(total) & set(local)), "word owned by two ranks"
        total.update(local)
    assert total == dict(cnt)
    top = out[0][2]
    want = sorted(cnt.values(), reverse=True)[:10]
    assert [c for _, c in top] == want
    assert all(cnt[w.encode()] == c for w, c in top)


@pytest.mark.parametrize("world", [2, 3])
def test_wordfreq_shuffle_distributed(world):
    _check_wordfreq_shuffle(run_world("case_wordfreq_shuffle", world))


def case_max_msg_mismatch(comm):
    """every rank asks for a different point-to-point piece size; the
    communicator must agree on rank 0's, and a shuffle whose per-peer bytes
    span many pieces must still deliver every pair exactly once"""
    import gpu_mapreduce_amd as g
    os.environ["MRH_RCCL_MAX_MSG"] = str(4096 if comm.rank == 0 else 1_000_000 + 7 * comm.rank)
    nc = comm.native  # built now, from this environment
    n = 40_000
    keys = torch.arange(comm.rank * n, (comm.rank + 1) * n, dtype=torch.int64)
    mr = g.MapReduce(comm)
    mr.map(comm.size, lambda i, kv: kv.add_tensors(keys.to(comm.device), keys.to(comm.device) * 3))
    mr.aggregate()
    got = sorted((struct.unpack("<q", k)[0], struct.unpack("<q", v)[0]) for k, v in mr.kv_pairs())
    return nc.max_msg, got


@pytest.mark.parametrize("world", [2, 3])
def test_max_msg_agreed_across_ranks(world):
    out = run_world("case_max_msg_mismatch", world)
    assert {m for m, _ in out.values()} == {4096}
    allp = sorted(p for _, got in out.values() for p in got)
    assert allp == [(k, 3 * k) for k in range(world * 40_000)]


def case_pagerank(comm):
    import numpy as np
    import gpu_mapreduce_amd as g
    from gpu_mapreduce_amd.models.pagerank import PageRank, rmat_map
    mr = g.MapReduce(comm)
    rmat_map(mr, 9, 8, seed=5)
    edges = mr.kv.kdata.view(torch.int64).view(-1, 2).cpu().numpy().copy()
    pr = PageRank(mr, 1 << 9).build()
    pr.run(12)
    ids, r = pr.ranks()
    return edges, ids.cpu().numpy(), r.cpu().numpy().copy()


def case_pagerank_ranges(comm):
    """RMAT-14 with the XCD source ranges forced on (tiny L2 budget): on
    device engines the replicated-c multi-GPU plan (graphplan.cpp
    build_device_dist) with several layers of ranges"""
    import numpy as np
    import gpu_mapreduce_amd as g
    from gpu_mapreduce_amd.models.pagerank import PageRank, rmat_map
    os.environ["MRH_PR_L2_BYTES"] = "4096"
    mr = g.MapReduce(comm)
    rmat_map(mr, 14, 16, seed=9)
    edges = mr.kv.kdata.view(torch.int64).view(-1, 2).cpu().numpy().copy()
    pr = PageRank(mr, 1 << 14).build()
    pr.run(15)
    ids, r = pr.ranks()
    return (edges, ids.cpu().numpy(), r.cpu().numpy().copy(), pr.layout, pr.xcd_ranges, pr.nedge, pr.overlapped,
            pr.comm_bytes_per_iter, pr.c_slice)


@pytest.mark.parametrize("world", [2, 3])
def test_pagerank_distributed(world):
    import numpy as np
    from gpu_mapreduce_amd.models.pagerank import reference_pagerank
    out = run_world("case_pagerank", world)
    edges = np.concatenate([out[r][0] for r in range(world)])
    ref = reference_pagerank(edges, 1 << 9, iters=12)
    got = np.zeros(1 << 9)
    for r in range(world):
        got[out[r][1]] = out[r][2]
    np.testing.assert_allclose(got, ref, rtol=2e-4, atol=1e-9)


def test_inverted_index_distributed():
    out = run_world("case_inverted_index", 2)
    got, ref = {}, collections.defaultdict(list)
    for r, (g_r, ref_r) in out.items():
        assert not (set(got) & set(g_r))
        got.update(g_r)
        for k, v in ref_r.items():
            ref[k].extend(v)
    assert {k: sorted(v) for k, v in got.items()} == {k: sorted(v) for k, v in ref.items()}


OINK_SCRIPT = """rmat 8 4 0.25 0.25 0.25 0.25 0.0 12345 -o tmp.rmat mre
edge_upper -i mre -o NULL mre
tri_find -i mre -o tmp.tri NULL
cc_find 0 -i mre -o tmp.cc mrc
cc_stats -i mrc
luby_find 7 -i mre -o tmp.mis NULL
degree_stats 0 -i mre
pagerank 0.0 8 0.85 -i mre -o tmp.pr NULL
"""


def oink_graph(comm):
    import io
    from gpu_mapreduce_amd.oink.interp import OINK
    os.chdir(os.environ["OINK_TEST_DIR"])
    out = io.StringIO()
    o = OINK(comm, screen=out, logfile="none")
    o.file(text=OINK_SCRIPT)
    return out.getvalue()


def _oink_files(d, stem):
    lines = []
    for f in sorted(os.listdir(d)):
        if f.startswith(stem + "."):
            lines += open(os.path.join(d, f)).read().split("\n")
    return sorted(ln for ln in lines if ln)


def test_oink_graph_commands_distributed(tmp_path, monkeypatch):
    import io
    from gpu_mapreduce_amd.oink.interp import OINK
    d1, d2 = tmp_path / "p1", tmp_path / "p2"
    d1.mkdir()
    d2.mkdir()
    monkeypatch.chdir(d1)
    out1 = io.StringIO()
    OINK(screen=out1, logfile="none").file(text=OINK_SCRIPT)
    monkeypatch.setenv("OINK_TEST_DIR", str(d2))
    res = run_world("oink_graph", 2)
    text1, text2 = out1.getvalue(), res[0]

    def counts(t):
        keep = ("Tri_find", "CC_find", "CCStats", "Luby_find", "  ", "EdgeUpper", "RMAT:")
        return [ln.split(" in ")[0] for ln in t.splitlines() if ln.startswith(keep)]
    assert counts(text1) == counts(text2)
    for stem in ("tmp.rmat", "tmp.tri", "tmp.cc", "tmp.mis"):
        assert _oink_files(d1, stem) == _oink_files(d2, stem), stem
    p1 = dict(ln.split() for ln in _oink_files(d1, "tmp.pr"))
    p2 = dict(ln.split() for ln in _oink_files(d2, "tmp.pr"))
    assert p1.keys() == p2.keys()
    for k in p1:
        assert abs(float(p1[k]) - float(p2[k])) <= 1e-5 * abs(float(p1[k])) + 1e-9


# the reference's MapReduce formulations of sssp and luby_find
# (oink/sssp.cpp:88-152, oink/luby_find.cpp:53-97): aggregate, cross-MR
# appends (open(1)/kv_open/close), compress as the combiner and the
# all-rank termination counts, at 2 ranks against 1
OINK_MR_SCRIPT = """rmat 8 4 0.25 0.25 0.25 0.25 0.0 4242 -o NULL mre
edge_upper -i mre -o NULL mre
luby_find_mr 99 -i mre -o tmp.mis NULL
mre map/mr mre add_weight
sssp_mr 2 31 -i mre -o tmp.sssp NULL
"""


def oink_graph_mr(comm):
    import io
    from gpu_mapreduce_amd.oink.interp import OINK
    os.chdir(os.environ["OINK_TEST_DIR"])
    out = io.StringIO()
    OINK(comm, screen=out, logfile="none").file(text=OINK_MR_SCRIPT)
    return out.getvalue()


def test_oink_graph_mr_commands_distributed(tmp_path, monkeypatch):
    import io
    import re
    from gpu_mapreduce_amd.oink.interp import OINK
    d1, d2 = tmp_path / "p1", tmp_path / "p2"
    d1.mkdir()
    d2.mkdir()
    monkeypatch.chdir(d1)
    out1 = io.StringIO()
    OINK(screen=out1, logfile="none").file(text=OINK_MR_SCRIPT)
    monkeypatch.setenv("OINK_TEST_DIR", str(d2))
    text1, text2 = out1.getvalue(), run_world("oink_graph_mr", 2)[0]
    pat = r"(Luby_find: \d+ MIS vertices in \d+ iterations|Source = \d+; Iterations = \d+; Num Vtx Labeled = \d+)"
    assert re.findall(pat, text1) == re.findall(pat, text2) and len(re.findall(pat, text1)) == 3
    assert _oink_files(d1, "tmp.mis") == _oink_files(d2, "tmp.mis")
    s1 = sorted(tuple(ln.split()[:2]) for ln in _oink_files(d1, "tmp.sssp"))
    s2 = sorted(tuple(ln.split()[:2]) for ln in _oink_files(d2, "tmp.sssp"))
    assert s1 == s2 and len(s1) > 100
