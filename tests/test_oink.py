"""OINK scripting layer + graph commands on the CPU engine (reference
examples/in.rmat, in.tri, in.cc, in.luby, in.sssp, in.wordfreq at reduced
scale; checked against brute-force numpy/scipy oracles, since the
reference ships no expected outputs for them)."""
import io
import os

import numpy as np
import pytest
import torch

from gpu_mapreduce_amd.oink.interp import OINK
from gpu_mapreduce_amd.oink.interp import OinkError


def run(script, tmp_path, monkeypatch, variables=None, comm=None):
    monkeypatch.chdir(tmp_path)
    out = io.StringIO()
    o = OINK(comm, screen=out, logfile="log.oink", variables=variables)
    o.file(text=script)
    return o, out.getvalue()


def load_edges(path):
    a = np.loadtxt(path, dtype=np.uint64, ndmin=2)
    return a.reshape(-1, 2).astype(np.int64)


RMAT = "rmat 8 4 0.25 0.25 0.25 0.25 0.0 12345 -o {out} mre\n"


def test_rmat_degree_stats(tmp_path, monkeypatch):
    s = RMAT.format(out="tmp.rmat") + "degree_stats 1 -i mre\ndegree 0 -i mre -o tmp.deg NULL\n"
    o, text = run(s, tmp_path, monkeypatch)
    e = load_edges(tmp_path / "tmp.rmat.0")
    assert len(e) == 256 * 4
    assert len({(a, b) for a, b in e}) == len(e)
    assert e.max() < 256
    assert "RMAT: 256 rows, 1024 non-zeroes" in text
    # degree_stats histogram over out-degrees
    deg = np.bincount(e[:, 0])
    deg = deg[deg > 0]
    vals, cnts = np.unique(deg, return_counts=True)
    for v, c in zip(vals, cnts):
        assert f"  {c} vertices with {v} edges" in text
    d = np.loadtxt(tmp_path / "tmp.deg.0", dtype=np.int64, ndmin=2)
    full = np.bincount(np.concatenate([e[:, 0], e[:, 1]]))
    assert dict(zip(d[:, 0], d[:, 1])) == {i: int(x) for i, x in enumerate(full) if x}


def test_rmat2_matches_count(tmp_path, monkeypatch):
    s = "rmat2 7 3 0.57 0.19 0.19 0.05 0.1 7 -o tmp.r2 mre\n"
    o, text = run(s, tmp_path, monkeypatch)
    e = load_edges(tmp_path / "tmp.r2.0")
    assert len(e) == 128 * 3 and len({(a, b) for a, b in e}) == len(e)


def _upper(e):
    lo, hi = np.minimum(e[:, 0], e[:, 1]), np.maximum(e[:, 0], e[:, 1])
    k = lo != hi
    return np.unique(np.stack([lo[k], hi[k]], 1), axis=0)


def test_edge_upper_tri_find(tmp_path, monkeypatch):
    s = (RMAT.format(out="tmp.rmat") + "edge_upper -i mre -o tmp.up mre\n"
         "tri_find -i mre -o tmp.tri mrt\n")
    o, text = run(s, tmp_path, monkeypatch)
    e = load_edges(tmp_path / "tmp.rmat.0")
    up = _upper(e)
    got = load_edges(tmp_path / "tmp.up.0")
    assert np.array_equal(np.unique(got, axis=0), up)
    n = int(e.max()) + 1
    A = np.zeros((n, n), dtype=np.int64)
    A[up[:, 0], up[:, 1]] = 1
    A = A + A.T
    ntri = int(np.trace(A @ A @ A) // 6)
    assert f"Tri_find: {ntri} triangles" in text
    t = np.loadtxt(tmp_path / "tmp.tri.0", dtype=np.int64, ndmin=2).reshape(-1, 3)
    assert len(t) == ntri
    ts = {tuple(sorted(r)) for r in t}
    assert len(ts) == ntri
    for a, b, c in ts:
        assert A[a, b] and A[b, c] and A[a, c]


def test_cc_find_stats(tmp_path, monkeypatch):
    from gpu_mapreduce_amd.models.graph import reference_cc
    s = ("rmat 8 1 0.25 0.25 0.25 0.25 0.0 99 -o tmp.rmat mre\n"
         "edge_upper -i mre -o NULL mre\n"
         "cc_find 0 -i mre -o tmp.cc mrc\n"
         "cc_stats -i mrc\n")
    o, text = run(s, tmp_path, monkeypatch)
    e = _upper(load_edges(tmp_path / "tmp.rmat.0"))
    n = int(e.max()) + 1
    lab = reference_cc(e, n)
    present = np.zeros(n, bool)
    present[e.ravel()] = True
    got = np.loadtxt(tmp_path / "tmp.cc.0", dtype=np.int64, ndmin=2)
    gd = dict(zip(got[:, 0], got[:, 1]))
    assert set(gd) == set(np.nonzero(present)[0])
    for v in gd:
        assert gd[v] == lab[v]
    ncc = len(set(lab[present]))
    assert f"CC_find: {ncc} components" in text
    assert f"CCStats: {ncc} components, {present.sum()} vertices" in text


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("nthresh", [1000000, 2])
def test_cc_find_mr_zone_salting(tmp_path, monkeypatch, nthresh, dev):
    """cc_find_mr: the reference's zone pipeline (oink/cc_find.cpp:38-109),
    callbacks as the ccmr kernels on cuda / their host twins on cpu. With
    nthresh = 2 nearly every zone becomes 'hot' and its vertices are salted
    over ranks; the components must not change."""
    from gpu_mapreduce_amd.models.graph import reference_cc
    from gpu_mapreduce_amd.parallel.comm import Comm
    scale = 8 if dev == "cpu" else 12
    s = (f"rmat {scale} 1 0.25 0.25 0.25 0.25 0.0 99 -o tmp.rmat mre\n"
         "edge_upper -i mre -o NULL mre\n"
         f"cc_find_mr {nthresh} -i mre -o tmp.ccmr mrc\n"
         "cc_stats -i mrc\n")
    o, text = run(s, tmp_path, monkeypatch, comm=Comm(device=dev))
    e = _upper(load_edges(tmp_path / "tmp.rmat.0"))
    n = int(e.max()) + 1
    lab = reference_cc(e, n)
    got = np.loadtxt(tmp_path / "tmp.ccmr.0", dtype=np.int64, ndmin=2)
    gd = dict(zip(got[:, 0], got[:, 1]))
    present = np.zeros(n, bool)
    present[e.ravel()] = True
    assert set(gd) == set(np.nonzero(present)[0])
    for v in gd:
        assert gd[v] == lab[v]
    ncc = len(set(lab[present]))
    assert f"CC_find: {ncc} components" in text


def test_luby_find(tmp_path, monkeypatch):
    s = (RMAT.format(out="tmp.rmat") + "edge_upper -i mre -o NULL mre\n"
         "luby_find 12345 -i mre -o tmp.mis NULL\n")
    o, text = run(s, tmp_path, monkeypatch)
    e = _upper(load_edges(tmp_path / "tmp.rmat.0"))
    mis = set(np.loadtxt(tmp_path / "tmp.mis.0", dtype=np.int64, ndmin=1).tolist())
    assert f"Luby_find: {len(mis)} MIS vertices" in text
    nbrs = {}
    for a, b in e:
        nbrs.setdefault(a, set()).add(b)
        nbrs.setdefault(b, set()).add(a)
    for a, b in e:                                   # independent
        assert not (a in mis and b in mis)
    for v, nb in nbrs.items():                       # maximal
        assert v in mis or nb & mis


def test_sssp(tmp_path, monkeypatch):
    """distances match Dijkstra, and the third column is the predecessor as the
    reference prints it (oink/sssp.cpp:405-411): 0 for the source, otherwise a
    u with an edge u -> v and d[u] + w == d[v] (the smallest such u: our
    deterministic tie-break)."""
    import re
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import dijkstra
    s = ("rmat 5 3 0.25 0.25 0.25 0.25 0.0 12345 -o tmp.rmat mre\n"
         "mre map/mr mre add_weight\n"
         "sssp 3 12345 -i mre -o tmp.sssp NULL\n")
    o, text = run(s, tmp_path, monkeypatch)
    e = load_edges(tmp_path / "tmp.rmat.0")
    n = int(e.max()) + 1
    G = csr_matrix((np.ones(len(e)), (e[:, 0], e[:, 1])), shape=(n, n))
    rows = np.loadtxt(tmp_path / "tmp.sssp.0", ndmin=2)
    blocks = [(int(a), int(b)) for a, b in re.findall(r"Source = (\d+); Iterations = \d+; Num Vtx Labeled = (\d+)", text)]
    assert len(blocks) == 3 and sum(b for _, b in blocks) == len(rows)
    inn = {}
    for a, b in e:
        inn.setdefault(int(b), set()).add(int(a))
    start = 0
    for sidx, cnt in blocks:
        r = rows[start:start + cnt]
        start += cnt
        d = dijkstra(G, indices=sidx)
        got = dict(zip(r[:, 0].astype(np.int64), r[:, 1]))
        want = {i: d[i] for i in range(n) if np.isfinite(d[i])}
        assert got.keys() == want.keys()
        for k in got:
            assert got[k] == pytest.approx(want[k])
        for v, dv, pv in zip(r[:, 0].astype(np.int64), r[:, 1], r[:, 2].astype(np.int64)):
            if v == sidx:
                assert pv == 0 and dv == 0
                continue
            cands = sorted(u for u in inn.get(int(v), ()) if np.isfinite(d[u]) and d[u] + 1 == d[v])
            assert cands and pv == cands[0], (v, pv, cands)


def test_wordfreq_histo(tmp_path, monkeypatch):
    files = []
    rng = np.random.default_rng(3)
    words = ["alpha", "beta", "gamma", "delta", "eps"]
    allw = []
    for i in range(3):
        w = [words[j] for j in rng.zipf(1.5, 200) % 5]
        allw += w
        p = tmp_path / f"f{i}.txt"
        p.write_text(" ".join(w) + "\n")
        files.append(str(p))
    s = ("wordfreq 3 -i v_files -o tmp.wf mrw\n"
         "histo -i mrw -o NULL NULL\n")
    o, text = run(s, tmp_path, monkeypatch, variables=[("files", files)])
    uniq, cnt = np.unique(allw, return_counts=True)
    assert f"WordFreq: 3 files, {len(allw)} words, {len(uniq)} unique" in text
    got = {}
    for line in open(tmp_path / "tmp.wf.0"):
        w, c = line.split()
        got[w] = int(c)
    assert got == dict(zip(uniq.tolist(), cnt.tolist()))
    top = sorted(cnt.tolist(), reverse=True)[:3]
    assert top[0] == max(cnt)


def test_pagerank_command(tmp_path, monkeypatch):
    from gpu_mapreduce_amd.models.pagerank import reference_pagerank
    s = (RMAT.format(out="tmp.rmat") + "pagerank 0.0 10 0.85 -i mre -o tmp.pr NULL\n")
    o, text = run(s, tmp_path, monkeypatch)
    e = load_edges(tmp_path / "tmp.rmat.0")
    n = int(e.max()) + 1
    ref = reference_pagerank(e, n, 0.85, 10)
    got = np.loadtxt(tmp_path / "tmp.pr.0", ndmin=2)
    r = np.zeros(n)
    r[got[:, 0].astype(np.int64)] = got[:, 1]
    assert np.allclose(r, ref, rtol=1e-4, atol=1e-7)


def test_neighbor_neigh_tri_vertex_extract(tmp_path, monkeypatch):
    s = ("rmat 6 3 0.25 0.25 0.25 0.25 0.0 5 -o tmp.rmat mre\n"
         "edge_upper -i mre -o NULL mre\n"
         "neighbor -i mre -o tmp.nb mrn\n"
         "tri_find -i mre -o NULL mrt\n"
         "neigh_tri nt -i mrn mrt -o NULL NULL\n"
         "vertex_extract -i mre -o tmp.vx NULL\n")
    o, text = run(s, tmp_path, monkeypatch)
    e = _upper(load_edges(tmp_path / "tmp.rmat.0"))
    nb = {}
    for a, b in e:
        nb.setdefault(a, set()).add(b)
        nb.setdefault(b, set()).add(a)
    got = {}
    for line in open(tmp_path / "tmp.nb.0"):
        t = [int(x) for x in line.split()]
        got[t[0]] = set(t[1:])
    assert got == nb
    vx = set(np.loadtxt(tmp_path / "tmp.vx.0", dtype=np.int64, ndmin=1).tolist())
    assert vx == set(nb)
    for v in list(nb)[:5]:
        lines = open(tmp_path / "nt" / str(v)).read().split("\n")
        assert sum(1 for ln in lines if ln.startswith(f"{v} ")) >= len(nb[v])


def test_script_control_flow(tmp_path, monkeypatch):
    s = ("variable a loop 3\n"
         "label top\n"
         "print \"iter $a\"\n"
         "next a\n"
         "jump SELF top\n")
    p = tmp_path / "in.loop"
    p.write_text(s)
    monkeypatch.chdir(tmp_path)
    out = io.StringIO()
    o = OINK(screen=out, logfile="none")
    o.file(str(p))
    assert [ln for ln in out.getvalue().splitlines() if ln.startswith("iter")] == ["iter 1", "iter 2", "iter 3"]


def test_script_if_equal_variables(tmp_path, monkeypatch):
    s = ("variable x equal 2*3+1\n"
         "variable p equal nprocs\n"
         "if \"$x > 5\" then \"print big\" else \"print small\"\n"
         "print \"x=$x p=$p v=${x}\"\n")
    o, text = run(s, tmp_path, monkeypatch)
    assert "big" in text and "x=7 p=1 v=7" in text


def test_named_mr_methods(tmp_path, monkeypatch):
    s = (RMAT.format(out="NULL") +
         "mr mv\n"
         "mv map/mr mre edge_to_vertices\n"
         "mv collate NULL\n"
         "mv reduce count\n"
         "histo -i mv -o NULL NULL\n")
    o, text = run(s, tmp_path, monkeypatch)
    assert "Histo:" in text


def test_bad_command_raises(tmp_path, monkeypatch):
    with pytest.raises(OinkError):
        run("frobnicate 1 2\n", tmp_path, monkeypatch)
    with pytest.raises(OinkError):
        run("rmat 8 4 0.5 0.5 0.5 0.5 0.0 1 -o NULL m\n", tmp_path, monkeypatch)
