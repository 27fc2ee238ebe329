"""Reference-style `mrmpi` Python interface (pickled keys/values) on the
native engine: examples/python/wordfreq.py and per-op semantics."""
import collections
import os
import runpy
import sys

from gpu_mapreduce_amd.mrmpi import mrmpi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_wordfreq_example(tmp_path, capsys):
    words = "the quick brown fox jumps over the lazy dog the end fox".split()
    (tmp_path / "a.txt").write_text(" ".join(words[:6]))
    (tmp_path / "b.txt").write_text(" ".join(words[6:]))
    mod = runpy.run_path(os.path.join(ROOT, "examples", "python", "wordfreq.py"))
    nwords, nunique, top = mod["main"]([str(tmp_path)], ntop=2)
    cnt = collections.Counter(words)
    assert nwords == len(words) and nunique == len(cnt)
    assert top[0] == ("the", 3) and top[1] == ("fox", 2)


def test_mrmpi_ops():
    mr = mrmpi()

    def gen(itask, m, ptr):
        for i in range(ptr):
            m.add(("k", i % 3), {"i": i})
    assert mr.map(2, gen, 5) == 10
    assert mr.collate() == 3
    seen = {}

    def red(key, mvalue, m):
        seen[key] = sorted(v["i"] for v in mvalue)
        m.add(key, sum(v["i"] for v in mvalue))
    assert mr.reduce(red) == 3
    assert seen[("k", 0)] == [0, 0, 3, 3]
    assert sorted(mr.pairs()) == [(("k", 0), 6), (("k", 1), 10), (("k", 2), 4)]
    mr.sort_keys(lambda a, b: (a > b) - (a < b))
    assert [k for k, _ in mr.pairs()] == [("k", 0), ("k", 1), ("k", 2)]
    other = mr.copy()
    assert mr.add(other) == 6
    got = []
    mr.scan_kv(lambda k, v: got.append(v))
    assert sorted(got) == [4, 4, 6, 6, 10, 10]


def test_rmat_python_example():
    """examples/python/rmat.py (reference examples/rmat.py) on the CPU engine"""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "rmat_example", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples",
                                     "python", "rmat.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    order, ntotal, histo = mod.main(["8", "4", "0.57", "0.19", "0.19", "0.05", "0.1", "3"])
    assert (order, ntotal) == (256, 1024)
    assert sum(k * v for k, v in histo) == ntotal
