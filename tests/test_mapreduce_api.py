"""MapReduce object semantics on the CPU engine (world size 1), checked
against plain-Python oracles. Mirrors the reference's example programs
(examples/wordfreq.cpp, oink pipelines) since the reference ships no tests."""
import collections
import os
import struct

import pytest
import torch

import gpu_mapreduce_amd as g
from gpu_mapreduce_amd import C, MapReduce


def mk():
    return MapReduce(g.Comm(device="cpu"))


def words_map(words):
    def fn(itask, kv):
        for w in words[itask::4]:
            kv.add(w)
    return fn


WORDS = ("the quick brown fox jumps over the lazy dog the end fox " * 7).split()


def test_hashlittle_vectors():
    # lookup3 driver5 test vectors (Bob Jenkins)
    kv = C.make_kv(torch.frombuffer(bytearray(b"Four score and seven years ago"), dtype=torch.uint8),
                   torch.tensor([0, 30]), torch.empty(0, dtype=torch.uint8), None, 1, "cpu")
    assert C.hash32_keys(kv, 0).view(torch.int32).numpy().astype("uint32")[0] == 0x17770551
    assert C.hash32_keys(kv, 1).numpy().astype("uint32")[0] == 0xcd628161
    e = C.make_kv(torch.empty(0, dtype=torch.uint8), torch.tensor([0, 0]), torch.empty(0, dtype=torch.uint8),
                  None, 1, "cpu")
    assert C.hash32_keys(e, 0).numpy().astype("uint32")[0] == 0xdeadbeef
    assert C.hash32_keys(e, 0xdeadbeef).numpy().astype("uint32")[0] == 0xbd5b7dde


def test_wordfreq_pipeline():
    mr = mk()
    n = mr.map(4, words_map(WORDS))
    assert n == len(WORDS)
    nu = mr.collate()
    cnt = collections.Counter(WORDS)
    assert nu == len(cnt)
    mr.reduce("count")
    mr.sort_values(-1)
    pairs = mr.kv_pairs()
    got = [(k[:-1].decode(), struct.unpack("<i", v)[0]) for k, v in pairs]
    assert dict(got) == dict(cnt)
    assert [c for _, c in got] == sorted(cnt.values(), reverse=True)


def test_host_reduce_callback_and_ptr():
    mr = mk()
    mr.map(4, words_map(WORDS))
    mr.collate()
    seen = {}

    def red(key, mv, kv, ptr):
        ptr[key] = len(mv)
        kv.add(key, struct.pack("<i", len(mv)))
    assert mr.reduce(red, seen) == len(set(WORDS))
    assert {k[:-1].decode(): v for k, v in seen.items()} == collections.Counter(WORDS)


def test_compress_then_collate_sum():
    mr = mk()
    mr.map(4, words_map(WORDS))
    mr.compress("count")
    # values are int32 counts now; collate + sum
    mr.collate()
    mr.reduce("sum:int32")
    got = {k[:-1].decode(): struct.unpack("<i", v)[0] for k, v in mr.kv_pairs()}
    assert got == collections.Counter(WORDS)


def test_clone_collapse_scan_print(capsys):
    mr = mk()
    mr.map(1, lambda i, kv: [kv.add(struct.pack("<i", j), struct.pack("<d", j * 0.5)) for j in range(5)])
    mr.clone()
    assert mr.kmv.nkey == 5 and mr.kmv.nval == 5
    out = []
    mr.scan_kmv(lambda k, vals: out.append((k, list(vals))))
    assert len(out) == 5 and all(len(v) == 1 for _, v in out)
    mr2 = mk()
    mr2.map(1, lambda i, kv: [kv.add(struct.pack("<i", j), struct.pack("<i", 10 * j)) for j in range(3)])
    mr2.collapse("all")
    (k, vals), = mr2.kmv_pairs()
    assert k == b"all\0"
    assert [struct.unpack("<i", v)[0] for v in vals] == [0, 0, 1, 10, 2, 20]
    mr2.print(-1, 1, 5, 1)
    assert "KMV pair: proc 0, nvalues 6" in capsys.readouterr().out


def test_add_copy_open_close():
    a = mk()
    a.map(1, lambda i, kv: [kv.add(b"k%d" % j, b"v") for j in range(10)])
    b = a.copy()
    assert b.add(a) == 20
    c = mk()
    kvo = c.open()
    a.map_mr(a, lambda i, k, v, kv: kvo.add(k, b"x"))
    assert c.close() == 10
    c.open(addflag=1)
    c.kv_open.add(b"extra", b"")
    assert c.close() == 11


def test_map_mr_and_sort_keys_callable():
    a = mk()
    a.map(1, lambda i, kv: [kv.add(struct.pack("<q", j), None) for j in (5, 3, 9, 1)])
    a.sort_keys(lambda x, y: (struct.unpack("<q", x)[0] > struct.unpack("<q", y)[0]) -
                (struct.unpack("<q", x)[0] < struct.unpack("<q", y)[0]))
    assert [struct.unpack("<q", k)[0] for k, _ in a.kv_pairs()] == [1, 3, 5, 9]
    a.sort_keys(-2)
    assert [struct.unpack("<q", k)[0] for k, _ in a.kv_pairs()] == [9, 5, 3, 1]
    b = mk()
    b.map_mr(a, lambda i, k, v, kv: kv.add(v, k))
    assert b.kv.n == 4


def test_sort_multivalues():
    mr = mk()
    mr.map(1, lambda i, kv: [kv.add(b"k%d" % (j % 3), struct.pack("<i", (j * 37) % 11)) for j in range(30)])
    mr.convert()
    mr.sort_multivalues(1)
    for k, vals in mr.kmv_pairs():
        xs = [struct.unpack("<i", v)[0] for v in vals]
        assert xs == sorted(xs)
    mr.sort_multivalues(-1)
    for k, vals in mr.kmv_pairs():
        xs = [struct.unpack("<i", v)[0] for v in vals]
        assert xs == sorted(xs, reverse=True)


def test_map_files_and_chunks(tmp_path):
    text = ("alpha beta gamma\n" * 500).encode()
    files = []
    for i in range(3):
        p = tmp_path / f"f{i}.txt"
        p.write_bytes(text)
        files.append(str(p))
    mr = mk()
    n = mr.map_file([str(tmp_path)], 0, 1, 0, lambda i, fname, kv: [kv.add(w) for w in open(fname).read().split()])
    assert n == 3 * 1500 and mr.mapfilecount == 3
    mr2 = mk()
    n2 = mr2.map_file_char(12, files, 0, 0, 0, "\n", 40, lambda i, chunk, kv: [kv.add(w) for w in chunk.split()])
    assert n2 == 3 * 1500
    mr3 = mk()
    n3 = mr3.map_file_str(7, files, 0, 0, 0, "gamma\n", 40,
                          lambda i, chunk, kv: [kv.add(w) for w in chunk.split()])
    assert n3 == 3 * 1500
    lst = tmp_path / "list.txt"
    lst.write_text("\n".join(files) + "\n")
    mr4 = mk()
    assert mr4.map_file([str(lst)], 0, 0, 1, lambda i, f, kv: kv.add(f)) == 3


def test_gather_broadcast_scrunch_single_rank():
    mr = mk()
    mr.map(2, lambda i, kv: kv.add(struct.pack("<i", i), b"v"))
    assert mr.gather(1) == 2
    assert mr.broadcast(0) == 2
    assert mr.scrunch(1, "key") == 1


def test_stats_output(capsys):
    mr = mk()
    mr.verbosity = 2
    mr.timer = 1
    mr.map(4, words_map(WORDS))
    mr.collate()
    mr.cummulative_stats(2, 0)
    out = capsys.readouterr().out
    assert "Map time (secs) =" in out and "Map KV = " in out and "KV pairs:" in out
    assert "Collate KMV = " in out and "Cummulative hi-water mem" in out


def test_tensor_fast_path_and_builtin_reduce():
    mr = mk()
    keys = torch.tensor([3, 1, 3, 2, 1, 3], dtype=torch.int64)
    vals = torch.tensor([1.0, 2.0, 3.0, 4.0, 5.0, 6.0], dtype=torch.float64)
    mr.map(1, lambda i, kv: kv.add_tensors(keys, vals))
    mr.convert()
    mr.reduce("sum:float64")
    got = {struct.unpack("<q", k)[0]: struct.unpack("<d", v)[0] for k, v in mr.kv_pairs()}
    assert got == {1: 7.0, 2: 4.0, 3: 10.0}
    # exact fixed-key group-by returns keys in sorted order
    assert list(got) == [1, 2, 3]


def test_mapstyle_stride_and_errors():
    mr = mk()
    mr.mapstyle = 1
    seen = []
    mr.map(5, lambda i, kv: seen.append(i))
    assert seen == [0, 1, 2, 3, 4]
    with pytest.raises(RuntimeError):
        mk().convert()
    with pytest.raises(RuntimeError):
        mk().reduce("count")
