"""String sorts (flags +-5 / +-6) with long shared prefixes: the first radix
pass only sees 8 bytes ("http://w" for every URL), so everything past it is the
tie-break. On the device engine the tie-break runs as device rounds of
(next 8-byte window, group id) radix sorts (engine.cpp str_tiebreak_device);
the CPU engine resolves tie groups with strcmp. Oracle: Python's stable sort
on the bytes up to the first NUL (reference compare_str / compare_strn,
src/mapreduce.cpp:2780-2803 — both compare up to the terminator)."""
import random
import struct

import pytest

import gpu_mapreduce_amd as g
from gpu_mapreduce_amd import MapReduce


def _urls(n, seed=3):
    rnd = random.Random(seed)
    hosts = [b"http://www.%s.org/" % bytes(rnd.choice(b"abcdefgh") for _ in range(rnd.randint(1, 4)))
             for _ in range(40)]
    out = []
    for i in range(n):
        h = rnd.choice(hosts)
        path = b"/".join(bytes(rnd.choice(b"abcxyz") for _ in range(rnd.randint(0, 6))) for _ in range(rnd.randint(0, 4)))
        u = h + path
        if i % 97 == 0:
            u = u + b"\0trailing-junk%d" % i     # bytes after a NUL do not count
        if i % 13 == 0 and out:
            u = out[rnd.randrange(len(out))]     # exact duplicates: ties must stay stable
        out.append(u)
    return out


def _cmpkey(b):
    z = b.find(b"\0")
    return b if z < 0 else b[:z]


def _run(dev, n, flag, by_value):
    urls = _urls(n)
    mr = MapReduce(g.Comm(device=dev))
    if by_value:
        mr.map(1, lambda i, kv: [kv.add(struct.pack("<i", j), u) for j, u in enumerate(urls)])
        mr.sort_values(flag)
        got = [(v, struct.unpack("<i", k)[0]) for k, v in mr.kv_pairs()]
    else:
        mr.map(1, lambda i, kv: [kv.add(u, struct.pack("<i", j)) for j, u in enumerate(urls)])
        mr.sort_keys(flag)
        got = [(k, struct.unpack("<i", v)[0]) for k, v in mr.kv_pairs()]
    want = sorted(((u, j) for j, u in enumerate(urls)), key=lambda t: _cmpkey(t[0]), reverse=flag < 0)
    assert got == want


@pytest.mark.parametrize("flag", [5, -5, 6, -6])
def test_string_sort_cpu(flag):
    _run("cpu", 20000, flag, False)


def test_string_sort_values_cpu():
    _run("cpu", 20000, -5, True)


@pytest.mark.gpu
@pytest.mark.parametrize("flag", [5, -5, 6, -6])
def test_string_sort_gpu(flag):
    _run("cuda:0", 200000, flag, False)


@pytest.mark.gpu
def test_string_sort_values_gpu():
    _run("cuda:0", 100000, 5, True)
