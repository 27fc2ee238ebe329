"""Property tests of the core MapReduce ops against plain-Python oracles
(SURVEY.md §4 plan, items 2-3: op-level differential tests with variable
keys, empty keys, keys containing NUL bytes, duplicate-heavy and
all-distinct inputs). Random inputs come from hypothesis; the same
properties run on the MI355X device engine under the gpu marker."""
import collections
import struct

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import gpu_mapreduce_amd as g

keys_st = st.lists(st.binary(min_size=0, max_size=14), min_size=0, max_size=300)
ints_st = st.lists(st.integers(min_value=-2 ** 31, max_value=2 ** 31 - 1), min_size=1, max_size=400)


def _mr(dev):
    return g.MapReduce(g.Comm(device=dev))


def _load(mr, pairs):
    def gen(i, kv):
        for k, v in pairs[i::3]:
            kv.add(k, v)
    return mr.map(3, gen)


def check_convert(dev, keys):
    pairs = [(k, struct.pack("<i", i)) for i, k in enumerate(keys)]
    mr = _mr(dev)
    assert _load(mr, pairs) == len(pairs)
    groups = collections.defaultdict(list)
    for k, v in pairs:
        groups[k].append(v)
    assert mr.convert() == len(groups)
    got = {k: sorted(vs) for k, vs in mr.kmv_pairs()}
    assert got == {k: sorted(vs) for k, vs in groups.items()}


def check_reduce_count_sum(dev, keys):
    pairs = [(k, struct.pack("<i", len(k) * 7 - 3)) for k in keys]
    mr = _mr(dev)
    _load(mr, pairs)
    mr.convert()
    c = mr.copy()
    mr.reduce("count")
    c.reduce("sum:int32")
    cnt = collections.Counter(k for k, _ in pairs)
    tot = collections.Counter()
    for k, v in pairs:
        tot[k] += struct.unpack("<i", v)[0]
    assert {k: struct.unpack("<i", v)[0] for k, v in mr.kv_pairs()} == dict(cnt)
    assert {k: struct.unpack("<i", v)[0] for k, v in c.kv_pairs()} == dict(tot)


def check_sort_int_values(dev, vals):
    pairs = [(struct.pack("<i", i), struct.pack("<i", v)) for i, v in enumerate(vals)]
    for flag in (1, -1):
        mr = _mr(dev)
        _load(mr, pairs)
        mr.sort_values(flag)
        got = [struct.unpack("<i", v)[0] for _, v in mr.kv_pairs()]
        assert got == sorted(vals, reverse=flag < 0)


def check_sort_string_keys(dev, keys):
    # MR-MPI flag 5 compares keys as C strings (strcmp, src/mapreduce.cpp:2770):
    # NUL-terminated words without embedded NULs
    words = [k.replace(b"\0", b"") + b"\0" for k in keys]
    pairs = [(w, b"") for w in words]
    for flag in (5, -5):
        mr = _mr(dev)
        _load(mr, pairs)
        mr.sort_keys(flag)
        got = [k for k, _ in mr.kv_pairs()]
        assert got == sorted(words, reverse=flag < 0)


CPU = settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])
GPU = settings(max_examples=12, deadline=None, suppress_health_check=[HealthCheck.too_slow])


@CPU
@given(keys_st)
def test_convert_groups_cpu(keys):
    check_convert("cpu", keys)


@CPU
@given(keys_st)
def test_reduce_count_sum_cpu(keys):
    check_reduce_count_sum("cpu", keys)


@CPU
@given(ints_st)
def test_sort_values_int_cpu(vals):
    check_sort_int_values("cpu", vals)


@CPU
@given(keys_st)
def test_sort_keys_str_cpu(keys):
    check_sort_string_keys("cpu", keys)


@pytest.mark.gpu
@GPU
@given(keys_st)
def test_convert_groups_gpu(keys):
    check_convert("cuda", keys)


@pytest.mark.gpu
@GPU
@given(keys_st)
def test_reduce_count_sum_gpu(keys):
    check_reduce_count_sum("cuda", keys)


@pytest.mark.gpu
@GPU
@given(ints_st)
def test_sort_values_int_gpu(vals):
    check_sort_int_values("cuda", vals)


@pytest.mark.gpu
@GPU
@given(keys_st)
def test_sort_keys_str_gpu(keys):
    check_sort_string_keys("cuda", keys)
