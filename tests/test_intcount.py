"""IntCount app (reference cpu/IntCount.cpp) vs a numpy bincount oracle."""
import pytest
import torch

import gpu_mapreduce_amd as g
from gpu_mapreduce_amd.models.intcount import IntCount, int_file, reference_counts


def _run(device, nbytes=400_000, key_range=5000):
    data = int_file(nbytes, key_range, seed=3)
    app = IntCount(g.MapReduce(g.Comm(device=device)), data)
    n = app.run()
    k, c = app.counts()
    return n, app.nunique, dict(zip(k.tolist(), c.tolist())), reference_counts([data])


def test_intcount_cpu():
    n, nu, got, ref = _run("cpu")
    assert n == 100_000
    assert nu == len(ref)
    assert got == ref


@pytest.mark.gpu
def test_intcount_gpu():
    n, nu, got, ref = _run("cuda:0", nbytes=4 << 20, key_range=1 << 16)
    assert n == 1 << 20
    assert got == ref


def case_intcount(comm):
    from gpu_mapreduce_amd.models.intcount import IntCount, int_file
    data = int_file(80_000, 3000, seed=9, rank=comm.rank)
    app = IntCount(g.MapReduce(comm), data)
    n = app.run()
    k, c = app.counts()
    return n, dict(zip(k.tolist(), c.tolist())), data.numpy().copy()


def test_intcount_distributed():
    from test_distributed_cpu import run_world
    out = run_world("test_intcount:case_intcount", 2)
    got = {}
    for n, d, _ in out.values():
        assert n == 40_000
        assert not (set(got) & set(d))
        got.update(d)
    assert got == reference_counts([torch.from_numpy(out[r][2]) for r in range(2)])
