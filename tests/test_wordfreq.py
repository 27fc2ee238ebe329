"""wordfreq app (reference examples/wordfreq.cpp) vs a Python Counter oracle."""
import collections

import pytest
import torch

import gpu_mapreduce_amd as g
from gpu_mapreduce_amd.models.wordfreq import WordFreq
from gpu_mapreduce_amd.utils import synth


def _oracle(chunks, ntop):
    c = collections.Counter()
    for t in chunks:
        c.update(bytes(t.cpu().numpy()).split())
    top = sorted(c.items(), key=lambda kv: -kv[1])
    return sum(c.values()), len(c), top[:ntop]


@pytest.mark.parametrize("combiner", [True, False])
def test_wordfreq_cpu(combiner):
    chunks = [synth.zipf_text(200_000, seed=s) for s in range(3)]
    app = WordFreq(g.MapReduce(g.Comm(device="cpu")), chunks, ntop=10, combiner=combiner)
    n = app.run()
    total, uniq, top = _oracle(chunks, 10)
    assert n == total and app.nunique == uniq
    assert [c for _, c in app.top] == [c for _, c in top]
    assert {w for w, _ in app.top[:3]} <= {w.decode() for w, _ in top[:5]}


@pytest.mark.gpu
def test_wordfreq_gpu():
    chunks = [synth.zipf_text(3_000_000, seed=s).pin_memory() for s in range(3)]
    app = WordFreq(g.MapReduce(g.Comm(device="cuda")), chunks, ntop=10)
    n = app.run()
    total, uniq, top = _oracle(chunks, 10)
    assert n == total and app.nunique == uniq
    assert [c for _, c in app.top] == [c for _, c in top]
