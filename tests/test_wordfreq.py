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


def _wc_counts(dev, chunks, init_slots=1 << 20):
    """run C.WordCounter over padded copies of the chunks -> {word: count}, words"""
    from gpu_mapreduce_amd import C
    wc = C.WordCounter(dev, init_slots)
    for t in chunks:
        buf = torch.zeros(t.numel() + 64, dtype=torch.uint8, device=dev)
        buf[: t.numel()] = t.to(dev)
        wc.add(buf, t.numel())
    words = wc.words
    kv = wc.finish()
    kd = bytes(kv.kdata.cpu().numpy())
    off = kv.koff.cpu().tolist()
    vals = kv.vdata.cpu().view(torch.int32).tolist()
    got = {kd[off[i]:off[i + 1] - 1]: vals[i] for i in range(kv.n)}
    assert len(got) == kv.n, "a word was emitted twice"
    return got, words


def _tricky_chunks():
    g_ = torch.Generator().manual_seed(3)
    # random lowercase words with a long tail (many distinct), very long words,
    # tabs/CR/FF separators, a word that ends exactly at the chunk end
    parts = []
    for i in range(4):
        n = 150_000
        letters = torch.randint(97, 100 + 2 * i, (n,), generator=g_, dtype=torch.uint8)
        sep = torch.rand(n, generator=g_) < 0.22
        seps = torch.tensor([32, 9, 10, 13, 12], dtype=torch.uint8)[torch.randint(0, 5, (n,), generator=g_)]
        t = torch.where(sep, seps, letters)
        t[5000:5300] = 120        # a 300-byte word
        t[-3:] = 122              # word touching the end of the chunk
        parts.append(t)
    return parts


def test_wordcounter_cpu_exact():
    chunks = _tricky_chunks()
    got, words = _wc_counts("cpu", chunks)
    c = collections.Counter()
    for t in chunks:
        c.update(bytes(t.numpy()).split())
    assert got == dict(c) and words == sum(c.values())


@pytest.mark.gpu
@pytest.mark.parametrize("init_slots", [1024, 1 << 20])
def test_wordcounter_gpu_exact(init_slots):
    """device in-mapper combiner == Counter, incl. table growth + rehash
    (init_slots=1024 forces several), long words, chunk-end words"""
    chunks = _tricky_chunks() + [synth.zipf_text(2_000_000, seed=9)]
    got, words = _wc_counts("cuda", chunks, init_slots)
    c = collections.Counter()
    for t in chunks:
        c.update(bytes(t.cpu().numpy()).split())
    assert words == sum(c.values())
    assert got == dict(c)


@pytest.mark.gpu
def test_wordfreq_gpu_combiner_matches_plain():
    chunks = [synth.zipf_text(3_000_000, seed=s).pin_memory() for s in range(2)]
    a = WordFreq(g.MapReduce(g.Comm(device="cuda")), chunks, ntop=20, combiner=True)
    b = WordFreq(g.MapReduce(g.Comm(device="cuda")), chunks, ntop=20, combiner=False)
    assert a.run() == b.run()
    total, uniq, top = _oracle(chunks, 20)
    assert a.nunique == b.nunique == uniq
    assert [c for _, c in a.top] == [c for _, c in b.top] == [c for _, c in top]
    ref = {w.decode(): c for w, c in top}
    assert all(ref.get(w, c) == c for w, c in a.top)


@pytest.mark.gpu
def test_wordfreq_gpu_job_pipeline_prefetch():
    """three jobs as a pipeline (each copies the next job's first chunk behind
    its own last one, ring slots continuing across jobs): every job's counts
    equal the oracle"""
    chunks = [synth.zipf_text(1_000_000, seed=10 + s).pin_memory() for s in range(4)]
    total, uniq, top = _oracle(chunks, 10)
    comm = g.Comm(device="cuda")
    for s in range(3):
        app = WordFreq(g.MapReduce(comm), chunks, ntop=10, prefetch_next=chunks if s < 2 else None)
        n = app.run()
        assert n == total and app.nunique == uniq
        assert [c for _, c in app.top] == [c for _, c in top]
