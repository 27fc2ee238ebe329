"""RingReader (gpu_mapreduce_amd/utils/fileio.py): part files of consecutive
wordfreq jobs streamed through a ring of fewer pinned buffers than files.
Every job must count exactly its files' words (a slot refilled before its copy
finished would corrupt a chunk), on the CPU engine and on the GPU."""
import os

import pytest

import gpu_mapreduce_amd as g
from gpu_mapreduce_amd.models.wordfreq import WordFreq
from gpu_mapreduce_amd.utils import synth
from gpu_mapreduce_amd.utils.fileio import RingReader
from test_wordfreq import _oracle


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_ring_reader_wordfreq_jobs(tmp_path, dev):
    chunks = [synth.zipf_text(150_000 + 977 * s, seed=40 + s) for s in range(11)]
    paths = []
    for i, t in enumerate(chunks):
        p = os.path.join(tmp_path, f"part-{i:05d}")
        t.numpy().tofile(p)
        paths.append((p, t.numel()))
    total, uniq, top = _oracle(chunks, 10)
    comm = g.Comm(device=dev)
    reader = RingReader(paths, slots=3, threads=4, piece=40_000, pin=dev == "cuda")
    try:
        nxt = reader.job()
        for s in range(3):
            entries, cb = nxt
            if s < 2:
                nxt = reader.job()  # queued while this job runs
            app = WordFreq(g.MapReduce(comm), entries, ntop=10, on_copied=cb)
            n = app.run()
            assert n == total and app.nunique == uniq, s
            assert [c for _, c in app.top] == [c for _, c in top], s
    finally:
        reader.close()
