"""InvertedIndex over part files read while the job runs: each file entry
carries a read future, the job waits for file i's read right before its copy
(reference cuda/InvertedIndex.cu:170-190 freads each part file in its map).
A deliberately slow read proves the wait: without it the job would copy an
all-zero buffer and lose that file's URLs."""
import os
import time
from concurrent.futures import ThreadPoolExecutor

import pytest
import torch

import gpu_mapreduce_amd as g
from gpu_mapreduce_amd.models.inverted_index import InvertedIndex, reference_inverted_index
from gpu_mapreduce_amd.utils import synth


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_inverted_index_waits_for_file_reads(tmp_path, dev):
    files = synth.html_corpus(3_000_000, file_bytes=600_000, seed=4, nurl=5_000)
    paths = []
    for name, t in files:
        p = os.path.join(tmp_path, name)
        t.numpy().tofile(p)
        paths.append((name, p, t.numel()))
    pin = dev == "cuda"
    bufs = [torch.zeros(n, dtype=torch.uint8, pin_memory=pin) for _, _, n in paths]

    def read(i):
        if i in (0, 3):
            time.sleep(0.3)  # the job reaches these files before their bytes are there
        with open(paths[i][1], "rb", buffering=0) as f:
            assert f.readinto(memoryview(bufs[i].numpy())) == paths[i][2]

    with ThreadPoolExecutor(2) as pool:
        futs = [pool.submit(read, i) for i in range(len(paths))]
        mr = g.MapReduce(g.Comm(device=dev))
        app = InvertedIndex(mr, [(paths[i][0], bufs[i], futs[i]) for i in range(len(paths))],
                            out_dir=str(tmp_path / "out"))
        app.run()
    got = {}
    for line in app.output_lines():
        url, rest = line.split("\t")
        got[url.encode()] = sorted(rest.split())
    assert got == reference_inverted_index(files)


def test_output_write_from_buffer(tmp_path):
    import numpy as np

    from gpu_mapreduce_amd.models.inverted_index import _write_file
    for n in (0, 5, 1 << 20, (48 << 20) + 7):
        a = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8)
        p = tmp_path / f"out{n}"
        _write_file(str(p), memoryview(a))
        assert p.read_bytes() == a.tobytes()
    # rewriting a path with less data leaves exactly the new bytes
    p = tmp_path / "again"
    _write_file(str(p), memoryview(np.full(1000, 7, dtype=np.uint8)))
    _write_file(str(p), memoryview(np.full(10, 3, dtype=np.uint8)))
    assert p.read_bytes() == bytes([3] * 10)


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_async_write_pipeline_files_equal_oracle(tmp_path, dev):
    """a job pipeline as bench.py's with_file_io runs it: job s's index is
    written by the writer thread while job s+1 runs (and its first file was
    prefetched by job s); every written file equals the oracle's index"""
    out = str(tmp_path / "out")
    comm = g.Comm(device=dev)
    jobs = [synth.html_corpus(2_000_000, file_bytes=500_000, seed=s, nurl=4_000) for s in (7, 8, 9)]
    if dev == "cuda":
        jobs = [[(n, t.pin_memory()) for n, t in f] for f in jobs]
    written = []
    for s, files in enumerate(jobs):
        nxt = jobs[s + 1] if s + 1 < len(jobs) else None
        app = InvertedIndex(g.MapReduce(comm), files, out_dir=out, async_write=True, prefetch_next=nxt)
        app.run()
        # the previous job's write may still run; this job's file name is the same,
        # so wait for it before reading (the writer thread keeps job order)
        app.wait_written()
        with open(os.path.join(out, "InvertedIndex-1-0"), "rb") as f:
            written.append(f.read())
    for files, data in zip(jobs, written):
        got = {}
        for line in data.decode().splitlines():
            url, rest = line.split("\t")
            got[url.encode()] = sorted(rest.split())
        assert got == reference_inverted_index(files)


@pytest.mark.gpu
def test_prefetch_void_when_next_job_has_larger_files():
    """advisor r3: the next job of a pipeline has a larger file, so its
    staging buffers are reallocated; the prefetched copy went to the old
    buffer and must not be taken (take_prefetch checks the buffer)"""
    comm = g.Comm(device="cuda")
    a = [(n, t.pin_memory()) for n, t in synth.html_corpus(1_000_000, file_bytes=250_000, seed=3, nurl=2_000)]
    # b's first file fits a's staging buffers (so job a prefetches it), a
    # later one does not (so job b reallocates them)
    small = synth.html_corpus(250_000, file_bytes=250_000, seed=4, nurl=2_000)[0]
    big = synth.html_corpus(2_000_000, file_bytes=1_000_000, seed=5, nurl=2_000)
    b = [(n, t.pin_memory()) for n, t in [("first-" + small[0], small[1])] + big]
    InvertedIndex(g.MapReduce(comm), a, prefetch_next=b).run()
    app = InvertedIndex(g.MapReduce(comm), b)
    app.run()
    got = {}
    for line in app.output_lines():
        url, rest = line.split("\t")
        got[url.encode()] = sorted(rest.split())
    assert got == reference_inverted_index(b)
