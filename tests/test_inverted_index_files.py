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
