"""MRH_GUARD device bounds-check mode (csrc/engine/guardalloc.h): every HBM
block gets canaries; an overrun is reported with the op that allocated the
block and fails the next MapReduce op. The GPU tests run in a child process
because the guarded allocator must be installed before the first HBM
allocation of the process."""
import os
import subprocess
import sys

import pytest
import torch

from gpu_mapreduce_amd import C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_guard_inactive_by_default_and_selftest_refused():
    assert not C.alloc_guard_active()
    with pytest.raises(RuntimeError):
        C._guard_selftest_overrun(torch.zeros(16, dtype=torch.int32), 8)
    assert C.guard_check("noop") == 0


CHILD = r'''
import torch, gpu_mapreduce_amd as g
from gpu_mapreduce_amd import C, MapReduce
from gpu_mapreduce_amd.models.inverted_index import InvertedIndex, reference_inverted_index
from gpu_mapreduce_amd.utils import synth
assert C.alloc_guard_active()
comm = g.Comm(device="cuda:0")
files = synth.html_corpus(1 << 20, file_bytes=256 << 10, seed=3, nurl=500, device="cuda:0")
files = [(n, t.cpu().pin_memory()) for n, t in files]
mr = MapReduce(comm)
app = InvertedIndex(mr, files)
app.run()
got = {l.split("\t")[0].encode(): sorted(l.split("\t")[1].split()) for l in app.output_lines()}
assert got == reference_inverted_index(files)
assert C.guard_check("after the job") == 0 and C.guard_reports() == [], C.guard_reports()
assert C.guard_blocks_live() > 0
# a deliberate 64-byte overrun past a block's end is caught
t = torch.zeros(1000, dtype=torch.int32, device="cuda")
C._guard_selftest_overrun(t, 64)
assert C.guard_check("selftest") == 1
r = C.guard_reports()[-1]
assert r["back_bad"] == 64 and r["front_bad"] == 0 and r["size"] == 4000, r
# ... and the next MapReduce op refuses to run on a corrupted heap
mr2 = MapReduce(comm)
try:
    mr2.map(1, lambda i, kv: kv.add(b"k", b"v"))
    raise SystemExit("op after an overrun did not fail")
except RuntimeError as e:
    assert "out-of-bounds" in str(e), e
print("guard ok")
'''


@pytest.mark.gpu
def test_guard_catches_overrun_gpu():
    env = dict(os.environ, MRH_GUARD="1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "guard ok" in r.stdout
    assert "out-of-bounds device write on a 4000-byte block" in r.stderr
