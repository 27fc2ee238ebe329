"""The pinned host arena (csrc/engine/hostarena.cpp): the out-of-core host
tier's pinned allocations are carved from one segment pinned at start-up
(gpu_mapreduce_amd/hostpin.py), falling back to the caching host allocator
when a request does not fit. tri_find_mr out of core with a small arena must
count exactly, take blocks from the arena, fall back for the rest, and give
every block back when the job's spools are gone. Runs in a child process: the
arena is per process, once."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import gc, json, sys, torch
import gpu_mapreduce_amd as g
from gpu_mapreduce_amd import C, hostpin
from gpu_mapreduce_amd.models.pagerank import GRAPH500
from gpu_mapreduce_amd.models.triangles import TriangleGraph, tri_find_mr
comm = g.Comm(device="cuda")
ms = hostpin.prepin(int(sys.argv[2]))
assert hostpin.prepin(64) == 0.0  # once per process
e = C.map_rmat((1 << 15) * 16, 15, *GRAPH500, 0.0, 3, 0, "cuda").kdata.view(torch.int64).view(-1, 2)
want = TriangleGraph(comm, e, 1 << 15).count()
r = tri_find_mr(comm, e, hbm_budget=8 << 20, host_budget=256 << 20, fpath=sys.argv[1], memsize=1)
del r["stages"]
gc.collect()
torch.cuda.synchronize()
print(json.dumps({"tri": int(r["triangles"]), "want": int(want), "host": int(r["spool_host_bytes"]),
                  "ms": ms, "arena": hostpin.stats()}))
"""


@pytest.mark.gpu
@pytest.mark.parametrize("mib", [8, 512])
def test_host_arena_serves_the_host_tier(tmp_path, mib):
    p = subprocess.run([sys.executable, "-c", CHILD, str(tmp_path), str(mib)], env=dict(os.environ, PYTHONPATH=ROOT),
                       cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    a = r["arena"]
    assert r["tri"] == r["want"] and r["host"] > 0
    assert a["reserved"] == mib << 20 and a["hits"] > 0 and 0 < a["peak"] <= a["reserved"]
    assert a["in_use"] == 0  # every block came back
    if mib == 8:
        assert a["misses"] > 0  # the caching host allocator took what did not fit
