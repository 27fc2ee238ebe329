"""The disk tier's background writes are bounded (csrc/engine/spool.cpp
DiskWriter): at most MRH_SPOOL_WRITERS threads and MRH_SPOOL_WRITE_INFLIGHT
bytes of drained-but-unwritten pinned pieces at a time, each pinned piece
released as soon as its file is written. tri_find_mr out of core with a host
budget far below the data spills most partition pieces to disk; the count
must stay exact and the writer pool within its bounds."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys, torch
import gpu_mapreduce_amd as g
from gpu_mapreduce_amd import C
from gpu_mapreduce_amd.models.pagerank import GRAPH500
from gpu_mapreduce_amd.models.triangles import TriangleGraph, tri_find_mr
comm = g.Comm(device="cuda")
e = C.map_rmat((1 << 15) * 16, 15, *GRAPH500, 0.0, 3, 0, "cuda").kdata.view(torch.int64).view(-1, 2)
want = TriangleGraph(comm, e, 1 << 15).count()
C.spool_writer_reset_peak()
r = tri_find_mr(comm, e, hbm_budget=8 << 20, host_budget=4 << 20, fpath=sys.argv[1], memsize=1)
w = dict(C.spool_writer_stats())
print(json.dumps({"tri": int(r["triangles"]), "want": int(want), "disk": int(r["spool_disk_bytes"]),
                  "files": int(r["spool_files"]), "writer": w, "live": C.spool_files_live()}))
"""


@pytest.mark.gpu
def test_disk_tier_writer_pool_is_bounded(tmp_path):
    cap = 2 << 20
    env = dict(os.environ, PYTHONPATH=ROOT, MRH_SPOOL_WRITERS="2", MRH_SPOOL_WRITE_INFLIGHT=str(cap))
    p = subprocess.run([sys.executable, "-c", CHILD, str(tmp_path)], env=env, cwd=ROOT, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["tri"] == r["want"], r
    w = r["writer"]
    assert r["disk"] > 8 * cap and w["jobs"] > 4, r          # the disk tier carried far more than the cap
    assert w["threads"] <= 2 and w["cap_bytes"] == cap, w
    # a piece larger than the cap is admitted alone; otherwise the cap holds
    # (a piece is at most one partition of one HBM-budget chunk)
    assert w["peak_inflight_bytes"] <= max(cap, 8 << 20), w
    assert w["inflight_bytes"] == 0, w
    assert r["live"] == 0 and not [f for f in os.listdir(tmp_path) if f.startswith("mrmpi.")], r
