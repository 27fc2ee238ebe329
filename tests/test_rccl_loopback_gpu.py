"""MRH_FORCE_RCCL=2: a one-rank RCCL communicator on which every collective
(allreduce, all-gather, broadcast, the scalar allreduce / bcast) and the
PageRank exchange ring call their nccl* functions instead of the one-rank
identity (csrc/engine/comm.cpp identity_coll, graphplan.cpp ring_start), so
every RCCL call site of the multi-GPU paths — including the RCCL operations
inside the PageRank iteration's HIP-graph capture — executes on one MI355X.

The child (tools/rccl_loopback.py) runs PageRank (replicated plan, graph
replay), the tri_find split build, tri_find_mr RMAT-16 and wordfreq without
the combiner in four modes; results must match the local path (bit for bit
where the arithmetic is the same) and every nccl* entry point's call counter
must be non-zero in mode 2. Reference collectives: src/mapreduce.cpp:539,
597-605; src/irregular.cpp:111-178."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = os.path.join(ROOT, "tools", "rccl_loopback.py")


def _run(mode, tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MRH_FORCE_RCCL", "MRH_PR_DIST_GRAPH", "MRH_PR_OVERLAP"):
        env.pop(k, None)
    prefix = str(tmp_path / mode)
    p = subprocess.run([sys.executable, "-u", CHILD, mode, prefix], env=env, cwd=ROOT, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-4000:]
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    return rec, dict(np.load(prefix + ".npz"))


@pytest.mark.gpu
def test_rccl_loopback_collectives_match_local(tmp_path):
    runs = {m: _run(m, tmp_path) for m in ("local", "force1", "force2", "force2_eager")}
    (lr, lo), (r1, o1), (r2, o2), (re, oe) = (runs[m] for m in ("local", "force1", "force2", "force2_eager"))
    assert lr["transport"] == "local" and not lr["loopback"]
    assert r1["transport"] == "rccl" and not r1["loopback"]
    assert r2["transport"] == "rccl" and r2["loopback"] and re["loopback"]
    fin = r2["counters_final"]
    # every nccl* entry point really ran in mode 2
    for k in ("all_reduce", "all_gather", "broadcast", "send", "recv", "group"):
        assert fin[k] > 0, (k, fin)
    # mode 1 never calls a collective (the identity), only send/recv rounds
    assert r1["counters_final"]["all_reduce"] == 0 and r1["counters_final"]["broadcast"] == 0, r1
    assert lr["counters_final"] == {k: 0 for k in fin}, lr
    # per workload, mode 2 made real collective calls
    pr2 = r2["counters_pagerank"]
    assert pr2["all_reduce"] > 0 and pr2["all_gather"] > 0 and pr2["send"] > 0 and pr2["recv"] > 0, pr2
    for a, b in (("pagerank", "trifind"), ("trifind", "trifind_mr"), ("trifind_mr", "wordfreq")):
        ca, cb = r2["counters_" + a], r2["counters_" + b]
        assert cb["all_reduce"] > ca["all_reduce"], (b, ca, cb)
        if b in ("trifind_mr", "wordfreq"):
            assert cb["send"] > ca["send"], (b, ca, cb)  # the shuffle went through RCCL
    # PageRank: the replicated plan with its self-ring replays as a HIP graph
    # (20-run: 2 eager + 18; 7-run: 1 eager + 6) and equals its eager run and
    # the mode-1 run bit for bit, the local plan to float32 accumulation order
    assert r2["pr_layout"] == "replicated" and r2["pr_graph_iters"] == 24, r2
    assert re["pr_graph_iters"] == 0, re
    assert np.array_equal(o2["pagerank"], oe["pagerank"])
    np.testing.assert_allclose(o2["pagerank"], o1["pagerank"], rtol=1e-4, atol=1e-10)  # mode 1: no source pieces
    np.testing.assert_allclose(o2["pagerank"], lo["pagerank"], rtol=1e-4, atol=1e-10)
    # tri_find: the split build at one rank; counts exact
    assert r2["tri_split"] and r1["tri_split"], (r1, r2)
    for m in (o1, o2):
        assert int(m["trifind"][0]) == int(lo["trifind"][0]) == int(lo["trifind_mr"][0])
        assert int(m["trifind_mr"][0]) == int(lo["trifind_mr"][0])
    # wordfreq without the combiner: the P > 1 route (no grouping in the map
    # shadow) with the same counts and top-10 as the local one-rank route
    assert lr["wf_route"] == "grouped in the map" and r2["wf_route"] == r1["wf_route"] == "exchanged per chunk", (lr, r2)
    for m, r in ((o1, r1), (o2, r2)):
        assert int(m["wf_nwords"][0]) == int(lo["wf_nwords"][0])
        assert int(m["wf_nunique"][0]) == int(lo["wf_nunique"][0])
        assert [c for _, c in r["wf_top"]] == [c for _, c in lr["wf_top"]]
    # broadcast / gather / scalar collectives: the one-rank identities
    for r in (lr, r1, r2):
        assert r["mr_broadcast"] == 300 and r["mr_gather"] == 300, r
        assert r["allreduce"] == [5, -3] and r["allgather_var_ok"], r
