"""bench.py's own multi-rank launcher (`--gpus N` without torchrun): it must
spawn N ranks that really join one job (n_gpus / ranks_joined = N, global
counts = N x the 1-rank counts for this weak-scaling workload) and keep the
single-rank path unchanged. CPU engine, gloo; the driver runs the same script
under torchrun on an 8-GPU node."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--bytes-per-gpu", "4e6", "--file-bytes", "1000000", "--steps", "1", "--warmup", "1", "--phases", "0",
        "--pagerank-scale", "10", "--pagerank-steps", "1"]


def _bench(n, tmp, extra=()):
    """the printed line merged over the detail file (the full record)"""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["HIP_VISIBLE_DEVICES"] = ""
    detail = os.path.join(str(tmp), f"detail_{n}.json")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), *ARGS, *extra,
                        "--detail-out", detail], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints exactly one JSON line
    line = json.loads(lines[0])
    # the printed line stays small enough for a driver's stdout tail
    assert len(lines[0]) < 4000, len(lines[0])
    assert line["detail_file"] == detail
    with open(detail) as f:
        full = json.load(f)
    return {**full, **line}


def test_bench_spawns_n_ranks(tmp_path):
    # the big in-HBM tri_find_mr run (BASELINE config 5 through the MapReduce
    # engine: RMAT-24 on 8 GPUs) rehearsed at a small scale on 1 and 3 ranks
    big = ("--trifind-mr-big-scale", "11")
    one, three = _bench(1, tmp_path, big), _bench(3, tmp_path, big)
    assert one["n_gpus"] == 1 and one["ranks_joined"] == 1
    assert three["n_gpus"] == 3 and three["ranks_joined"] == 3
    assert three["config"]["parallelism"] == "dp3"
    assert three["kv_pairs_per_step"] == 3 * one["kv_pairs_per_step"]
    assert three["config"]["global_batch"] == 3 * one["config"]["global_batch"]
    # the PageRank extra is strong scaling: same graph, same edge count
    assert three["pagerank_config"]["edges"] == one["pagerank_config"]["edges"] == 16 * 1024
    for k in ("metric", "value", "unit", "ms_per_step", "higher_is_better", "scaling", "vs_baseline", "dtype",
              "data", "pagerank_kvps", "pagerank_ms", "pagerank_setup_ms",
              # BASELINE configs 5 and 3 ride in the same record
              "trifind_kvps", "trifind_ms", "trifind_setup_ms", "trifind_triangles",
              "wordfreq_kvps", "wordfreq_ms", "wordfreq_setup_ms", "wordfreq_words"):
        assert k in three, k
    assert three["trifind_triangles"] == one["trifind_triangles"] > 0   # strong scaling: same graph
    assert three["wordfreq_words"] == 3 * one["wordfreq_words"]          # weak scaling: text per rank
    # every extra ran (a failing extra is recorded as <name>_error, not fatal)
    for rec in (one, three):
        assert not [k for k in rec if k.endswith("_error")], [k for k in rec if k.endswith("_error")]
        assert rec["trifind_mr_triangles"] == rec["trifind_mr_triangles_check"] > 0
        assert "ms_per_step" in rec["with_file_io"] and "ms_per_step" in rec["wordfreq_with_file_io"]
        # driver-visible (printed) keys of every BASELINE config
        for k in ("pagerank_ms", "pagerank_setup_ms", "trifind_ms", "trifind_triangles", "trifind_mr_ms",
                  "trifind_mr_big_ms", "trifind_mr_big_triangles_ok", "wordfreq_ms", "wordfreq_shuffle_ms",
                  "with_file_io_ms", "wordfreq_with_file_io_ms"):
            assert k in rec, k
        assert rec["trifind_mr_big_scale"] == 11 and rec["trifind_mr_big_triangles_ok"] is True
        assert rec["trifind_mr_big"]["triangles"] == one["trifind_mr_big"]["triangles"] > 0  # same graph


def test_bench_eight_ranks(tmp_path):
    """the driver's largest scaling point, N = 8 (one node), rehearsed on the
    CPU engine: 8 ranks join, global counts are 8x, PageRank keeps its graph"""
    one, eight = _bench(1, tmp_path), _bench(8, tmp_path)
    assert eight["n_gpus"] == eight["ranks_joined"] == 8 and eight["config"]["parallelism"] == "dp8"
    assert eight["kv_pairs_per_step"] == 8 * one["kv_pairs_per_step"]
    assert eight["pagerank_config"]["edges"] == one["pagerank_config"]["edges"]
    assert "pagerank_error" not in eight


def test_bench_rejects_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", *ARGS], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


@pytest.mark.gpu
def test_bench_two_ranks_on_one_gpu():
    """bench.py --gpus 2 on a 1-GPU box: both ranks share cuda:0 (RCCL refuses
    two ranks on one device, so torch.distributed runs gloo and the engine its
    store transport); every multi-rank engine path of the headline job runs
    on the GPU — per-file exchange, grouped collate, GPU output formatting,
    PageRank plan with owner exchange — and the global counts double"""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(MRH_DIST_BACKEND="gloo", MRH_TRANSPORT="pg", MRH_NUMA_BIND="0")
    args = ["--bytes-per-gpu", "32e6", "--file-bytes", "8000000", "--steps", "2", "--warmup", "1", "--phases", "0",
            "--pagerank-scale", "16", "--pagerank-steps", "1"]
    out = {}
    for n in (1, 2):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), *args], cwd=ROOT,
                           env=env, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
        assert len(lines) == 1, r.stdout
        line = json.loads(lines[0])
        with open(line["detail_file"]) as f:
            out[n] = {**json.load(f), **line}
    one, two = out[1], out[2]
    assert two["n_gpus"] == two["ranks_joined"] == 2 and two["backend"]["torch.distributed"].startswith("gloo")
    # ranks share the GPU: the engine runs the pg transport; the RCCL facts come
    # from a one-rank probe communicator per rank
    assert two["engine_transport"].startswith("pg") and two["rccl_comm_count"] == 1
    assert two["kv_pairs_per_step"] == 2 * one["kv_pairs_per_step"]
    assert two["pagerank_config"]["edges"] == one["pagerank_config"]["edges"]
