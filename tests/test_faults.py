"""Failure detection, fault injection and check mode (csrc/engine/guard.h;
SURVEY.md §5). The reference has none of these (Error::one -> MPI_Abort,
src/error.cpp:47-57); the tests here are ours:

* a rank that dies mid-job (MRH_FAULT=abort) is detected by the surviving
  ranks within the collective timeout (MRH_COMM_TIMEOUT) — they exit with an
  error instead of hanging;
* an HBM out-of-memory inside an op (MRH_FAULT=oom) spills the other live
  MapReduce objects to host memory and retries, with the same result;
* MRH_CHECK=1 validates KV/KMV invariants after every op of a full C API run.
Each case runs in its own process because the knobs are read once per process.
"""
import os
import subprocess
import sys
import textwrap
import time

import pytest

from test_native_multiproc import PKG, ROOT, _cc, _docs, _port

ENV0 = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}


def _py(code, env, gpu=False):
    e = dict(ENV0, PYTHONPATH=ROOT, **env)
    if not gpu:
        e["HIP_VISIBLE_DEVICES"] = ""
    return subprocess.run([sys.executable, "-c", textwrap.dedent(code)], env=e, capture_output=True, text=True,
                          timeout=300)


def test_dead_rank_is_detected_not_hung(tmp_path):
    exe = _cc(os.path.join(ROOT, "examples", "c", "cwordfreq.c"), tmp_path / "cwordfreq")
    _docs(tmp_path / "docs")
    port = _port()
    procs = []
    t0 = time.time()
    for r in range(2):
        env = dict(ENV0, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HIP_VISIBLE_DEVICES="", MRH_FAULT="abort:exchange_round:1")
        procs.append(subprocess.Popen([exe, "docs"], cwd=tmp_path, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    try:
        res = [p.communicate(timeout=120) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    elapsed = time.time() - t0
    # rank 1 dies inside the shuffle (a round of the collate exchange)
    assert procs[1].returncode == 3 and "rank 1 aborts at exchange_round" in res[1][1]
    assert procs[0].returncode != 0, "the surviving rank must fail, not report success"
    assert elapsed < 30, f"failure took {elapsed:.0f} s to surface (MRH_COMM_TIMEOUT left at 600 s)"


OOM_SCRIPT = """
import collections, struct
import gpu_mapreduce_amd as g
from gpu_mapreduce_amd import MapReduce
dev = "{dev}"
comm = g.Comm(device=dev)
words = ("a bb ccc a dddd bb a eeeee " * 50).split()
other = MapReduce(comm)
other.map(1, lambda i, kv: [kv.add(w) for w in words])       # a second live MR holding device data
mr = MapReduce(comm)
mr.map(2, lambda i, kv: [kv.add(w) for w in words[i::2]])
mr.collate()                                                 # convert hits the injected OOM
mr.reduce("count")
got = {{k[:-1].decode(): struct.unpack("<i", v)[0] for k, v in mr.kv_pairs()}}
assert got == dict(collections.Counter(words)), got
assert other.collate() == 5                                   # the spilled MR comes back and works
print("OOM-RETRY-OK", other.kv is None)
"""


def test_oom_spills_other_mrs_and_retries():
    r = _py(OOM_SCRIPT.format(dev="cpu"), {"MRH_FAULT": "oom:convert:0"})
    assert r.returncode == 0, r.stderr
    assert "OOM-RETRY-OK" in r.stdout
    assert "spilled 1 MapReduce object(s) to host and retrying" in r.stderr


def test_injected_throw_surfaces_as_error():
    code = """
    import gpu_mapreduce_amd as g
    mr = g.MapReduce(g.Comm(device="cpu"))
    mr.map(1, lambda i, kv: kv.add(b"k", b"v"))
    try:
        mr.convert()
    except RuntimeError as e:
        print("CAUGHT", "injected failure in convert" in str(e))
    """
    r = _py(code, {"MRH_FAULT": "throw:convert:-1"})
    assert r.returncode == 0, r.stderr
    assert "CAUGHT True" in r.stdout


def test_bad_fault_spec_is_rejected():
    r = _py("import gpu_mapreduce_amd as g; mr = g.MapReduce(g.Comm(device='cpu')); mr.map(1, lambda i, kv: None)",
            {"MRH_FAULT": "explode:map"})
    assert r.returncode != 0 and "MRH_FAULT must be" in r.stderr


def test_check_mode_full_capi_run(tmp_path):
    exe = _cc(os.path.join(ROOT, "tests", "capi", "capi_test.c"), tmp_path / "capi_test")
    env = dict(ENV0, HIP_VISIBLE_DEVICES="", MRH_CHECK="1")
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout and "MRH_CHECK" not in r.stderr


@pytest.mark.gpu
def test_oom_spill_retry_gpu():
    r = _py(OOM_SCRIPT.format(dev="cuda:0"), {"MRH_FAULT": "oom:convert:0", "MRH_CHECK": "1"}, gpu=True)
    assert r.returncode == 0, r.stderr
    # the victim was moved to host memory: its next op brought it back to HBM
    assert "OOM-RETRY-OK" in r.stdout and "spilled 1 MapReduce object(s)" in r.stderr


@pytest.mark.gpu
def test_serialize_mode_gpu():
    """MRH_SYNC=1: every kernel launch is followed by a device sync (faults are
    reported at their launch site); the job's results must not change."""
    code = """
    import collections, struct
    import gpu_mapreduce_amd as g
    words = ("a bb ccc a dddd bb a eeeee https://x.org/y " * 300).split()
    mr = g.MapReduce(g.Comm(device="cuda:0"))
    mr.map(3, lambda i, kv: [kv.add(w.encode() + b"\\0") for w in words[i::3]])
    mr.collate()
    mr.reduce("count")
    mr.sort_values(-1)
    got = {k[:-1].decode(): struct.unpack("<i", v)[0] for k, v in mr.kv_pairs()}
    assert got == dict(collections.Counter(words)), got
    print("SYNC-OK")
    """
    r = _py(code, {"MRH_SYNC": "1", "MRH_CHECK": "1"}, gpu=True)
    assert r.returncode == 0, r.stderr
    assert "SYNC-OK" in r.stdout


@pytest.mark.skipif(os.environ.get("MRH_ASAN") != "1", reason="slow (rebuilds the host code with ASan); MRH_ASAN=1")
def test_host_asan_clean():
    """host AddressSanitizer build of the engine + C API + OINK runs the C API
    test, a 2-rank C job and two OINK scripts cleanly (tools/asan_check.sh)"""
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "asan_check.sh")], capture_output=True, text=True,
                       timeout=1800)
    assert r.returncode == 0 and "ASAN CLEAN" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


def test_op_trace_two_ranks(tmp_path):
    """MRH_TRACE: every MapReduce op of every rank is one JSON line; the
    summary tool groups them into the reference's stages"""
    import importlib.util
    exe = _cc(os.path.join(ROOT, "examples", "c", "cwordfreq.c"), tmp_path / "cwordfreq")
    _docs(tmp_path / "docs")
    port = _port()
    procs = []
    for r in range(2):
        env = dict(ENV0, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HIP_VISIBLE_DEVICES="", MRH_TRACE=str(tmp_path / "trace"))
        procs.append(subprocess.Popen([exe, "docs"], cwd=tmp_path, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    for p in procs:
        p.communicate(timeout=120)
        assert p.returncode == 0
    spec = importlib.util.spec_from_file_location("trace_summary", os.path.join(ROOT, "tools", "trace_summary.py"))
    ts = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ts)
    recs = ts.load(str(tmp_path / "trace"))
    assert {r["rank"] for r in recs} == {0, 1}
    ops = {r["op"] for r in recs}
    assert {"map_file", "collate", "reduce", "gather", "sort_values"} <= ops
    # the pipelined collate is one leaf op (shuffle rounds + per-round group-by);
    # with MRH_PIPELINE_COLLATE=0 it nests aggregate + convert one level deeper
    col = [r for r in recs if r["op"] == "collate" and r["rank"] == 0][0]
    assert "aggregate" not in ops or any(r["op"] == "aggregate" and r["depth"] == col["depth"] + 1 for r in recs)
    assert sum(r["sent"] for r in recs if r["op"] in ("aggregate", "collate")) > 0
    s = ts.summarise(recs)
    assert {"Map", "Network I/O", "Sort/Hash", "Reduce"} <= set(s["stages_ms"])


def _run_ranks(exe, args, n, cwd, extra, timeout=120):
    """n native ranks; returns [(returncode, stderr, exit_time)] with exit
    times measured by polling, so the test can bound how long the survivors
    outlive the failed rank."""
    port = _port()
    procs = []
    for r in range(n):
        env = dict(ENV0, WORLD_SIZE=str(n), RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HIP_VISIBLE_DEVICES="", **extra)
        procs.append(subprocess.Popen([exe, *args], cwd=cwd, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    t_exit = [None] * n
    t0 = time.time()
    try:
        while any(t is None for t in t_exit) and time.time() - t0 < timeout:
            for i, p in enumerate(procs):
                if t_exit[i] is None and p.poll() is not None:
                    t_exit[i] = time.time()
            time.sleep(0.02)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return [(p.returncode, p.communicate()[1], t) for p, t in zip(procs, t_exit)]


@pytest.mark.parametrize("kind", ["abort", "throw"])
def test_rank_failure_inside_shuffle_ends_job_fast(tmp_path, kind):
    """One rank fails INSIDE the chunked exchange (first round of the first
    aggregate); MRH_COMM_TIMEOUT stays at its 600 s default. Every rank must
    exit non-zero within 10 s of the failure: a crash ("abort", no chance to
    say goodbye) is seen through the stopped heartbeat, an error ("throw") is
    broadcast by poisoning the job (reference Error::one -> MPI_Abort,
    src/error.cpp:47-57)."""
    exe = _cc(os.path.join(ROOT, "examples", "c", "cwordfreq.c"), tmp_path / "cwordfreq")
    _docs(tmp_path / "docs")
    res = _run_ranks(exe, ["docs"], 3, tmp_path, {"MRH_FAULT": f"{kind}:exchange_round:1"})
    codes = [r[0] for r in res]
    assert all(t is not None for _, _, t in res), f"a rank hung: {codes}"
    assert all(c != 0 for c in codes), codes
    t_fail = res[1][2]
    for r in (0, 2):
        assert res[r][2] - t_fail < 10.0, f"rank {r} outlived the failure by {res[r][2] - t_fail:.1f} s"
        msg = res[r][1]
        # a crash: the heartbeat sees it, or a survivor's exchange with the
        # dead peer errors first and that rank poisons the job with its own error
        ok = ("stopped responding" in msg or "failed:" in msg) if kind == "abort" else ("rank 1 failed" in msg)
        assert ok, msg[-2000:]
    if kind == "abort":
        assert codes[1] == 3 and "rank 1 aborts at exchange_round" in res[1][1]


DRAIN_SCRIPT = """
import os, sys, time, torch
sys.path.insert(0, os.environ["PYTHONPATH"])
from gpu_mapreduce_amd.parallel import comm as pcomm
from gpu_mapreduce_amd._ext import C
comm = pcomm.init()
assert comm.native.transport.startswith("pg"), comm.native.transport   # two ranks share the GPU
n = 200000
keys = torch.arange(n, dtype=torch.int64) * 2654435761 + comm.rank
kv = C.make_kv(keys.view(torch.uint8), None, keys.view(torch.uint8), None, n, "cuda:0")
t0 = time.time()
try:
    out, st = C.aggregate(kv, comm.native, chunk_bytes=1 << 16, host_sink=True)
    torch.cuda.synchronize()
    print("NO-ERROR", flush=True)
except Exception as e:
    print(f"RAISED after {time.time() - t0:.1f}s: {e}", flush=True)
    os._exit(1)
"""


@pytest.mark.gpu
def test_forced_drain_failure_ends_every_rank_fast(tmp_path):
    """MRH_FAULT=hip:drain_copy:0 fails the first device->host drain copy of a
    host-sink (out-of-core) aggregate on rank 0: the checked HIP call raises,
    the job is poisoned, and BOTH ranks end with an error within seconds —
    no rank reports success over garbage output, none hangs."""
    port = _port()
    procs = []
    t0 = time.time()
    for r in range(2):
        env = dict(ENV0, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONPATH=ROOT, MRH_NUMA_BIND="0",
                   MRH_COMM_TIMEOUT="60", MRH_FAULT="hip:drain_copy:0")
        procs.append(subprocess.Popen([sys.executable, "-c", DRAIN_SCRIPT], cwd=tmp_path, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    try:
        res = [p.communicate(timeout=150) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    elapsed = time.time() - t0
    assert all(p.returncode != 0 for p in procs), res
    assert "HIP error at drain_copy on rank 0" in res[0][0] + res[0][1], res[0]
    assert "NO-ERROR" not in res[1][0], res[1]
    assert elapsed < 60, f"failure took {elapsed:.0f} s to surface"


def test_hip_fault_kind_is_accepted():
    """kind 'hip' parses (it fires only at checked HIP call sites of device paths)"""
    code = """
    import gpu_mapreduce_amd as g
    mr = g.MapReduce(g.Comm(device="cpu"))
    print(mr.map(1, lambda i, kv: kv.add(b"k", b"v")))
    """
    r = _py(code, {"MRH_FAULT": "hip:drain_copy:0"})
    assert r.returncode == 0 and r.stdout.strip() == "1", r.stderr


POOL_SCRIPT = """
import os, sys, time, struct, torch
sys.path.insert(0, os.environ["PYTHONPATH"])
from gpu_mapreduce_amd.parallel import comm as pcomm
import gpu_mapreduce_amd as g
comm = pcomm.init()
t0 = time.time()
try:
    for it in range(40):
        mr = g.MapReduce(comm)
        mr.map(2, lambda i, kv: [kv.add(b"w%d" % (j % 97), struct.pack("<i", j)) for j in range(2000)])
        mr.collate()
        mr.reduce("count")
        torch.cuda.synchronize()
    print("NO-ERROR", flush=True)
except Exception as e:
    print(f"RAISED after {time.time() - t0:.1f}s: {e}", flush=True)
    os._exit(1)
"""


@pytest.mark.gpu
def test_pool_fault_poisons_every_rank(tmp_path):
    """MRH_FAULT=hip:pool:1:200: rank 1's page pool reports a failed event /
    stream wait at its 200th allocation. The pool is then faulted for good
    (the block is never reused, no later allocation is served), the op raises,
    the job is poisoned and both ranks end with an error within seconds."""
    port = _port()
    procs = []
    t0 = time.time()
    for r in range(2):
        env = dict(ENV0, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONPATH=ROOT, MRH_NUMA_BIND="0",
                   MRH_COMM_TIMEOUT="60", MRH_FAULT="hip:pool:1:200")
        procs.append(subprocess.Popen([sys.executable, "-c", POOL_SCRIPT], cwd=tmp_path, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    try:
        res = [p.communicate(timeout=150) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    elapsed = time.time() - t0
    assert all(p.returncode != 0 for p in procs), res
    assert "page pool" in res[1][0] + res[1][1], res[1]
    assert "NO-ERROR" not in res[0][0], res[0]
    assert elapsed < 90, f"failure took {elapsed:.0f} s to surface"
