"""Native programs (oink executable, C examples on the MR_* API) as real
multi-process jobs: N processes launched like torchrun ranks (RANK /
WORLD_SIZE / LOCAL_RANK / MASTER_ADDR=127.0.0.1 / MASTER_PORT). On the CPU the
ranks talk through the store transport (csrc/engine/storepg.h); on a GPU box
the same binaries use RCCL. This is the reference's own test method — run
the example programs and OINK scripts (examples/in.*) with mpirun -np N and
compare the printed results — with the P=1 run as the oracle.
"""
import collections
import os
import socket
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gpu_mapreduce_amd")
OINK = os.path.join(PKG, "bin", "oink")
SCRIPTS = os.path.join(ROOT, "examples", "oink")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(cmd, n, cwd, gpu=False, timeout=240):
    """run `cmd` as an n-rank job; returns rank 0's stdout (all ranks must exit 0)"""
    port = _port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(WORLD_SIZE=str(n), RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if not gpu:
            env["HIP_VISIBLE_DEVICES"] = ""
        procs.append(subprocess.Popen(cmd, cwd=cwd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    outs = []
    try:
        for p in procs:
            out, err = p.communicate(timeout=timeout)
            outs.append((p.returncode, out, err))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, (rc, out, err) in enumerate(outs):
        assert rc == 0, f"rank {r} exited {rc}\n{out}\n{err[-3000:]}"
    return outs[0][1]


def _cc(src, out):
    subprocess.run(["gcc", "-O1", "-Wall", src, "-I", os.path.join(ROOT, "csrc", "capi"), "-L", PKG, "-lmrhip",
                    f"-Wl,-rpath,{PKG}", "-o", str(out)], check=True)
    return str(out)


def _lines(out, *prefixes):
    return [ln for ln in out.splitlines() if ln.startswith(prefixes)]


def _docs(d):
    words = ["alpha", "beta", "gamma", "delta", "epsilon", "zeta", "eta"]
    cnt = collections.Counter()
    d.mkdir()
    for i in range(5):
        ws = [words[(i * 5 + j * j + j // 3) % 7] for j in range(400 + 13 * i)]
        cnt.update(ws)
        (d / f"f{i}.txt").write_text(" ".join(ws) + "\n")
    return cnt


@pytest.mark.parametrize("n", [2, 3])
def test_cwordfreq_ranks(tmp_path, n):
    exe = _cc(os.path.join(ROOT, "examples", "c", "cwordfreq.c"), tmp_path / "cwordfreq")
    cnt = _docs(tmp_path / "docs")
    one = launch([exe, "-n", "4", "docs"], 1, tmp_path)
    many = launch([exe, "-n", "4", "docs"], n, tmp_path)
    assert many == one
    assert many.splitlines()[-1] == f"{sum(cnt.values())} total words, {len(cnt)} unique words"
    for ln in many.splitlines()[:4]:
        c, w = ln.split()
        assert cnt[w] == int(c)


def test_crmat_ranks(tmp_path):
    exe = _cc(os.path.join(ROOT, "examples", "c", "crmat.c"), tmp_path / "crmat")
    out = launch([exe, "9", "4", "0.57", "0.19", "0.19", "0.05", "0.1", "3"], 2, tmp_path)
    lines = out.splitlines()
    assert lines[0] == "512 rows in matrix" and lines[1] == "2048 nonzeroes in matrix"
    assert sum(int(ln.split()[0]) * int(ln.split()[3]) for ln in lines[3:]) == 2048


# (script, extra -var args, result-line prefixes that must not depend on P)
SCRIPTS_CASES = [
    ("in.tri", [], ("EdgeUpper", "Tri_find")),
    ("in.cc", [], ("EdgeUpper", "CC_find", "CCStats", "  ")),
    ("in.ccmr", [], ("EdgeUpper", "CC_find", "CCStats", "  ")),
    ("in.luby", [], ("EdgeUpper", "Luby_find")),
    ("in.pagerank", [], ("PageRank: 2",)),
    ("in.rmat", [], ("RMAT: 256", "DegreeStats", "  ")),
    ("in.sssp", [], ("SSSP:",)),
    ("in.luby_mr", [], ("EdgeUpper", "Luby_find")),
    ("in.sssp_mr", [], ("SSSP_MR:",)),
]


def _oink(script, n, cwd, extra, gpu=False):
    return launch([OINK, "-in", os.path.join(SCRIPTS, script), "-var", "scale", "8", *extra], n, cwd, gpu=gpu)


@pytest.mark.parametrize("script,extra,keys", SCRIPTS_CASES, ids=[c[0] for c in SCRIPTS_CASES])
def test_oink_scripts_native_ranks(tmp_path, script, extra, keys):
    one = _oink(script, 1, tmp_path, extra)
    two = _oink(script, 2, tmp_path, extra)
    if script in ("in.sssp", "in.sssp_mr"):
        # sources are drawn per run; the per-source label counts must agree
        pick = lambda o: sorted(ln.split(";")[0] + ";" + ln.split(";")[2] for ln in o.splitlines()
                                if "Source =" in ln)
        assert pick(one) and pick(one) == pick(two)
        return
    if script == "in.pagerank":
        # float sums in a different order: vertex count and iteration count agree
        pick = lambda o: [ln.split(" L1")[0] for ln in _lines(o, "PageRank: 2")]
        assert pick(one) and pick(one) == pick(two)
        return
    assert _lines(one, *keys) and _lines(one, *keys) == _lines(two, *keys)


def test_cc_find_mr_salted_matches_plan_3_ranks(tmp_path):
    """hot-zone splitting across 3 ranks (every zone above 2 vertices is
    salted) gives the same components as the edge-plan cc_find"""
    plan = _oink("in.cc", 3, tmp_path, [])
    mr = _oink("in.ccmr", 3, tmp_path, ["-var", "nthresh", "2"])
    keys = ("CC_find", "CCStats", "  ")
    pick = lambda o: [ln.split(" in ")[0] for ln in _lines(o, *keys)]
    assert pick(plan) and pick(plan) == pick(mr)


def test_oink_wordfreq_script_ranks(tmp_path):
    cnt = _docs(tmp_path / "docs")
    one = launch([OINK, "-in", os.path.join(SCRIPTS, "in.wordfreq"), "-var", "files", "docs"], 1, tmp_path)
    three = launch([OINK, "-in", os.path.join(SCRIPTS, "in.wordfreq"), "-var", "files", "docs"], 3, tmp_path)
    key = lambda o: [ln for ln in o.splitlines() if not ln.startswith("WordFreq:")]
    assert key(one) == key(three)
    assert str(sum(cnt.values())) in one


def test_python_oink_matches_native(tmp_path):
    """the Python OINK binding and the oink executable run the same script to
    the same result"""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(["python", "-m", "gpu_mapreduce_amd.oink", "-in", os.path.join(SCRIPTS, "in.tri"), "-var",
                        "scale", "8"], cwd=tmp_path, env={**env, "PYTHONPATH": ROOT}, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr
    native = _oink("in.tri", 1, tmp_path, [])
    assert _lines(r.stdout, "Tri_find") == _lines(native, "Tri_find") != []


@pytest.mark.gpu
@pytest.mark.parametrize("script", ["in.tri", "in.cc", "in.luby", "in.pagerank", "in.rmat", "in.luby_mr", "in.sssp_mr"])
def test_oink_scripts_native_gpu(tmp_path, script):
    """the same scripts on the MI355X device engine agree with the CPU engine
    (sssp_mr: the per-source iteration and label counts)"""
    keys = dict((c[0], c[2]) for c in SCRIPTS_CASES)[script]
    if script == "in.sssp_mr":
        keys = ("0:  Source", "1:  Source", "2:  Source", "3:  Source")
    cpu = _oink(script, 1, tmp_path, [])
    gpu = _oink(script, 1, tmp_path, [], gpu=True)
    if script == "in.pagerank":
        keys = ("RMAT",)
    assert _lines(cpu, *keys) == _lines(gpu, *keys) != []


# ---------------------------------------------------------------- native apps (csrc/apps)
BIN = os.path.join(PKG, "bin")


def _synth(*args):
    env = dict(os.environ, PYTHONPATH=ROOT, HIP_VISIBLE_DEVICES="")
    subprocess.run(["python", "-m", "gpu_mapreduce_amd.utils.synth", *map(str, args)], check=True, env=env,
                   timeout=240)


def _ii_oracle(d, nfile):
    import re
    idx = {}
    for i in range(nfile):
        name = f"part-{i:05d}"
        b = (d / name).read_bytes()
        for m in re.finditer(rb'<a href="', b):
            e = b.find(b'"', m.end())
            idx.setdefault(b[m.end():e if e >= 0 else len(b)], []).append(name)
    return {k: sorted(v) for k, v in idx.items()}


def _ii_output(outdir):
    got = {}
    for f in sorted(os.listdir(outdir)):
        for ln in (outdir / f).read_bytes().splitlines():
            url, rest = ln.split(b"\t")
            assert url not in got, "a URL must be reduced on exactly one rank"
            got[url] = sorted(x.decode() for x in rest.split())
    return got


def _run_invertedindex(tmp_path, n, gpu):
    d = tmp_path / "html"
    _synth("html", d, 5, 60000, "--nurl", 500)
    out = tmp_path / f"out{n}"
    out.mkdir()
    log = launch([os.path.join(BIN, "invertedindex"), str(d), "5", str(out)], n, tmp_path, gpu=gpu)
    ref = _ii_oracle(d, 5)
    assert _ii_output(out) == ref
    assert f"{sum(len(v) for v in ref.values())} URL KVs, {len(ref)} unique URLs" in log


@pytest.mark.parametrize("n", [1, 2])
def test_invertedindex_app(tmp_path, n):
    _run_invertedindex(tmp_path, n, gpu=False)


def test_intcount_app(tmp_path):
    import numpy as np
    _synth("ints", tmp_path / "ints.bin", 80000, 3000)
    v = np.fromfile(tmp_path / "ints.bin", dtype=np.int32)
    one = launch([os.path.join(BIN, "intcount"), "ints.bin"], 1, tmp_path)
    two = launch([os.path.join(BIN, "intcount"), "ints.bin"], 2, tmp_path)
    assert f"IntCount: {v.size} ints, {np.unique(v).size} unique" in one
    assert f"IntCount: {2 * v.size} ints, {np.unique(v).size} unique" in two   # every rank maps the file
    assert f"Counts sum: {2 * v.size}" in two


def test_wordfreq_app(tmp_path):
    cnt = _docs(tmp_path / "docs")
    one = launch([os.path.join(BIN, "wordfreq"), "-n", "3", "docs"], 1, tmp_path)
    two = launch([os.path.join(BIN, "wordfreq"), "-n", "3", "docs"], 2, tmp_path)
    top = [ln for ln in one.splitlines()[:3]]
    assert [int(x.split()[0]) for x in top] == sorted(cnt.values(), reverse=True)[:3]
    assert two.splitlines()[:4] == one.splitlines()[:4]
    assert f"{sum(cnt.values())} total words, {len(cnt)} unique words" in two
    assert "Time to process 5 files on 2 procs" in two


def test_rmat_app(tmp_path):
    args = [os.path.join(BIN, "rmat"), "10", "4", "0.57", "0.19", "0.19", "0.05", "0.1", "3", "m.mtx"]
    one = launch(args, 1, tmp_path)
    two = launch(args, 2, tmp_path)
    assert one.splitlines()[:2] == ["1024 rows in matrix", "4096 nonzeroes in matrix"]
    histo = lambda o: [ln for ln in o.splitlines() if "rows with" in ln]
    assert sum(int(h.split()[0]) * int(h.split()[3]) for h in histo(one)) == 4096
    # the generator is counter-based: the matrix does not depend on the rank count
    assert histo(one) == histo(two)
    lines = (tmp_path / "m.mtx").read_text().splitlines()
    assert lines[1] == "1024 1024 4096" and len(lines) == 2 + 4096


@pytest.mark.gpu
def test_native_apps_gpu(tmp_path):
    _run_invertedindex(tmp_path, 1, gpu=True)
    _synth("ints", tmp_path / "ints.bin", 80000, 3000)
    out = launch([os.path.join(BIN, "intcount"), "ints.bin"], 1, tmp_path, gpu=True)
    assert "Counts sum: 20000" in out and "(gpu)" in out
    cnt = _docs(tmp_path / "docs")
    out = launch([os.path.join(BIN, "wordfreq"), "-n", "3", "docs"], 1, tmp_path, gpu=True)
    assert f"{sum(cnt.values())} total words, {len(cnt)} unique words" in out
    cpu = launch([os.path.join(BIN, "rmat"), "10", "4", "0.57", "0.19", "0.19", "0.05", "0.1", "3"], 1, tmp_path)
    gpu = launch([os.path.join(BIN, "rmat"), "10", "4", "0.57", "0.19", "0.19", "0.05", "0.1", "3"], 1, tmp_path,
                 gpu=True)
    histo = lambda o: [ln for ln in o.splitlines() if "rows with" in ln]
    assert histo(cpu) == histo(gpu) != []


@pytest.mark.gpu
def test_c_api_device_functors_gpu(tmp_path):
    """MR_map_device_tasks + MR_collate + MR_reduce_device (examples/c/cdevice.c):
    map and reduce are device source strings compiled at run time"""
    exe = _cc(os.path.join(ROOT, "examples", "c", "cdevice.c"), tmp_path / "cdevice")
    out = launch([exe, "1000003", "101"], 1, tmp_path, gpu=True)
    assert "keys 101 sum 1000003 count0 9902 first 9902" in out, out  # sorted by count, largest first
