"""MR_* C API (csrc/capi/cmapreduce.h over libmrhip.so): a C test program
covering every op family, and the C example apps (examples/c), compiled with
the system C compiler and run as separate processes. The CPU variant runs
here; the gpu variant runs the same binaries on an MI355X (the native
communicator binds the process to the GPU and the engine runs HIP kernels)."""
import collections
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gpu_mapreduce_amd")


def _cc(src, out):
    subprocess.run(["gcc", "-O1", "-Wall", src, "-I", os.path.join(ROOT, "csrc", "capi"), "-L", PKG, "-lmrhip",
                    f"-Wl,-rpath,{PKG}", "-o", str(out)], check=True)
    return str(out)


def _env(gpu):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    if not gpu:
        env["HIP_VISIBLE_DEVICES"] = ""   # force the CPU engine
    return env


def _run_capi_test(tmp_path, gpu):
    exe = _cc(os.path.join(ROOT, "tests", "capi", "capi_test.c"), tmp_path / "capi_test")
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, env=_env(gpu), timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout


def _run_wordfreq(tmp_path, gpu):
    exe = _cc(os.path.join(ROOT, "examples", "c", "cwordfreq.c"), tmp_path / "cwordfreq")
    words = ["alpha", "beta", "gamma", "delta", "epsilon", "zeta"]
    cnt = collections.Counter()
    d = tmp_path / "docs"
    d.mkdir()
    for i in range(4):
        ws = [words[(i * 7 + j * j) % 6] for j in range(300 + i)]
        cnt.update(ws)
        (d / f"f{i}.txt").write_text(" ".join(ws) + "\n")
    r = subprocess.run([exe, "-n", "3", str(d)], capture_output=True, text=True, env=_env(gpu), timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().splitlines()
    top = [(int(a), b) for a, b in (ln.split() for ln in lines[:3])]
    assert [c for c, _ in top] == sorted(cnt.values(), reverse=True)[:3]
    for c, w in top:
        assert cnt[w] == c
    assert lines[3] == f"{sum(cnt.values())} total words, {len(cnt)} unique words"


def _run_crmat(tmp_path, gpu):
    exe = _cc(os.path.join(ROOT, "examples", "c", "crmat.c"), tmp_path / "crmat")
    r = subprocess.run([exe, "9", "4", "0.57", "0.19", "0.19", "0.05", "0.1", "3"], capture_output=True, text=True,
                       env=_env(gpu), timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[0] == "512 rows in matrix" and lines[1] == "2048 nonzeroes in matrix"
    tot = 0
    for ln in lines[3:]:
        rows, _, _, nz, _ = ln.split()
        tot += int(rows) * int(nz)
    assert tot == 2048


def test_capi_cpu(tmp_path):
    _run_capi_test(tmp_path, gpu=False)


def test_capi_examples_cpu(tmp_path):
    _run_wordfreq(tmp_path, gpu=False)
    _run_crmat(tmp_path, gpu=False)


@pytest.mark.gpu
def test_capi_gpu(tmp_path):
    _run_capi_test(tmp_path, gpu=True)
    _run_wordfreq(tmp_path, gpu=True)
    _run_crmat(tmp_path, gpu=True)
