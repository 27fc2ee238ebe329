"""HBM page pool (csrc/engine/hbmpool.h): the engine's device allocator with a
hard cap (reference page pool, src/mapreduce.cpp:3318-3547).

The pool must be installed before the process allocates device memory, so
every GPU case runs in a child process with MRH_HBM_POOL=1."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _child(code, timeout=240):
    env = dict(os.environ, PYTHONPATH=ROOT, MRH_HBM_POOL="1")
    env.pop("MRH_GUARD", None)
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def test_pool_stats_shape_cpu():
    from gpu_mapreduce_amd.runtime import hbm_pool
    s = hbm_pool.stats(0)
    assert set(s) == {"in_use", "peak", "reserved", "reserved_peak", "cap", "allocs", "frees", "failures", "cached",
                      "cross_stream_reuse", "faulted", "grows", "grow_ms", "releases", "oom_retries"}


BASIC = r'''
import torch
import gpu_mapreduce_amd as g
from gpu_mapreduce_amd.runtime import hbm_pool
assert hbm_pool.installed()
s0 = hbm_pool.stats(0)
x = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
s1 = hbm_pool.stats(0)
assert s1["in_use"] - s0["in_use"] >= 64 << 20, (s0, s1)
# a block used on a side stream is freed behind that stream's work
side = torch.cuda.Stream()
y = torch.ones(1 << 24, device="cuda")
with torch.cuda.stream(side):
    z = y * 2
y.record_stream(side)
del y
torch.cuda.synchronize()
assert float(z.sum()) == 2.0 * (1 << 24)
del x, z
torch.cuda.synchronize()
s2 = hbm_pool.stats(0)
assert s2["in_use"] <= s0["in_use"] + 4096 and s2["peak"] >= s1["in_use"], (s0, s2)
# an end-to-end job on pool memory, checked against the host oracle
from gpu_mapreduce_amd.models.inverted_index import InvertedIndex, reference_inverted_index
from gpu_mapreduce_amd.utils import synth
files = synth.html_corpus(4 << 20, file_bytes=1 << 20, seed=3, nurl=3000, device="cuda")
files = [(n, t.cpu().pin_memory()) for n, t in files]
app = InvertedIndex(g.MapReduce(g.Comm(device="cuda")), files)
app.run()
got = {}
for line in app.output_lines():
    url, rest = line.split("\t")
    got[url.encode()] = sorted(rest.split())
assert got == reference_inverted_index(files)
hbm_pool.trim(0)
print("ok", hbm_pool.stats(0))
'''

CAP = r'''
import torch
import gpu_mapreduce_amd as g
from gpu_mapreduce_amd import C
from gpu_mapreduce_amd.runtime import hbm_pool
comm = g.Comm(device="cuda")
# hard cap: a tensor past it fails with the page-pool error
hbm_pool.set_cap(hbm_pool.stats(0)["in_use"] + (8 << 20), 0)
try:
    torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
    raise SystemExit("allocation past the cap succeeded")
except torch.OutOfMemoryError as e:
    assert "Cannot allocate page" in str(e), e
hbm_pool.set_cap(0, 0)
assert hbm_pool.stats(0)["failures"] >= 1
# a MapReduce op under a page budget (1 MiB pages, maxpage 4): the map's
# 64 MiB of pairs are spooled to pinned host. clone() has an out-of-core
# path and clones them where they live; collapse() has none and must bring
# them back to HBM: 64 MiB of new device memory > 2 x 4 MiB + 16 MiB of
# scratch -> Cannot allocate page
n = 8 << 20
mr = g.MapReduce(comm)
mr.memsize = -(1 << 20)  # 1 MiB pages
mr.maxpage = 4
k = torch.arange(n, dtype=torch.int64, device="cuda")
emit = lambda itask, kv: kv.add_kv(C.make_kv(k, None, k, None, n, "cuda"))
mr.map(1, emit)
assert mr.clone() == n
assert not mr.kmv.vdata.is_cuda
mr.map(1, emit)
try:
    mr.collapse(b"all")
    raise SystemExit("collapse past the page budget succeeded")
except Exception as e:
    assert "Cannot allocate page" in str(e), e
# the same budget large enough: the op runs in HBM
mr.maxpage = 256
mr.map(1, emit)
mr.clone()
assert mr.kmv.nkey == n and mr.kmv.vdata.is_cuda
print("ok", hbm_pool.stats(0))
'''


@pytest.mark.gpu
def test_pool_basic_and_stream_order_gpu():
    assert _child(BASIC).startswith("ok")


@pytest.mark.gpu
def test_pool_cap_and_page_budget_gpu():
    assert _child(CAP).startswith("ok")


CROSS = r'''
import torch
import gpu_mapreduce_amd as g
from gpu_mapreduce_amd.runtime import hbm_pool
assert hbm_pool.installed()
side = torch.cuda.Stream()
# blocks freed on the side stream serve the main stream's requests of their
# class (behind an event) instead of growing the pool
with torch.cuda.stream(side):
    xs = [torch.full((1 << 22,), float(i), device="cuda") for i in range(8)]
    ref = [float(x.sum()) for x in xs]
with torch.cuda.stream(side):
    del xs
torch.cuda.synchronize()
r0 = hbm_pool.stats(0)
ys = [torch.ones(1 << 22, device="cuda") for _ in range(8)]
torch.cuda.synchronize()
r1 = hbm_pool.stats(0)
assert r1["cross_stream_reuse"] - r0["cross_stream_reuse"] >= 8, (r0, r1)
assert r1["reserved"] <= r0["reserved"], (r0, r1)   # no growth
assert all(float(y.sum()) == float(1 << 22) for y in ys)
# concurrent op caps never leave a stale cap behind (advisor r3)
from gpu_mapreduce_amd import C
import threading
def op():
    mr = g.MapReduce(g.Comm(device="cuda"))
    mr.memsize = -(1 << 20)
    mr.maxpage = 64
    k = torch.arange(1 << 18, dtype=torch.int64, device="cuda")
    for _ in range(5):
        mr.map(1, lambda i, kv: kv.add_kv(C.make_kv(k, None, k, None, k.numel(), "cuda")))
        mr.convert()
ts = [threading.Thread(target=op) for _ in range(4)]
[t.start() for t in ts]
[t.join() for t in ts]
assert hbm_pool.stats(0)["cap"] == 0, hbm_pool.stats(0)
print("ok", hbm_pool.stats(0))
'''


@pytest.mark.gpu
def test_pool_cross_stream_reuse_and_concurrent_caps_gpu():
    assert _child(CROSS).startswith("ok")


ARENA = r'''
import torch
import gpu_mapreduce_amd as g
from gpu_mapreduce_amd.runtime import hbm_pool
comm = g.Comm(device="cuda:0")
GiB = 1 << 30
st0 = hbm_pool.stats(0)
# a job's mix of big sizes: once a segment holds the peak, later sizes are cut
# from it (best fit) and coalesce again when freed: no new device allocation
big = torch.empty(6 * GiB, dtype=torch.uint8, device="cuda")
del big
grows = hbm_pool.stats(0)["grows"]
a = torch.empty(3 * GiB, dtype=torch.uint8, device="cuda")
b = torch.empty(2 * GiB, dtype=torch.uint8, device="cuda")
a.fill_(1); b.fill_(2)
assert hbm_pool.stats(0)["grows"] == grows
del a, b
c = torch.empty(6 * GiB - (64 << 20), dtype=torch.uint8, device="cuda")  # the freed pieces coalesced
c.fill_(3)
assert hbm_pool.stats(0)["grows"] == grows, hbm_pool.stats(0)
del c
# data written on another stream before a free is not overwritten by the next user early
s = torch.cuda.Stream()
x = torch.empty(GiB, dtype=torch.uint8, device="cuda")
with torch.cuda.stream(s):
    x.fill_(7)
    x.record_stream(s)
del x
y = torch.zeros(GiB, dtype=torch.uint8, device="cuda")  # waits for the fill on s
torch.cuda.synchronize()
assert int(y.max().item()) == 0
del y
st3 = hbm_pool.stats(0)
assert st3["reserved_peak"] <= int(1.5 * max(st3["peak"], 6 * GiB)) + 2 * GiB, st3
hbm_pool.trim(0)
st4 = hbm_pool.stats(0)
assert st4["reserved"] < st3["reserved"], (st3, st4)
print("ok", st4)
'''


@pytest.mark.gpu
def test_pool_big_block_arena_gpu():
    """big blocks (>= 256 MiB) are cut best-fit from segments and coalesce, so
    a new mix of sizes reuses the memory held (no growth); a block freed
    after use on another stream is handed out behind that stream's work;
    reserved stays within 1.5x of the bytes in use; trim returns segments"""
    assert _child(ARENA).startswith("ok")


@pytest.mark.gpu
def test_pool_retired_stream_is_forgotten():
    """Blocks cached on an engine stream that is destroyed (a PageRank plan's
    exchange stream, an RCCL communicator's stream) are released by
    forget_stream first: a later allocation of the same class from another
    stream must not record an event on the dead stream (that was a segfault
    inside the HIP runtime at 2 ranks, bench.py --gpus 2 on one GPU)"""
    assert _child(RETIRE).startswith("ok")


RETIRE = r"""
import torch
import gpu_mapreduce_amd as g
from gpu_mapreduce_amd.runtime import hbm_pool
assert hbm_pool.installed()
n = 3 << 20
for _ in range(3):
    assert g._ext.C.hbm_pool_stream_retire_check(0, n) == 2 * n
print("ok")
"""
