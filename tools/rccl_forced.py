#!/usr/bin/env python3
"""Forced-RCCL single-rank check (MRH_FORCE_RCCL=1): every distributed code
path of the engine through a real RCCL communicator on one MI355X, compared
with the local path. Run by tests/test_rccl_gpu.py; also the program profiled
for the RCCL kernel trace under profiles/ (rocprofv3 --kernel-trace)."""
import collections, os, struct, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gpu_mapreduce_amd as g
from gpu_mapreduce_amd import MapReduce
from gpu_mapreduce_amd.models.pagerank import PageRank, rmat_map
C = g._ext.C
dev = "cuda:0"

def comm(force):
    os.environ["MRH_FORCE_RCCL"] = "1" if force else "0"
    c = g.Comm(device=dev)
    c.native  # the native communicator (and its RCCL transport) is created here, under this env
    return c

rc, lc = comm(True), comm(False)
assert rc.native.transport == "rccl", rc.native.transport
assert lc.native.transport == "local"
# what RCCL itself reports about the forced communicator and a probe one
info = rc.rccl_info()
assert (info["comm_count"], info["cu_device"], info["user_rank"]) == (1, 0, 0), info
assert info["live_comms"] == 1, info          # exactly one RCCL communicator in this process
assert lc.rccl_info()["comm_count"] == -1
probe = C.rccl_self_probe(0)
assert (probe["comm_count"], probe["cu_device"]) == (1, 0), probe
assert C.live_rccl_comms() == 1               # the probe is gone again

def var_kv(keys, vals):
    import itertools
    kd = torch.tensor(list(b"".join(keys)), dtype=torch.uint8)
    vd = torch.tensor(list(b"".join(vals)), dtype=torch.uint8)
    ko = torch.tensor([0] + list(itertools.accumulate(len(k) for k in keys)), dtype=torch.int64)
    vo = torch.tensor([0] + list(itertools.accumulate(len(v) for v in vals)), dtype=torch.int64)
    return C.make_kv(kd, ko, vd, vo, len(keys), dev)

def pairs(kv):
    out = []
    C.kv_iter(kv, lambda i, k, v: out.append((bytes(k), bytes(v))))
    return out

keys = [(b"hot" if j % 3 == 0 else b"key%05d" % (j * 7919 % 5003)) + b"\0" for j in range(20000)]
vals = [b"v" * (1 + j % 29) for j in range(20000)]
want = pairs(var_kv(keys, vals))
# P = 1: every pair stays, in input order (stable partition), whatever the rounds
for kw in (dict(), dict(chunk_bytes=4096), dict(chunk_bytes=8192, all2all=0), dict(chunk_bytes=16384, host_sink=True)):
    out, st = C.aggregate(var_kv(keys, vals), rc.native, **kw)
    assert pairs(out) == want, kw
    if kw.get("chunk_bytes"):
        assert st.rounds >= 10, (kw, st.rounds)
    if kw.get("host_sink"):
        assert not out.kdata.is_cuda and out.kdata.is_pinned()
# fixed-width keys / values
fk = torch.arange(100000, dtype=torch.int64).mul_(2654435761).remainder_(1 << 40)
fkv = C.make_kv(fk.view(torch.uint8), None, (fk * 3).view(torch.uint8), None, fk.numel(), dev)
fo, st = C.aggregate(fkv, rc.native, chunk_bytes=65536)
assert torch.equal(fo.kdata.cpu(), fkv.kdata.cpu()) and torch.equal(fo.vdata.cpu(), fkv.vdata.cpu()) and st.rounds >= 10

# scalar collectives and the raw data-plane helpers
assert rc.native.allreduce([5, -3], 0) == [5, -3]
assert rc.native.alltoall_counts([7]) == [7]
x = torch.arange(1000, dtype=torch.float32, device=dev)
assert torch.equal(rc.native.alltoallv(x, [1000], [1000]), x)
assert torch.equal(rc.native.allgather_var(x), x)

# MapReduce ops through RCCL vs local
def wordcount(c, chunk):
    mr = MapReduce(c)
    mr.chunk_bytes = chunk
    mr.map(4, lambda i, kv: [kv.add(w) for w in keys[i::4]])
    n = mr.collate()
    mr.reduce("count")
    return n, sorted((k, struct.unpack("<i", v)[0]) for k, v in mr.kv_pairs())
a, b = wordcount(rc, 0), wordcount(lc, 0)
assert a == b and a[0] == len(set(keys))
assert wordcount(rc, 2048) == b
mr = MapReduce(rc)
mr.map(1, lambda i, kv: [kv.add(k, v) for k, v in zip(keys[:500], vals[:500])])
assert mr.gather(1) == 500 and mr.broadcast(0) == 500
assert sorted(mr.kv_pairs()) == sorted(zip(keys[:500], vals[:500]))

# PageRank and the edge plan: same numbers through the RCCL all-to-all path
def pagerank(c):
    mr = MapReduce(c)
    rmat_map(mr, 14, 8, seed=3)
    pr = PageRank(mr, 1 << 14).build()
    pr.run(20)
    ids, r = pr.ranks()
    return torch.zeros(1 << 14, dtype=torch.float32).index_put_((ids.cpu(),), r.cpu())
pa, pb = pagerank(rc), pagerank(lc)
assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-9), (pa - pb).abs().max()
assert abs(float(pa.sum()) - 1.0) < 1e-3
e = torch.randint(0, 4000, (20000, 2), dtype=torch.int64)
pl_r = C.EdgePlan(rc.native, e, 4000, None, True)
pl_l = C.EdgePlan(lc.native, e, 4000, None, True)
lr, _ = C.connected_components(pl_r, 1000)
ll, _ = C.connected_components(pl_l, 1000)
assert torch.equal(lr.cpu(), ll.cpu())
print("RCCL-FORCED-OK", flush=True)
