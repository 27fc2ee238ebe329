#!/usr/bin/env python3
"""Probe: can two processes share the one GPU of a gpurun box through the
native RCCL communicator? If RCCL accepts two ranks on one device, the
multi-rank RCCL shuffle (header allgather + grouped send/recv rounds between
different processes) is exercised for real on the 1-GPU box; if it refuses
(duplicate-GPU check), the refusal is printed and the probe exits 0 — that is
a property of the box, not a failure of the engine.

    timeout -k 10 120 python tools/rccl_probe.py
"""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys, collections, struct
import torch, torch.distributed as dist
sys.path.insert(0, ROOT)
dist.init_process_group("gloo")
import gpu_mapreduce_amd as g
from gpu_mapreduce_amd.parallel.comm import Comm
C = g._ext.C
r, P = dist.get_rank(), dist.get_world_size()
torch.cuda.set_device(0)
store = dist.distributed_c10d._get_default_store()
try:
    nc = C.NativeComm(dist.group.WORLD, "cuda:0", store, "")
except Exception as e:
    print(f"PROBE rank {r}: RCCL refused two ranks on one GPU: {e}", flush=True)
    sys.exit(0)
print(f"PROBE rank {r}: transport {nc.transport}", flush=True)
keys = [b"k%d-%d\0" % (j % 997, r) for j in range(50000)]
import itertools
kd = torch.tensor(list(b"".join(keys)), dtype=torch.uint8)
ko = torch.tensor([0] + list(itertools.accumulate(len(k) for k in keys)), dtype=torch.int64)
vd = torch.full((len(keys) * 4,), r, dtype=torch.uint8)
kv = C.make_kv(kd, ko, vd, None, len(keys), "cuda:0")
out, st = C.aggregate(kv, nc, chunk_bytes=32768)
tot = nc.allreduce([out.n], 0)[0]
assert tot == P * len(keys), tot
print(f"PROBE rank {r}: RCCL aggregate OK, {st.rounds} rounds, {out.n} pairs received, total {tot}", flush=True)
'''


def main():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), MRH_PEER_TIMEOUT="20")
        procs.append(subprocess.Popen([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + CHILD], env=env))
    rc = 0
    for p in procs:
        try:
            rc |= p.wait(timeout=100)
        except subprocess.TimeoutExpired:
            p.kill()
            rc |= 1
    print("PROBE exit", rc, flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
