"""The RCCL data path on a real MI355X (VERDICT r1 "exercise the real RCCL
code path on the 1-GPU box").

MRH_FORCE_RCCL=1 gives a world-size-1 job a real RCCL communicator (comm.h):
every distributed code path runs exactly as on 8 GPUs — header allgather,
grouped ncclSend/ncclRecv rounds (chunked, ring-ordered, host-sink), scalar
ncclAllReduce, ncclBroadcast, and the PageRank / edge-plan all-to-alls — and
its results must equal the local (non-RCCL) path bit for bit. Each case runs
in a child process so the RCCL communicator is created and torn down cleanly.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = os.path.join(ROOT, "tools", "rccl_forced.py")


@pytest.mark.gpu
def test_forced_rccl_single_rank_matches_local():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, SCRIPT], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-5000:]
    assert "RCCL-FORCED-OK" in r.stdout


_BIG = r"""
import os, sys, torch
os.environ["MRH_FORCE_RCCL"] = "1"
os.environ.pop("MRH_RCCL_MAX_MSG", None)   # the default piece size
sys.path.insert(0, sys.argv[1])
import gpu_mapreduce_amd as g
C = g._ext.C
comm = g.Comm(device="cuda:0")
nc = comm.native
assert nc.transport == "rccl", nc.transport
assert nc.max_msg == 1 << 28, nc.max_msg
n = (3 << 27) + 5                      # 1.5 GiB of int64 + 40 bytes
x = torch.arange(n, dtype=torch.int64, device="cuda").mul_(2654435761)
y = nc.alltoallv(x, [n], [n])
assert torch.equal(x, y), "alltoallv of 1.5 GiB not bitwise equal"
del y
kv = C.make_kv(x.view(torch.uint8), None, torch.empty(0, dtype=torch.uint8, device="cuda"), None, n, "cuda:0")
out, st = C.exchange(kv, torch.zeros(n, dtype=torch.int32, device="cuda"), nc)
assert torch.equal(x, out.kdata.view(torch.int64)), "exchange of 1.5 GiB not bitwise equal"
print("BIG-OK")
"""


@pytest.mark.gpu
def test_forced_rccl_large_transfers_bitwise():
    """RCCL 2.26.6 corrupted single point-to-point messages of ~1 GiB and more
    (profiles/r4_rccl_big_messages.txt); the transport cuts every transfer into
    pieces of the communicator's agreed size (256 MiB by default): a 1.5 GiB
    alltoallv and a 1.5 GiB exchange through a forced RCCL communicator must
    come back bit for bit"""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", _BIG, ROOT], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-5000:]
    assert "BIG-OK" in r.stdout
