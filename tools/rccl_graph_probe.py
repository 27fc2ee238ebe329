#!/usr/bin/env python3
"""Which RCCL operations survive HIP-graph capture on a one-rank communicator?
Each op runs in its own child process (a crash names the op and the step).
usage: rccl_graph_probe.py [op[:mode] ...]   (mode: 0 global, 1 thread-local (default), 2 relaxed)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OPS = sys.argv[1:] or ["allreduce", "allgather", "broadcast", "self", "self_inplace"]
CHILD = ("import sys; sys.path.insert(0, %r); from gpu_mapreduce_amd import C; "
         "op, _, m = sys.argv[1].partition(':'); "
         "print('RESULT', sys.argv[1], C.rccl_graph_probe(0, op, True, int(m or 1)), flush=True)") % ROOT
for op in OPS:
    p = subprocess.run([sys.executable, "-c", CHILD, op], capture_output=True, text=True, timeout=120)
    steps = [ln for ln in p.stderr.splitlines() if ln.startswith("[rccl_graph_probe]")]
    res = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT")]
    nodes = [ln.split(":")[-1].strip() for ln in steps if "graph nodes" in ln]
    print(f"{op:15s} rc={p.returncode} {res[-1] if res else ''} graph_nodes={nodes[-1] if nodes else '-'} "
          f"last={steps[-1] if steps else ''}", flush=True)
    if p.returncode != 0:  # a crashed child: nothing more on the GPU in this run
        print(p.stderr[-2000:], flush=True)
        sys.exit(1)
