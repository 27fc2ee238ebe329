#!/bin/bash
# wordfreq 1 GiB copy/kernel timeline (rocprofv3 kernel + memory-copy trace)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_wf_tl -o p -- python3 bench.py --workload wordfreq --steps 3 --warmup 1 > gpurun_out/wf_tl.log 2>&1
