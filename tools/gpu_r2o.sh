#!/bin/bash
# wordfreq: phase timing (map vs collate/reduce vs sort) and a kernel trace
# of the bench to find the time above the 19 ms H2D floor.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/wf_time.py > gpurun_out/wf_time.log 2>&1 && cat gpurun_out/wf_time.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_wf -o wf -- python bench.py --workload wordfreq --steps 3 --warmup 1 > gpurun_out/prof_wf.log 2>&1 && echo "prof wf ok"
