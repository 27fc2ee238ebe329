#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_wf2 -o wf -- python bench.py --workload wordfreq --steps 3 --warmup 1 > gpurun_out/prof_wf2.log 2>&1 && echo "prof wf ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_ii2 -o ii -- python bench.py --steps 3 --warmup 1 --phases 0 --pagerank-scale 0 > gpurun_out/prof_ii2.log 2>&1 && echo "prof ii ok"
