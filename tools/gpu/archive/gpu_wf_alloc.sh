#!/bin/bash
# wordfreq: memory allocations (HSA-level, pool growth) against the copy
# timeline, to see whether fresh device memory coincides with the slow copy
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "start $(date)" > $P
rm -rf gpurun_out/prof_wf_alloc
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --memory-allocation-trace -d gpurun_out/prof_wf_alloc -o p -- python3 bench.py --workload wordfreq --steps 3 --warmup 6 > gpurun_out/wf_alloc.log 2>&1
echo "alloc trace rc=$? $(date)" >> $P
exit 0
