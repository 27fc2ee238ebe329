#!/bin/bash
# tri_find RMAT-24 kernel trace at the current defaults
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --workload trifind --steps 3 --warmup 1 > gpurun_out/tri_now.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tri_now -o p -- python3 bench.py --workload trifind --steps 2 --warmup 0 > gpurun_out/tri_now_prof.log 2>&1 || exit $?
exit 0
