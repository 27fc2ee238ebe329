#!/bin/bash
# rocprofv3 kernel stats of the wordfreq and InvertedIndex benches (1 GPU)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wf -o wf -- python3 bench.py --workload wordfreq --steps 6 --warmup 1 > gpurun_out/prof_wf.log 2>&1
rc=$?; echo "wf rc=$rc" > gpurun_out/progress.txt; [ $rc -eq 0 ] || exit $rc
exit 0
