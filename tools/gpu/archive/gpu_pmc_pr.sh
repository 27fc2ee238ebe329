#!/bin/bash
# PMC counters for the PageRank gather-reduce kernel (L2 hit rate, HBM bytes)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_pr1 -o pr -- python3 bench.py --workload pagerank --steps 1 --warmup 0 --iters 3 > gpurun_out/pmc_pr1.log 2>&1
rc=$?; echo "pmc1 rc=$rc" > gpurun_out/progress.txt; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_pr2 -o pr -- python3 bench.py --workload pagerank --steps 1 --warmup 0 --iters 3 > gpurun_out/pmc_pr2.log 2>&1
rc=$?; echo "pmc2 rc=$rc" >> gpurun_out/progress.txt
exit $rc
