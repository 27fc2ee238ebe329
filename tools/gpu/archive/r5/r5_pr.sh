#!/bin/bash
# PageRank hot-prefix gather: correctness test, RMAT-26 x20 timing with the
# LDS hot prefix on / off / smaller, kernel stats and L2 counters of the gather
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "start $(date)" > $P
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_pagerank.py -m gpu -k "hot_prefix or xcd or graph" > gpurun_out/pr_test.log 2>&1
rc=$?; echo "test rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
run() {  # name env...
  local name=$1; shift
  timeout -k 10 200 env "$@" python bench.py --workload pagerank --steps 3 --warmup 1 > gpurun_out/pr_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc $(date)" >> $P; return $rc
}
run hot MRH_X=0 || exit $?
run off MRH_PR_HOT=0 || exit $?
run h16k MRH_PR_HOT=16384 || exit $?
run h8k MRH_PR_HOT=8192 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pr_prof -o pr -- python3 bench.py --workload pagerank --steps 1 --warmup 0 > gpurun_out/pr_prof.log 2>&1
rc=$?; echo "prof rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum SQ_WAVES --kernel-include-regex gather -d gpurun_out/pr_pmc_hot -o pr -- python3 bench.py --workload pagerank --steps 1 --warmup 0 --iters 3 > gpurun_out/pr_pmc_hot.log 2>&1
rc=$?; echo "pmc hot rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
MRH_PR_HOT=0 timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum SQ_WAVES --kernel-include-regex gather -d gpurun_out/pr_pmc_off -o pr -- python3 bench.py --workload pagerank --steps 1 --warmup 0 --iters 3 > gpurun_out/pr_pmc_off.log 2>&1
rc=$?; echo "pmc off rc=$rc $(date)" >> $P
exit $rc
