#!/bin/bash
# full GPU pass: every gpu test, smoke, the default bench record (headline +
# extras), PageRank kernel trace + L2 counters. Usage: gpu_full.sh [tag]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:-full}
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "start $(date)" > $P
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(date)" >> $P
  return $rc
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench_$T 300 python bench.py || exit $?
step pr_prof_$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pr_$T -o p -- python3 bench.py --workload pagerank --steps 1 --warmup 0 || exit $?
step pr_pmc_$T 120 timeout -s KILL 110 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_pr_$T -o p -- python3 bench.py --workload pagerank --steps 1 --warmup 0 --iters 3 || exit $?
exit 0
