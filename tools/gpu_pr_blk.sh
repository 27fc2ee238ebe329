#!/bin/bash
# PageRank source-range blocking (MRH_PR_SRC_BLOCKS) sweep + scale sweep + L2 PMC passes
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
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
step prb_tests 300 env MRH_PR_SRC_BLOCKS=3 python -u -m pytest tests/test_pagerank.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
for b in 1 2 4 8; do
  step prb_$b 300 env MRH_PR_SRC_BLOCKS=$b python bench.py --workload pagerank --steps 3 --warmup 1 || exit $?
done
for sc in 24 25; do
  step prs_$sc 300 python bench.py --workload pagerank --scale $sc --steps 3 --warmup 1 || exit $?
done
step pmc_hit 120 timeout -s KILL 110 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_pr1 -o p -- python3 bench.py --workload pagerank --steps 1 --warmup 0 --iters 3 || exit $?
step pmc_hit4 120 env MRH_PR_SRC_BLOCKS=4 timeout -s KILL 110 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_pr4 -o p -- python3 bench.py --workload pagerank --steps 1 --warmup 0 --iters 3 || exit $?
exit 0
