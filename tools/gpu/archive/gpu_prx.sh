#!/bin/bash
# PageRank XCD source ranges: tests, layer sweep, kernel trace
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
step tests 400 python -u -m pytest tests/test_pagerank.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
step prx 300 python bench.py --workload pagerank --steps 3 --warmup 1 || exit $?
step prx_off 300 env MRH_PR_XCD=0 python bench.py --workload pagerank --steps 3 --warmup 1 || exit $?
for l in 1 2 4; do
  step prx_l$l 300 env MRH_PR_XCD_LAYERS=$l python bench.py --workload pagerank --steps 3 --warmup 1 || exit $?
done
step prx_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_prx -o p -- python3 bench.py --workload pagerank --steps 1 --warmup 0 || exit $?
step pmc_prx 120 timeout -s KILL 110 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_prx -o p -- python3 bench.py --workload pagerank --steps 1 --warmup 0 --iters 3 || exit $?
exit 0
