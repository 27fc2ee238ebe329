#!/bin/bash
# PageRank fused tile step: tests, bench, kernel trace; tri_find hub kernel
# counters (one counter group per pass); available counter list
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
step pr_tests 400 python -u -m pytest tests/test_pagerank.py tests/test_graph_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
step pr_bench 300 python bench.py --workload pagerank --steps 3 --warmup 1 || exit $?
step pr_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pr_b -o p -- python3 bench.py --workload pagerank --steps 1 --warmup 0 || exit $?
step avail 60 rocprofv3 --list-avail || exit $?
step tri_pmc1 120 timeout -s KILL 110 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_tri1 -o p -- python3 bench.py --workload trifind --steps 1 --warmup 0 || exit $?
step tri_pmc2 120 timeout -s KILL 110 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/pmc_tri2 -o p -- python3 bench.py --workload trifind --steps 1 --warmup 0 || exit $?
exit 0
