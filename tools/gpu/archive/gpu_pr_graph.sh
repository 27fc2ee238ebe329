#!/bin/bash
# PageRank HIP-graph replay: tests, bench with and without, kernel trace
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
step pr_tests 400 python -u -m pytest tests/test_pagerank.py tests/test_graph_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
step pr_graph 200 python bench.py --workload pagerank --steps 5 --warmup 1 || exit $?
step pr_nograph 200 env MRH_PR_GRAPH=0 python bench.py --workload pagerank --steps 5 --warmup 1 || exit $?
step pr_graph2 200 python bench.py --workload pagerank --steps 5 --warmup 1 || exit $?
step pr_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pr_graph -o p -- python3 bench.py --workload pagerank --steps 1 --warmup 0 || exit $?
exit 0
