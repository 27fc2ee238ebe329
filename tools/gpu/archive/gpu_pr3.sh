#!/bin/bash
# PageRank plan build (device kernels) + InvertedIndex timeline: GPU tests,
# setup split, benches, kernel traces
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
step pr_tests 400 python -u -m pytest tests/test_pagerank.py tests/test_distributed_gpu.py tests/test_rccl_gpu.py tests/test_native_multiproc.py tests/test_faults.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
step pr_setup 300 python tools/pr_setup_time.py 26 || exit $?
step pr_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pr -o pr -- python3 tools/pr_setup_time.py 26 || exit $?
step bench 400 python bench.py || exit $?
tail -1 gpurun_out/bench.log > gpurun_out/bench.json
step ii_prof 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_ii -o ii -- python3 bench.py --steps 4 --warmup 1 --phases 0 --pagerank-scale 0 --trifind-scale 0 --wordfreq-bytes 0 || exit $?
exit 0
