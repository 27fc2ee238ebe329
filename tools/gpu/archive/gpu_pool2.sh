#!/bin/bash
# page pool with the per-stream size-class cache: tests, suites with the pool, headline with the pool
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
NOX="--pagerank-scale 0 --trifind-scale 0 --wordfreq-bytes 0"
step pool_tests 400 python -u -m pytest tests/test_hbm_pool.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
step pool_suite 600 env MRH_HBM_POOL=1 python -u -m pytest tests/test_outofcore.py tests/test_kernels_gpu.py tests/test_wordfreq.py tests/test_pagerank.py tests/test_triangles.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
step ii_pool 200 env MRH_HBM_POOL=1 python bench.py $NOX || exit $?
step ii_nopool 200 python bench.py $NOX || exit $?
step pr_pool 200 env MRH_HBM_POOL=1 python bench.py --workload pagerank --steps 3 --warmup 1 || exit $?
step tri_pool 200 env MRH_HBM_POOL=1 python bench.py --workload trifind --steps 3 --warmup 1 || exit $?
step wf_pool 200 env MRH_HBM_POOL=1 python bench.py --workload wordfreq --steps 5 --warmup 2 || exit $?
exit 0
