#!/bin/bash
# tri_find sparse-hub kernel (sorted words, flattened pairs) + HBM page pool:
# tests, tri_find bench + trace, page-pool tests, headline bench with the pool
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
step tri_tests 600 python -u -m pytest tests/test_triangles.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
step tri_bench 300 python bench.py --workload trifind --steps 3 --warmup 1 || exit $?
step tri_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tri_s2 -o p -- python3 bench.py --workload trifind --steps 2 --warmup 0 || exit $?
step pool_tests 400 python -u -m pytest tests/test_hbm_pool.py tests/test_outofcore.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
step pool_ooc 300 env MRH_HBM_POOL=1 python -u -m pytest tests/test_outofcore.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
step ii_pool 300 env MRH_HBM_POOL=1 python bench.py --pagerank-scale 0 --trifind-scale 0 --wordfreq-bytes 0 || exit $?
exit 0
