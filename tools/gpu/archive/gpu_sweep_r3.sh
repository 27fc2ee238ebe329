#!/bin/bash
# InvertedIndex staging-ring depth sweep (MRH_II_BUFS), tri_find degree
# kernel variants (MRH_TRI_DEG), wordfreq job pipeline
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
for b in 2 3 4; do
  step ii_b$b 200 env MRH_II_BUFS=$b python bench.py $NOX || exit $?
done
step tri_deg_atomic 200 python bench.py --workload trifind --steps 3 --warmup 1 || exit $?
step tri_deg_lds 200 env MRH_TRI_DEG=lds python bench.py --workload trifind --steps 3 --warmup 1 || exit $?
step wf 200 python bench.py --workload wordfreq --steps 10 --warmup 2 || exit $?
step tri_tests 400 env MRH_TRI_DEG=lds python -u -m pytest tests/test_triangles.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
step pool_tests 400 python -u -m pytest tests/test_hbm_pool.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
step pool_suite 400 env MRH_HBM_POOL=1 python -u -m pytest tests/test_outofcore.py tests/test_kernels_gpu.py tests/test_wordfreq.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
step ii_pool 200 env MRH_HBM_POOL=1 python bench.py $NOX || exit $?
exit 0
