#!/bin/bash
# tri_find v-major hub kernel: tests (vs CPU merge / brute force, every hub
# kernel), RMAT-24 bench (pull vs bitmap), kernel trace; oracle tests
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
step tri_tests 600 python -u -m pytest tests/test_triangles.py tests/test_oracles.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
step tri_pull 300 python bench.py --workload trifind --steps 3 --warmup 1 || exit $?
step tri_bitmap 300 env MRH_TRI_HUB_KERNEL=bitmap python bench.py --workload trifind --steps 3 --warmup 1 || exit $?
step tri_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tri_pull -o p -- python3 bench.py --workload trifind --steps 2 --warmup 0 || exit $?
step tri_stats 200 python tools/tri_hub_stats.py 24 || exit $?
exit 0
