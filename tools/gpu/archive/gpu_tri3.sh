#!/bin/bash
# tri_find hub kernel: LDS bitmap vs global bitmaps (MRH_TRI_HUB_KERNEL), tests, kernel trace
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
step tri_tests 400 python -u -m pytest tests/test_triangles.py tests/test_oink.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
step tri_lds 300 python bench.py --workload trifind --steps 3 --warmup 1 || exit $?
step tri_bitmap 300 env MRH_TRI_HUB_KERNEL=bitmap python bench.py --workload trifind --steps 3 --warmup 1 || exit $?
step tri_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tri -o tri -- python3 bench.py --workload trifind --steps 2 --warmup 1 || exit $?
exit 0
