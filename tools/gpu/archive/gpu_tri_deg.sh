#!/bin/bash
# tri_find partitioned degree count: tests, bench, trace; dense core re-test
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
step tri_tests 500 python -u -m pytest tests/test_triangles.py tests/test_oink.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
step tri_bench 200 python bench.py --workload trifind --steps 3 --warmup 1 || exit $?
step tri_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tri_deg -o p -- python3 bench.py --workload trifind --steps 2 --warmup 0 || exit $?
for c in 4096 16384; do
  step tri_core_$c 200 env MRH_TRI_CORE=$c python bench.py --workload trifind --steps 3 --warmup 1 || exit $?
done
exit 0
