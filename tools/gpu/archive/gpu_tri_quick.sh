#!/bin/bash
# tri_find: GPU tests, RMAT-24 bench, kernel trace
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-q}
timeout -k 10 400 python -u -m pytest tests/test_triangles.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tri_tests_$T.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --workload trifind --steps 3 --warmup 1 > gpurun_out/tri_bench_$T.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tri_$T -o p -- python3 bench.py --workload trifind --steps 2 --warmup 0 > gpurun_out/tri_prof_$T.log 2>&1 || exit $?
exit 0
