#!/bin/bash
# tri_find + graph GPU tests, RMAT-24 bench + kernel summary
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_triangles.py tests/test_graph_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tri_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/tri_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload trifind --steps 2 --warmup 1 > gpurun_out/tri.json 2>gpurun_out/tri.err || exit 1
cut -c1-300 gpurun_out/tri.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tri -o tri -- python3 bench.py --workload trifind --steps 1 --warmup 1 > gpurun_out/prof_tri.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
