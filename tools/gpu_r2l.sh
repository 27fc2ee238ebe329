#!/bin/bash
# rerun of gpu_r2k after the hub-size test fix: triangle tests first, then
# the rest of the GPU tier, headline bench, tri_find bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_triangles.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_tri.log 2>&1 && echo "tri ok" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest gpu ok" &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json &&
timeout -k 10 200 python -u bench.py --workload trifind --steps 2 --warmup 1 > gpurun_out/bench_tri.json 2>/dev/null && cut -c1-300 gpurun_out/bench_tri.json
rc=$?
tail -n 3 gpurun_out/pytest_gpu.log
exit $rc
