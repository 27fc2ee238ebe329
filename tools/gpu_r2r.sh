#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_triangles.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_tri.log 2>&1 && echo "tri ok" &&
timeout -k 10 300 python -u bench.py --workload wordfreq --steps 5 --warmup 2 > gpurun_out/bench_wf.json 2>/dev/null && cut -c1-400 gpurun_out/bench_wf.json &&
timeout -k 10 200 python -u bench.py --workload trifind --steps 2 --warmup 1 > gpurun_out/bench_tri.json 2>/dev/null && cut -c1-300 gpurun_out/bench_tri.json && grep -o '"hub_vertices": [0-9]*' gpurun_out/bench_tri.json &&
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "bench_scale" -x -q --timeout 250 --timeout-method thread > gpurun_out/pytest_ii.log 2>&1 && echo "ii bench-scale ok"
rc=$?
tail -n 3 gpurun_out/pytest_ii.log
exit $rc
