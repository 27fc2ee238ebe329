#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/h2d_chunks.py > gpurun_out/h2d_chunks.log 2>&1 && cat gpurun_out/h2d_chunks.log &&
timeout -k 10 400 python -u -m pytest tests/test_triangles.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_tri.log 2>&1 && echo "tri ok" &&
timeout -k 10 200 python -u bench.py --workload trifind --steps 2 --warmup 1 > gpurun_out/bench_tri.json 2>/dev/null && cut -c1-300 gpurun_out/bench_tri.json &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tri -o tri -- python bench.py --workload trifind --steps 1 --warmup 0 > gpurun_out/prof_tri.log 2>&1 && echo "prof tri ok"
