#!/bin/bash
# pipelined collate + hub default: forced single-rank RCCL path, full GPU
# tier, headline bench, tri_find bench at the default hub size.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/rccl_forced.py > gpurun_out/rccl_forced.log 2>&1 && echo "forced rccl ok" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest gpu ok" &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json &&
timeout -k 10 200 python -u bench.py --workload trifind --steps 2 --warmup 1 > gpurun_out/bench_tri.json 2>/dev/null && cut -c1-300 gpurun_out/bench_tri.json
rc=$?
tail -n 3 gpurun_out/pytest_gpu.log
exit $rc
