#!/bin/bash
# radix sort variants (2048 vs 4096-pair tiles) + grouper insert change:
# micro-bench, grouper/radix tests, II bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -u -m pytest tests/test_kernels_gpu.py tests/test_grouper.py -k "radix or group" -x -q --timeout 60 --timeout-method thread > gpurun_out/pytest_radix.log 2>&1 && echo "radix+grouper gpu ok" &&
timeout -k 10 200 python -u tools/radix_bench.py > gpurun_out/radix_it8.log 2>&1 && cat gpurun_out/radix_it8.log &&
MRH_RX_IT=16 timeout -k 10 200 python -u tools/radix_bench.py > gpurun_out/radix_it16.log 2>&1 && cat gpurun_out/radix_it16.log &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --pagerank-scale 0 > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json
