#!/bin/bash
# host->HBM copy engines: SDMA (default) vs blit kernels (HSA_ENABLE_SDMA=0),
# then the headline bench under each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/h2d_bw.py > gpurun_out/h2d_sdma.log 2>&1 && cat gpurun_out/h2d_sdma.log &&
HSA_ENABLE_SDMA=0 timeout -k 10 120 python -u tools/h2d_bw.py > gpurun_out/h2d_blit.log 2>&1 && cat gpurun_out/h2d_blit.log &&
HSA_ENABLE_SDMA=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --pagerank-scale 0 > gpurun_out/bench_blit.json 2>/dev/null && cut -c1-400 gpurun_out/bench_blit.json
