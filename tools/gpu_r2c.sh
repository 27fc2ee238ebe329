#!/bin/bash
# Round-2 check after the pipelined InvertedIndex: headline bench (with the
# PageRank extra), a timed-path kernel trace of InvertedIndex, then the GPU
# test tier. Every GPU step has its own limit; steps chained with &&.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ii -o ii -- python bench.py --steps 4 --warmup 1 --phases 0 --pagerank-scale 0 > gpurun_out/prof_ii.log 2>&1 && echo "prof ii ok" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest gpu ok"
rc=$?
tail -3 gpurun_out/pytest_gpu.log 2>/dev/null
exit $rc
