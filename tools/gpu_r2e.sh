#!/bin/bash
# One-sweep radix sort check: the radix GPU tests alone first under a short
# limit (a look-back bug would hang), then the bench (InvertedIndex +
# PageRank), a timed-path kernel trace, the full GPU tier.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -u -m pytest tests/test_kernels_gpu.py -k radix -x -v --timeout 60 --timeout-method thread > gpurun_out/pytest_radix.log 2>&1 && echo "radix gpu ok" &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ii -o ii -- python bench.py --steps 4 --warmup 1 --phases 0 --pagerank-scale 0 > gpurun_out/prof_ii.log 2>&1 && echo "prof ii ok" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest gpu ok"
rc=$?
tail -3 gpurun_out/pytest_radix.log gpurun_out/pytest_gpu.log 2>/dev/null
exit $rc
