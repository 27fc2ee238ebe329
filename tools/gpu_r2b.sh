#!/bin/bash
# GPU tier + library-kernel audit: pytest -m gpu, then kernel traces of the
# InvertedIndex and wordfreq benches (no rocPRIM / bincount / index kernels
# may appear), each step time-limited and chained with &&.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest gpu ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ii -o ii -- python bench.py --steps 4 --warmup 1 --phases 0 --pagerank-scale 0 > gpurun_out/prof_ii.log 2>&1 && echo "prof ii ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wf -o wf -- python bench.py --workload wordfreq --steps 3 --warmup 1 > gpurun_out/prof_wf.log 2>&1 && echo "prof wf ok"
rc=$?
tail -3 gpurun_out/pytest_gpu.log
exit $rc
