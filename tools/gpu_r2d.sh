#!/bin/bash
# Grouped-convert check: the new GPU tests first (grouper + InvertedIndex),
# then the headline bench and a timed-path kernel trace, then the full tier.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_grouper.py tests/test_mapreduce_api.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_grp.log 2>&1 && echo "grouper gpu ok" &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ii -o ii -- python bench.py --steps 4 --warmup 1 --phases 0 --pagerank-scale 0 > gpurun_out/prof_ii.log 2>&1 && echo "prof ii ok" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest gpu ok"
rc=$?
tail -3 gpurun_out/pytest_grp.log gpurun_out/pytest_gpu.log 2>/dev/null
exit $rc
