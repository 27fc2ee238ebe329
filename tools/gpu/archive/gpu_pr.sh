#!/bin/bash
# PageRank: graph GPU tests, RMAT-26 bench, kernel summary
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_pagerank.py tests/test_graph_gpu.py tests/test_wavesegred_gpu.py tests/test_bench_launcher.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pr_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pr_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload pagerank --steps 5 --warmup 1 > gpurun_out/pr.json 2>gpurun_out/pr.err || exit 1
cut -c1-250 gpurun_out/pr.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pr -o pr -- python3 bench.py --workload pagerank --steps 1 --warmup 0 > gpurun_out/prof_pr.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
