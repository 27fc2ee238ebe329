#!/bin/bash
# PageRank propagation blocking: tests, bench (blocking vs pull), kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_pagerank.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_pr.log 2>&1 && echo "pagerank gpu ok" &&
timeout -k 10 300 python -u bench.py --workload pagerank --steps 3 --warmup 1 > gpurun_out/bench_pr_pb.json 2>/dev/null && cut -c1-500 gpurun_out/bench_pr_pb.json &&
MRH_PR_BLOCKING=0 timeout -k 10 300 python -u bench.py --workload pagerank --steps 3 --warmup 1 > gpurun_out/bench_pr_pull.json 2>/dev/null && cut -c1-500 gpurun_out/bench_pr_pull.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pr -o pr -- python bench.py --workload pagerank --steps 1 --warmup 0 > gpurun_out/prof_pr.log 2>&1 && echo "prof pr ok"
rc=$?
tail -n 3 gpurun_out/pytest_pr.log
exit $rc
