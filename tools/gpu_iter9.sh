#!/bin/bash
# static-segment wave kernel: numerics, graph/pagerank tests, PageRank bench old vs new, rocprof
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "start $(date)" > $P
timeout -k 10 300 python -u -m pytest tests/test_wavesegred_gpu.py tests/test_graph_gpu.py tests/test_pagerank.py tests/test_oink.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ws.log 2>&1
rc=$?; echo "pytest rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload pagerank --steps 3 --warmup 1 > gpurun_out/bench_pr_ws.log 2>&1
rc=$?; echo "bench pr ws rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
MRH_PLAN_KERNEL=tiles timeout -k 10 300 python bench.py --workload pagerank --steps 3 --warmup 1 > gpurun_out/bench_pr_tiles.log 2>&1
rc=$?; echo "bench pr tiles rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_pr" -o pr -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload pagerank --steps 1 --warmup 0 > "$GRAFT_REPO_ROOT/gpurun_out/bench_pr_prof.log" 2>&1
rc=$?; echo "prof pr rc=$rc $(date)" >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
exit $rc
