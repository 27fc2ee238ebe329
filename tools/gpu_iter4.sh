#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "start $(date)" > gpurun_out/progress.txt
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_pagerank.py tests/test_wordfreq.py -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(date)" >> gpurun_out/progress.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload pagerank --steps 3 --warmup 1 > gpurun_out/bench_pr.log 2>&1
rc=$?; echo "bench pr rc=$rc $(date)" >> gpurun_out/progress.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload wordfreq --steps 3 --warmup 1 > gpurun_out/bench_wf.log 2>&1
rc=$?; echo "bench wf rc=$rc $(date)" >> gpurun_out/progress.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_pr" -o pr -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload pagerank --steps 1 --warmup 0 > "$GRAFT_REPO_ROOT/gpurun_out/bench_pr_prof.log" 2>&1
rc=$?; echo "prof pr rc=$rc $(date)" >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_wf" -o wf -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload wordfreq --steps 1 --warmup 0 > "$GRAFT_REPO_ROOT/gpurun_out/bench_wf_prof.log" 2>&1
rc=$?; echo "prof wf rc=$rc $(date)" >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
exit $rc
