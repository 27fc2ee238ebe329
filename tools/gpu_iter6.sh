#!/bin/bash
# full GPU test suite + 1-GPU benches (long InvertedIndex run to see steady state)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "start $(date)" > $P
timeout -k 10 500 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_ii.log 2>&1
rc=$?; echo "bench ii rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload pagerank --steps 3 --warmup 1 > gpurun_out/bench_pr.log 2>&1
rc=$?; echo "bench pr rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload wordfreq --steps 5 --warmup 2 > gpurun_out/bench_wf.log 2>&1
rc=$?; echo "bench wf rc=$rc $(date)" >> $P
exit $rc
