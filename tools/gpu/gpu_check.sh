#!/bin/bash
# full GPU check: every gpu-marked test, smoke, 1-GPU benches (headline, pagerank, wordfreq)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "start $(date)" > $P
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_ii.log 2>&1
rc=$?; echo "bench ii rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload pagerank --steps 3 --warmup 1 > gpurun_out/bench_pr.log 2>&1
rc=$?; echo "bench pr rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload wordfreq --steps 10 --warmup 2 > gpurun_out/bench_wf.log 2>&1
rc=$?; echo "bench wf rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wf3 -o wf -- python3 bench.py --workload wordfreq --steps 6 --warmup 1 > gpurun_out/prof_wf3.log 2>&1
rc=$?; echo "prof wf rc=$rc $(date)" >> $P
exit $rc
