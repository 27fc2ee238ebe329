#!/bin/bash
# GPU: wordfreq tests (in-mapper combiner), bench, kernel profile
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "start $(date)" > $P
timeout -k 10 300 python -u -m pytest tests/test_wordfreq.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_wf.log 2>&1
rc=$?; echo "pytest rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload wordfreq --steps 10 --warmup 2 > gpurun_out/bench_wf.log 2>&1
rc=$?; echo "bench rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wf2 -o wf -- python3 bench.py --workload wordfreq --steps 6 --warmup 1 > gpurun_out/prof_wf2.log 2>&1
rc=$?; echo "prof rc=$rc $(date)" >> $P
exit $rc
