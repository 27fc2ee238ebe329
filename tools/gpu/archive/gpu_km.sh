#!/bin/bash
# GPU: kmeans tests + bench (GPMR K-means baseline), intcount bench (GPMR IntegerCount baseline)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "start $(date)" > $P
timeout -k 10 300 python -u -m pytest tests/test_kmeans.py tests/test_checkpoint.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_km.log 2>&1
rc=$?; echo "pytest rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload kmeans --steps 5 --warmup 1 > gpurun_out/bench_km.log 2>&1
rc=$?; echo "bench km rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload intcount --steps 10 --warmup 2 > gpurun_out/bench_ic.log 2>&1
rc=$?; echo "bench ic rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_km -o km -- python3 bench.py --workload kmeans --steps 2 --warmup 1 > gpurun_out/prof_km.log 2>&1
rc=$?; echo "prof km rc=$rc $(date)" >> $P
exit $rc
