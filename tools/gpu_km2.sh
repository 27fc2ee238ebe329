#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/km_sweep.txt
timeout -k 10 300 python -u -m pytest tests/test_kmeans.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_km.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/km_sweep.txt; [ $rc -eq 0 ] || exit $rc
for v in 0 3 1; do
  MRH_KMEANS_KERNEL=$v timeout -k 10 200 python bench.py --workload kmeans --steps 5 --warmup 1 > gpurun_out/km_$v.log 2>&1
  rc=$?; echo "variant $v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/km_$v.log)" >> gpurun_out/km_sweep.txt
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_km3 -o km -- python3 bench.py --workload kmeans --steps 1 --warmup 1 > gpurun_out/prof_km3.log 2>&1
echo "prof rc=$?" >> gpurun_out/km_sweep.txt
