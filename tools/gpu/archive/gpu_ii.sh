#!/bin/bash
# convert/kvops GPU tests + headline bench + kernel profile
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_property_ops.py tests/test_distributed_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ii.log 2>&1
rc=$?; echo "pytest rc=$rc" > gpurun_out/progress.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_ii.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/progress.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ii -o ii -- python3 bench.py --steps 4 --warmup 1 --phases 0 > gpurun_out/prof_ii.log 2>&1
rc=$?; echo "prof rc=$rc" >> gpurun_out/progress.txt
exit $rc
