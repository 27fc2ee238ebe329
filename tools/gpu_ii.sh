#!/bin/bash
# convert/kvops GPU tests + headline bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_property_ops.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ii.log 2>&1
rc=$?; echo "pytest rc=$rc" > gpurun_out/progress.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_ii.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/progress.txt
exit $rc
