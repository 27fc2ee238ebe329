#!/bin/bash
# iteration GPU pass: kernel tests, bench with stage breakdown, H2D floor
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "start $(date)" > gpurun_out/progress.txt
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(date)" >> gpurun_out/progress.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/h2d_bw.py > gpurun_out/h2d.log 2>&1
rc=$?; echo "h2d rc=$rc $(date)" >> gpurun_out/progress.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench1.log 2>&1
rc=$?; echo "bench rc=$rc $(date)" >> gpurun_out/progress.txt
exit $rc
