#!/bin/bash
# first GPU pass: kernel numerics, smoke, 1-GPU bench, rocprof kernel stats
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "start $(date)" > gpurun_out/progress.txt
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(date)" >> gpurun_out/progress.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(date)" >> gpurun_out/progress.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench1.log 2>&1
rc=$?; echo "bench rc=$rc $(date)" >> gpurun_out/progress.txt
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o ii -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof.log" 2>&1
rc=$?; echo "prof rc=$rc $(date)" >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
exit $rc
