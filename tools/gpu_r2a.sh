#!/bin/bash
# Round-2 GPU check: forced-RCCL data path, the GPU test tier, the headline
# bench, an RCCL kernel trace, and the two-ranks-on-one-GPU RCCL probe.
# Every GPU step has its own time limit; the steps are chained with && so a
# failure (or a fault) ends the call there.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/rccl_forced.py > gpurun_out/rccl_forced.log 2>&1 && echo "forced rccl ok" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest gpu ok" &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rccl -o rccl -- python tools/rccl_forced.py > gpurun_out/prof_rccl.log 2>&1 && echo "rocprof rccl ok" &&
timeout -k 10 150 python -u tools/rccl_probe.py > gpurun_out/probe.log 2>&1; rc=$?
echo "last rc=$rc"
tail -5 gpurun_out/rccl_forced.log gpurun_out/pytest_gpu.log gpurun_out/probe.log 2>/dev/null
exit $rc
