#!/bin/bash
# triangle kernels: GPU tests, tri_find bench (scale 20 then 24), rocprof summary
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "start $(date)" > $P
timeout -k 10 300 python -m pytest tests/test_triangles.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_tri.log 2>&1
rc=$?; echo "pytest rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload trifind --scale 20 --steps 3 --warmup 1 > gpurun_out/bench_tri20.log 2>&1
rc=$?; echo "bench tri20 rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload trifind --scale 24 --steps 3 --warmup 1 > gpurun_out/bench_tri24.log 2>&1
rc=$?; echo "bench tri24 rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_tri" -o tri -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload trifind --scale 24 --steps 1 --warmup 0 > "$GRAFT_REPO_ROOT/gpurun_out/bench_tri_prof.log" 2>&1
rc=$?; echo "prof tri rc=$rc $(date)" >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
exit $rc
