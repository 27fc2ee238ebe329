#!/bin/bash
# guard allocator + radix (4096-pair tiles default) + full GPU tier + the
# other workload benches (PageRank, wordfreq, tri_find, intcount, kmeans).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_guard_alloc.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_guard.log 2>&1 && echo "guard+kernels gpu ok" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest gpu ok" &&
timeout -k 10 300 python -u bench.py --workload pagerank --steps 3 --warmup 1 > gpurun_out/bench_pr.json 2> gpurun_out/bench_pr.err && cat gpurun_out/bench_pr.json &&
timeout -k 10 300 python -u bench.py --workload wordfreq --steps 5 --warmup 2 > gpurun_out/bench_wf.json 2> gpurun_out/bench_wf.err && cat gpurun_out/bench_wf.json &&
timeout -k 10 300 python -u bench.py --workload trifind --steps 2 --warmup 1 > gpurun_out/bench_tri.json 2> gpurun_out/bench_tri.err && cat gpurun_out/bench_tri.json &&
timeout -k 10 300 python -u bench.py --workload intcount --steps 5 --warmup 2 > gpurun_out/bench_ic.json 2> gpurun_out/bench_ic.err && cat gpurun_out/bench_ic.json
rc=$?
tail -3 gpurun_out/pytest_guard.log gpurun_out/pytest_gpu.log 2>/dev/null
exit $rc
