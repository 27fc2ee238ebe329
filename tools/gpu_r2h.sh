#!/bin/bash
# K-means matrix-core kernel: tests, bench D=64/K=128 (MFMA vs library GEMM),
# D=2 (unchanged kernel), kernel trace of the MFMA run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kmeans.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_km.log 2>&1 && echo "kmeans gpu ok" &&
timeout -k 10 200 python -u bench.py --workload kmeans --kmeans-points 8388608 --kmeans-dim 64 --kmeans-k 128 --steps 3 --warmup 1 > gpurun_out/bench_km64.json 2>/dev/null && cat gpurun_out/bench_km64.json &&
MRH_KMEANS_GEMM=1 timeout -k 10 200 python -u bench.py --workload kmeans --kmeans-points 8388608 --kmeans-dim 64 --kmeans-k 128 --steps 3 --warmup 1 > gpurun_out/bench_km64_gemm.json 2>/dev/null && cat gpurun_out/bench_km64_gemm.json &&
timeout -k 10 200 python -u bench.py --workload kmeans --kmeans-points 8388608 --kmeans-dim 16 --kmeans-k 32 --steps 3 --warmup 1 > gpurun_out/bench_km16.json 2>/dev/null && cat gpurun_out/bench_km16.json &&
MRH_KMEANS_GEMM=1 timeout -k 10 200 python -u bench.py --workload kmeans --kmeans-points 8388608 --kmeans-dim 16 --kmeans-k 32 --steps 3 --warmup 1 > gpurun_out/bench_km16_gemm.json 2>/dev/null && cat gpurun_out/bench_km16_gemm.json &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_km -o km -- python bench.py --workload kmeans --kmeans-points 8388608 --kmeans-dim 64 --kmeans-k 128 --steps 1 --warmup 1 > gpurun_out/prof_km.log 2>&1 && echo "prof km ok"
