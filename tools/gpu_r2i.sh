#!/bin/bash
# tri_find hub bitmaps: triangle GPU tests, RMAT-24 bench at several hub
# sizes (0 = hash kernels only), kernel trace of the default.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_triangles.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_tri.log 2>&1 && echo "tri gpu ok" &&
for K in 0 32768 65536 131072 262144; do
  MRH_TRI_HUB=$K timeout -k 10 200 python -u bench.py --workload trifind --steps 2 --warmup 1 > gpurun_out/bench_tri_$K.json 2>/dev/null || exit 1
  echo "K=$K $(cut -c1-330 gpurun_out/bench_tri_$K.json)"
done &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tri -o tri -- python bench.py --workload trifind --steps 1 --warmup 0 > gpurun_out/prof_tri.log 2>&1 && echo "prof tri ok" &&
timeout -k 10 150 python -u -m pytest tests/test_kmeans.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_km.log 2>&1 && echo "kmeans gpu ok" &&
MRH_KMEANS_GEMM=1 timeout -k 10 150 python -u bench.py --workload kmeans --kmeans-points 8388608 --kmeans-dim 64 --kmeans-k 128 --steps 3 --warmup 1 > gpurun_out/bench_km64_gemm2.json 2>/dev/null && cut -c1-300 gpurun_out/bench_km64_gemm2.json
