#!/bin/bash
# hub kernel with sparse-row lists: triangle tests, then the hub-size sweep.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_triangles.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_tri.log 2>&1 && echo "tri ok" &&
for K in 131072 262144 393216 524288; do
  MRH_TRI_HUB=$K timeout -k 10 200 python -u bench.py --workload trifind --steps 2 --warmup 1 > gpurun_out/bench_tri_s$K.json 2>/dev/null || exit 1
  echo "K=$K $(cut -c170-260 gpurun_out/bench_tri_s$K.json)"
done
