#!/bin/bash
# hub-size sweep beyond 262144 (bitmap of K*K/8 bytes: 32 GB at 524288)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for K in 262144 393216 524288; do
  MRH_TRI_HUB=$K timeout -k 10 200 python -u bench.py --workload trifind --steps 2 --warmup 1 > gpurun_out/bench_tri_$K.json 2>/dev/null || exit 1
  echo "K=$K $(cut -c1-330 gpurun_out/bench_tri_$K.json)"
done
