#!/bin/bash
# tri_find RMAT-24 bench + kernel summary
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload trifind --steps 2 --warmup 1 > gpurun_out/tri.json 2>gpurun_out/tri.err || exit 1
cut -c1-300 gpurun_out/tri.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tri -o tri -- python3 bench.py --workload trifind --steps 1 --warmup 1 > gpurun_out/prof_tri.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
