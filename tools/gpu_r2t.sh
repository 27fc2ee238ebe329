#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for nb in 2 3 4; do
  MRH_WF_BUFS=$nb timeout -k 10 200 python -u bench.py --workload wordfreq --steps 5 --warmup 2 > gpurun_out/bench_wf_b$nb.json 2>/dev/null || exit 1
  echo "bufs=$nb $(cut -c200-300 gpurun_out/bench_wf_b$nb.json)"
done &&
MRH_WF_BUFS=3 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_wf3 -o wf -- python bench.py --workload wordfreq --steps 3 --warmup 1 > gpurun_out/prof_wf3.log 2>&1 && echo "prof wf ok"
