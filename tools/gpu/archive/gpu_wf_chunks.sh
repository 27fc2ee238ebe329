#!/bin/bash
# wordfreq 1 GiB/GPU: chunk (file) size x staging ring depth sweep
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for fb in 16777216 33554432 67108864 134217728; do
  for nb in 3 4; do
    MRH_WF_BUFS=$nb timeout -k 10 150 python bench.py --workload wordfreq --steps 10 --warmup 3 --file-bytes $fb > gpurun_out/wf_${fb}_${nb}.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/wf_${fb}_${nb}.json')); print('chunk=$fb bufs=$nb', round(d['ms_per_step'],3), 'ms/step')"
  done
done
