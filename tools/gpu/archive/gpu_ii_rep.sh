#!/bin/bash
# headline bench repeated (step-time spread / outliers)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --pagerank-scale 0 > gpurun_out/ii_rep$r.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ii_rep$r.json')); s=d['step_ms_rank0']; print('run $r', round(d['ms_per_step'],3), 'ms/step, max step', max(s), 'min', min(s))"
done
