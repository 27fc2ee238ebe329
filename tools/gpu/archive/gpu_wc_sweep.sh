#!/bin/bash
# wordfreq bench for each in-mapper combiner kernel configuration
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/wc_sweep.txt
for c in 5 6 7 8 9; do
  MRH_WC_CFG=$c timeout -k 10 200 python bench.py --workload wordfreq --steps 8 --warmup 2 > gpurun_out/wc_$c.log 2>&1
  rc=$?; echo "cfg $c rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/wc_$c.log)" >> gpurun_out/wc_sweep.txt
  [ $rc -eq 0 ] || exit $rc
done
