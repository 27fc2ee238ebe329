#!/bin/bash
# K-means map kernel variants: transposed reduction (default) vs the batched LDS-atomic kernel
# with one (MRH_KMEANS_KERNEL=5) or 16 (=6) partial copies: tests, benches, kernel trace, one PMC pass
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kmeans.py -x -q --timeout 120 --timeout-method thread > gpurun_out/km_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/km_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 5 6; do
  MRH_KMEANS_KERNEL=$v timeout -k 10 120 python bench.py --workload kmeans --steps 10 --warmup 2 > gpurun_out/km_v$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/km_v$v.json')); print('variant=$v', round(d['ms_per_step'],3), 'ms/step', '%.3g points/s' % d['value'], 'shift', d.get('final_shift'))"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kmv -o km -- python3 bench.py --workload kmeans --steps 3 --warmup 1 > gpurun_out/prof_kmv.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmc_kmv -o km -- python3 bench.py --workload kmeans --steps 1 --warmup 0 --iters 3 > gpurun_out/pmc_kmv.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
