#!/bin/bash
# SQ counters of the K-means map kernel (what bounds it): one counter group
# per rocprofv3 pass
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmc_km -o km -- python3 bench.py --workload kmeans --steps 1 --warmup 0 --iters 3 > gpurun_out/pmc_km.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
