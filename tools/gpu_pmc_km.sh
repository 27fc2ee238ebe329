#!/bin/bash
# SQ counters of the K-means map kernel (what bounds it)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES -d gpurun_out/pmc_km -o km -- python3 bench.py --workload kmeans --steps 1 --warmup 0 --iters 3 > gpurun_out/pmc_km.log 2>&1
