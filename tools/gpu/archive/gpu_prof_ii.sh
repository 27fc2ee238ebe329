#!/bin/bash
# rocprofv3 kernel stats of the headline InvertedIndex bench (1 GPU)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ii -o ii -- python3 bench.py --steps 4 --warmup 1 --phases 0 > gpurun_out/prof_ii.log 2>&1
