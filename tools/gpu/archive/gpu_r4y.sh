# r4: PMC counters of the PageRank gather and of tri_find_mr's collate (L2 hits/misses; VMEM reads, busy cycles)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -s KILL 110 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/pmc_pr4 -o p -- python3 bench.py --workload pagerank --steps 1 --warmup 0 --iters 3 > $O/pmc_pr4.log 2>&1 &&
timeout -s KILL 110 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $O/pmc_pr4b -o p -- python3 bench.py --workload pagerank --steps 1 --warmup 0 --iters 3 > $O/pmc_pr4b.log 2>&1
