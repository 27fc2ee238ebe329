# L2 request counters: the gather microbenchmark and the PageRank gather (3 iterations)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6g; mkdir -p $o
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum SQ_WAVES --kernel-include-regex k_bench -d $o/pmc_bench -o b -- tools/bin/l2_gather_bench > $o/pmc_bench.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum SQ_WAVES --kernel-include-regex gather -d $o/pmc_pr -o pr -- python3 bench.py --workload pagerank --steps 1 --warmup 0 --iters 3 > $o/pmc_pr.log 2>&1
