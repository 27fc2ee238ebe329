# per-kernel time of the headline InvertedIndex step and of the PageRank workload on the final round-6 code
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6k; mkdir -p $o
EX="--pagerank-scale 0 --trifind-scale 0 --trifind-mr-scale 0 --trifind-mr-big-scale 0 --trifind-mr-ooc-scale 0 --wordfreq-bytes 0 --file-io-steps 0 --dist-extras 0"
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pii -o t -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 $EX --detail-out '' > $GRAFT_REPO_ROOT/$o/ii.out 2>&1 || exit $?
cp /tmp/pii/t_kernel_stats.csv $GRAFT_REPO_ROOT/$o/ii_kernel_stats.csv
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ppr -o t -- python3 $GRAFT_REPO_ROOT/bench.py --workload pagerank --steps 3 --warmup 1 $EX --detail-out '' > $GRAFT_REPO_ROOT/$o/pr.out 2>&1 || exit $?
cp /tmp/ppr/t_kernel_stats.csv $GRAFT_REPO_ROOT/$o/pr_kernel_stats.csv
