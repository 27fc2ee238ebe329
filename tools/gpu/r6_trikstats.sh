# per-kernel time of the tri_find workload (RMAT-24) on the final round-6 code
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6k2; mkdir -p $o
EX="--pagerank-scale 0 --trifind-scale 0 --trifind-mr-scale 0 --trifind-mr-big-scale 0 --trifind-mr-ooc-scale 0 --wordfreq-bytes 0 --file-io-steps 0 --dist-extras 0"
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ptri -o t -- python3 $GRAFT_REPO_ROOT/bench.py --workload trifind --steps 3 --warmup 1 $EX --detail-out '' > $GRAFT_REPO_ROOT/$o/tri.out 2>&1 || exit $?
cp /tmp/ptri/t_kernel_stats.csv $GRAFT_REPO_ROOT/$o/tri_kernel_stats.csv
