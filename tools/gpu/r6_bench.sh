# the full 1-GPU bench (the driver's command) with its detail file
cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 1000 python -u bench.py --detail-out $o/bench_detail.json > $o/bench.out 2> $o/bench.err
