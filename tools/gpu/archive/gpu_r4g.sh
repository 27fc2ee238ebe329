# r4: pool cap test (clone out of core, collapse past the cap), faults, OOC, chunked wedges; trifind_mr extra
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_hbm_pool.py tests/test_faults.py tests/test_outofcore.py tests/test_ops.py > $O/t_pool.log 2>&1 &&
timeout -k 10 500 python bench.py --steps 2 --warmup 1 --pagerank-scale 0 --trifind-scale 0 --wordfreq-bytes 0 --file-io-steps 0 --dist-extras 0 > $O/trimr.json 2> $O/trimr.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_prsetup -o prsetup -- python tools/pr_setup_time.py 26 > $O/prof_prsetup.log 2>&1
