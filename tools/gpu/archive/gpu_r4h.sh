# r4: PageRank setup (bitmap unpack, dangling count, Philox-7 R-MAT, keys-only tiles): tests, radix tile sweep, stages, kernel profile; trifind_mr
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_ops.py tests/test_pagerank.py tests/test_distributed_gpu.py tests/test_triangles.py tests/test_hbm_pool.py > $O/t_h.log 2>&1 &&
for kit in 16 24 32; do MRH_RX_KIT=$kit timeout -k 10 120 python tools/radix_keys_bench.py >> $O/radix_kit.log 2>&1 || exit 1; done &&
bash tools/pr_setup_stages.sh &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_prsetup2 -o prsetup -- python tools/pr_setup_time.py 26 > $O/prof_prsetup2.log 2>&1 &&
timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/pr_local.json 2> $O/pr_local.err &&
timeout -k 10 500 python bench.py --steps 2 --warmup 1 --pagerank-scale 0 --trifind-scale 0 --wordfreq-bytes 0 --file-io-steps 0 --dist-extras 0 > $O/trimr.json 2> $O/trimr.err
