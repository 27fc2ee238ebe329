# r4: narrow-key grouping, pool counters, windowed out-degrees, unaligned radix digits
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_ops.py tests/test_grouper.py tests/test_pagerank.py tests/test_distributed_gpu.py tests/test_triangles.py tests/test_hbm_pool.py > $O/t_j.log 2>&1 &&
bash tools/pr_setup_stages.sh &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_prsetup3 -o prsetup -- python tools/pr_setup_time.py 26 > $O/prof_prsetup3.log 2>&1 &&
timeout -k 10 300 python tools/trimr_time.py 20 > $O/trimr_time.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_trimr2 -o trimr -- python tools/trimr_time.py 20 > $O/prof_trimr2.log 2>&1
