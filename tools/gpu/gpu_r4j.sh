# r4: narrow-key exact grouping + pool counters: tests, tri_find_mr RMAT-20 timing + profile
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_grouper.py tests/test_triangles.py tests/test_hbm_pool.py tests/test_oracles.py > $O/t_j.log 2>&1 &&
timeout -k 10 300 python tools/trimr_time.py 20 > $O/trimr_time.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_trimr2 -o trimr -- python tools/trimr_time.py 20 > $O/prof_trimr2.log 2>&1
