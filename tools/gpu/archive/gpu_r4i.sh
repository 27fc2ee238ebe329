# r4: tiled wedge kernel: wedge tests, tri_find_mr RMAT-20 stage times + kernel profile
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_ops.py tests/test_triangles.py > $O/t_i.log 2>&1 &&
timeout -k 10 300 python tools/trimr_time.py 20 > $O/trimr_time.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_trimr -o trimr -- python tools/trimr_time.py 20 > $O/prof_trimr.log 2>&1
