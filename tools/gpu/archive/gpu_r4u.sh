# r4: tri_find_mr with fixed-width edge markers: tests, timing, kernel profile
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_triangles.py tests/test_oink.py > $O/t_u.log 2>&1 &&
timeout -k 10 300 python tools/trimr_time.py 20 > $O/trimr_time.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_trimr3 -o trimr -- python tools/trimr_time.py 20 > $O/prof_trimr3.log 2>&1
