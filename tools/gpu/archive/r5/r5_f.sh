# r5: emit LDS key map; tri_find_mr RMAT-20/22 + kernel profile
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_triangles.py > $O/f_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/trimr_time.py 20 > $O/f_trimr20.txt 2>&1 &&
timeout -k 10 400 python -u tools/trimr_time.py 22 > $O/f_trimr22.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ftri -o run -- python -u tools/trimr_time.py 20 > $O/f_ptri.txt 2>&1
