# r5: wedge tile groups + LDS map (tests, RMAT-20/22 timing); out-of-core RMAT-18 host-phase trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_triangles.py tests/test_ops.py > $O/j_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/trimr_time.py 20 > $O/j_trimr20.txt 2>&1 &&
timeout -k 10 400 python -u tools/trimr_time.py 22 > $O/j_trimr22.txt 2>&1 &&
MRH_OOC_TRACE=1 timeout -k 10 300 python -u tools/trimr_time.py 18 ooc > $O/i_ooc18.txt 2>&1
