# r5: retired-stream fix: pool tests + the 2-rank bench launcher test
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
MRH_SEGV_TRACE=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_hbm_pool.py tests/test_bench_launcher.py > $O/x_tests.txt 2>&1
