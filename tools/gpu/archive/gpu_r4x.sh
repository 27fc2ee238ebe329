# r4: packed-pairs convert test on the GPU
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_grouper.py > $O/t_x.log 2>&1
