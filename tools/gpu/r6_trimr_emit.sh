# tri_find_mr wedge / triangle emit kernels: the triangle tests, stage times
# (RMAT-20, checked) and per-kernel stats
cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_triangles.py tests/test_ooc_hot_key.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1 &&
CHECK=1 REPS=3 timeout -k 10 300 python -u tools/trimr_time.py 20 > $o/time20.log 2>&1 &&
REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 tools/trimr_time.py 20 > $o/prof.log 2>&1
