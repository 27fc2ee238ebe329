# r5: compact wedges + bucketed packed convert: tests, tri_find_mr RMAT-20 and RMAT-22 stage times
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_append_parts.py tests/test_triangles.py > $O/b_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/trimr_time.py 20 > $O/b_trimr20.txt 2>&1 &&
timeout -k 10 400 python -u tools/trimr_time.py 22 > $O/b_trimr22.txt 2>&1
