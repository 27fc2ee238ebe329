# device functors after the single-column count pass: GPU tests (functors, C API, OINK methods), then timings
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6f11; mkdir -p $o
timeout -k 10 500 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_device_functors.py tests/test_graph_mr.py tests/test_native_multiproc.py > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/devfn_time.py 27 20 > $o/time_27_20.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/devfn_time.py 27 10 > $o/time_27_10.log 2>&1 || exit $?
