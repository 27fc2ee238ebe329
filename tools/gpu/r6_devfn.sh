# device functors + the segmented reduce's single-segment tiles: GPU tests, then timing against the built-ins
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6f3; mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_device_functors.py tests/test_kernels_gpu.py tests/test_oracles.py tests/test_wavesegred_gpu.py tests/test_pagerank.py > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/devfn_time.py 27 20 > $o/time_27_20.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/devfn_time.py 27 10 > $o/time_27_10.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/devfn_time.py 27 0 > $o/time_27_0.log 2>&1 || exit $?
