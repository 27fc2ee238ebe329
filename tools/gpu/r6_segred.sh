# the builtin segmented reduce from one hot key to a million small ones (multi-level carry fold),
# its GPU tests, and the device-functor timings
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6s8; mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_oracles.py tests/test_wavesegred_gpu.py tests/test_pagerank.py tests/test_device_functors.py > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/segred_keys_bench.py > $o/keys.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/devfn_time.py 27 0 > $o/devfn_27_0.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/devfn_time.py 27 10 > $o/devfn_27_10.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/devfn_time.py 27 20 > $o/devfn_27_20.log 2>&1 || exit $?
