# segred with the wave-parallel partial fold: its GPU tests, then the key-count microbench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6s6; mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_oracles.py tests/test_wavesegred_gpu.py tests/test_pagerank.py tests/test_device_functors.py tests/test_wordfreq.py > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/segred_keys_bench.py > $o/keys.log 2>&1 || exit $?
