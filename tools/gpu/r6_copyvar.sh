# the block-tiled var-width gather (k_copy_var_blk): shuffle / wordfreq GPU tests, then wordfreq's
# P > 1 route with it and with the wave version (MRH_COPY_VAR=wave)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6c; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_shuffle.py tests/test_wordfreq.py tests/test_distributed_gpu.py tests/test_rccl_loopback_gpu.py tests/test_kernels_gpu.py > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/tests.log
[ $rc -eq 0 ] || exit 1
MRH_FORCE_RCCL=2 timeout -k 10 200 python -u tools/wf_shuffle_time.py 8 3 0 > $o/wf_dist_blk.log 2>&1 || exit $?
MRH_COPY_VAR=wave MRH_FORCE_RCCL=2 timeout -k 10 200 python -u tools/wf_shuffle_time.py 8 3 0 > $o/wf_dist_wave.log 2>&1 || exit $?
