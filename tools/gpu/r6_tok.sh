# the LDS-staged tokenizer emit (k_tok_emit2): map_words / wordfreq GPU tests, then both no-combiner routes
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6t; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_wordfreq.py tests/test_kernels_gpu.py tests/test_shuffle.py tests/test_dict_group.py tests/test_oracles.py > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/wf_shuffle_time.py 8 3 0 > $o/wf_local.log 2>&1 || exit $?
MRH_FORCE_RCCL=2 timeout -k 10 200 python -u tools/wf_shuffle_time.py 8 3 0 > $o/wf_dist.log 2>&1 || exit $?
