# wave-aggregated partition counts (k_part_count) vs per-lane byte atomics (MRH_PART_COUNT=atomic), same box:
# wordfreq's P > 1 route, then the shuffle GPU tests
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6t3; mkdir -p $o
MRH_FORCE_RCCL=2 timeout -k 10 200 python -u tools/wf_shuffle_time.py 8 3 0 > $o/wf_dist_wave.log 2>&1 || exit $?
MRH_PART_COUNT=atomic MRH_FORCE_RCCL=2 timeout -k 10 200 python -u tools/wf_shuffle_time.py 8 3 0 > $o/wf_dist_atomic.log 2>&1 || exit $?
MRH_FORCE_RCCL=2 timeout -k 10 200 python -u tools/wf_shuffle_time.py 8 3 0 > $o/wf_dist_wave2.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_shuffle.py tests/test_distributed_gpu.py > $o/tests.log 2>&1
