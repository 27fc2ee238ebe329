# GPU tests of the shuffle / wordfreq / tri_find_mr paths, wordfreq timings of both no-combiner
# routes, then the ATen-window profiles
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6j; mkdir -p $o
timeout -k 10 700 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_shuffle.py tests/test_wordfreq.py tests/test_dict_group.py tests/test_distributed_gpu.py tests/test_rccl_loopback_gpu.py tests/test_triangles.py tests/test_kernels_gpu.py tests/test_rccl_gpu.py > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/wf_shuffle_time.py 8 3 0 > $o/wf_local.log 2>&1 || exit $?
MRH_FORCE_RCCL=2 timeout -k 10 200 python -u tools/wf_shuffle_time.py 8 3 0 > $o/wf_dist.log 2>&1 || exit $?
prof() {  # name marker-kernel command...
  local name=$1 mark=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_$name -o t -- "$@" > $o/$name.log 2>&1 || return $?
  python3 tools/aten_window.py $(find /tmp/prof_$name -name "*.db" | head -1) --after-kernel "$mark" > $o/${name}_kernels.txt 2>&1
  rm -rf /tmp/prof_$name
}
prof trimr20 k_rmat python3 tools/trimr_time.py 20 || exit $?
prof ooc18 k_rmat python3 tools/trimr_time.py 18 ooc || exit $?
export MRH_FORCE_RCCL=2
prof wfd k_tok python3 tools/wf_shuffle_time.py 8 2 0
