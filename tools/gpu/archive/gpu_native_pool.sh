#!/bin/bash
# native programs / C API / OINK on the GPU with the page pool installed by Comm construction
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "start $(date)" > $P
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(date)" >> $P
  return $rc
}
step native_tests 500 python -u -m pytest tests/test_native_multiproc.py tests/test_capi.py tests/test_oink.py tests/test_faults.py tests/test_guard_alloc.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
D=/tmp/mrh_html
step synth 300 python -m gpu_mapreduce_amd.utils.synth html $D 8 134217728 --device cuda --nurl 1048576 || exit $?
step ii_native_pool 120 gpu_mapreduce_amd/bin/invertedindex $D 8 NULL || exit $?
step ii_native_nopool 120 env MRH_HBM_POOL=0 gpu_mapreduce_amd/bin/invertedindex $D 8 NULL || exit $?
exit 0
