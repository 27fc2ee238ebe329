#!/bin/bash
# build the C API test with a crash reporter and run it on the GPU box
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
gcc -g -O0 -rdynamic tests/capi/capi_test.c tools/segv_trace.c -Icsrc/capi -Lgpu_mapreduce_amd -lmrhip \
  -Wl,-rpath,$GRAFT_REPO_ROOT/gpu_mapreduce_amd -o /tmp/capi_test || exit 1
gcc -g -O0 -rdynamic examples/c/cwordfreq.c tools/segv_trace.c -Icsrc/capi -Lgpu_mapreduce_amd -lmrhip \
  -Wl,-rpath,$GRAFT_REPO_ROOT/gpu_mapreduce_amd -o /tmp/cwordfreq || exit 1
printf "a b c a\n" > /tmp/w.txt
timeout -k 10 120 /tmp/cwordfreq /tmp/w.txt > gpurun_out/cwf.log 2>&1
echo "cwordfreq rc=$?" >> gpurun_out/cwf.log
timeout -k 10 120 /tmp/capi_test /tmp > gpurun_out/capi.log 2>&1
echo "capi rc=$?" >> gpurun_out/capi.log
exit 0
