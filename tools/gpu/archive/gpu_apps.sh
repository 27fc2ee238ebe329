#!/bin/bash
# GPU check of the native programs: their gpu tests, then the native
# InvertedIndex app on 1 GiB (8 x 128 MiB part files) vs the Python bench path
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "start $(date)" > $P
timeout -k 10 400 python -u -m pytest tests/test_native_multiproc.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_native_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
D=/tmp/mrh_html
timeout -k 10 300 python -m gpu_mapreduce_amd.utils.synth html $D 8 134217728 --device cuda --nurl 1048576 > gpurun_out/synth.log 2>&1
rc=$?; echo "synth rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 120 gpu_mapreduce_amd/bin/invertedindex $D 8 NULL > gpurun_out/ii_native_$i.log 2>&1
  rc=$?; echo "ii native $i rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
done
exit 0
