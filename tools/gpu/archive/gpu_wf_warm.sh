#!/bin/bash
# wordfreq: does a longer warmup explain the faster second window? serial loop
# timed first after 1 / 2 / 6 warmup jobs; then the headline with the
# overlapped file-I/O extra
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "start $(date)" > $P
for w in 1 2 6; do
  timeout -k 10 200 python bench.py --workload wordfreq --steps 6 --warmup $w > gpurun_out/wfw_$w.log 2>&1 || exit $?
  echo "wf warmup $w $(date)" >> $P
done
timeout -k 10 300 python bench.py --pagerank-scale 0 --trifind-scale 0 --wordfreq-bytes 0 > gpurun_out/ii_fileio2.log 2>&1 || exit $?
echo "ii file io $(date)" >> $P
exit 0
