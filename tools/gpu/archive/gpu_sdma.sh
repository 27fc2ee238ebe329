#!/bin/bash
# H2D engine experiment: SDMA copies (default) vs blit-kernel copies (HSA_ENABLE_SDMA=0)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "start $(date)" > $P
NOX="--pagerank-scale 0 --trifind-scale 0 --wordfreq-bytes 0"
for mode in 1 0; do
  timeout -k 10 200 env HSA_ENABLE_SDMA=$mode python bench.py $NOX > gpurun_out/ii_sdma$mode.log 2>&1 || exit $?
  echo "ii sdma=$mode $(date)" >> $P
  timeout -k 10 200 env HSA_ENABLE_SDMA=$mode python bench.py --workload wordfreq --steps 10 --warmup 2 > gpurun_out/wf_sdma$mode.log 2>&1 || exit $?
  echo "wf sdma=$mode $(date)" >> $P
done
timeout -k 10 100 env HSA_ENABLE_SDMA=0 python tools/h2d_bw.py > gpurun_out/h2d_sdma0.log 2>&1
echo "h2d rc=$? $(date)" >> $P
exit 0
