#!/bin/bash
# SDMA engine selection for the H2D streams: ROCr defaults vs the
# recommended-engine and ganged-engine modes (wordfreq + InvertedIndex)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "start $(date)" > $P
NOX="--pagerank-scale 0 --trifind-scale 0 --wordfreq-bytes 0 --file-io-steps 0"
for v in "none" "HSA_ENABLE_SDMA_RECOMMENDED_ENG=1" "HSA_ENABLE_SDMA_RECOMMENDED_ENG=0" "HSA_ENABLE_SDMA_GANG=1" "HSA_ENABLE_SDMA_GANG=0"; do
  tag=${v//=/_}
  if [ "$v" = none ]; then E=(); else E=("$v"); fi
  timeout -k 10 200 env "${E[@]}" python bench.py --workload wordfreq --steps 10 --warmup 2 > gpurun_out/wfe_$tag.log 2>&1 || exit $?
  echo "wf $v $(date)" >> $P
  timeout -k 10 200 env "${E[@]}" python bench.py $NOX > gpurun_out/iie_$tag.log 2>&1 || exit $?
  echo "ii $v $(date)" >> $P
done
timeout -k 10 300 python bench.py --pagerank-scale 0 --trifind-scale 0 --wordfreq-bytes 0 > gpurun_out/ii_fileio.log 2>&1 || exit $?
echo "ii file io $(date)" >> $P
exit 0
