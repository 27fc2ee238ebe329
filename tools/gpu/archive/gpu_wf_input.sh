#!/bin/bash
# wordfreq input placement: one pinned allocation per 128 MiB chunk (default)
# vs views of one pinned 1 GiB allocation (MRH_WF_INPUT=contig); plus a copy
# timeline of the contiguous variant
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "wf start $(date)" >> $P
for mode in split contig; do
  timeout -k 10 200 env MRH_WF_INPUT=$mode python bench.py --workload wordfreq --steps 10 --warmup 2 > gpurun_out/wf_in_$mode.log 2>&1 || exit $?
  echo "wf $mode $(date)" >> $P
done
rm -rf gpurun_out/prof_wf_contig
MRH_WF_INPUT=contig timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_wf_contig -o p -- python3 bench.py --workload wordfreq --steps 3 --warmup 1 > gpurun_out/wf_tl_contig.log 2>&1
echo "timeline rc=$? $(date)" >> $P
exit 0
