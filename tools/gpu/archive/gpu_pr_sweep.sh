#!/bin/bash
# PageRank RMAT-26 x20 with the fused tile step: XCD range size (MRH_PR_L2_BYTES) and layer count sweep
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "start $(date)" > $P
run() {  # name env...
  local name=$1; shift
  timeout -k 10 200 env "$@" python bench.py --workload pagerank --steps 3 --warmup 1 > gpurun_out/pr_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc $(date)" >> $P; return $rc
}
run base MRH_X=0 || exit $?
for b in 2097152 3145728 5242880 6291456; do run l2_$b MRH_PR_L2_BYTES=$b || exit $?; done
for l in 1 2 3; do run layers_$l MRH_PR_XCD_LAYERS=$l || exit $?; done
run xcd_off MRH_PR_XCD=0 || exit $?
exit 0
