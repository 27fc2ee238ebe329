#!/bin/bash
# r5 full pass: every gpu test, smoke, the default bench record, out-of-core
# tri_find_mr RMAT-18 timing. Usage: r5_final.sh [tag]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:-final}
mkdir -p gpurun_out
P=gpurun_out/progress_$T.txt
echo "start $(date)" > $P
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(date)" >> $P
  return $rc
}
step pytest_gpu_$T 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
step smoke_$T 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step ooc18_$T 300 python -u tools/trimr_time.py 18 ooc || exit $?
step bench_$T 400 python bench.py || exit $?
exit 0
