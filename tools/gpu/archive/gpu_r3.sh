#!/bin/bash
# round-3 GPU pass: every gpu test, smoke, the default bench (headline + the
# PageRank / tri_find / wordfreq extras). Each step has its own time limit and
# the script stops at the first failing step.
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
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 400 python bench.py || exit $?
tail -1 gpurun_out/bench.log > gpurun_out/bench.json
step strsort 300 python tools/strsort_bench.py 10000000 || exit $?
step strsort_prof 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_ss -o ss -- python3 tools/strsort_bench.py 10000000 || exit $?
exit 0
