#!/bin/bash
# PageRank XCD ranges with the fixed-point combine; tri_find hub kernel per-chunk trace
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
step tests 500 python -u -m pytest tests/test_pagerank.py tests/test_triangles.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
step prx 300 python bench.py --workload pagerank --steps 3 --warmup 1 || exit $?
step prx_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_prx2 -o p -- python3 bench.py --workload pagerank --steps 1 --warmup 0 || exit $?
step tri 300 python bench.py --workload trifind --steps 3 --warmup 1 || exit $?
step tri_prof 300 env MRH_TRI_HUB_CHUNKS=16 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tri2 -o p -- python3 bench.py --workload trifind --steps 1 --warmup 0 || exit $?
step ii1 300 python bench.py --workload invertedindex --extra-steps 0 --pagerank-scale 0 --trifind-scale 0 --wordfreq-bytes 0 || exit $?
step ii2 300 python bench.py --workload invertedindex --extra-steps 0 --pagerank-scale 0 --trifind-scale 0 --wordfreq-bytes 0 || exit $?
exit 0
