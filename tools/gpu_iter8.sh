#!/bin/bash
# intcount GPU test + bench + rocprof; 2-rank bench.py rehearsal over gloo on one GPU
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "start $(date)" > $P
timeout -k 10 200 python -u -m pytest tests/test_intcount.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ic.log 2>&1
rc=$?; echo "pytest rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --workload intcount --steps 10 --warmup 3 > gpurun_out/bench_ic.log 2>&1
rc=$?; echo "bench ic rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
MRH_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_ii_2r.log 2>&1
rc=$?; echo "bench ii 2 ranks rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_ic" -o ic -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload intcount --steps 3 --warmup 1 --phases 0 > "$GRAFT_REPO_ROOT/gpurun_out/bench_ic_prof.log" 2>&1
rc=$?; echo "prof ic rc=$rc $(date)" >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
exit $rc
