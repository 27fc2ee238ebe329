#!/bin/bash
# Multi-rank rehearsal on the 1-GPU box: two ranks share cuda:0.
#  1. can RCCL join two ranks on one device (tools/rccl_probe.py)?
#  2. bench.py --gpus 2 over gloo + the engine's store transport (every
#     multi-rank engine path on the GPU except the RCCL data plane)
#  3. the same with the native RCCL transport (only if the probe joined)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
SMALL="--bytes-per-gpu 256e6 --file-bytes 33554432 --steps 3 --warmup 1 --pagerank-scale 20 --pagerank-steps 1"
timeout -k 10 150 python -u tools/rccl_probe.py > gpurun_out/probe.log 2>&1
rc=$?; echo "probe rc=$rc"; grep PROBE gpurun_out/probe.log; [ $rc -eq 0 ] || exit $rc
MRH_DIST_BACKEND=gloo MRH_TRANSPORT=pg MRH_NUMA_BIND=0 timeout -k 10 300 python -u bench.py --gpus 2 $SMALL \
  > gpurun_out/bench_g2_pg.json 2> gpurun_out/bench_g2_pg.err
rc=$?; echo "bench g2 pg rc=$rc"; cut -c1-400 gpurun_out/bench_g2_pg.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_g2_pg.err; exit $rc; }
if grep -q "RCCL aggregate OK" gpurun_out/probe.log; then
  MRH_DIST_BACKEND=gloo MRH_NUMA_BIND=0 timeout -k 10 300 python -u bench.py --gpus 2 $SMALL \
    > gpurun_out/bench_g2_rccl.json 2> gpurun_out/bench_g2_rccl.err
  rc=$?; echo "bench g2 rccl rc=$rc"; cut -c1-400 gpurun_out/bench_g2_rccl.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_g2_rccl.err; exit $rc; }
fi
exit 0
