#!/bin/bash
# tri_find dense core (MRH_TRI_CORE top ranks on the int8 GEMM): hub/core
# correctness test, then an RMAT-24 sweep of the core size
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_triangles.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tri_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/tri_tests.log; [ $rc -eq 0 ] || exit $rc
for T in 0 4096 8192 16384 32768; do
  MRH_TRI_CORE=$T timeout -k 10 200 python bench.py --workload trifind --steps 2 --warmup 1 > gpurun_out/tri_c$T.json 2>gpurun_out/tri_c$T.err || { tail -5 gpurun_out/tri_c$T.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/tri_c$T.json')); print('core=$T', round(d['ms_per_step'],1), 'ms/step', d.get('triangles'))"
done
