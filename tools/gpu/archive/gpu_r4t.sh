# r4: one-sort triangle build: tests, local and forced tri_find, kernel summary
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_triangles.py tests/test_oink.py tests/test_distributed_gpu.py > $O/t_t.log 2>&1 &&
timeout -k 10 300 python bench.py --workload trifind --steps 3 --warmup 1 > $O/tri_local.json 2> $O/tri_local.err &&
MRH_TRI_ONESORT=0 timeout -k 10 300 python bench.py --workload trifind --steps 3 --warmup 1 > $O/tri_twosort.json 2> $O/tri_twosort.err &&
MRH_FORCE_RCCL=1 timeout -k 10 300 python bench.py --workload trifind --steps 3 --warmup 1 > $O/tri_forced.json 2> $O/tri_forced.err
