# r4: multi-GPU PageRank / tri_find plans: tests, then local vs forced-RCCL benches
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_pagerank.py tests/test_distributed_gpu.py tests/test_triangles.py > $O/t_pr.log 2>&1 &&
timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/pr_local.json 2> $O/pr_local.err &&
MRH_FORCE_RCCL=1 timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/pr_forced.json 2> $O/pr_forced.err &&
timeout -k 10 200 python bench.py --workload trifind --steps 3 --warmup 1 > $O/tri_local.json 2> $O/tri_local.err &&
MRH_FORCE_RCCL=1 timeout -k 10 200 python bench.py --workload trifind --steps 3 --warmup 1 > $O/tri_forced.json 2> $O/tri_forced.err
