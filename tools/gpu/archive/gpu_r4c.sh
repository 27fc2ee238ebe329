# r4: full GPU test suite, then local vs forced-RCCL PageRank / tri_find benches
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/t_all.log 2>&1 ; echo "rc=$?" >> $O/t_all.log
timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/pr_local.json 2> $O/pr_local.err &&
MRH_FORCE_RCCL=1 timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/pr_forced.json 2> $O/pr_forced.err &&
timeout -k 10 200 python bench.py --workload trifind --steps 3 --warmup 1 > $O/tri_local.json 2> $O/tri_local.err &&
MRH_FORCE_RCCL=1 timeout -k 10 200 python bench.py --workload trifind --steps 3 --warmup 1 > $O/tri_forced.json 2> $O/tri_forced.err
