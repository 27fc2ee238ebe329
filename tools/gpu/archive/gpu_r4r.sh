# r4: PageRank gather with sources in ascending order inside each group (experiment)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/pr_base.json 2> $O/pr_base.err &&
MRH_PR_SRC_ORDER=1 timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/pr_srcorder.json 2> $O/pr_srcorder.err &&
timeout -k 10 1000 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ > $O/t_all.log 2>&1
