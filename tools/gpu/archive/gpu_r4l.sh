# r4: full default bench record + rocprof kernel summaries of the forced-RCCL PageRank / tri_find runs + setup stages
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python bench.py > $O/bench_full.json 2> $O/bench_full.err &&
bash tools/pr_setup_stages.sh &&
MRH_FORCE_RCCL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_forced_pr -o pr -- python bench.py --workload pagerank --steps 2 --warmup 1 > $O/prof_forced_pr.log 2>&1 &&
MRH_FORCE_RCCL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_forced_tri -o tri -- python bench.py --workload trifind --steps 2 --warmup 1 > $O/prof_forced_tri.log 2>&1
