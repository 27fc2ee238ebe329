# r4: PageRank with histogram out-degrees: tests, setup stages, iteration time (local, forced, old sort build)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_pagerank.py tests/test_distributed_gpu.py tests/test_triangles.py > $O/t_f.log 2>&1 &&
bash tools/pr_setup_stages.sh &&
timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/pr_local.json 2> $O/pr_local.err &&
MRH_PR_DEGREES=sort timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/pr_sort.json 2> $O/pr_sort.err &&
MRH_FORCE_RCCL=1 timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/pr_forced.json 2> $O/pr_forced.err
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_hbm_pool.py tests/test_faults.py tests/test_outofcore.py > $O/t_pool.log 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_triangles.py -k tri_find_mr > $O/t_trimr.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --pagerank-scale 0 --trifind-scale 0 --wordfreq-bytes 0 --file-io-steps 0 --dist-extras 0 > $O/trimr.json 2> $O/trimr.err
