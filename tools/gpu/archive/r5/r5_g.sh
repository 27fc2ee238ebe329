# r5: multi-GPU PageRank pieces + ring overlap (gloo ranks on one GPU), forced-RCCL plans, pagerank record keys
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_distributed_gpu.py tests/test_pagerank.py tests/test_rccl_gpu.py > $O/g_tests.txt 2>&1 &&
timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/g_pr.log 2>&1
