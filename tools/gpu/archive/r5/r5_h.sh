# r5: multi-GPU PageRank chunk rounds (gloo ranks on one GPU), forced-RCCL plans,
# pagerank record keys; out-of-core tri_find_mr RMAT-18 with per-stage PCIe bytes + a copy/kernel trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_distributed_gpu.py tests/test_pagerank.py tests/test_rccl_gpu.py > $O/h_tests.txt 2>&1 &&
timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/h_pr.log 2>&1 &&
timeout -k 10 300 python -u tools/trimr_time.py 18 ooc > $O/h_ooc18.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/hooc -o run -- python -u tools/trimr_time.py 18 ooc > $O/h_pooc.txt 2>&1
