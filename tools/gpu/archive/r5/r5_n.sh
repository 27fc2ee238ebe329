# r5: chunked multi-GPU PageRank plan from grouped one-GPU ranges: tests (forced RCCL, gloo ranks), one-rank cost at K = 1 / 4; wordfreq shuffle job vs teardown
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_pagerank.py tests/test_distributed_gpu.py -k "pagerank" > $O/n_tests.txt 2>&1 &&
MRH_FORCE_RCCL=1 MRH_PR_OVERLAP=2 MRH_PR_PIECES=1 timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/n_pr_pieces1.log 2>&1 &&
MRH_FORCE_RCCL=1 MRH_PR_OVERLAP=2 timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/n_pr_pieces4.log 2>&1 &&
timeout -k 10 300 python -u tools/wf_shuffle_time.py 8 3 0 > $O/n_wf.txt 2>&1
