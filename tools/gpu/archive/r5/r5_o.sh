# r5: one-pass word keys (tests + wordfreq shuffle / combiner timing); PageRank chunks of whole layers (forced RCCL K=4 timing, tests)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_wordfreq.py tests/test_dict_group.py tests/test_pagerank.py tests/test_distributed_gpu.py > $O/o_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/wf_shuffle_time.py 8 3 0 > $O/o_wf.txt 2>&1 &&
MRH_FORCE_RCCL=1 MRH_PR_OVERLAP=2 timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/o_pr_pieces4.log 2>&1
