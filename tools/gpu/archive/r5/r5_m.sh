# r5: forced-RCCL PageRank with the overlapped chunk plan at one rank (test + RMAT-26 timing vs the plain replicated plan)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_pagerank.py -k "forced" > $O/m_tests.txt 2>&1 &&
MRH_FORCE_RCCL=1 timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/m_pr_forced.log 2>&1 &&
MRH_FORCE_RCCL=1 MRH_PR_OVERLAP=2 timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/m_pr_pieces.log 2>&1 &&
MRH_FORCE_RCCL=1 MRH_PR_OVERLAP=2 MRH_PR_PIECES=8 timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/m_pr_pieces8.log 2>&1
