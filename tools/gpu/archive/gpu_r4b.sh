# r4: large RCCL transfers on one rank (pieces of 1 GiB vs one message); kernel trace of the forced-RCCL PageRank
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
MRH_RCCL_MAX_MSG=0 timeout -k 10 200 python -u tools/rccl_big.py > $O/rccl_big_whole.log 2>&1 ; echo "rc=$?" >> $O/rccl_big_whole.log
timeout -k 10 200 python -u tools/rccl_big.py > $O/rccl_big.log 2>&1 ; echo "rc=$?" >> $O/rccl_big.log
MRH_FORCE_RCCL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_prf -o prf -- python3 bench.py --workload pagerank --steps 1 --warmup 1 > $O/prof_prf.log 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_inverted_index_files.py > $O/t_ii.log 2>&1
