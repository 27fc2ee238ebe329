# r5: find the 2-rank bench crash (test_bench_two_ranks_on_one_gpu args, faulthandler on)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
MRH_DIST_BACKEND=gloo MRH_TRANSPORT=pg MRH_NUMA_BIND=0 PYTHONFAULTHANDLER=1 MRH_SEGV_TRACE=1 timeout -k 10 400 python -u bench.py --gpus 2 --bytes-per-gpu 32e6 --file-bytes 8000000 --steps 2 --warmup 1 --phases 0 --pagerank-scale 16 --pagerank-steps 1 > $O/w_g2.json 2> $O/w_g2.err
echo "rc=$?" >> $O/w_g2.err
