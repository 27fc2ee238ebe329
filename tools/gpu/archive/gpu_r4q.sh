# r4: one-rank tensor collectives as the identity: RCCL/PageRank/distributed/fault tests, dist extras probe
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_rccl_gpu.py tests/test_pagerank.py tests/test_distributed_gpu.py tests/test_faults.py tests/test_triangles.py > $O/t_q.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --wordfreq-bytes 0 --trifind-mr-scale 0 --file-io-steps 0 > $O/dist_a.json 2> $O/dist_a.err
