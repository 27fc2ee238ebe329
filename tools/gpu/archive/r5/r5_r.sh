# r5: multi-rank rehearsal of the driver's bench (2 and 3 ranks sharing the one GPU, gloo process group + the
# engine's store transport; RCCL cannot join ranks on one device): every extra at small sizes, incl. the
# chunked PageRank exchange and the per-occurrence wordfreq shuffle across ranks
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
SMALL="--bytes-per-gpu 256e6 --file-bytes 33554432 --steps 3 --warmup 1 --pagerank-scale 20 --pagerank-steps 1 --trifind-scale 18 --trifind-mr-scale 16 --trifind-mr-big-scale 0 --trifind-mr-ooc-scale 0 --wordfreq-bytes 268435456 --file-io-steps 2 --extra-steps 1"
MRH_DIST_BACKEND=gloo MRH_TRANSPORT=pg MRH_NUMA_BIND=0 timeout -k 10 500 python -u bench.py --gpus 2 $SMALL > $O/r_g2.json 2> $O/r_g2.err &&
MRH_DIST_BACKEND=gloo MRH_TRANSPORT=pg MRH_NUMA_BIND=0 timeout -k 10 500 python -u bench.py --gpus 3 $SMALL > $O/r_g3.json 2> $O/r_g3.err
