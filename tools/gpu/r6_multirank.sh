# multi-rank rehearsal of the driver's bench on the one-GPU box: 2 and 3 ranks sharing cuda:0 over a gloo
# process group + the engine's host transport (RCCL cannot join two ranks on one device); every extra at
# small sizes, incl. the out-of-core run (pinned host arena per rank) and the big tri_find_mr run
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6m; mkdir -p $o
SMALL="--bytes-per-gpu 256e6 --file-bytes 33554432 --steps 3 --warmup 1 --pagerank-scale 20 --pagerank-steps 1 --trifind-scale 18 --trifind-mr-scale 16 --trifind-mr-big-scale 17 --trifind-mr-ooc-scale 14 --wordfreq-bytes 268435456 --file-io-steps 2 --extra-steps 1"
MRH_DIST_BACKEND=gloo MRH_TRANSPORT=pg MRH_NUMA_BIND=0 MRH_PIN_RESERVE_MB=2048 timeout -k 10 500 python -u bench.py --gpus 2 $SMALL --detail-out $o/g2_detail.json > $o/g2.json 2> $o/g2.err &&
MRH_DIST_BACKEND=gloo MRH_TRANSPORT=pg MRH_NUMA_BIND=0 MRH_PIN_RESERVE_MB=2048 timeout -k 10 500 python -u bench.py --gpus 3 $SMALL --detail-out $o/g3_detail.json > $o/g3.json 2> $o/g3.err
