# r4: forced-RCCL PageRank extra: right after the local PageRank extra vs in the full record
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --trifind-scale 0 --wordfreq-bytes 0 --trifind-mr-scale 0 --file-io-steps 0 > $O/dist_a.json 2> $O/dist_a.err &&
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --pagerank-scale 26 --trifind-scale 24 --wordfreq-bytes 0 --trifind-mr-scale 0 --file-io-steps 0 > $O/dist_b.json 2> $O/dist_b.err
