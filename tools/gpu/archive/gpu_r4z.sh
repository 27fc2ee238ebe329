# r4: tri_find_mr extra with 64 MB pages in its out-of-core run
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --pagerank-scale 0 --trifind-scale 0 --wordfreq-bytes 0 --file-io-steps 0 --dist-extras 0 > $O/trimr64.json 2> $O/trimr64.err
