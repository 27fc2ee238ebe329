# r4: wordfreq at 8 GiB and at 1 GiB per GPU in the record
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --pagerank-scale 0 --trifind-scale 0 --trifind-mr-scale 0 --file-io-steps 0 --dist-extras 0 > $O/wf1g.json 2> $O/wf1g.err
