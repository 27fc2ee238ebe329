# r4: kernel trace of the record's local + forced PageRank extras (where the forced 10 % goes)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_dist -o dist -- python bench.py --steps 3 --warmup 1 --trifind-scale 0 --wordfreq-bytes 0 --trifind-mr-scale 0 --file-io-steps 0 > $O/prof_dist.log 2>&1
