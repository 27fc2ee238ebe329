# r4: with_file_io alone vs after the PageRank extra; dist extras after trifind_mr with a trimmed pool
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --pagerank-scale 0 --trifind-scale 0 --wordfreq-bytes 0 --trifind-mr-scale 0 --dist-extras 0 > $O/fio_a.json 2> $O/fio_a.err &&
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --trifind-scale 0 --wordfreq-bytes 0 --trifind-mr-scale 0 --dist-extras 0 > $O/fio_b.json 2> $O/fio_b.err &&
timeout -k 10 500 python bench.py --steps 3 --warmup 1 --pagerank-scale 0 --trifind-scale 0 --wordfreq-bytes 0 --file-io-steps 0 > $O/dist_c.json 2> $O/dist_c.err
