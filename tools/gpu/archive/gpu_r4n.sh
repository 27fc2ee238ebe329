# r4: why with_file_io is slower after the PageRank extra: pool off / caches kept / OMP threads 1
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
A="--steps 3 --warmup 1 --trifind-scale 0 --wordfreq-bytes 0 --trifind-mr-scale 0 --dist-extras 0"
MRH_HBM_POOL=0 timeout -k 10 300 python bench.py $A > $O/fio_pool0.json 2> $O/fio_pool0.err &&
MRH_BENCH_KEEP_CACHE=1 timeout -k 10 300 python bench.py $A > $O/fio_keep.json 2> $O/fio_keep.err &&
OMP_NUM_THREADS=1 timeout -k 10 300 python bench.py $A > $O/fio_omp1.json 2> $O/fio_omp1.err &&
timeout -k 10 300 python bench.py $A --file-io-steps 16 > $O/fio_16.json 2> $O/fio_16.err
