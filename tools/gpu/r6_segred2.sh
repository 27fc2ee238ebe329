# the segmented reduce microbench with the engine's HBM pool as allocator vs without
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6s3; mkdir -p $o
POOL=1 timeout -k 10 200 python -u tools/segred_keys_bench.py > $o/keys_pool.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/segred_keys_bench.py > $o/keys_nopool.log 2>&1 || exit $?
