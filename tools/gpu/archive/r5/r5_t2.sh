# r5: kernel + copy trace of out-of-core tri_find_mr RMAT-18 with the final pipelined partition pass
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/t2ooc -o run -- python -u $GRAFT_REPO_ROOT/tools/trimr_time.py 18 ooc > $O/t2_pooc.txt 2>&1
