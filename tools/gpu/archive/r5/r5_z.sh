# r5: out-of-core tri_find_mr RMAT-18 after an in-HBM RMAT-22 run (the bench's order), with and without a pool trim between
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
BIG=22 timeout -k 10 400 python -u tools/trimr_time.py 18 ooc > $O/z_big.txt 2>&1 &&
BIG=22 TRIM=1 timeout -k 10 400 python -u tools/trimr_time.py 18 ooc > $O/z_bigtrim.txt 2>&1
