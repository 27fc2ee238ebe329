# r5: OOC RMAT-18 after RMAT-22 in HBM, pool trimmed and the pinned host cache emptied between
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
BIG=22 TRIM=2 timeout -k 10 400 python -u tools/trimr_time.py 18 ooc > $O/z2_bigtrim2.txt 2>&1
