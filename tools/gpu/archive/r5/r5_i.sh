# r5: out-of-core tri_find_mr RMAT-18 host-phase trace (MRH_OOC_TRACE=1)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
MRH_OOC_TRACE=1 timeout -k 10 300 python -u tools/trimr_time.py 18 ooc > $O/i_ooc18.txt 2>&1
