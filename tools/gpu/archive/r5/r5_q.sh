# r5: per-occurrence wordfreq at 8 GiB (NUMA-bound) by staging ring depth 3 / 4 / 6
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
MRH_WF_BUFS=4 timeout -k 10 300 python -u tools/wf_shuffle_time.py 8 1 0 > $O/q4_b4.txt 2>&1 &&
MRH_WF_BUFS=6 timeout -k 10 300 python -u tools/wf_shuffle_time.py 8 1 0 > $O/q4_b6.txt 2>&1
