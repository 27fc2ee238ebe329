# r5: baseline of the per-occurrence wordfreq (no combiner) at 1 and 8 GiB
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u tools/wf_shuffle_time.py 1 3 0 > $O/wf0_1g.txt 2>&1 &&
timeout -k 10 400 python -u tools/wf_shuffle_time.py 8 2 0 > $O/wf0_8g.txt 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/wf0prof -o run -- python -u $GRAFT_REPO_ROOT/tools/wf_shuffle_time.py 1 2 0 > $GRAFT_REPO_ROOT/$O/wf0_prof.txt 2>&1
