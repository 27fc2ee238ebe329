# r5: kernel profiles of the per-occurrence wordfreq (8 GiB) and tri_find_mr RMAT-20
cd /tmp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pwf -o run -- python -u $R/tools/wf_shuffle_time.py 8 1 0 > $O/pwf.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ptri -o run -- python -u $R/tools/trimr_time.py 20 > $O/ptri.txt 2>&1
