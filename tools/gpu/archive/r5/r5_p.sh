# r5: per-occurrence wordfreq timeline (kernels + memory copies) at 2 GiB: why the map runs at 3 ms per 128 MiB chunk
cd /tmp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/pwf2 -o run -- python -u $R/tools/wf_shuffle_time.py 2 2 0 > $O/p_wf2.txt 2>&1
