# sssp_mr out-of-core repetitions with the pinned pieces uploaded by hipMemcpyAsync
# (MRH_GATHER_KERNEL=0), then the out-of-core tri_find_mr time that way
cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o
MRH_GATHER_KERNEL=0 timeout -k 10 500 python -u tools/sssp_ooc_repeat.py 40 > $o/repeat.log 2>&1 &&
MRH_GATHER_KERNEL=0 CHECK=1 REPS=3 timeout -k 10 300 python -u tools/trimr_time.py 18 ooc > $o/ooc18.log 2>&1
