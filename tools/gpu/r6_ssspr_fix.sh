# host gather with system-scope loads: sssp_mr out-of-core repetitions, then
# the out-of-core tri_find_mr (RMAT-18, 256 MiB HBM / 2 GiB host) for its time
cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 500 python -u tools/sssp_ooc_repeat.py 40 > $o/repeat.log 2>&1 &&
CHECK=1 REPS=3 timeout -k 10 300 python -u tools/trimr_time.py 18 ooc > $o/ooc18.log 2>&1
