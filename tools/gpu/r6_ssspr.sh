# sssp_mr out-of-core nondeterminism: repetitions under diagnostic switches
cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o
MRH_SYNC=1 timeout -k 10 300 python -u tools/sssp_ooc_repeat.py 20 > $o/sync.log 2>&1 &&
MRH_GATHER_KERNEL=0 timeout -k 10 240 python -u tools/sssp_ooc_repeat.py 20 > $o/nogather.log 2>&1 &&
MRH_PACKED_PAIRS=0 timeout -k 10 240 python -u tools/sssp_ooc_repeat.py 20 > $o/nopacked.log 2>&1
