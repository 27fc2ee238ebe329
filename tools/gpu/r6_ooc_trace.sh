# out-of-core RMAT-18: host wall time per phase without device syncs (MRH_OOC_TRACE=2), alone and after RMAT-22
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6k; mkdir -p $o
MRH_OOC_TRACE=2 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/alone.log 2>&1 || exit $?
BIG=22 MRH_OOC_TRACE=2 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/big.log 2>&1
