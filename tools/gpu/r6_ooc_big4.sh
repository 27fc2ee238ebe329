# out-of-core: staging waits vs memcpy alone / after RMAT-22; then RMAT-21 under 8 GiB HBM / 4 GiB host
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6l; mkdir -p $o
MRH_OOC_TRACE=2 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/alone.log 2>&1 || exit $?
BIG=22 MRH_OOC_TRACE=2 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/big.log 2>&1 || exit $?
HEARTBEAT=20 MRH_OOC_TRACE=2 REPS=1 CHECK=1 FPATH=/tmp timeout -k 10 400 python -u tools/trimr_time.py 21 ooc 8192 4096 > $o/ooc21.log 2>&1
