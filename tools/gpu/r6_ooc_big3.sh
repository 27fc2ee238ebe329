# (1) out-of-core RMAT-18 host phase clocks alone / after RMAT-22 (upload totals),
# (2) the capacity tier at scale: tri_find_mr RMAT-22 then RMAT-23 out of core with the
#     TriangleGraph count as the check, per-stage PCIe and disk bytes
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6k; mkdir -p $o
MRH_OOC_TRACE=2 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/alone.log 2>&1 || exit $?
BIG=22 MRH_OOC_TRACE=2 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/big.log 2>&1 || exit $?
{ df -h /tmp; free -g; nproc; } > $o/box.txt 2>&1
REPS=1 CHECK=1 FPATH=/tmp timeout -k 10 300 python -u tools/trimr_time.py 22 ooc 32768 16384 > $o/ooc22.log 2>&1 || exit $?
REPS=1 CHECK=1 FPATH=/tmp timeout -k 10 500 python -u tools/trimr_time.py 23 ooc 204800 49152 > $o/ooc23.log 2>&1
