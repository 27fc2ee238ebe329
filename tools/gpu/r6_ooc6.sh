# out of core with the HBM tier and the zero-copy gather upload: GPU tests, RMAT-18 alone (gather kernel
# on / off) and after RMAT-22, then tri_find_mr RMAT-23 under a 200 GB HBM / 128 GB host budget
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6o; mkdir -p $o
timeout -k 10 500 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_outofcore.py tests/test_ooc_hot_key.py tests/test_spool_writer.py tests/test_checkpoint.py tests/test_triangles.py > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/tests.log; [ $rc -eq 0 ] || exit 1
MRH_OOC_TRACE=2 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/alone.log 2>&1 || exit $?
MRH_GATHER_KERNEL=0 MRH_OOC_TRACE=2 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/alone_nokernel.log 2>&1 || exit $?
BIG=22 MRH_OOC_TRACE=2 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/big.log 2>&1 || exit $?
HEARTBEAT=20 MRH_OOC_TRACE=2 REPS=1 CHECK=1 FPATH=/tmp timeout -k 10 700 python -u tools/trimr_time.py 23 ooc 131072 131072 > $o/ooc23.log 2>&1
