# out-of-core after the staged multi-threaded pageable uploads: GPU tests, RMAT-18 alone / after
# RMAT-22, RMAT-21 under an 8 GiB HBM / 4 GiB host budget (disk tier)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6m; mkdir -p $o
timeout -k 10 500 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_outofcore.py tests/test_ooc_hot_key.py tests/test_spool_writer.py tests/test_checkpoint.py tests/test_triangles.py tests/test_append_parts.py > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/tests.log; [ $rc -eq 0 ] || exit 1
MRH_OOC_TRACE=2 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/alone.log 2>&1 || exit $?
BIG=22 MRH_OOC_TRACE=2 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/big.log 2>&1 || exit $?
HEARTBEAT=20 MRH_OOC_TRACE=2 REPS=1 CHECK=1 FPATH=/tmp timeout -k 10 400 python -u tools/trimr_time.py 21 ooc 8192 4096 > $o/ooc21.log 2>&1
