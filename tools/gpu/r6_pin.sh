# the pinned host arena: its GPU test, then out-of-core RMAT-18 cold / warm with the arena
# pinned before the job (8 GiB) and without
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6p3; mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_hostarena.py tests/test_spool_writer.py tests/test_graph_mr.py > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/tests.log
[ $rc -eq 0 ] || exit 1
PREPIN=8192 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/arena8192.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/noarena.log 2>&1 || exit $?
