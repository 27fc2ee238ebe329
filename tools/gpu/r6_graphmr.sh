# GPU tests of sssp_mr / luby_find_mr, then their timings on R-MAT graphs
# next to the plan-based sssp / luby_find commands
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}
o=gpurun_out/r6g; mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_graph_mr.py tests/test_oink.py > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/tests.log
[ $rc -eq 0 ] || exit 1
mkdir -p /tmp/oinkrun && cp examples/oink/in.* /tmp/oinkrun/ && cd /tmp/oinkrun || exit 1
for sc in 16 18 20; do
  for s in in.sssp_mr in.sssp in.luby_mr in.luby; do
    echo "== $s scale $sc" >> $GRAFT_REPO_ROOT/$o/timings.log
    timeout -k 10 300 python -u -m gpu_mapreduce_amd.oink -in $s -var scale $sc -log none >> $GRAFT_REPO_ROOT/$o/timings.log 2>&1 || exit $?
  done
done
