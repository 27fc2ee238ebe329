# the whole GPU test suite, as the driver runs it at round end, plus smoke()
cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 1500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $o/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc" >> $o/gpu_suite.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
