# device functors (fold tree merge): GPU tests + timings, then a kernel profile of the 1024-key case
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6f4; mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_device_functors.py > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $o/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/devfn_time.py 27 0 > $o/time_27_0.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/devfn_time.py 27 10 > $o/time_27_10.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pf -o t -- python3 $GRAFT_REPO_ROOT/tools/devfn_time.py 27 10 > $GRAFT_REPO_ROOT/$o/prof.log 2>&1 || exit $?
find /tmp/pf -name "*kernel_stats.csv" -exec cp {} $GRAFT_REPO_ROOT/$o/kernel_stats.csv \;
ls -R /tmp/pf | head -20 > $GRAFT_REPO_ROOT/$o/pf_ls.txt
