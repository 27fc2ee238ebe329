# r5: raw pinned uploads + deferred spool syncs: OOC tests, out-of-core tri_find_mr RMAT-18 (timing, phase trace, kernel + copy trace)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_outofcore.py tests/test_ooc_hot_key.py tests/test_triangles.py tests/test_append_parts.py tests/test_hbm_pool.py > $O/u_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/trimr_time.py 18 ooc > $O/u_ooc18.txt 2>&1 &&
MRH_OOC_TRACE=1 timeout -k 10 300 python -u tools/trimr_time.py 18 ooc > $O/u_ooc18_trace.txt 2>&1 && cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/uooc -o run -- python -u $GRAFT_REPO_ROOT/tools/trimr_time.py 18 ooc > $O/u_pooc.txt 2>&1
