# r5: KMV parts / pwrite spools: OOC + triangle tests, out-of-core tri_find_mr RMAT-18 (plain + phase trace), then the full default record
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_outofcore.py tests/test_ooc_hot_key.py tests/test_triangles.py tests/test_append_parts.py tests/test_mapreduce_api.py > $O/k_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/trimr_time.py 18 ooc > $O/k_ooc18.txt 2>&1 &&
MRH_OOC_TRACE=1 timeout -k 10 300 python -u tools/trimr_time.py 18 ooc > $O/k_ooc18_trace.txt 2>&1 &&
timeout -k 10 900 python -u bench.py > $O/l_bench.json 2> $O/l_bench.err
