# r5: big-block arena + compact wedge kernel: tests, tri_find_mr RMAT-20 / RMAT-22, the trifind_mr extra
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_hbm_pool.py tests/test_append_parts.py tests/test_triangles.py > $O/c_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/trimr_time.py 20 > $O/c_trimr20.txt 2>&1 &&
timeout -k 10 400 python -u tools/trimr_time.py 22 > $O/c_trimr22.txt 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --pagerank-scale 0 --trifind-scale 0 --wordfreq-bytes 0 --file-io-steps 0 --dist-extras 0 > $O/c_bench.json 2> $O/c_bench.err
