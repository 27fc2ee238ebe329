# r5: GPU tests of this round's changes (dict group-by, parts, piece size, distributed wordfreq),
# the wordfreq extras of the record at 8 GiB, and tri_find_mr RMAT-20 stage times
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_distributed_gpu.py tests/test_rccl_gpu.py tests/test_append_parts.py tests/test_triangles.py tests/test_dict_group.py -k "wordfreq or inverted or collate or rccl or append or add or tri_find_mr or dict or convert" > $O/a_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/trimr_time.py 20 > $O/a_trimr20.txt 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --pagerank-scale 0 --trifind-scale 0 --trifind-mr-scale 0 --file-io-steps 0 --dist-extras 0 > $O/a_bench.json 2> $O/a_bench.err
