# r5: fused packed segmentation + wave-match radix histogram + ordered buckets:
# tests (packed convert, dict group, triangles, kernels), tri_find_mr RMAT-20 / 22, PageRank default
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_append_parts.py tests/test_triangles.py tests/test_kernels_gpu.py tests/test_dict_group.py tests/test_mapreduce_api.py tests/test_ooc_hot_key.py tests/test_outofcore.py > $O/d_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/trimr_time.py 20 > $O/d_trimr20.txt 2>&1 &&
timeout -k 10 400 python -u tools/trimr_time.py 22 > $O/d_trimr22.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dtri -o run -- python -u tools/trimr_time.py 20 > $O/d_ptri.txt 2>&1 &&
timeout -k 10 200 python bench.py --workload pagerank --steps 3 --warmup 1 > $O/d_pr.log 2>&1
