# r4: packed (key, value) grouping: GPU suite parts, tri_find_mr timing + profile, graph benches
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 800 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_triangles.py tests/test_oink.py tests/test_grouper.py tests/test_oracles.py tests/test_graph_gpu.py tests/test_outofcore.py tests/test_mapreduce_api.py tests/test_shuffle.py > $O/t_w.log 2>&1 &&
timeout -k 10 300 python tools/trimr_time.py 20 > $O/trimr_time.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_trimr4 -o trimr -- python tools/trimr_time.py 20 > $O/prof_trimr4.log 2>&1
