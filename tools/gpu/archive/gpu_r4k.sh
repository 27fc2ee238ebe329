# r4: pool big blocks: pool/fault/OOC tests, tri_find_mr timing, PageRank setup stages
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_hbm_pool.py tests/test_faults.py tests/test_outofcore.py tests/test_pagerank.py > $O/t_k.log 2>&1 &&
timeout -k 10 300 python tools/trimr_time.py 20 > $O/trimr_time.log 2>&1 &&
bash tools/pr_setup_stages.sh
