# r5: dictionary group-by — GPU tests, per-occurrence wordfreq times, kernel profile
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_dict_group.py tests/test_grouper.py tests/test_wordfreq.py tests/test_inverted_index_files.py > $O/wf1_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/wf_shuffle_time.py 1 3 0 > $O/wf1_1g.txt 2>&1 &&
timeout -k 10 400 python -u tools/wf_shuffle_time.py 8 3 0 > $O/wf1_8g.txt 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/wf1prof -o run -- python -u $GRAFT_REPO_ROOT/tools/wf_shuffle_time.py 8 1 0 > $GRAFT_REPO_ROOT/$O/wf1_prof.txt 2>&1
