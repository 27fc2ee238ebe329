# r5: grouped per chunk in the map — tests, timings, kernel profile, PMC of the insert
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_dict_group.py tests/test_grouper.py tests/test_wordfreq.py tests/test_inverted_index_files.py > $O/wf3_tests.txt 2>&1 &&
timeout -k 10 400 python -u tools/wf_shuffle_time.py 8 3 0 > $O/wf3_8g.txt 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/wf3prof -o run -- python -u $GRAFT_REPO_ROOT/tools/wf_shuffle_time.py 8 1 0 > $GRAFT_REPO_ROOT/$O/wf3_prof.txt 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "dict" -d $GRAFT_REPO_ROOT/$O/wf3pmc -o pmc -- python -u $GRAFT_REPO_ROOT/tools/wf_shuffle_time.py 1 1 0 > $GRAFT_REPO_ROOT/$O/wf3_pmc.txt 2>&1
