# r5: single-copy pinned to_host (spill tier): spill/checkpoint/fault GPU tests + OOC
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_checkpoint.py tests/test_faults.py tests/test_outofcore.py tests/test_ooc_hot_key.py tests/test_append_parts.py tests/test_triangles.py > $O/pin_tests.txt 2>&1
