cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6f10; mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_device_functors.py > $o/tests.log 2>&1
