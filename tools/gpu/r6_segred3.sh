cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6s4; mkdir -p $o
timeout -k 10 200 python -u tools/segred_mr_probe.py > $o/probe.log 2>&1 || exit $?
