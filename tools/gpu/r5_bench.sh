# r5: default bench record + smoke
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/bb_smoke.txt 2>&1 &&
timeout -k 10 500 python bench.py > $O/bb_bench.txt 2>&1
