# r4: final: full GPU test suite, default record, smoke
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ > $O/t_final.log 2>&1 &&
timeout -k 10 600 python bench.py > $O/bench_final.json 2> $O/bench_final.err &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
