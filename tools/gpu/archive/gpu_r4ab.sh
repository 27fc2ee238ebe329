# r4: final record after the wordfreq 1 GiB extra: bench launcher GPU test, default record, smoke
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_bench_launcher.py > $O/t_ab.log 2>&1 &&
timeout -k 10 600 python bench.py > $O/bench_final.json 2> $O/bench_final.err &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
