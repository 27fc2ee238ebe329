# r4: final default record (bench.py, no flags) + smoke()
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python bench.py > $O/bench_final.json 2> $O/bench_final.err &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
