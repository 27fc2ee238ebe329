# r4: new GPU tests, then the default bench record
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_fileio.py tests/test_inverted_index_files.py tests/test_wordfreq.py > $O/t_d.log 2>&1 &&
timeout -k 10 500 python bench.py > $O/bench_d.json 2> $O/bench_d.err
