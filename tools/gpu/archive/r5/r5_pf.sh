# r5: out-of-core tri_find_mr RMAT-18 at partition factors 4 / 3 / 2.5 (MRH_OOC_PART_FACTOR), then the OOC tests at 3
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
for f in 4 3 2.5; do
  MRH_OOC_PART_FACTOR=$f timeout -k 10 300 python -u tools/trimr_time.py 18 ooc > $O/pf_$f.txt 2>&1 || exit $?
done
MRH_OOC_PART_FACTOR=3 timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_outofcore.py tests/test_ooc_hot_key.py > $O/pf_tests.txt 2>&1
