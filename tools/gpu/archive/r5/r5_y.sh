# r5: out-of-core tri_find_mr RMAT-18 with and without bench.py's NUMA binding; then the bench's trifind_mr extra alone (RMAT-22 before it, then OOC)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
nproc > $O/y_nproc.txt; python -c "import os; print(len(os.sched_getaffinity(0)))" >> $O/y_nproc.txt
timeout -k 10 300 python -u tools/trimr_time.py 18 ooc > $O/y_plain.txt 2>&1 &&
NUMA=1 timeout -k 10 300 python -u tools/trimr_time.py 18 ooc > $O/y_numa.txt 2>&1
