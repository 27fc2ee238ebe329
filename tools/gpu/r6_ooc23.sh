# (1) pinned-pieces upload microbenchmark: SDMA per piece vs one zero-copy gather kernel, fresh / after
#     180 GB of HBM was touched; (2) the capacity tier at 100+ GB: tri_find_mr RMAT-23 out of core under a
#     200 GB HBM / 64 GB pinned-host budget, the disk tier for the rest, TriangleGraph count as the check
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6n; mkdir -p $o
timeout -k 10 200 tools/bin/h2d_pieces_bench 40 1.6 40 180 > $o/h2d_pieces.log 2>&1 || exit $?
{ df -h /tmp; free -g; } > $o/box.txt 2>&1
HEARTBEAT=20 MRH_OOC_TRACE=2 REPS=1 CHECK=1 FPATH=/tmp timeout -k 10 1000 python -u tools/trimr_time.py 23 ooc 204800 65536 > $o/ooc23.log 2>&1
