# the capacity tier at 100+ GB: tri_find_mr RMAT-23 (17.7 G wedge pairs, ~212 GB) out of core under a
# 128 GB HBM / 128 GB pinned-host budget, the disk tier for the rest, TriangleGraph count as the check
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6p; mkdir -p $o
{ df -h /tmp; free -g; } > $o/box.txt 2>&1
HEARTBEAT=20 MRH_OOC_TRACE=2 REPS=1 CHECK=1 FPATH=/tmp timeout -k 10 900 python -u tools/trimr_time.py 23 ooc 131072 131072 > $o/ooc23.log 2>&1
