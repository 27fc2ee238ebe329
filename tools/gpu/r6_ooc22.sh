# the capacity tier at ~100 GB: tri_find_mr RMAT-22 (7.27 G wedge pairs, ~87 GB through collate 4) out of
# core under a 48 GB HBM / 32 GB pinned-host budget, the disk tier for the rest, TriangleGraph count as the check
# (RMAT-23 does not fit this box: 79 GB of disk, 270 GiB of host memory per command)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6q; mkdir -p $o
{ df -h /tmp; free -g; } > $o/box.txt 2>&1
HEARTBEAT=20 MRH_OOC_TRACE=2 REPS=1 CHECK=1 FPATH=/tmp timeout -k 10 900 python -u tools/trimr_time.py 22 ooc 49152 32768 > $o/ooc22.log 2>&1
