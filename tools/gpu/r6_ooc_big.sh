# is the post-big-job slowdown in the disk tier? RMAT-18 out of core after RMAT-22 in HBM:
# pageable uploads through the staging ring (default) vs the runtime's path, and with a
# host budget that keeps everything off disk
set -e
o=gpurun_out/r6e; mkdir -p $o
BIG=22 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/big_stage.log 2>&1
BIG=22 MRH_STAGE_PAGEABLE=0 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/big_nostage.log 2>&1
BIG=22 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc 256 16384 > $o/big_nodisk.log 2>&1
timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/alone_stage.log 2>&1
