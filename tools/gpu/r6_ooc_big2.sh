# post-big-job slowdown: copy rates and phase clocks, alone vs after RMAT-22 in HBM
set -e
o=gpurun_out/r6f; mkdir -p $o
COPYBW=1 MRH_OOC_TRACE=1 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/alone.log 2>&1
BIG=22 COPYBW=1 MRH_OOC_TRACE=1 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/big.log 2>&1
