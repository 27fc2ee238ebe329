# out-of-core tri_find_mr RMAT-18: writer-pool A/B, phase clocks, after a big job
set -e
o=gpurun_out/r6d; mkdir -p $o
timeout -k 10 120 python -u tools/trimr_time.py 18 ooc > $o/a_default.log 2>&1
MRH_SPOOL_WRITERS=64 MRH_SPOOL_WRITE_INFLIGHT=100000000000 timeout -k 10 120 python -u tools/trimr_time.py 18 ooc > $o/b_wide.log 2>&1
MRH_OOC_TRACE=1 timeout -k 10 120 python -u tools/trimr_time.py 18 ooc > $o/c_trace.log 2>&1
BIG=22 timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/d_big.log 2>&1
