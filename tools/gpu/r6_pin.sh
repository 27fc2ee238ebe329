# out-of-core RMAT-18 cold / warm with the pinned host reserve allocated before the job
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6p2; mkdir -p $o
PREPIN=1 PYTORCH_HIP_ALLOC_CONF=pinned_use_hip_host_register:True,pinned_num_register_threads:16,pinned_reserve_segment_size_mb:4096 \
  timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/reg_reserve4096.log 2>&1 || exit $?
PREPIN=1 PYTORCH_HIP_ALLOC_CONF=pinned_reserve_segment_size_mb:4096 \
  timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/reserve4096.log 2>&1 || exit $?
PREPIN=1 PYTORCH_HIP_ALLOC_CONF=pinned_use_hip_host_register:True,pinned_num_register_threads:16,pinned_reserve_segment_size_mb:8192 \
  timeout -k 10 200 python -u tools/trimr_time.py 18 ooc > $o/reg_reserve8192.log 2>&1 || exit $?
