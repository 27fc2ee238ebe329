# PageRank RMAT-26 setup stages (MRH_PR_STAGES=1), local and forced-RCCL plan; run from the repo root on a GPU box
export TMPDIR=/tmp
MRH_PR_STAGES=1 timeout -k 10 200 python tools/pr_setup_time.py 26 > gpurun_out/pr_stages_local.log 2>&1 &&
MRH_PR_STAGES=1 MRH_FORCE_RCCL=1 timeout -k 10 200 python tools/pr_setup_time.py 26 > gpurun_out/pr_stages_forced.log 2>&1
