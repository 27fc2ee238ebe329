# kernel traces of the three engine workloads whose timed windows must hold no ATen / rocPRIM kernel:
# tri_find_mr RMAT-20, its out-of-core run at RMAT-18, wordfreq without the combiner (both routes).
# Summaries are written on the box and the databases deleted (gpurun_out must stay < 64 MiB).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6h; mkdir -p $o
prof() {  # name marker-kernel command...
  local name=$1 mark=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_$name -o t -- "$@" > $o/$name.log 2>&1 || return $?
  python3 tools/aten_window.py /tmp/prof_$name/*/t_results.db --after-kernel "$mark" > $o/${name}_kernels.txt 2>&1 ||
    python3 tools/aten_window.py $(find /tmp/prof_$name -name "*.db" | head -1) --after-kernel "$mark" > $o/${name}_kernels.txt 2>&1
  rm -rf /tmp/prof_$name
}
prof trimr20 k_rmat python3 tools/trimr_time.py 20 || exit $?
prof ooc18 k_rmat python3 tools/trimr_time.py 18 ooc || exit $?
prof wf k_tok python3 tools/wf_shuffle_time.py 8 2 0 || exit $?
export MRH_FORCE_RCCL=2
prof wfd k_tok python3 tools/wf_shuffle_time.py 8 2 0
