# kernel time of wordfreq's P > 1 route (one-rank RCCL communicator, 8 GiB, 2 jobs)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6w2; mkdir -p $o
cd /tmp && MRH_FORCE_RCCL=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pf -o t -- python3 $GRAFT_REPO_ROOT/tools/wf_shuffle_time.py 8 2 0 > $GRAFT_REPO_ROOT/$o/run.log 2>&1 || exit $?
cp /tmp/pf/t_kernel_stats.csv $GRAFT_REPO_ROOT/$o/kernel_stats.csv
python3 - <<'PY' > $GRAFT_REPO_ROOT/$o/last_job.txt
import csv
rows = list(csv.DictReader(open("/tmp/pf/t_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last job: from the last k_tok-ish kernel window; print the last 3000 dispatches aggregated by name
tail = rows[-4000:]
agg = {}
for r in tail:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    n = r["Kernel_Name"][:100]
    a = agg.setdefault(n, [0, 0.0])
    a[0] += 1
    a[1] += d
span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e6
print(f"last {len(tail)} dispatches span {span:.1f} ms")
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:30]:
    print(f"{t:9.2f} ms {c:6d}  {n}")
PY
