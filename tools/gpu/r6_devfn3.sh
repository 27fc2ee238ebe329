cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6f5; mkdir -p $o
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/pf -o t -- python3 $GRAFT_REPO_ROOT/tools/devfn_map_prof.py > $GRAFT_REPO_ROOT/$o/prof.log 2>&1 || exit $?
python3 - <<'PY' > $GRAFT_REPO_ROOT/$o/trace.txt
import csv
rows = list(csv.DictReader(open("/tmp/pf/t_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = None
for r in rows[-40:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    t0 = t0 or s
    print(f"{(s - t0) / 1e6:9.3f} {(e - s) / 1e6:8.3f} ms {r['Grid_Size_X']:>10} {r['Kernel_Name'][:90]}")
PY
