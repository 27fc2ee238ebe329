cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r6s4; mkdir -p $o
timeout -k 10 200 python -u tools/segred_keys_bench.py > $o/keys.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/pf -o t -- python3 $GRAFT_REPO_ROOT/tools/segred_keys_bench.py > $GRAFT_REPO_ROOT/$o/prof.log 2>&1 || exit $?
python3 - <<'PY' > $GRAFT_REPO_ROOT/$o/trace.txt
import csv
rows = list(csv.DictReader(open("/tmp/pf/t_kernel_trace.csv")))
print(list(rows[0].keys()))
for r in rows:
    nm = r.get("Kernel_Name", "")
    if "segred" in nm or "carry" in nm:
        print(nm[:50], r.get("Grid_Size", r.get("Grid_Size_X", "")), r.get("Workgroup_Size", ""), r.get("LDS_Block_Size", r.get("Lds_Size", "")),
              (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
PY
