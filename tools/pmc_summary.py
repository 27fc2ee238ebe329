"""Per-kernel PMC counter totals from a rocprofv3 --pmc database.

usage: python tools/pmc_summary.py <p_results.db> [kernel-substring ...]
Prints, per kernel name (truncated), the dispatch count, the mean duration and
the per-dispatch mean of every collected counter."""
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sqlite3.connect(sys.argv[1])
    pats = sys.argv[2:]
    rows = db.execute("select dispatch_id, kernel_name, counter_name, value, duration from counters_collection")
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    dur = defaultdict(dict)
    for did, name, cname, val, d in rows:
        if pats and not any(p in name for p in pats):
            continue
        agg[name][cname] += val
        disp[name].add(did)
        dur[name][did] = d
    for name in sorted(agg, key=lambda n: -sum(dur[n].values())):
        n = len(disp[name])
        ms = sum(dur[name].values()) / max(n, 1) / 1e6
        cs = "  ".join(f"{c}={v / n:.4g}" for c, v in sorted(agg[name].items()))
        print(f"{name[:90]}\n    dispatches={n} mean_ms={ms:.3f}  {cs}")


if __name__ == "__main__":
    main()
