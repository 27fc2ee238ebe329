"""Allocations against the H2D copy timeline of a wordfreq trace
(tools/gpu/archive/gpu_wf_alloc.sh): for the last 3 jobs, every 128 MiB copy (start,
duration) interleaved with every device allocation or free that started
within 1 ms of a copy.

    python tools/wf_alloc_tl.py gpurun_out/prof_wf_alloc/*/p_results.db
"""
import sqlite3
import sys


def main(path):
    db = sqlite3.connect(path)
    names = [r[0] for r in db.execute("select name from sqlite_master where type in ('table','view')")]
    alloc_tab = next((n for n in names if n == "memory_allocations"), None) or \
        next((n for n in names if "alloc" in n.lower()), None)
    print("# allocation table:", alloc_tab)
    cols = [r[1] for r in db.execute(f"pragma table_info({alloc_tab})")]
    print("# columns:", cols)
    cp = db.execute("select start,end from memory_copies where size >= 100000000 order by start").fetchall()
    al = db.execute(f"select * from {alloc_tab} order by start").fetchall()
    ci = {c: i for i, c in enumerate(cols)}
    print(f"# {len(cp)} big copies, {len(al)} allocation records")
    win = cp[-24:]
    t0 = win[0][0]
    ev = [(a, "COPY", (b - a) / 1e3, "") for a, b in win]
    for r in al:
        a = r[ci["start"]]
        if a < t0 - 1e6:
            continue
        desc = " ".join(f"{k}={r[ci[k]]}" for k in ("operation", "name", "size", "agent_type", "category")
                        if k in ci and r[ci[k]] is not None)
        ev.append((a, "ALLOC", (r[ci["end"]] - a) / 1e3 if "end" in ci else 0.0, desc))
    for a, kind, d, desc in sorted(ev):
        print(f"{(a - t0) / 1e3:10.1f} us  {kind:5s} {d:8.1f} us  {desc}")


if __name__ == "__main__":
    main(sys.argv[1])
