#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --kernel-trace run (rocpd SQLite output).

    python tools/rocpd_summary.py DB [--top N] [--skip-first-ms T] [--title "..."]

Prints total ms / calls / avg us / % per kernel name (demangled name cut to
90 chars), plus the host<->device copy totals. --after-marker-kernel K keeps
only dispatches after the first dispatch whose name contains K (to drop
setup / data generation before the timed region)."""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--title", default="")
    ap.add_argument("--after-kernel", default=None,
                    help="only count dispatches starting after the first dispatch of a kernel containing this")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    t0 = 0
    if a.after_kernel:
        r = c.execute("select min(start) from kernels where name like ?", (f"%{a.after_kernel}%",)).fetchone()
        t0 = r[0] or 0
    rows = c.execute("select name, count(*), sum(duration) from kernels where start >= ? group by name "
                     "order by sum(duration) desc", (t0,)).fetchall()
    tot = sum(r[2] for r in rows) or 1
    if a.title:
        print(f"# {a.title}")
    print(f"# kernels: {sum(r[1] for r in rows)} dispatches, {tot / 1e6:.3f} ms GPU time")
    print(f"{'total_ms':>10} {'calls':>6} {'avg_us':>9} {'pct':>6}  kernel")
    for name, n, d in rows[: a.top]:
        print(f"{d / 1e6:10.3f} {n:6d} {d / n / 1e3:9.1f} {100 * d / tot:6.2f}  {name[:90]}")
    cp = c.execute("select src_agent_type, dst_agent_type, count(*), sum(size), sum(duration) from memory_copies "
                   "where start >= ? group by src_agent_type, dst_agent_type", (t0,)).fetchall()
    for s, d, n, b, dur in cp:
        bw = (b / dur) if dur else 0
        print(f"# copies {s}->{d}: {n} x, {b / 1e6:.1f} MB, {dur / 1e6:.3f} ms, {bw:.1f} GB/s")


if __name__ == "__main__":
    main()
