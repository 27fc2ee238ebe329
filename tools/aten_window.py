#!/usr/bin/env python3
"""ATen / rocPRIM kernels in a rocprofv3 --kernel-trace database (rocpd
SQLite), optionally only after the first dispatch of a marker kernel (the
start of the timed window, after synthetic-data generation).

    python tools/aten_window.py DB [--after-kernel NAME] [--top N]

Prints the top kernels by time, then every at::native / rocprim / hipcub
kernel in the window with its count and time (the engine's own kernels are
mrh::*)."""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--after-kernel", default=None)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    t0 = 0
    if a.after_kernel:
        r = c.execute("select min(start) from kernels where name like ?", (f"%{a.after_kernel}%",)).fetchone()
        t0 = r[0] or 0
    rows = c.execute("select name, count(*), sum(duration), min(start), max(end) from kernels where start >= ? "
                     "group by name order by sum(duration) desc", (t0,)).fetchall()
    tot = sum(r[2] for r in rows) or 1
    span = (max(r[4] for r in rows) - min(r[3] for r in rows)) / 1e6 if rows else 0
    print(f"window: {len(rows)} kernel names, {sum(r[1] for r in rows)} dispatches, kernel time {tot / 1e6:.2f} ms, "
          f"span {span:.1f} ms")
    for name, n, d, _, _ in rows[:a.top]:
        print(f"{d / 1e6:10.3f} ms {n:7d}  {100 * d / tot:5.1f}%  {name[:110]}")
    foreign = [r for r in rows if any(s in r[0] for s in ("at::native", "rocprim", "hipcub", "at::cuda"))]
    ft = sum(r[2] for r in foreign)
    print(f"\nATen / rocPRIM kernels in the window: {len(foreign)} names, {sum(r[1] for r in foreign)} dispatches, "
          f"{ft / 1e6:.3f} ms ({100 * ft / tot:.1f}% of kernel time)")
    for name, n, d, _, _ in foreign:
        print(f"{d / 1e6:10.3f} ms {n:7d}  {name[:150]}")
    # where they come from: the engine kernels dispatched just before the
    # first dispatch of each foreign kernel
    if foreign:
        print("\ncontext (the 3 kernels dispatched before the first dispatch of each):")
        for name, _, _, first, _ in foreign[:20]:
            prev = c.execute("select name from kernels where start < ? and start >= ? order by start desc limit 3",
                             (first, t0)).fetchall()
            print(f"  {name[:70]}  <-  " + "  <-  ".join(p[0][:50] for p in prev))


if __name__ == "__main__":
    main()
