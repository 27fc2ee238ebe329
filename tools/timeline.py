"""Timeline of the last job in a rocprofv3 trace (kernels + memory copies):
start offset, duration, gap; long kernels and all copies only.

    python tools/timeline.py DB --copies N   (N = big H2D copies per job)"""
import argparse
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--copies", type=int, default=8)
ap.add_argument("--min-us", type=float, default=20.0)
a = ap.parse_args()
db = sqlite3.connect(a.db)
k = db.execute("select name,start,end from kernels order by start").fetchall()
try:
    m = db.execute("select name,start,end,size from memory_copies order by start").fetchall()
except sqlite3.OperationalError:
    m = []
ev = [(s, e, "K", n.split("(")[0].replace("mrh::k::(anonymous namespace)::", "")[-44:]) for n, s, e in k]
ev += [(s, e, "M", f"{n.replace('MEMORY_COPY_', '')} {sz >> 20} MiB") for n, s, e, sz in m]
ev.sort()
big = [i for i, x in enumerate(ev) if x[2] == "M" and int(x[3].split()[-2]) >= 64]
start = big[-a.copies] if len(big) >= a.copies else 0
t0 = ev[start][0]
for s, e, t, n in ev[start:]:
    if t == "K" and (e - s) / 1e3 < a.min_us:
        continue
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {t} {n}")
