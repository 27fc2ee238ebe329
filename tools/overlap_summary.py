#!/usr/bin/env python3
"""Copy / kernel overlap in a window of a rocprofv3 trace (--kernel-trace
--memory-copy-trace, rocpd SQLite): busy time of kernels, of host->device and
device->host copies, the part of the copy time during which a kernel ran, and
the idle time (neither). The window runs from the end of the last dispatch of
kernel --after to the start of the next dispatch of kernel --before (the
second such window when --rep 1). Copies the runtime runs as blit kernels
(__amd_rocclr_copyBuffer*, small or pageable transfers) are counted as
copies of their own, not as compute.

    python tools/overlap_summary.py DB --after k_wedges --before k_emit_tiles [--rep 1]
"""
import argparse
import sqlite3


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def length(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    i = j = 0
    out = []
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--after", required=True)
    ap.add_argument("--before", required=True)
    ap.add_argument("--rep", type=int, default=-1, help="which window (default: the last)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    K = c.execute("select start, end, name from kernels order by start").fetchall()
    M = c.execute("select start, end, size, src_agent_type, dst_agent_type from memory_copies order by start").fetchall()
    wins = []
    last_after = None
    for s, e, n in K:
        if a.after in n:
            last_after = e
        elif a.before in n and last_after is not None:
            wins.append((last_after, s))
            last_after = None
    if not wins:
        raise SystemExit("no window found")
    w0, w1 = wins[a.rep]
    clip = lambda s, e: [max(s, w0), min(e, w1)]
    blit_names = ("__amd_rocclr_copyBuffer", "__amd_rocclr_copyBufferAligned", "__amd_rocclr_copyBufferRect")
    is_blit = lambda n: n.startswith(blit_names)
    kern = union([clip(s, e) for s, e, n in K if e > w0 and s < w1 and not is_blit(n)])
    blit = union([clip(s, e) for s, e, n in K if e > w0 and s < w1 and is_blit(n)])
    nblit = sum(1 for s, e, n in K if e > w0 and s < w1 and is_blit(n))
    h2d = union([clip(s, e) for s, e, _, sa, da in M if e > w0 and s < w1 and sa == "CPU"])
    d2h = union([clip(s, e) for s, e, _, sa, da in M if e > w0 and s < w1 and sa == "GPU" and da == "CPU"])
    hb = sum(sz for s, e, sz, sa, da in M if e > w0 and s < w1 and sa == "CPU")
    db = sum(sz for s, e, sz, sa, da in M if e > w0 and s < w1 and sa == "GPU" and da == "CPU")
    copies = union(h2d + d2h + blit)
    busy = union(kern + copies)
    ms = lambda x: x / 1e6
    print(f"window {ms(w1 - w0):.2f} ms (windows found: {len(wins)})")
    print(f"kernels busy          {ms(length(kern)):9.2f} ms")
    print(f"H2D copies busy       {ms(length(h2d)):9.2f} ms  {hb / 1e6:9.1f} MB  {hb / max(length(h2d), 1):6.1f} GB/s")
    print(f"D2H copies busy       {ms(length(d2h)):9.2f} ms  {db / 1e6:9.1f} MB  {db / max(length(d2h), 1):6.1f} GB/s")
    print(f"blit-kernel copies    {ms(length(blit)):9.2f} ms  ({nblit} dispatches)")
    print(f"copies under kernels  {ms(length(intersect(copies, kern))):9.2f} ms  "
          f"({100 * length(intersect(copies, kern)) / max(length(copies), 1):.0f} % of the copy time)")
    print(f"H2D under D2H         {ms(length(intersect(h2d, d2h))):9.2f} ms")
    print(f"H2D under blit copies {ms(length(intersect(h2d, blit))):9.2f} ms")
    print(f"GPU busy (any)        {ms(length(busy)):9.2f} ms")
    print(f"idle (no kernel, no copy) {ms((w1 - w0) - length(busy)):9.2f} ms")


if __name__ == "__main__":
    main()
