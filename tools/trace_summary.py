#!/usr/bin/env python3
"""Summarise an MRH_TRACE op trace (one JSON line per MapReduce op, one file
per rank: PATH.<rank>) into per-op and per-stage tables. Stages follow the
reference's breakdown (chapter_final.pdf Fig. 4/5): Map, Network I/O,
Sort/Hash, Reduce, Other.

    MRH_TRACE=/tmp/job python my_job.py          (or any native program)
    python tools/trace_summary.py /tmp/job [--json]
"""
import argparse
import collections
import glob
import json
import sys

STAGE = {
    "map": "Map", "map_file": "Map", "map_file_char": "Map", "map_file_str": "Map", "map_mr": "Map",
    "map_mr_batch": "Map", "map_chunks": "Map",
    "aggregate": "Network I/O", "aggregate_dest": "Network I/O", "gather": "Network I/O",
    "broadcast": "Network I/O",
    # a pipelined collate is one leaf op: the shuffle rounds with the
    # group-by of each round hidden under the next one
    "collate": "Network I/O",
    "convert": "Sort/Hash", "clone": "Sort/Hash", "collapse": "Sort/Hash", "sort_keys": "Sort/Hash",
    "sort_values": "Sort/Hash", "sort_multivalues": "Sort/Hash",
    "reduce": "Reduce", "reduce_builtin": "Reduce", "reduce_batch": "Reduce", "compress": "Reduce",
    "compress_builtin": "Reduce",
}


def load(prefix):
    recs = []
    for f in sorted(glob.glob(prefix + ".*")):
        rank = f.rsplit(".", 1)[1]
        if not rank.isdigit():
            continue
        with open(f) as fh:
            for ln in fh:
                r = json.loads(ln)
                r["rank"] = int(rank)
                recs.append(r)
    return recs


def summarise(recs):
    """per-op and per-stage totals over leaf ops (an op's nested ops, e.g.
    collate = aggregate + convert, are counted once, at the deepest level)"""
    ranks = sorted({r["rank"] for r in recs})
    by_rank_op = collections.defaultdict(float)
    calls = collections.Counter()
    sent = collections.Counter()
    # a record is a leaf if no deeper record of the same rank lies inside its time window
    per_rank = collections.defaultdict(list)
    for r in recs:
        per_rank[r["rank"]].append(r)
    for rk, rs in per_rank.items():
        for r in rs:
            t0, t1 = r["t0"], r["t0"] + r["ms"] / 1e3
            inner = [q for q in rs if q["depth"] > r["depth"] and q["t0"] >= t0 and q["t0"] < t1]
            if inner:
                continue
            by_rank_op[(rk, r["op"])] += r["ms"]
            calls[r["op"]] += 1
            sent[r["op"]] += r["sent"]
    ops = sorted({op for _, op in by_rank_op})
    table = []
    for op in ops:
        ms = [by_rank_op.get((rk, op), 0.0) for rk in ranks]
        table.append({"op": op, "stage": STAGE.get(op, "Other"), "calls": calls[op] // max(1, len(ranks)),
                      "ms_max": max(ms), "ms_avg": sum(ms) / len(ms), "sent_bytes": sent[op]})
    stages = collections.defaultdict(float)
    for row in table:
        stages[row["stage"]] += row["ms_max"]
    return {"ranks": len(ranks), "ops": table, "stages_ms": dict(stages)}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)
    recs = load(a.prefix)
    if not recs:
        sys.exit(f"no trace files {a.prefix}.<rank>")
    s = summarise(recs)
    if a.json:
        print(json.dumps(s))
        return
    print(f"# {s['ranks']} rank(s)")
    print(f"{'op':<18} {'stage':<12} {'calls':>6} {'ms(max rank)':>13} {'ms(avg)':>9} {'sent MB':>9}")
    for r in sorted(s["ops"], key=lambda r: -r["ms_max"]):
        print(f"{r['op']:<18} {r['stage']:<12} {r['calls']:>6} {r['ms_max']:>13.3f} {r['ms_avg']:>9.3f} "
              f"{r['sent_bytes'] / 1e6:>9.2f}")
    print("stages (ms):", ", ".join(f"{k} {v:.3f}" for k, v in s["stages_ms"].items()))


if __name__ == "__main__":
    main()
