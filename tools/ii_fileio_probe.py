#!/usr/bin/env python3
"""Where the time of bench.py's with_file_io goes: the same pipelined job
window with reads and writes (the record), without the index write, without
the part-file reads (buffers filled once before), and with neither."""
import argparse, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench
from gpu_mapreduce_amd.parallel import comm as pcomm

comm = pcomm.init()
ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=5)
a = ap.parse_args()
args = argparse.Namespace(bytes_per_gpu=float(1 << 30), file_bytes=128 << 20, seed=1, link_gap=200, steps=a.steps,
                          warmup=2)
out = {}
for name, rd, wr in (("read+write", True, True), ("read only", True, False), ("write only", False, True),
                     ("neither", False, False)):
    args.fileio_read, args.fileio_write = rd, wr
    r = bench.bench_inverted_index_files(comm, args)
    out[name] = {k: round(v, 2) if isinstance(v, float) else v for k, v in r.items() if k != "note"}
    print(name, json.dumps(out[name]), flush=True)
