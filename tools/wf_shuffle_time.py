"""wordfreq without the in-mapper combiner (one (word, NULL) pair per
occurrence through collate -> reduce("count") -> top-N) on one GPU: per-stage
device-synced times of a few jobs, then the plain job time.

    python tools/wf_shuffle_time.py [GiB] [jobs] [combiner 0/1]
"""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import gpu_mapreduce_amd as g  # noqa: E402
from gpu_mapreduce_amd.models.wordfreq import WordFreq  # noqa: E402
from gpu_mapreduce_amd.utils import synth  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
jobs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
comb = bool(int(sys.argv[3])) if len(sys.argv) > 3 else False
nb = int(gib * (1 << 30))
chunk = 128 << 20
chunks = []
for i, o in enumerate(range(0, nb, chunk)):
    chunks.append(synth.zipf_text(min(chunk, nb - o), seed=7919 + i, device="cuda").cpu().pin_memory())
torch.cuda.empty_cache()
comm = g.Comm(device="cuda:0")
print(f"{gib} GiB, {len(chunks)} chunks, combiner={comb}", flush=True)
for rep in range(jobs):
    ph = {}
    app = WordFreq(g.MapReduce(comm), chunks, combiner=comb)
    t0 = time.perf_counter()
    app.run(ph)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) * 1e3
    print(f"job {rep}: {t:.1f} ms  " + "  ".join(f"{k} {v * 1e3:.1f}" for k, v in ph.items())
          + f"  pairs {app.npairs} unique {app.nunique} top {app.top[:3]}", flush=True)
for rep in range(jobs):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    app = WordFreq(g.MapReduce(comm), chunks, combiner=comb)
    app.run()
    torch.cuda.synchronize()
    print(f"plain job {rep}: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
