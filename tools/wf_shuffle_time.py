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
from gpu_mapreduce_amd.parallel.comm import bind_numa_local  # noqa: E402
bind_numa_local(0)  # as bench.py: host buffers on the GPU's NUMA node
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
from gpu_mapreduce_amd.runtime import hbm_pool  # noqa: E402
for rep in range(jobs):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    del app  # the previous job's MapReduce goes away here (inside the bench's timed loop too)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    app = WordFreq(g.MapReduce(comm), chunks, combiner=comb)
    app.run()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    st = hbm_pool.stats(0) if hbm_pool.installed() else {}
    print(f"plain job {rep}: {(t2 - t0) * 1e3:.1f} ms (teardown of the previous {(t1 - t0) * 1e3:.1f}, job "
          f"{(t2 - t1) * 1e3:.1f}); pool grows {st.get('grows')} grow_ms {st.get('grow_ms')} releases "
          f"{st.get('releases')} reserved {st.get('reserved', 0) / 1e9:.1f} GB", flush=True)
# H2D into each staging slot of the ring, from one pinned chunk (is one slot slow?)
src = chunks[0]
for b, buf in enumerate(app.bufs):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        buf[: src.numel()].copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    print(f"slot {b}: {src.numel() / dt / 1e9:.1f} GB/s  ptr {buf.data_ptr():#x}", flush=True)
for i in range(min(6, len(chunks))):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    app.bufs[0][: chunks[i].numel()].copy_(chunks[i], non_blocking=True)
    torch.cuda.synchronize()
    print(f"chunk {i} -> slot 0: {chunks[i].numel() / (time.perf_counter() - t0) / 1e9:.1f} GB/s  host ptr {chunks[i].data_ptr():#x}", flush=True)
