#!/usr/bin/env python3
"""sort_keys(+-5) on ~10 M synthetic URLs that share a 29-byte prefix
("http://en.wikipedia.org/wiki/", the InvertedIndex corpus): the first radix
pass sees only "http://e", so the order comes from the device tie-break
rounds. Prints ms per sort and checks the order of a sample against strcmp.
Run under rocprofv3 --memory-copy-trace to see that no key column goes D2H."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpu_mapreduce_amd._ext import C  # noqa: E402
from gpu_mapreduce_amd.utils import synth  # noqa: E402

dev = "cuda:0"
want = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
parts = []
n = 0
seed = 0
while n < want:
    files = synth.html_corpus(256 << 20, file_bytes=256 << 20, seed=11 + seed, device=dev, nurl=4_000_000)
    for _, t in files:
        buf = torch.zeros(t.numel() + 64, dtype=torch.uint8, device=dev)
        buf[: t.numel()].copy_(t)
        kv = C.map_urls(buf, t.numel(), seed)
        parts.append(kv)
        n += kv.n
    seed += 1
kv = C.concat(parts, dev)
del parts
torch.cuda.synchronize()
print(f"{kv.n} URL keys, {kv.kdata.numel() / kv.n:.1f} bytes avg", flush=True)
for flag in (5, -5):
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = C.sort_kv(kv, flag, False)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        print(f"flag {flag} rep {rep}: {ms:.1f} ms", flush=True)
    # check a contiguous sample of the result against strcmp order
    ko = out.koff[: 200001].cpu()
    kd = out.kdata[: int(ko[-1])].cpu().numpy().tobytes()
    keys = [kd[int(ko[i]):int(ko[i + 1])] for i in range(200000)]
    keys = [k.split(b"\0", 1)[0] for k in keys]
    ok = all((keys[i] <= keys[i + 1]) if flag > 0 else (keys[i] >= keys[i + 1]) for i in range(len(keys) - 1))
    print(f"flag {flag} sample order ok: {ok}", flush=True)
    assert ok
