"""Per-chunk host->HBM copy time of the wordfreq bench's 8 pinned chunks,
each copied alone (is any chunk's memory slower to read over PCIe?), then
with a wordcount kernel running concurrently."""
import sys
import time

import torch

sys.path.insert(0, ".")
import gpu_mapreduce_amd as g  # noqa: E402
from gpu_mapreduce_amd import C  # noqa: E402
from gpu_mapreduce_amd.parallel import comm as pcomm  # noqa: E402
from gpu_mapreduce_amd.utils import synth  # noqa: E402

comm = pcomm.init()
chunks = [synth.zipf_text(128 << 20, seed=7 + 1000 * comm.rank + i, device="cuda").cpu().pin_memory() for i in range(8)]
torch.cuda.empty_cache()
d = torch.empty((128 << 20) + 64, dtype=torch.uint8, device="cuda")
d2 = torch.zeros((128 << 20) + 64, dtype=torch.uint8, device="cuda")
d2[: 128 << 20].copy_(chunks[0])
s = torch.cuda.Stream()
for rep in range(2):
    line = []
    for i, h in enumerate(chunks):
        torch.cuda.synchronize()
        t = time.perf_counter()
        d[: h.numel()].copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        line.append(f"{(time.perf_counter() - t) * 1e3:.2f}")
    print("alone ms:", " ".join(line), flush=True)
wc = C.WordCounter("cuda:0")
line = []
for i, h in enumerate(chunks):
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        wc.add(d2, 128 << 20)
    t = time.perf_counter()
    d[: h.numel()].copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    line.append(f"{(time.perf_counter() - t) * 1e3:.2f}")
print("with wc_count ms:", " ".join(line), flush=True)
