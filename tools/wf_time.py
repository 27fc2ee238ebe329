import sys, time, torch
sys.path.insert(0, "/root/repo")
import gpu_mapreduce_amd as g
from gpu_mapreduce_amd.models.wordfreq import WordFreq
from gpu_mapreduce_amd.utils import synth
chunks = [synth.zipf_text(128 << 20, seed=7919 + i, device="cuda").cpu().pin_memory() for i in range(8)]
comm = g.Comm(device="cuda:0")
for rep in range(4):
    app = WordFreq(g.MapReduce(comm), chunks)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    app.mr.map(1, app._map); torch.cuda.synchronize(); t1 = time.perf_counter()
    app.mr.collate(); app.mr.reduce("sum:int32"); torch.cuda.synchronize(); t2 = time.perf_counter()
    app.mr.sort_values(-1); torch.cuda.synchronize(); t3 = time.perf_counter()
    print(f"map {1e3*(t1-t0):.2f} ms  collate+reduce {1e3*(t2-t1):.2f}  sort {1e3*(t3-t2):.2f}", flush=True)
# per-chunk timing inside the map
from gpu_mapreduce_amd import C
wc = C.WordCounter("cuda:0")
buf = torch.zeros((128 << 20) + 64, dtype=torch.uint8, device="cuda")
buf[: 128 << 20].copy_(chunks[0])
for i in range(4):
    torch.cuda.synchronize(); t = time.perf_counter()
    wc.add(buf, 128 << 20); torch.cuda.synchronize()
    print(f"add {1e3*(time.perf_counter()-t):.3f} ms", flush=True)
t = time.perf_counter(); kv = wc.finish(); torch.cuda.synchronize(); print(f"finish {1e3*(time.perf_counter()-t):.3f} ms")
