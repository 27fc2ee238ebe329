"""wordfreq job phases on one GPU (1 GiB, 8 x 128 MiB chunks): host wall time
of each step of WordFreq.run with the device synchronised at every boundary,
plus the time from job construction to the first H2D issue."""
import sys
import time

import torch

sys.path.insert(0, ".")
import gpu_mapreduce_amd as g  # noqa: E402
from gpu_mapreduce_amd.models.wordfreq import WordFreq  # noqa: E402
from gpu_mapreduce_amd.utils import synth  # noqa: E402

chunks = [synth.zipf_text(128 << 20, seed=7919 + i, device="cuda").cpu().pin_memory() for i in range(8)]
torch.cuda.empty_cache()
comm = g.Comm(device="cuda:0")


def T():
    torch.cuda.synchronize()
    return time.perf_counter()


for rep in range(5):
    t0 = T()
    mr = g.MapReduce(comm)
    app = WordFreq(mr, chunks)
    t1 = T()
    mr.map(mr.nprocs, app._map)
    t2 = T()
    mr.collate()
    t3 = T()
    mr.reduce("sum:int32")
    t4 = T()
    mr.sort_values(-1)
    t5 = T()

    def keep_top(src, kv):
        n = min(10, src.n)
        koff = src.koff[: n + 1]
        kv.add_tensors(src.kdata[: int(koff[-1].item())], src.vdata[: 4 * n].view(torch.int32), koff=koff)
    mr.map_mr_batch(mr, keep_top)
    mr.gather(1)
    mr.sort_values(-1)
    top = mr.kv_pairs()
    t6 = T()
    ms = lambda a, b: round((b - a) * 1e3, 3)  # noqa: E731
    print(f"rep {rep}: construct {ms(t0, t1)}  map {ms(t1, t2)}  collate {ms(t2, t3)}  reduce {ms(t3, t4)}  "
          f"sort {ms(t4, t5)}  top-N {ms(t5, t6)}  total {ms(t0, t6)}", flush=True)
