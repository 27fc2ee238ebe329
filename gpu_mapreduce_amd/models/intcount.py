"""IntCount: count occurrences of 4-byte integers (reference cpu/IntCount.cpp).

Reference (cpu/IntCount.cpp:75-81, 150-190): every rank reads a 128 MB file
of raw ints (32 M 4-byte ints), emits KV(int, int 1) per int with a host
`kv->add` loop, then `aggregate` + `convert` (the reduce is commented out).
The chapter's GPMR IntegerCount (same shape: 32 M ints per GPU) also counts,
so this app finishes with `reduce(count)`.

MI355X pipeline per rank:
  map        the 128 MB "file" streams host(pinned) -> HBM; the key array IS
             the file (4-byte fixed-width keys, no per-pair work), values are
             int32 1 (fixed width): one `add_tensors` call, no host loop;
  aggregate  hashlittle partition kernel + RCCL all-to-all (N > 1);
  convert    exact-bit LSD radix sort of the 4-byte keys + head flags + scan;
  reduce     "count" segmented reduce kernel -> (int, int32 count).
"""
from __future__ import annotations

import time

import numpy as np
import torch

from ..runtime.mapreduce import MapReduce

# GPMR IntegerCount (chapter_final.pdf p.14, Fig. 6(b)): 32 M ints per GPU,
# 3.94 s total at 20 GK104 nodes -> 162 M KV/s aggregate, 8.1 M KV/s per GPU
REF_KVPS_PER_GPU = 20 * 32 * (1 << 20) / 3.94 / 20


def int_file(nbytes: int, key_range: int, seed: int, rank: int = 0) -> torch.Tensor:
    """Synthetic stand-in for the reference's intcount_data: `nbytes` of
    uniform random little-endian int32 keys in [0, key_range) (uint8 view)."""
    g = torch.Generator().manual_seed(seed * 1000003 + rank)
    n = nbytes // 4
    return torch.randint(0, key_range, (n,), generator=g, dtype=torch.int32).view(torch.uint8)


class IntCount:
    def __init__(self, mr: MapReduce, data: torch.Tensor, reduce=True):
        """data: this rank's raw int file (uint8 tensor, host pinned or device)."""
        self.mr = mr
        self.data = data
        self.do_reduce = reduce

    def _map(self, itask, kv):
        # the reference emits one pair per 4-byte int (cpu/IntCount.cpp:179-180)
        keys = self.data.to(self.mr.device, non_blocking=True).view(torch.int32)
        ones = torch.ones(keys.numel(), dtype=torch.int32, device=keys.device)
        kv.add_tensors(keys, ones)

    def run(self, phases=None):
        mr = self.mr
        sync = (lambda: torch.cuda.synchronize()) if mr.device.startswith("cuda") else (lambda: None)
        t = [time.perf_counter()]

        def mark():
            if phases is not None:
                sync()
                t.append(time.perf_counter())
        # mapstyle 0 with nmap = nprocs: task i runs on rank i, like the reference
        self.nkv = mr.map(mr.nprocs, self._map)
        mark()
        mr.aggregate()
        mark()
        self.nunique = mr.convert()
        mark()
        if self.do_reduce:
            mr.reduce("count")
        mark()
        if phases is not None:
            for name, a, b in zip(("Map", "Network I/O", "Sort/Hash", "Reduce"), t, t[1:]):
                phases[name] = b - a
        return self.nkv

    def counts(self):
        """(keys int32, counts int32) of this rank's reduced KV (host tensors)."""
        kv = self.mr.kv
        return kv.kdata.view(torch.int32).cpu(), kv.vdata.view(torch.int32).cpu()


def reference_counts(datas) -> dict:
    a = np.concatenate([d.cpu().numpy().view(np.int32) for d in datas])
    k, c = np.unique(a, return_counts=True)
    return dict(zip(k.tolist(), c.tolist()))


def bench_intcount(comm, args):
    per_gpu = int(args.intcount_bytes)
    data = int_file(per_gpu, args.key_range, args.seed, comm.rank)
    if comm.is_cuda:
        data = data.pin_memory()

    def step():
        app = IntCount(MapReduce(comm), data)
        app.run()
        return app

    for _ in range(args.warmup):
        step()
    if comm.is_cuda:
        torch.cuda.synchronize()
    comm.barrier()
    if comm.is_cuda:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        app = step()
    if comm.is_cuda:
        torch.cuda.synchronize()
    comm.barrier()
    if comm.is_cuda:
        torch.cuda.synchronize()
    dt = comm.allreduce((time.perf_counter() - t0) / args.steps, "max", dtype=torch.float64)
    phases = {}
    if args.phases:
        IntCount(MapReduce(comm), data).run(phases)
        phases = {k: round(v * 1e3, 3) for k, v in phases.items()}
    value = app.nkv / dt
    return {
        "metric": "KV-pairs/sec (whole node), IntCount (map -> aggregate -> convert -> reduce count)",
        "value": value,
        "unit": "KV/s",
        "ms_per_step": dt * 1e3,
        "vs_baseline": value / (REF_KVPS_PER_GPU * comm.size),
        "baseline_note": "GPMR IntegerCount, 32M ints/GPU: 162M KV/s on 20x GK104 = 8.1M KV/s per GPU "
                         "(BASELINE.md); vs_baseline = our KV/s / (8.1M x n_gpus)",
        "kv_pairs_per_step": app.nkv,
        "unique_keys": app.nunique,
        "stage_ms": phases,
        "config": {"model": "IntCount", "global_batch": app.nkv, "seq_len": 1,
                   "parallelism": f"dp{comm.size}", "bytes_per_gpu": per_gpu, "key_range": args.key_range},
    }
