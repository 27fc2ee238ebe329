#!/usr/bin/env python3
"""Headline benchmark: KV-pairs/sec (whole node) of InvertedIndex on MI355X.

BASELINE.json metric: "KV-pairs/sec (whole node) for InvertedIndex +
RMAT-2^26 PageRank at 1/2/4/8 MI355X"; config "InvertedIndex on 1 GB
synthetic docs, 1xMI355X (map + local sort/reduce)" — weak scaling: every
GPU owns 1 GiB of synthetic Wikipedia-like HTML in eight 128 MiB part files
(the reference's part-file shape, cuda/InvertedIndex.cu:282).

One step = the whole job, end to end, as the reference times it
(cuda/InvertedIndex.cu:170-205): stream the part files host(pinned)->HBM,
map (find `<a href="`, emit URL->file KVs), aggregate (RCCL all-to-all when
N>1), convert (group by URL), reduce (format "url\\tfile ...\\n" lines on the
GPU and copy the text back to host memory). Nothing is cached across steps.

value = total URL KV pairs processed by all ranks / seconds per step.
The reference publishes no KV/s; its end-to-end input throughput is
0.85 GB/s aggregate on 20 GK104 GPUs (50 GB in 59.0 s), so
`vs_baseline` compares our aggregate input GB/s with that number.

The same invocation also runs the BASELINE headline's second workload,
PageRank on RMAT-2^26 (edge factor 16, 20 iterations, strong scaling: the
same graph for every N), and reports it in extra keys: pagerank_kvps (edge
contributions per second over the timed iterations), pagerank_ms (one
20-iteration run), pagerank_setup_ms (R-MAT generation + aggregate to the
source owner + plan build) and pagerank_kvps_incl_setup.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload invertedindex|pagerank|wordfreq|trifind|intcount]
    torchrun --nproc-per-node N bench.py --gpus N ...

`--gpus N` without torchrun spawns the N ranks itself (one process per GPU,
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set per
child, before anything touches the GPU), like the reference's one MPI rank
per GPU (cuda/InvertedIndex.cu:142-145, cuda/nodefile).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

REF_GBPS = 50.0 * 1e9 / 59.0 / 1e9  # reference end-to-end InvertedIndex, 50 GB in 59.0 s (decimal GB)


def _quiesce():
    """Before a timed loop: collect once and freeze the survivors (gc.freeze),
    so a generation-2 collection inside the loop does not walk the ~10^5
    objects of torch and the engine bindings — a 10 ms pause in one 21 ms
    step otherwise (the allocation pattern of the loop is unchanged)."""
    import gc
    gc.collect()
    gc.freeze()


def _sync(comm):
    if comm.is_cuda:
        torch.cuda.synchronize()
    comm.barrier()
    if comm.is_cuda:
        torch.cuda.synchronize()


def bench_inverted_index(comm, args):
    from gpu_mapreduce_amd import MapReduce
    from gpu_mapreduce_amd.models.inverted_index import InvertedIndex
    from gpu_mapreduce_amd.utils import synth

    per_gpu = int(args.bytes_per_gpu)
    gen_dev = comm.device
    files = synth.html_corpus(per_gpu, file_bytes=args.file_bytes, seed=args.seed, rank=comm.rank, device=gen_dev,
                              link_gap=args.link_gap)
    if comm.is_cuda:
        files = [(n, t.cpu().pin_memory()) for n, t in files]
    in_bytes = sum(t.numel() for _, t in files)

    def step(prefetch_next=None):
        mr = MapReduce(comm)
        app = InvertedIndex(mr, files, prefetch_next=prefetch_next)
        n = app.run()
        return n, app

    def steps(k, pipelined):
        """k back-to-back jobs; pipelined: job s copies job s+1's first part
        file behind its own last one (input prefetch, like a serving loop or a
        data loader) — never the last job, so nothing of a later job starts
        before this window ends and nothing of this window's jobs ran before it"""
        nurl, app, ms = 0, None, []
        for s in range(k):
            del app
            ts = time.perf_counter()
            nurl, app = step(files if (pipelined and s < k - 1) else None)
            ms.append(round((time.perf_counter() - ts) * 1e3, 3))
        return nurl, app, ms

    steps(args.warmup, True)
    _quiesce()
    _sync(comm)
    t0 = time.perf_counter()
    nurl, app, step_ms = steps(args.steps, True)
    _sync(comm)
    dt = (time.perf_counter() - t0) / args.steps
    dt = comm.allreduce(dt, "max", dtype=torch.float64)
    # the same jobs strictly one after another (no cross-job prefetch), for reference
    _sync(comm)
    t1 = time.perf_counter()
    steps(args.steps, False)
    _sync(comm)
    dt_serial = comm.allreduce((time.perf_counter() - t1) / args.steps, "max", dtype=torch.float64)
    total_in = comm.allreduce(in_bytes, "sum")
    phases = {}
    if args.phases:  # separate, device-synced run for the stage breakdown (not the timed steps)
        mr = MapReduce(comm)
        InvertedIndex(mr, files).run(phases)
        phases = {k: round(v * 1e3, 3) for k, v in phases.items()}
    value = nurl / dt
    gbps = total_in / dt / 1e9
    return {
        "metric": "KV-pairs/sec (whole node), InvertedIndex end-to-end",
        "value": value,
        "unit": "KV/s",
        "ms_per_step": dt * 1e3,
        "vs_baseline": gbps / REF_GBPS,
        "baseline_note": "reference publishes no KV/s; vs_baseline = aggregate input GB/s "
                         f"({gbps:.2f}) / reference end-to-end 0.847 GB/s (50 GB in 59 s on 20x GK104)",
        "input_GBps": gbps,
        "timed_step": "host(pinned)->HBM part files, map, aggregate (RCCL when N>1), convert, reduce; the reduce "
                      "formats url\\tfile lines on the GPU into pinned host memory (not written to a file). Jobs run "
                      "as a pipeline: job s copies job s+1's first part file behind its own last one (the link does "
                      "not idle during job s's tail); the last timed job prefetches nothing and the first timed job "
                      "copies all its files inside the window",
        "ms_per_step_no_prefetch": dt_serial * 1e3,
        "kv_pairs_per_step": nurl,
        "unique_urls": app.nunique,
        "stage_ms": phases,
        "step_ms_rank0": step_ms,
        "config": {"model": "InvertedIndex", "global_batch": total_in, "seq_len": args.file_bytes,
                   "parallelism": f"dp{comm.size}", "bytes_per_gpu": per_gpu,
                   "file_bytes": args.file_bytes, "link_gap": args.link_gap},
    }


def bench_inverted_index_files(comm, args):
    """The headline job with its file I/O, like the reference's end-to-end time
    (cuda/InvertedIndex.cu:170-205 freads the part files and the reduce writes
    the index): each step reads this rank's 8 part files from the page cache
    (a RAM-backed directory, parallel reads into pinned buffers), runs the job
    and writes the output text to a file. Part files are written once before
    the timed steps."""
    import shutil
    import tempfile
    from concurrent.futures import ThreadPoolExecutor

    from gpu_mapreduce_amd import MapReduce
    from gpu_mapreduce_amd.models.inverted_index import InvertedIndex
    from gpu_mapreduce_amd.utils import synth
    # a RAM-backed directory with room for the part files and the output (on
    # every rank: one rank without room would leave its peers waiting in the
    # job's collectives, so all ranks agree before any of them starts)
    # the node's ranks share the directory: room for all of them, with a margin
    nloc = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    need = 2 * int(args.bytes_per_gpu) + (256 << 20)
    base = next((d for d in ("/dev/shm", tempfile.gettempdir())
                 if os.path.isdir(d) and shutil.disk_usage(d).free >= nloc * need + (4 << 30)), None)
    root = None
    files_ok = 0
    try:
        if base is not None:
            root = tempfile.mkdtemp(prefix=f"mrh_ii_{comm.rank}_", dir=base)
            files = synth.html_corpus(int(args.bytes_per_gpu), file_bytes=args.file_bytes, seed=args.seed,
                                      rank=comm.rank, device=comm.device, link_gap=args.link_gap)
            paths = []
            for name, t in files:
                pth = os.path.join(root, name)
                t.cpu().numpy().tofile(pth)
                paths.append((name, pth, t.numel()))
            del files
            files_ok = 1
    except OSError as e:
        print(f"bench.py rank {comm.rank}: with_file_io: {e}", file=sys.stderr, flush=True)
    try:
        if comm.allreduce(files_ok, "min") == 0:
            return {"skipped": f"a rank had no directory with {need >> 20} MiB free for the part files"}
        # two sets of pinned read buffers: job s+1's files are read while job s
        # copies and maps its own (a job pipeline, like the headline's)
        bufsets = [[torch.empty(n, dtype=torch.uint8, pin_memory=comm.is_cuda) for _, _, n in paths]
                   for _ in range(2)]
        outdir = os.path.join(root, "out")

        # reads in 32 MiB pieces (os.preadv releases the GIL), spread over
        # this rank's share of the host CPUs
        piece = 32 << 20
        jobs = [(i, o, min(piece, n - o)) for i, (_, _, n) in enumerate(paths) for o in range(0, n, piece)]
        nloc = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
        nthr = max(4, min(16, (os.cpu_count() or 8) // nloc))
        fds = [os.open(pth, os.O_RDONLY) for _, pth, _ in paths]
        views = [[memoryview(b.numpy()) for b in bs] for bs in bufsets]

        def read_piece(job, k=0):
            i, o, n = job
            got = os.preadv(fds[i], [views[k][i][o:o + n]], o)
            if got != n:
                raise OSError(f"short read of {paths[i][1]} at {o}: {got} of {n} bytes")

        pool = ThreadPoolExecutor(max_workers=nthr)

        class _FileRead:  # ready.result() for InvertedIndex: every piece of one file read
            def __init__(self, futs):
                self.futs = futs

            def result(self):
                for f in self.futs:
                    f.result()

        def reads(s):
            """queue job s's reads (file order) into buffer set s % 2"""
            k = s % 2
            futs = [pool.submit(read_piece, j, k) for j in jobs]
            ready = [_FileRead([f for f, j in zip(futs, jobs) if j[0] == i]) for i in range(len(paths))]
            return [(paths[i][0], bufsets[k][i], ready[i]) for i in range(len(paths))]

        do_read = getattr(args, "fileio_read", True)    # probes (tools/ii_fileio_probe.py): drop one side
        do_write = getattr(args, "fileio_write", True)
        if not do_read:
            for k in range(2):
                for i in range(len(paths)):
                    for j in jobs:
                        if j[0] == i:
                            read_piece(j, k)

        def window(k):
            """k jobs back to back: job s's part files are read while job s-1
            runs, job s copies job s+1's first file behind its own last one and
            its index is written by the writer thread during job s+1; the
            window ends when the last job's index is on disk"""
            def get(s):
                if do_read:
                    return reads(s)
                return [(paths[i][0], bufsets[s % 2][i]) for i in range(len(paths))]
            files = get(0)
            apps = []
            for s in range(k):
                nxt = get(s + 1) if s < k - 1 else None
                app = InvertedIndex(MapReduce(comm), files, out_dir=outdir if do_write else None, async_write=True,
                                    prefetch_next=nxt)
                app.run()
                apps.append(app)
                files = nxt
            for app in apps:
                app.wait_written()
            return apps

        window(max(1, args.warmup))
        _sync(comm)
        t0 = time.perf_counter()
        apps = window(args.steps)
        _sync(comm)
        dt = comm.allreduce((time.perf_counter() - t0) / args.steps, "max", dtype=torch.float64)
        write_s = [a.write_s for a in apps]
        out_bytes = [a.output.numel() if a.output is not None else 0 for a in apps]
        wr = comm.allreduce(sum(write_s) / max(1, len(write_s)), "max", dtype=torch.float64)
        # the reads alone (untimed above: they overlap the job)
        t0 = time.perf_counter()
        list(pool.map(read_piece, jobs))
        rd = comm.allreduce(time.perf_counter() - t0, "max", dtype=torch.float64)
        for fd in fds:
            os.close(fd)
        pool.shutdown()
        total_in = comm.allreduce(sum(n for _, _, n in paths), "sum")
        return {"ms_per_step": dt * 1e3, "read_ms": rd * 1e3, "read_threads": nthr,
                "write_ms": wr * 1e3, "output_bytes": out_bytes[-1] if out_bytes else 0, "input_GBps": total_in / dt / 1e9,
                "vs_reference_end_to_end": total_in / dt / 1e9 / REF_GBPS,
                "note": "part files read from the page cache (RAM-backed directory) into pinned memory (32 MiB pieces "
                        "over read_threads threads; job s+1's files are read while job s copies and maps its own; "
                        "read_ms: the reads alone), the index text written to a file by a writer thread during the "
                        "next job (write_ms: one write); the window ends when the last index is written; "
                        "steps=%d" % args.steps}
    finally:
        if root is not None:
            shutil.rmtree(root, ignore_errors=True)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n, argv):
    """One child process per rank (this process never touches the GPU);
    returns the first non-zero child exit code, or 0."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                c = p.poll()
                if c is None:
                    continue
                procs.remove(p)
                if c != 0 and rc == 0:
                    rc = c
                    for q in procs:  # a failed rank ends the job (the others fail fast anyway)
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


def _round16(x):
    return (x + 15) // 16 * 16


def bench_pagerank_extra(comm, args):
    """PageRank RMAT-2^scale x iters inside the headline run (extra keys)."""
    from gpu_mapreduce_amd import MapReduce
    from gpu_mapreduce_amd.models.pagerank import PageRank, rmat_map
    scale, ef, iters = args.pagerank_scale, args.edgefactor, args.iters

    def setup_once():
        """R-MAT generation (map) + aggregate to the owners + plan build, timed"""
        _sync(comm)
        t0 = time.perf_counter()
        mr = MapReduce(comm)
        rmat_map(mr, scale, ef, seed=args.seed)
        p = PageRank(mr, 1 << scale).build()
        del mr
        _sync(comm)
        return p, comm.allreduce(time.perf_counter() - t0, "max", dtype=torch.float64)
    # the first setup of the process is the warm-up (cold: the pool grows by
    # the graph's ~30 GB, kernels load) and is reported as
    # pagerank_setup_cold_ms; the record's pagerank_setup_ms is the second,
    # like every timed step of this file follows its warm-up steps
    pr, setup_cold = setup_once()
    del pr
    pr, setup = setup_once()
    nedge = comm.allreduce(pr.nedge, "sum")
    for _ in range(max(1, args.pagerank_warmup)):
        pr.reset()
        pr.run(iters)
    _quiesce()
    _sync(comm)
    t0 = time.perf_counter()
    for _ in range(args.pagerank_steps):
        pr.reset()
        pr.run(iters)
    _sync(comm)
    dt = comm.allreduce((time.perf_counter() - t0) / args.pagerank_steps, "max", dtype=torch.float64)
    out = {
        "pagerank_kvps": nedge * iters / dt,
        "pagerank_ms": dt * 1e3,
        "pagerank_setup_ms": setup * 1e3,
        "pagerank_setup_cold_ms": setup_cold * 1e3,
        "pagerank_kvps_incl_setup": nedge * iters / (dt + setup),
        "pagerank_hip_graph_iterations": pr.graph_iterations,
        "pagerank_layout": pr.layout,
        "pagerank_comm_bytes_per_iter": comm.allreduce(pr.comm_bytes_per_iter, "max"),
        "pagerank_comm_overlapped": bool(pr.overlapped),
        # what the replicated plan moves per rank and iteration at P = 8: the
        # other 7 ranks' c slices (active sources / 8, 64-byte aligned), fp32
        "pagerank_comm_bytes_per_iter_p8_predicted": 7 * 4 * _round16(-(-((1 << scale) - pr.ndangling) // 8)) + 16,
        "pagerank_config": {"graph": f"RMAT-2^{scale}", "edgefactor": ef, "edges": nedge, "iters": iters,
                            "runs_timed": args.pagerank_steps, "alpha": 0.85, "scaling": "strong",
                            "rank_dtype": "fp32 ranks, fp64 L1/dangling reductions"},
    }
    # the pool keeps its caches (it releases them itself when the device fills
    # up): trimming 45 GB here and regrowing made the next job 7 ms slower per
    # step (with_file_io 21.3 -> 28.5 ms, the same with the ATen allocator)
    del pr
    return out


def _extra(comm, prefix, fn, args, **over):
    """Run another BASELINE workload inside the headline invocation and report
    it under prefixed keys; a failure is recorded, not fatal (the failing
    rank's native op poisons the job, so its peers fail fast too)."""
    import copy
    a = copy.copy(args)
    for k, v in over.items():
        setattr(a, k, v)
    try:
        r = fn(comm, a)
    except Exception as e:  # noqa: BLE001
        print(f"bench.py rank {comm.rank}: {prefix} extra failed: {e}", file=sys.stderr, flush=True)
        return {f"{prefix}_error": f"{type(e).__name__}: {e}"[:500]}
    out = {f"{prefix}_kvps": r["value"], f"{prefix}_ms": r["ms_per_step"], f"{prefix}_setup_ms": r.get("setup_ms"),
           f"{prefix}_config": dict(r["config"], steps=a.steps, warmup=a.warmup, scaling=r.get("scaling", "weak"),
                                    metric=r["metric"])}
    for k in ("triangles", "unique_edges", "words", "unique_words", "input_GBps", "hub_vertices", "build",
              "triangles_check", "stages", "wedge_pairs", "ooc", "ms_per_step_prefetch", "pairs",
              "pairs_per_s_by_stage", "top10", "top10_equals_combiner", "big", "compact_vb", "route", "cfg5"):
        if k in r:
            out[f"{prefix}_{k}"] = r[k]
    return out


def bench_wordfreq_files(comm, args):
    """wordfreq with its file reads (the reference maps files,
    examples/wordfreq.cpp:64, 104-130): this rank's text as 128 MiB part files
    in the page cache (a RAM-backed directory), streamed by a RingReader into
    8 pinned buffers while the job copies and counts the earlier ones; the
    next job's reads queue behind this job's. Part files are written once
    before the timed steps (same synthetic text as the wordfreq extra)."""
    import shutil
    import tempfile

    from gpu_mapreduce_amd import MapReduce
    from gpu_mapreduce_amd.models.wordfreq import WordFreq
    from gpu_mapreduce_amd.utils import synth
    from gpu_mapreduce_amd.utils.fileio import RingReader
    per_gpu = int(args.wordfreq_bytes)
    chunk = min(int(args.file_bytes), per_gpu)
    nloc = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))  # ranks of this node share the directory
    base = next((d for d in ("/dev/shm", tempfile.gettempdir())
                 if os.path.isdir(d) and shutil.disk_usage(d).free >= nloc * (per_gpu + (1 << 30)) + (4 << 30)),
                None)
    if comm.allreduce(0 if base is None else 1, "min") == 0:
        return {"skipped": f"a rank had no directory with room for its node's part files "
                           f"({nloc} x {(per_gpu >> 20) + 1024} MiB + 4 GiB)"}
    root = tempfile.mkdtemp(prefix=f"mrh_wf_{comm.rank}_", dir=base)
    reader = None
    try:
        paths, left, i = [], per_gpu, 0
        while left > 0:
            n = min(chunk, left)
            t = synth.zipf_text(n, seed=args.seed * 7919 + comm.rank * 1000 + i, device=comm.device)
            pth = os.path.join(root, f"part-{i:05d}")
            t.cpu().numpy().tofile(pth)
            paths.append((pth, n))
            left -= n
            i += 1
        del t
        nloc = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
        nthr = max(4, min(16, (os.cpu_count() or 8) // nloc))
        reader = RingReader(paths, slots=8, threads=nthr, pin=comm.is_cuda)

        def window(k):
            nxt = reader.job()
            app = None
            for s in range(k):
                entries, cb = nxt
                if s < k - 1:
                    nxt = reader.job()  # queued behind this job's reads
                app = WordFreq(MapReduce(comm), entries, on_copied=cb)
                app.run()
            return app

        window(2)
        _sync(comm)
        t0 = time.perf_counter()
        app = window(args.extra_steps)
        _sync(comm)
        dt = comm.allreduce((time.perf_counter() - t0) / args.extra_steps, "max", dtype=torch.float64)
        total = comm.allreduce(per_gpu, "sum")
        return {"ms_per_step": dt * 1e3, "kvps": app.nwords / dt, "input_GBps": total / dt / 1e9,
                "bytes_per_gpu": per_gpu, "part_file_bytes": chunk, "read_threads": nthr, "ring_slots": 8,
                "words": app.nwords,
                "steps": args.extra_steps,
                "note": "part files read from the page cache into a ring of 8 pinned buffers (32 MiB pieces over "
                        "read_threads threads) while the job copies and counts earlier files; the next job's reads "
                        "queue behind; nothing cached between jobs"}
    finally:
        if reader is not None:
            reader.close()
        shutil.rmtree(root, ignore_errors=True)


def _forced_rccl_comm(comm, level="2"):
    """A one-rank communicator on this rank's GPU that runs the native RCCL
    transport (csrc/engine/comm.h): every multi-GPU code path — the
    exchanges, the all-gathers and allreduces of the PageRank and tri_find
    plans — runs through a real RCCL communicator on one GPU. Level 2
    (MRH_FORCE_RCCL=2): the collectives call ncclAllReduce / ncclAllGather /
    ncclBroadcast too (level 1: they are the one-rank identity)."""
    from gpu_mapreduce_amd.parallel.comm import Comm
    prev = os.environ.get("MRH_FORCE_RCCL")
    os.environ["MRH_FORCE_RCCL"] = level
    try:
        c = Comm(group=None, device=comm.device)
        c.__dict__["_force"] = True
        if c.native.transport != "rccl":
            raise RuntimeError(f"forced communicator has transport {c.native.transport}")
    finally:
        if prev is None:
            os.environ.pop("MRH_FORCE_RCCL", None)
        else:
            os.environ["MRH_FORCE_RCCL"] = prev
    return c


def bench_dist_plans(comm, args):
    """One GPU (N=1): PageRank RMAT-26 x20 and tri_find RMAT-24 again through
    the multi-GPU plans on a forced one-rank RCCL communicator (the paths the
    8-GPU BASELINE configs run), reported next to the local-path numbers"""
    from gpu_mapreduce_amd._ext import C
    out = {}
    fc = _forced_rccl_comm(comm)
    c0 = dict(C.rccl_counters())
    try:
        try:
            r = bench_pagerank_extra(fc, args)
            out.update({"pagerank_dist_ms": r["pagerank_ms"], "pagerank_dist_setup_ms": r["pagerank_setup_ms"],
                        "pagerank_dist_layout": r.get("pagerank_layout"),
                        "pagerank_dist_comm_bytes_per_iter": r.get("pagerank_comm_bytes_per_iter")})
        except Exception as e:  # noqa: BLE001
            out["pagerank_dist_error"] = f"{type(e).__name__}: {e}"[:500]
        if args.trifind_scale > 0:
            from gpu_mapreduce_amd.models.triangles import bench_trifind
            r = _extra(fc, "trifind_dist", bench_trifind, args, scale=args.trifind_scale, steps=args.extra_steps,
                       warmup=1)
            out.update({k: v for k, v in r.items() if k in ("trifind_dist_ms", "trifind_dist_triangles",
                                                             "trifind_dist_error", "trifind_dist_build")})
        if args.wordfreq_bytes > 0 and getattr(args, "wordfreq_dist", 1):
            # BASELINE config 3's P > 1 route at full size on one GPU: the
            # (word, NULL) pairs are materialised, hash-partitioned, sent
            # through RCCL (to this rank) and grouped as the rounds land
            from gpu_mapreduce_amd.models.wordfreq import bench_wordfreq
            from gpu_mapreduce_amd.runtime import hbm_pool
            dev = torch.device(comm.device).index or 0
            hbm_pool.reset_peak(dev)
            r = _extra(fc, "wordfreq_shuffle_dist", bench_wordfreq, args, bytes_per_gpu=args.wordfreq_bytes,
                       file_bytes=min(args.file_bytes, int(args.wordfreq_bytes)), steps=args.extra_steps,
                       warmup=1, combiner=False)
            out.update(r)
            out["wordfreq_shuffle_dist_hbm_peak"] = hbm_pool.stats(dev)["peak"]
        c1 = dict(C.rccl_counters())
        out["dist_rccl_calls"] = {k: c1[k] - c0.get(k, 0) for k in c1}
        out["dist_plans_note"] = ("MRH_FORCE_RCCL=2 one-rank RCCL communicator: the PageRank plan of several GPUs "
                                  "(destination-owned edges, source pieces exchanged in side-stream rounds sent to "
                                  "this rank itself, per-iteration stats ncclAllReduce; the iteration replays as a "
                                  "HIP graph that holds those RCCL operations), the tri_find split build (key-range "
                                  "exchange, allreduced degrees, row-range exchange, column all-gather) and "
                                  "wordfreq without the combiner on its P > 1 route; every collective calls its "
                                  "nccl* function (dist_rccl_calls counts them)")
    finally:
        del fc
    return out


def rccl_record(comm):
    """What RCCL itself reports about the job's communicator, from every rank:
    ncclCommCount (must equal N on every rank), ncclCommCuDevice, the GPU's
    PCI bus id (N distinct GPUs must have joined) and how many RCCL
    communicators each process holds (exactly one). At N=1 the engine runs the
    local transport, so a one-rank probe communicator answers instead."""
    from gpu_mapreduce_amd._ext import C
    rec = {"engine_transport": comm.native.transport}
    if not comm.is_cuda:
        return rec
    dev = torch.device(comm.device).index or 0
    if comm.native.transport == "rccl":
        info, probe = comm.rccl_info(), False
    else:
        info, probe = dict(C.rccl_self_probe(dev)), True
        info["live_comms"] = C.live_rccl_comms()
    mine = {"comm_count": info["comm_count"], "cu_device": info["cu_device"], "user_rank": info["user_rank"],
            "live_comms": info["live_comms"], "pci": C.gpu_pci_bus_id(dev)}
    allr = comm.allgather_object(mine)
    rec.update({
        "rccl_comm_count": allr[0]["comm_count"],
        "rccl_cu_devices": [r["cu_device"] for r in allr],
        "rccl_user_ranks": [r["user_rank"] for r in allr],
        "rccl_live_comms_per_rank": [r["live_comms"] for r in allr],
        "gpu_pci_bus_ids": [r["pci"] for r in allr],
    })
    if probe:
        rec["rccl_note"] = "engine transport is not RCCL at this N (local/pg); counts from a one-rank probe communicator"
        return rec
    bad = []
    if any(r["comm_count"] != comm.size for r in allr):
        bad.append(f"ncclCommCount {[r['comm_count'] for r in allr]} != {comm.size}")
    if sorted(r["user_rank"] for r in allr) != list(range(comm.size)):
        bad.append(f"ncclCommUserRank {[r['user_rank'] for r in allr]}")
    if len(set(r["pci"] for r in allr)) != comm.size:
        bad.append(f"{len(set(r['pci'] for r in allr))} distinct GPUs for {comm.size} ranks")
    if any(r["live_comms"] != 1 for r in allr):
        bad.append(f"RCCL communicators per process {[r['live_comms'] for r in allr]} (expected 1)")
    # a failed check is reported in the record (and on stderr), not fatal: the
    # headline line of an otherwise complete run must not be lost to it
    rec["rccl_check"] = "ok" if not bad else "FAILED: " + "; ".join(bad)
    if bad and comm.rank == 0:
        print("bench.py: RCCL communicator check failed: " + "; ".join(bad), file=sys.stderr, flush=True)
    return rec


def trifind_mr_big_scale_for(n_gpus, hbm_bytes=288e9):
    """R-MAT scale of the big in-HBM tri_find_mr run at N GPUs (strong
    scaling): the largest scale <= 24 (BASELINE config 5: tri_find on RMAT-24
    over 8 GPUs) whose estimated per-GPU peak fits 65 % of one GPU's HBM.
    Wedge pairs grow ~5.9x per two scales (RMAT-20: 1.23 G, RMAT-22: 7.27 G,
    measured); the pipeline peaks at ~25 bytes per pair on one GPU (RMAT-22:
    ~180 GB). N = 1, 2 -> 22; N = 4 -> 23; N = 8 -> 24 (the config-5 graph,
    ~5.4 G pairs per GPU)."""
    best = 20
    for sc in range(20, 25):
        pairs = 1.23e9 * (7.27 / 1.23) ** ((sc - 20) / 2)
        if 25.0 * pairs / max(1, n_gpus) <= 0.65 * hbm_bytes:
            best = sc
    return best


def _r(x, nd=2):
    return None if x is None else round(float(x), nd)


def compact_record(res):
    """The driver-visible subset of the record: one number per BASELINE
    config and extra workload, with its correctness check; no stage arrays.
    (The full record, stage by stage, is written to --detail-out.)"""
    out = {}

    def put(key, src=None, nd=2):
        v = res.get(src or key)
        if v is not None and not isinstance(v, (dict, list)):
            out[key] = _r(v, nd) if isinstance(v, float) else v
    for k in ("ms_per_step_no_prefetch", "input_GBps", "kv_pairs_per_step", "unique_urls",
              "pagerank_ms", "pagerank_setup_ms", "pagerank_setup_cold_ms", "pagerank_hip_graph_iterations",
              "pagerank_dist_ms", "pagerank_dist_setup_ms",
              "trifind_ms", "trifind_triangles", "trifind_build", "trifind_dist_ms", "trifind_dist_triangles",
              "wordfreq_ms", "wordfreq_input_GBps", "wordfreq_words", "wordfreq_1gib_ms",
              "wordfreq_shuffle_ms", "wordfreq_shuffle_top10_equals_combiner",
              "wordfreq_shuffle_dist_ms", "wordfreq_shuffle_dist_hbm_peak", "wordfreq_shuffle_dist_top10_equals_combiner",
              "wordfreq_shuffle_dist_route",
              "trifind_mr_ms", "trifind_mr_triangles", "trifind_mr_triangles_check"):
        put(k)
    if "pagerank_kvps" in res:
        out["pagerank_Gedges_per_s"] = _r(res["pagerank_kvps"] / 1e9)
    if "stage_ms" in res and isinstance(res["stage_ms"], dict):
        out["ii_stage_ms"] = {k: _r(v) for k, v in res["stage_ms"].items()}
    for src, dst in (("with_file_io", "with_file_io_ms"), ("wordfreq_with_file_io", "wordfreq_with_file_io_ms")):
        v = res.get(src)
        if isinstance(v, dict):
            out[dst] = _r(v["ms_per_step"]) if "ms_per_step" in v else str(v.get("error") or v.get("skipped"))[:120]
    for tag, key in (("big", "trifind_mr_big"), ("ooc", "trifind_mr_ooc"), ("cfg5", "trifind_mr_cfg5")):
        v = res.get(f"trifind_mr_{tag}")
        if isinstance(v, dict):
            out[f"{key}_scale"] = v.get("scale")
            out[f"{key}_ms"] = _r(v.get("ms"))
            if "ms_cold" in v:
                out[f"{key}_ms_cold"] = _r(v["ms_cold"])
            out[f"{key}_triangles_ok"] = v.get("triangles") == v.get("triangles_check")
            for st in v.get("stages", []):
                if st.get("op") == "collate 4" and "x_floor" in st:
                    out[f"{key}_collate4_ms"] = st["ms"]
                    out[f"{key}_collate4_x_floor"] = st["x_floor"]
            if "spool_disk_bytes" in v:
                out[f"{key}_disk_bytes"] = v["spool_disk_bytes"]
    hp = res.get("host_pin_reserve")
    if isinstance(hp, dict) and hp.get("mib"):
        out["host_pin_reserve_ms"] = hp["ms"]  # the start-up pinning of the out-of-core host tier's reserve
    for k in ("pagerank_error", "pagerank_dist_error", "trifind_error", "trifind_dist_error", "wordfreq_error",
              "wordfreq_shuffle_error", "wordfreq_shuffle_dist_error", "trifind_mr_error"):
        if k in res:
            out[k] = str(res[k])[:200]
    for k in ("engine_transport", "rccl_comm_count", "rccl_check", "rccl_calls", "hbm_pool_peak_bytes",
              "hbm_pool_reserved_peak_bytes", "ranks_joined"):
        if k in res:
            out[k] = res[k]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="invertedindex", choices=["invertedindex", "pagerank", "wordfreq", "trifind", "intcount", "kmeans"])
    ap.add_argument("--bytes-per-gpu", type=float, default=float(1 << 30))
    ap.add_argument("--file-bytes", type=int, default=128 << 20)
    ap.add_argument("--link-gap", type=int, default=200)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--phases", type=int, default=1, help="also report a per-stage breakdown (extra run)")
    ap.add_argument("--scale", type=int, default=None, help="RMAT scale (pagerank 26, trifind 24)")
    ap.add_argument("--edgefactor", type=int, default=16, help="RMAT edges per vertex")
    ap.add_argument("--intcount-bytes", type=int, default=128 << 20, help="intcount: raw int32 bytes per GPU")
    ap.add_argument("--key-range", type=int, default=1 << 24, help="intcount: keys uniform in [0, key_range)")
    ap.add_argument("--iters", type=int, default=20, help="pagerank / kmeans iterations per step")
    ap.add_argument("--kmeans-points", type=int, default=32 << 20, help="kmeans: points per GPU")
    ap.add_argument("--kmeans-dim", type=int, default=2)
    ap.add_argument("--kmeans-k", type=int, default=32)
    ap.add_argument("--pagerank-scale", type=int, default=None,
                    help="RMAT scale of the PageRank extra (26 on GPU, 14 on CPU; 0 = skip)")
    ap.add_argument("--pagerank-steps", type=int, default=3, help="timed 20-iteration PageRank runs")
    ap.add_argument("--pagerank-warmup", type=int, default=1)
    ap.add_argument("--trifind-scale", type=int, default=None,
                    help="RMAT scale of the tri_find extra (BASELINE config 5: 24 on GPU, 12 on CPU; 0 = skip)")
    ap.add_argument("--trifind-mr-scale", type=int, default=None,
                    help="RMAT scale of the tri_find_mr extra (the 4-collate MapReduce pipeline: 20 on GPU, 10 on "
                         "CPU; 0 = skip)")
    ap.add_argument("--trifind-mr-big-scale", type=int, default=None,
                    help="RMAT scale of a second, larger tri_find_mr run in HBM (22 on GPU: ~7 G wedge pairs as "
                         "12-byte compact pairs; 0 = skip)")
    ap.add_argument("--trifind-mr-ooc-scale", type=int, default=None,
                    help="RMAT scale of its out-of-core run under a 256 MiB HBM budget (18 on GPU, 0 on CPU)")
    ap.add_argument("--wordfreq-bytes", type=float, default=None,
                    help="text bytes per GPU of the wordfreq extra (BASELINE config 3: 64 GB over 8 GPUs = 8 GiB "
                         "per GPU, the default on GPU; 4e6 on CPU; 0 = skip)")
    ap.add_argument("--extra-steps", type=int, default=3, help="timed steps of the tri_find / wordfreq extras")
    ap.add_argument("--dist-extras", type=int, default=1,
                    help="N=1: also time PageRank / tri_find through the multi-GPU plans on a forced one-rank RCCL "
                         "communicator (pagerank_dist_* / trifind_dist_* keys)")
    ap.add_argument("--file-io-steps", type=int, default=8,
                    help="timed steps of the headline job with part-file reads and output write (0 = skip)")
    ap.add_argument("--detail-out", default="gpurun_out/bench_detail.json",
                    help="rank 0 writes the full record (stage arrays, notes) here; '' = don't")
    args = ap.parse_args()
    if args.scale is None:
        args.scale = 24 if args.workload == "trifind" else 26

    ws_env = os.environ.get("WORLD_SIZE")
    if ws_env is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    if ws_env is not None and int(ws_env) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws_env}", file=sys.stderr)
        sys.exit(2)

    from gpu_mapreduce_amd.parallel import comm as pcomm
    comm = pcomm.init()
    if comm.size != args.gpus:
        raise SystemExit(f"bench.py: {comm.size} ranks joined, expected {args.gpus}")
    # the out-of-core host tier's pinned arena (gpu_mapreduce_amd/hostpin.py),
    # pinned at start-up like the HBM pool: outside every timed region
    from gpu_mapreduce_amd import hostpin
    pin_mb = int(os.environ.get("MRH_PIN_RESERVE_MB", "8192"))
    pin_ms = hostpin.prepin(pin_mb) if comm.is_cuda else 0.0
    if args.pagerank_scale is None:
        args.pagerank_scale = 26 if comm.is_cuda else 14
    if args.trifind_scale is None:
        args.trifind_scale = 24 if comm.is_cuda else 12
    if args.trifind_mr_scale is None:
        args.trifind_mr_scale = 20 if comm.is_cuda else 10
    if args.trifind_mr_ooc_scale is None:
        args.trifind_mr_ooc_scale = 18 if comm.is_cuda else 0
    if args.trifind_mr_big_scale is None:
        args.trifind_mr_big_scale = trifind_mr_big_scale_for(comm.size) if comm.is_cuda else 0
    if args.wordfreq_bytes is None:
        args.wordfreq_bytes = float(8 << 30) if comm.is_cuda else 4e6
    if args.workload == "invertedindex":
        res = bench_inverted_index(comm, args)
    elif args.workload == "pagerank":
        from gpu_mapreduce_amd.models.pagerank import bench_pagerank
        res = bench_pagerank(comm, args)
    elif args.workload == "intcount":
        from gpu_mapreduce_amd.models.intcount import bench_intcount
        res = bench_intcount(comm, args)
    elif args.workload == "trifind":
        from gpu_mapreduce_amd.models.triangles import bench_trifind
        res = bench_trifind(comm, args)
    elif args.workload == "kmeans":
        from gpu_mapreduce_amd.models.kmeans import bench_kmeans
        res = bench_kmeans(comm, args)
    else:
        from gpu_mapreduce_amd.models.wordfreq import bench_wordfreq
        res = bench_wordfreq(comm, args)
    # before the extras: a failing extra poisons (aborts) the communicator
    rrec = rccl_record(comm)
    peaks = {}

    def mark(part):
        """hi-water of pool bytes in use during `part`, then a fresh mark"""
        from gpu_mapreduce_amd.runtime import hbm_pool
        if hbm_pool.installed() and comm.is_cuda:
            dev = torch.device(comm.device).index or 0
            peaks[part] = hbm_pool.stats(dev)["peak"]
            hbm_pool.reset_peak(dev)
    mark(args.workload)
    if args.workload == "invertedindex" and args.pagerank_scale > 0:
        # the headline line is printed even if the PageRank extra fails (its
        # peers fail fast through the engine's peer monitor); the error is
        # reported in the record instead of the PageRank keys
        try:
            res.update(bench_pagerank_extra(comm, args))
        except Exception as e:  # noqa: BLE001
            res["pagerank_error"] = f"{type(e).__name__}: {e}"[:500]
            print(f"bench.py rank {comm.rank}: PageRank extra failed: {e}", file=sys.stderr, flush=True)
        mark("pagerank")
    if args.workload == "invertedindex" and args.file_io_steps > 0:
        # the headline job again with its file reads and output write (the
        # reference's end-to-end scope), failure-isolated
        try:
            import copy
            a = copy.copy(args)
            a.steps, a.warmup = args.file_io_steps, 1
            res["with_file_io"] = bench_inverted_index_files(comm, a)
        except Exception as e:  # noqa: BLE001
            res["with_file_io"] = {"error": f"{type(e).__name__}: {e}"[:500]}
        mark("with_file_io")
    if args.workload == "invertedindex":
        # BASELINE configs 5 and 3 in the same driver-measured record
        if args.trifind_scale > 0:
            from gpu_mapreduce_amd.models.triangles import bench_trifind
            res.update(_extra(comm, "trifind", bench_trifind, args, scale=args.trifind_scale,
                              steps=args.extra_steps, warmup=1))
            mark("trifind")
        if args.wordfreq_bytes > 0:
            from gpu_mapreduce_amd.models.wordfreq import bench_wordfreq
            res.update(_extra(comm, "wordfreq", bench_wordfreq, args, bytes_per_gpu=args.wordfreq_bytes,
                              file_bytes=min(args.file_bytes, int(args.wordfreq_bytes)),
                              steps=args.extra_steps, warmup=6))  # steady state after ~6 jobs:
            # warmup 1 / 2 / 6 -> 27.1 / 24.7 / 22.8 ms (profiles/r3_wordfreq_input.txt)
            mark("wordfreq")
            # BASELINE config 3 as the reference runs it: one (word, NULL) pair
            # per occurrence through the shuffle (no in-mapper combiner;
            # examples/wordfreq.cpp:64-67, 104-130; oink/wordfreq.cpp:40-90)
            res.update(_extra(comm, "wordfreq_shuffle", bench_wordfreq, args, bytes_per_gpu=args.wordfreq_bytes,
                              file_bytes=min(args.file_bytes, int(args.wordfreq_bytes)), steps=args.extra_steps,
                              warmup=2, combiner=False))
            mark("wordfreq_shuffle")
            if comm.is_cuda and args.wordfreq_bytes > (1 << 30):
                # the round-3 shape too (1 GiB per GPU), for comparison with earlier records
                r1 = _extra(comm, "wordfreq_1gib", bench_wordfreq, args, bytes_per_gpu=float(1 << 30),
                            file_bytes=args.file_bytes, steps=args.extra_steps, warmup=6)
                res.update({k: v for k, v in r1.items() if k in ("wordfreq_1gib_ms", "wordfreq_1gib_kvps",
                                                                   "wordfreq_1gib_error", "wordfreq_1gib_input_GBps",
                                                                   "wordfreq_1gib_ms_per_step_prefetch")})
        if args.wordfreq_bytes > 0 and args.file_io_steps > 0:
            try:
                res["wordfreq_with_file_io"] = bench_wordfreq_files(comm, args)
            except Exception as e:  # noqa: BLE001
                res["wordfreq_with_file_io"] = {"error": f"{type(e).__name__}: {e}"[:500]}
            mark("wordfreq_with_file_io")
        if comm.size == 1 and comm.is_cuda and args.dist_extras:
            res.update(bench_dist_plans(comm, args))
            mark("dist_extras")
        # last: the generic-engine pipeline holds ~120 GB at its peak, and a
        # job run on device memory handed back after such a peak was measured
        # slower (PageRank gathers 125 -> 135 ms)
        if args.trifind_mr_scale > 0:
            from gpu_mapreduce_amd.models.triangles import bench_trifind_mr
            r = _extra(comm, "trifind_mr", bench_trifind_mr, args, scale=args.trifind_mr_scale, steps=1, warmup=1,
                       mr_ooc_scale=args.trifind_mr_ooc_scale, mr_big_scale=args.trifind_mr_big_scale)
            res.update(r)
            mark("trifind_mr")

    res.update(rrec)
    res["ranks_joined"] = comm.size
    from gpu_mapreduce_amd.runtime import hbm_pool
    res["host_pin_reserve"] = {"mib": pin_mb if comm.is_cuda else 0, "ms": round(pin_ms, 1),
                               **(hostpin.stats() if comm.is_cuda else {})}
    res["device_allocator"] = "mrhip HBM page pool (csrc/engine/hbmpool.cpp)" if hbm_pool.installed() else "ATen caching allocator"
    if hbm_pool.installed() and comm.is_cuda:
        st = hbm_pool.stats(torch.device(comm.device).index or 0)
        res["hbm_pool_peak_bytes"] = max([st["peak"], *peaks.values()])  # hi-water of bytes in use
        res["hbm_pool_reserved_peak_bytes"] = st["reserved_peak"]  # hi-water of bytes held from the driver
        res["hbm_pool_cross_stream_reuse"] = st["cross_stream_reuse"]
        res["hbm_pool_peak_bytes_by_part"] = peaks  # the hi-water of each workload of the record
    res["backend"] = {"torch.distributed": (comm.backend or "none (world size 1)") + " (host objects/scalars only)",
                      "engine_transport": rrec["engine_transport"]}
    from gpu_mapreduce_amd._ext import C
    if comm.is_cuda:
        res["rccl_calls"] = dict(C.rccl_counters())
    out = {
        "metric": res["metric"], "value": res["value"], "unit": res["unit"], "n_gpus": comm.size,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": res["ms_per_step"],
        "higher_is_better": True, "scaling": res.get("scaling", "weak"), "vs_baseline": res.get("vs_baseline"),
        "dtype": res.get("dtype", "bytes+int32 (no float compute in MapReduce)"), "data": "synthetic",
        "config": res["config"],
    }
    full = dict(out)
    for k, v in res.items():
        if k not in full:
            full[k] = v
    if comm.rank == 0:
        # the whole record (per-stage arrays, notes, configs) goes to a side
        # file; the printed line carries every BASELINE-config number in a few
        # kB so that all of it is inside the driver's stdout tail
        detail = args.detail_out
        if detail:
            try:
                os.makedirs(os.path.dirname(os.path.abspath(detail)), exist_ok=True)
                with open(detail, "w") as f:
                    json.dump(full, f, indent=1)
            except OSError as e:
                print(f"bench.py: could not write {detail}: {e}", file=sys.stderr, flush=True)
        out.update(compact_record(res))
        if detail:
            out["detail_file"] = detail
        print(json.dumps(out, separators=(",", ":")), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
