"""wordfreq: word counts + global top-N (reference examples/wordfreq.cpp:42-97,
oink/wordfreq.cpp:40-90).

Reference pipeline: map(files, strtok words) -> collate -> reduce(count) ->
sort_values(-1) -> local top 10 -> gather(1) -> sort_values(-1) -> print.

MI355X pipeline (same op sequence on device-resident data):
  map       text chunks stream host->HBM (double buffered); with the combiner
            (default) the in-mapper combining kernels (csrc/kernels/
            wordcount.hip) tokenize and count every chunk into a device hash
            table (LDS pre-aggregation, exact byte-compare matching) and the
            map emits KV(word+NUL, int32 count) once per distinct word — the
            pairs map + compress(count) would leave, without materialising a
            KV per occurrence; without it the tokenizer kernel emits
            KV(word+NUL, NULL) per occurrence (the reference's pairs), and on
            one rank the KeyValue groups them chunk by chunk on a device hash
            dictionary while the next chunk is on the PCIe link;
  collate   hashlittle partition + RCCL all-to-all + group-by (as the rounds
            land: the same hash dictionary, csrc/engine/grouper.h);
  reduce    "sum:int32" (or "count" without the combiner) segmented reduce;
  top-N     sort_values(-1) (radix on negated counts) -> slice -> gather(1) ->
            sort_values(-1).
"""
from __future__ import annotations

import struct
import time

import torch

from .._ext import C
from ..runtime import pools
from ..runtime.mapreduce import MapReduce

PAD = 64


class WordFreq:
    def __init__(self, mr: MapReduce, chunks, ntop=10, combiner=True, prefetch_next=None, on_copied=None):
        """chunks: list of uint8 text tensors for this rank (host, ideally
        pinned), or of (tensor, ready) pairs where ready.result() blocks until
        the tensor holds the chunk (a file read in flight: it is waited for
        right before that chunk's copy, so reading chunk i+1 overlaps the copy
        and count of chunk i — the reference's fileread, examples/wordfreq.cpp:
        104-130). on_copied(i, event): called once chunk i's host->HBM copy is
        issued, event completing with it (a streaming reader reuses the host
        buffer after that).

        prefetch_next: the chunks of the job that runs next on this rank (a job
        pipeline): the copy of its first chunk is issued behind this job's
        last one, so the PCIe link does not idle during this job's tail
        (collate, reduce, top-N); the next job finds that copy and does not
        repeat it."""
        self.prefetch_next = prefetch_next
        self.on_copied = on_copied
        self.mr = mr
        self.ready = [c[1] if isinstance(c, (tuple, list)) else None for c in chunks]
        chunks = [c[0] if isinstance(c, (tuple, list)) else c for c in chunks]
        self.chunks = chunks
        self.ntop = ntop
        self.combiner = combiner
        self.is_cuda = mr.device.startswith("cuda")
        maxlen = max((t.numel() for t in chunks), default=0)
        # staging ring depth = the MR's `streams` setting (0 = auto, or
        # MRH_WF_BUFS) — with two buffers the copy of chunk i+2 waits for the
        # count kernel of chunk i; 1 GiB step 29.0 / 24.5 / 25.3 ms with 2 / 3 /
        # 4 buffers on one MI355X (profiles/r2_wordfreq_ring.txt). Without the
        # combiner every chunk's pairs are grouped too, and a copy behind a
        # buffer still read ran at half speed: 8 GiB 197 / 188 / 180 ms with
        # 3 / 4 / 6 buffers (profiles/r5_wordfreq_ring.txt) — 6 there, 3 with
        # the combiner. streams = 1 copies and counts one chunk at a time
        import os
        st = int(mr.streams)
        auto = 3 if combiner else 6
        self.nbuf = st if st > 0 else max(2, int(os.environ.get("MRH_WF_BUFS", str(auto))))
        self.bufs = [pools.device_buffer(mr.device, maxlen + PAD, 8 + s) for s in range(self.nbuf if chunks else 0)]
        # the process's persistent H2D stream (a new stream per job would be
        # a new HIP queue each time)
        self.copy_stream = pools.stream(mr.device, "h2d") if self.is_cuda else None

    def _map(self, itask, kv):
        self.local_words = 0
        if not self.chunks:
            return
        wc = C.WordCounter(self.mr.device) if self.combiner else None
        # no combiner, on a GPU: the pairs are grouped chunk by chunk as the
        # map emits them (the KeyValue's hash dictionary, csrc/engine/
        # grouper.h) in the shadow of the next chunk's H2D copy, so the
        # collate's convert only ranks the groups. With several ranks each
        # chunk's pairs are first hash-partitioned and exchanged (the chunked
        # RCCL aggregate, as InvertedIndex does per part file) and grouped as
        # they land, all under the next chunk's copy; the collate is then a
        # local convert. A forced one-rank RCCL communicator (MRH_FORCE_RCCL=1/2)
        # is "distributed" and takes that route (pairs sent to itself).
        dist = self.mr.comm.native.distributed
        group = wc is None and self.is_cuda
        exchange = group and dist
        self.route = ("combiner" if wc is not None else "exchanged per chunk" if exchange else
                      "grouped in the map" if group else "shuffle")
        self.exchanged = exchange
        if group:
            kv.enable_grouping()
        total = sum(t.numel() for t in self.chunks)
        reserved = [False]
        native = self.mr.comm.native

        def consume(buf, n):
            if wc is not None:
                wc.add(buf, n)
                return
            part = C.map_words(buf, n)
            if exchange:
                part, _ = C.aggregate(part, native, chunk_bytes=self.mr.chunk_bytes)
            if group and not reserved[0] and part.n > 0:
                # arenas for the whole map from the first chunk's density
                # (+15 %); the table is sized from a sample of its words
                reserved[0] = True
                f = 1.15 * total / max(1, n)
                kv.reserve_grouping(int(part.n * f) + 1024, int(part.kdata.numel() * f) + 4096, 0, groups=0)
            kv.add_kv(part)
        if not self.is_cuda:
            for i, t in enumerate(self.chunks):
                if self.ready[i] is not None:
                    self.ready[i].result()
                b = self.bufs[0]
                b[: t.numel()].copy_(t)
                if self.on_copied is not None:
                    self.on_copied(i, None)  # copied synchronously: the host buffer is free
                b[t.numel():t.numel() + PAD].zero_()
                consume(b, t.numel())
        else:
            self._stream_chunks(consume)
        if exchange:
            # lock-step exchanges: a rank with fewer chunks joins with empty parts
            more = int(self.mr.comm.allreduce(len(self.chunks), "max")) - len(self.chunks)
            for _ in range(more):
                consume(torch.zeros(PAD, dtype=torch.uint8, device=self.mr.device), 0)
        if wc is not None:
            self.local_words = wc.words
            kv.add_kv(wc.finish())

    def _stream_chunks(self, consume):
        main = torch.cuda.current_stream()
        cs = self.copy_stream
        nb = self.nbuf
        ready = [torch.cuda.Event() for _ in range(nb)]
        dev = self.mr.device
        n = len(self.chunks)
        # the staging ring continues across jobs (chunk i lands in slot
        # (base + i) % nb), so a job pipeline's prefetch of the next job's
        # first chunk goes to the slot after this job's last one
        base = pools.ring_cursor(dev, "wf") % nb

        def copy_into(b, t, ev):
            with torch.cuda.stream(cs):
                prev = pools.last_use(dev, 8 + b)  # the last kernel (any job) that read this buffer
                if prev is not None:
                    cs.wait_event(prev)
                self.bufs[b][: t.numel()].copy_(t, non_blocking=True)
                ev.record(cs)

        def issue(i):
            b = (base + i) % nb
            ev = pools.take_prefetch(dev, 8 + b, self.chunks[i], self.bufs[b])  # copied by the previous job of a pipeline
            if ev is not None:
                ready[b] = ev
            else:
                if self.ready[i] is not None:
                    self.ready[i].result()  # the chunk's bytes are in its host buffer
                ready[b] = torch.cuda.Event()  # one per copy: a reader may still wait on the previous one
                copy_into(b, self.chunks[i], ready[b])
            if self.on_copied is not None:
                self.on_copied(i, ready[b])

        ahead = max(1, nb - 1)
        for i in range(min(ahead, n)):
            issue(i)
        for i in range(n):
            if nb > 1 and i + ahead < n:
                issue(i + ahead)
            elif nb == 1 and i > 0:
                issue(i)
            if i == n - 1 and nb > 1 and self.prefetch_next:
                first = self.prefetch_next[0]
                # entries as in `chunks`: a tensor or (tensor, ready)
                nxt = first[0] if isinstance(first, (tuple, list)) else first
                if nxt.numel() + PAD <= self.bufs[0].numel():
                    if isinstance(first, (tuple, list)) and len(first) > 1 and first[1] is not None:
                        first[1].result()  # its bytes are read into the host buffer
                    slot = (base + n) % nb
                    ev = torch.cuda.Event()
                    copy_into(slot, nxt, ev)
                    pools.set_prefetch(dev, 8 + slot, nxt, ev, self.bufs[slot])
            b = (base + i) % nb
            main.wait_event(ready[b])
            consume(self.bufs[b], self.chunks[i].numel())
            pools.mark_use(dev, 8 + b, main)
        pools.ring_cursor(dev, "wf", advance=n, n=nb)

    def run(self, phases=None):
        """phases: optional dict; if given, per-stage seconds (device-synced,
        barrier between stages) are added under map / collate / reduce / top_n"""
        from .inverted_index import _Ticker
        mr = self.mr
        tick = _Ticker(phases, mr.comm)
        nkv = mr.map(mr.nprocs, self._map)
        tick("map")
        if self.combiner:
            # pairs are (word, local count): total words = sum of the counts
            self.nwords = int(mr.comm.allreduce(self.local_words, "sum"))
            self.npairs = nkv  # map returns the global pair count
            self.nunique = mr.collate()
            tick("collate")
            mr.reduce("sum:int32")
        else:
            # one (word, NULL) pair per occurrence through the shuffle
            # (reference examples/wordfreq.cpp:64-67, 104-130); exchanged
            # chunk by chunk during the map already: the collate's aggregate
            # is done, its convert remains
            self.nwords = self.npairs = nkv
            self.nunique = mr.convert() if getattr(self, "exchanged", False) else mr.collate()
            tick("collate")
            mr.reduce("count")
        tick("reduce")
        mr.sort_values(-1)
        ntop = self.ntop

        def keep_top(src, kv):
            n = min(ntop, src.n)
            if n == 0:
                return
            koff = src.koff[: n + 1]
            kv.add_tensors(src.kdata[: int(koff[-1].item())], src.vdata[: 4 * n].view(torch.int32), koff=koff)
        mr.map_mr_batch(mr, keep_top)
        mr.gather(1)
        mr.sort_values(-1)
        self.top = [(k.rstrip(b"\0").decode("utf-8", "replace"), struct.unpack("<i", v)[0])
                    for k, v in mr.kv_pairs()][:ntop]
        tick("top_n")
        return self.nwords


def bench_wordfreq(comm, args):
    from ..utils import synth
    per_gpu = int(args.bytes_per_gpu)
    chunk = int(args.file_bytes)
    ts = time.perf_counter()
    chunks = []
    left = per_gpu
    i = 0
    # MRH_WF_INPUT=contig: the input chunks as views of one pinned allocation
    # (default: one pinned allocation per chunk, as a reader of separate files
    # would hold them)
    import os
    contig = comm.is_cuda and os.environ.get("MRH_WF_INPUT", "") == "contig"
    host = torch.empty(per_gpu, dtype=torch.uint8, pin_memory=True) if contig else None
    while left > 0:
        n = min(chunk, left)
        t = synth.zipf_text(n, seed=args.seed * 7919 + comm.rank * 1000 + i, device=comm.device)
        if contig:
            off = per_gpu - left
            host[off:off + n].copy_(t)
            chunks.append(host[off:off + n])
        else:
            chunks.append(t.cpu().pin_memory() if comm.is_cuda else t)
        left -= n
        i += 1
    setup = comm.allreduce(time.perf_counter() - ts, "max", dtype=torch.float64)

    combiner = bool(getattr(args, "combiner", True))

    def steps(k, pipelined):
        """k back-to-back jobs; pipelined: job s copies job s+1's first chunk
        behind its own last one (never the last job of the window)"""
        app = None
        for s in range(k):
            app = WordFreq(MapReduce(comm), chunks, combiner=combiner,
                           prefetch_next=chunks if (pipelined and s < k - 1) else None)
            app.run()
        return app

    def timed(k, pipelined):
        if comm.is_cuda:
            torch.cuda.synchronize()
        comm.barrier()
        t0 = time.perf_counter()
        app = steps(k, pipelined)
        if comm.is_cuda:
            torch.cuda.synchronize()
        comm.barrier()
        return app, comm.allreduce((time.perf_counter() - t0) / k, "max", dtype=torch.float64)

    # the timed number is the strictly serial loop. The cross-job prefetch is
    # reported only: it measured 20.5 ms when timed after the serial window but
    # 25.0 ms when timed first (the serial loop 23.7 first, 22.9 second) — the
    # second window of a process runs faster whichever loop it is, so the
    # prefetch shows no robust gain (profiles/r3_wordfreq_input.txt,
    # r3_wordfreq_prefetch.txt)
    steps(args.warmup, False)
    app, dt = timed(args.steps, False)
    _, dt_pipe = timed(args.steps, True)
    total = comm.allreduce(per_gpu, "sum")
    out = {
        "metric": "KV-pairs/sec (whole node), wordfreq words counted end-to-end",
        "value": app.nwords / dt,
        "unit": "KV/s",
        "ms_per_step": dt * 1e3,
        "ms_per_step_prefetch": dt_pipe * 1e3,
        "timed_step": ("host(pinned)->HBM chunks, in-mapper count, collate, reduce, top-N" if combiner else
                       "host(pinned)->HBM chunks, one (word, NULL) pair per occurrence, collate (hash partition + "
                       "all-to-all when N>1, group-by), reduce(count), sort_values, top-N, gather") +
                      "; jobs strictly one after another (ms_per_step_prefetch: job s copies job s+1's first chunk "
                      "behind its own last one)",
        "vs_baseline": None,
        "baseline_note": "reference publishes no wordfreq number",
        "input_GBps": total / dt / 1e9,
        "words": app.nwords,
        "pairs": app.npairs,
        "unique_words": app.nunique,
        "top3": app.top[:3],
        "route": getattr(app, "route", None),
        "setup_ms": setup * 1e3,
        "config": {"model": "wordfreq" if combiner else "wordfreq (no combiner: a pair per occurrence)",
                   "global_batch": total, "seq_len": chunk, "parallelism": f"dp{comm.size}",
                   "bytes_per_gpu": per_gpu, "combiner": combiner},
    }
    if not combiner:
        # one more job with device-synced stage boundaries (not the timed
        # steps): per-stage times and pair rates, and the combiner's top-10
        # as the check
        ph = {}
        a2 = WordFreq(MapReduce(comm), chunks, combiner=False)
        a2.run(ph)
        st = {k: comm.allreduce(v, "max", dtype=torch.float64) for k, v in ph.items()}
        out["stages"] = {k: round(v * 1e3, 3) for k, v in st.items()}
        out["pairs_per_s_by_stage"] = {k: (a2.npairs / v if v > 0 else None) for k, v in st.items()}
        comb = WordFreq(MapReduce(comm), chunks, combiner=True)
        comb.run()
        out["top10"] = app.top
        out["top10_equals_combiner"] = comb.top == app.top
    return out
