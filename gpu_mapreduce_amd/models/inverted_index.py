"""InvertedIndex: URL -> list of files that link to it.

Reference: cuda/InvertedIndex.cu (GPU map) — per rank, files
part-%05d in [me*fpp, (me+1)*fpp) are read, every `<a href="URL"` is found on
the GPU, URLs are copied back and added to the KV one by one on the host
(:254-410), then aggregate (:182) -> convert (:186) -> reduce writes
"url\\tfile file ... \\n" lines with one fopen per key (:463-513).

MI355X design, pipelined per part file:
  map       files stream host(pinned) -> HBM on a side HIP stream, double
            buffered; the fused scan/extract kernels (csrc/kernels/text.hip)
            emit KV(url+NUL, int32 file id) directly into HBM — no D2H, no
            per-URL host loop;
  aggregate (P > 1) each file's URLs go through the chunked RCCL exchange as
            soon as they are mapped, while the next file is still on the PCIe
            link — the shuffle hides behind the input stream instead of
            following it (the map chunk k+1 || shuffle chunk k pipeline of
            SURVEY.md §2.10);
  group     each file's (received) URLs are grouped by key in the same shadow
            of the H2D: the map's KeyValue has grouping enabled, so every
            part is appended to device arenas (no final concat), hashed, and
            inserted into an exact HBM hash table (byte check per pair)
            (csrc/engine/grouper.h, csrc/kernels/group.hip);
  convert   finds the group-by done: it only orders the ~600 K groups by hash
            and the pairs by group (two short radix sorts);
  reduce    the output text is formatted on the GPU (apps.hip) and drains to
            pinned host memory on a D2H copy stream (the PCIe link is full
            duplex: the drain overlaps the next job's input stream); the
            output is complete once `output_ready()` (or any device sync).
            Optionally written to `out_dir/InvertedIndex-P-me`.

`output` lives in a pinned host buffer of a two-slot pool (no
hipHostMalloc per job): it stays valid until two more InvertedIndex jobs
have run in this process. `output_lines()` / `output_bytes()` refuse to read
an overwritten slot; pass `own_output=True` to get a private buffer.
"""
from __future__ import annotations

import os
import time

import torch

from .._ext import C
from ..runtime import pools
from ..runtime.mapreduce import MapReduce

PAD = 64


def _write_file(path, data):
    """write `data` (a memoryview of the pinned output) to `path` straight
    from the buffer, no bytes copy. One writer: 16 MiB pieces pwritten by 8
    threads measured slower into a RAM-backed directory (27.8 vs 21.1 ms for
    the 98 MB index, profiles/r3_gpu_full_g.txt)"""
    # overwrite in place: a job writing the same path again reuses the file's
    # cached pages instead of freeing them (O_TRUNC) and faulting in fresh
    # zeroed ones. A longer old file is cut first, so a write that dies
    # midway leaves a file no longer than the new index (never stale lines
    # past its end); an equal-size overwrite that dies midway leaves old bytes
    # behind the new ones, which a reader cannot detect — write elsewhere and
    # rename if that matters
    fd = os.open(path, os.O_WRONLY | os.O_CREAT, 0o644)
    try:
        if os.fstat(fd).st_size > len(data):
            os.ftruncate(fd, len(data))
        done = 0
        while done < len(data):
            done += os.pwrite(fd, data[done:], done)
        os.ftruncate(fd, len(data))
    finally:
        os.close(fd)


_WRITER = []
_SLOT_WRITE = {}  # pinned output slot -> the pending write of the job that filled it


def _writer():
    """the index writer thread (one: writes land in job order)"""
    if not _WRITER:
        from concurrent.futures import ThreadPoolExecutor
        _WRITER.append(ThreadPoolExecutor(max_workers=1, thread_name_prefix="mrh-ii-write"))
    return _WRITER[0]


class InvertedIndex:
    def __init__(self, mr: MapReduce, files, out_dir=None, pipelined=True, own_output=False, prefetch_next=None,
                 async_write=False):
        """files: list of (name, uint8 tensor) for THIS rank (host tensors —
        ideally pinned — or device tensors), or (name, tensor, ready) where
        ready.result() blocks until the tensor holds the file's bytes (e.g. the
        future of a read into a pinned buffer): it is waited for right before
        that file's copy is issued, so reading file i+1 overlaps the copy and
        map of file i (the reference freads each part file in its map,
        cuda/InvertedIndex.cu:170-190).

        prefetch_next: the (name, tensor) files of the job that will run next on
        this rank (a job pipeline, e.g. a serving loop). While this job maps
        its last file, the next job's first file is already copied into the
        following staging slot, so the PCIe link does not idle during this
        job's tail (its last file's map and group-by, the group ordering, the
        output formatting); the next job finds that copy and does not repeat
        it. Every job still copies all of its own files. A (name, tensor,
        ready) entry is waited for (ready.result()) before that copy.

        async_write (with out_dir): the index file is written by a writer
        thread once the output text has drained to host memory, so the write
        overlaps the next job (the reference writes it inside its reduce,
        cuda/InvertedIndex.cu:463-513); wait_written() blocks until it is on
        disk. The pinned output slot is not reused before its write is done."""
        self.prefetch_next = prefetch_next
        self.async_write = async_write
        self._write = None
        self.mr = mr
        self.files = files
        self.out_dir = out_dir
        self.pipelined = pipelined
        self.own_output = own_output
        self._gen = None
        self._mapped = False
        self._reserved = False
        # doc ids are global (rank-major) so a value means the same file name on
        # every rank after the shuffle; the reference ships the name string itself
        all_names = mr.comm.allgather_object([f[0] for f in files])
        self.doc_base = sum(len(x) for x in all_names[: mr.me])
        self.max_files = max(len(x) for x in all_names)
        names = [n.encode() for lst in all_names for n in lst]
        self.names = torch.frombuffer(bytearray(b"".join(names) or b"\0"), dtype=torch.uint8).clone()
        lens = torch.tensor([0] + [len(n) for n in names], dtype=torch.int64)
        self.name_off = torch.cumsum(lens, 0)
        dev = mr.device
        self.dev = dev
        self.is_cuda = dev.startswith("cuda")
        self.names_dev = pools.device_constant(dev, self.names)
        self.name_off_dev = pools.device_constant(dev, self.name_off)
        maxlen = max((f[1].numel() for f in files), default=0)
        # persistent staging buffers: a ring of `streams` (0 = auto: 3, or
        # MRH_II_BUFS) so streams - 1 file copies are in flight while one file
        # maps: with the cross-job prefetch 2 / 3 / 4 buffers measured 19.75 /
        # 19.25 / 19.22 ms per 1 GiB job (profiles/r3_ii_ring_depth.txt); the
        # PAD bytes past each file are read by the 16-byte scan windows but
        # never matched
        st = int(mr.streams)
        self.nbuf = st if st > 0 else max(1, int(os.environ.get("MRH_II_BUFS", "3")))
        self.bufs = [pools.device_buffer(dev, maxlen + PAD, slot) for slot in range(self.nbuf if files else 0)]
        self.copy_stream = pools.stream(dev, "h2d") if self.is_cuda else None
        self.output = None
        self._done = None
        self.exchanged = False
        self.nurls = 0
        self.write_s = 0.0

    # -------------------------------------------------------------- map
    def _emit(self, kv, part):
        """one file's KV: shuffled right away (P > 1) and grouped (the
        KeyValue's GroupIndex), in the shadow of the next file's H2D"""
        mr = self.mr
        if self.pipelined and mr.nprocs > 1:
            part, _ = C.aggregate(part, mr.comm.native, chunk_bytes=mr.chunk_bytes)
        kv.add_kv(part)
        if self.pipelined and not self._reserved and part.n > 0:
            # size the grouped arenas once for the whole job from the first
            # part (+25 %): no x1.5 regrow copies or table rehash under the H2D
            self._reserved = True
            f = 1.25 * max(1, len(self.files), self.max_files)
            kv.reserve_grouping(int(part.n * f) + 1024, int(part.kdata.numel() * f) + 4096,
                                int(part.vdata.numel() * f) + 4096)

    def _wait_read(self, i):
        f = self.files[i]
        if len(f) > 2 and f[2] is not None:
            f[2].result()

    def _map(self, itask, kv):
        if self._mapped:
            raise RuntimeError("InvertedIndex: a rank was given two map tasks (its files are mapped once)")
        self._mapped = True
        files = self.files
        if self.pipelined:
            kv.enable_grouping()
        empty = lambda: C.map_urls(torch.zeros(PAD, dtype=torch.uint8, device=self.dev), 0, 0)
        if not self.is_cuda:
            for fid, f in enumerate(files):
                self._wait_read(fid)
                t = f[1]
                buf = self.bufs[0]
                buf[: t.numel()].copy_(t)
                buf[t.numel():t.numel() + PAD].zero_()
                self._emit(kv, C.map_urls(buf, t.numel(), self.doc_base + fid))
        else:
            main = torch.cuda.current_stream()
            cs = self.copy_stream
            nb = self.nbuf
            ready = [torch.cuda.Event() for _ in range(nb)]
            # the staging ring continues across jobs: file i of this job lands
            # in slot (base + i) % nb, so a job pipeline's prefetch of the next
            # job's first file goes to the slot after this job's last one
            base = pools.ring_cursor(self.dev, "ii") % nb

            def copy_into(b, t, ev):
                with torch.cuda.stream(cs):
                    prev = pools.last_use(self.dev, b)  # the last kernel (any job) that read this buffer
                    if prev is not None:
                        cs.wait_event(prev)
                    self.bufs[b][: t.numel()].copy_(t, non_blocking=True)
                    ev.record(cs)

            def issue(i):
                b = (base + i) % nb
                t = files[i][1]
                self._wait_read(i)
                ev = pools.take_prefetch(self.dev, b, t, self.bufs[b])  # copied by the previous job of a pipeline
                if ev is not None:
                    ready[b] = ev
                else:
                    copy_into(b, t, ready[b])

            ahead = max(1, nb - 1)
            for i in range(min(ahead, len(files))):
                issue(i)
            for i in range(len(files)):
                if nb > 1 and i + ahead < len(files):
                    issue(i + ahead)
                elif nb == 1 and i > 0:
                    issue(i)
                if i == len(files) - 1 and nb > 1 and self.prefetch_next:
                    # the next job's first file, behind this job's last copy
                    first = self.prefetch_next[0]
                    nxt = first[1]
                    if nxt.numel() + PAD <= self.bufs[0].numel():
                        if len(first) > 2 and first[2] is not None:
                            first[2].result()  # its bytes are read into the host buffer
                        slot = (base + len(files)) % nb
                        ev = torch.cuda.Event()
                        copy_into(slot, nxt, ev)
                        pools.set_prefetch(self.dev, slot, nxt, ev, self.bufs[slot])
                b = (base + i) % nb
                main.wait_event(ready[b])
                n = files[i][1].numel()
                part = C.map_urls(self.bufs[b], n, self.doc_base + i)
                pools.mark_use(self.dev, b, main)
                self._emit(kv, part)
            pools.ring_cursor(self.dev, "ii", advance=len(files), n=nb)
        # lock-step exchanges: ranks with fewer files join with empty parts
        if self.pipelined and self.mr.nprocs > 1:
            for _ in range(len(files), self.max_files):
                self._emit(kv, empty())
            self.exchanged = True

    # -------------------------------------------------------------- reduce
    def _reduce(self, kmv, kv):
        text = C.inverted_index_format(kmv, self.names_dev, self.name_off_dev)
        if self.is_cuda:
            slot = None
            if self.own_output:
                host = torch.empty(text.numel(), dtype=torch.uint8, pin_memory=True)
            else:
                slot = 100 + pools.next_slot("ii_out")
                pending = _SLOT_WRITE.pop(slot, None)
                if pending is not None:
                    pending.result()  # an earlier job's index is still being written from this slot
                host = pools.pinned_buffer(text.numel(), slot=slot)
                self._gen = pools.generation("ii_out")
            d2h = pools.stream(self.dev, "d2h")
            d2h.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(d2h):
                host.copy_(text, non_blocking=True)
            text.record_stream(d2h)
            self._done = torch.cuda.Event()
            self._done.record(d2h)
        else:
            host = text
            slot = None
        self.output = host
        if self.out_dir is not None:
            os.makedirs(self.out_dir, exist_ok=True)
            path = os.path.join(self.out_dir, f"InvertedIndex-{self.mr.nprocs}-{self.mr.me}")
            MapReduce.count_io(write=host.numel())
            done = self._done

            def write():
                if done is not None:
                    done.synchronize()  # the D2H drain (releases the GIL)
                t = time.perf_counter()
                _write_file(path, memoryview(host.numpy()))
                return time.perf_counter() - t
            if self.async_write:
                self._write = _writer().submit(write)
                if slot is not None:
                    _SLOT_WRITE[slot] = self._write
            else:
                self.write_s = write()

    def wait_written(self):
        """block until the index file is written (async_write); returns the
        write's seconds"""
        if self._write is not None:
            self.write_s = self._write.result()
            self._write = None
        return self.write_s

    def output_ready(self):
        """block until the output text has drained to host memory"""
        if self._done is not None:
            self._done.synchronize()

    def run(self, phases=None):
        """phases: optional dict; if given, per-stage seconds (device-synced)
        are recorded under the reference's stage names (Map, Network I/O,
        Sort/Hash, Reduce — chapter_final.pdf Fig. 4/5). With the pipelined
        map the per-file shuffle runs inside Map (Network I/O = 0)."""
        mr = self.mr
        tick = _Ticker(phases, mr.comm)
        # one map task per rank, each maps its own files (reference :175,
        # :278-284). The files are rank-local and the per-file exchange inside
        # the callback is lock-step across ranks, so the task of rank r must
        # run on rank r: mapstyle 2 (dynamic assignment: a rank could get none
        # or two) is overridden for this map
        ms = mr.mapstyle
        if ms not in (0, 1):
            mr.mapstyle = 0
        try:
            self.nurls = mr.map(mr.nprocs, self._map)
        finally:
            mr.mapstyle = ms
        tick("Map")
        if not self.exchanged:
            mr.aggregate()
        tick("Network I/O")
        self.nunique = mr.convert()
        tick("Sort/Hash")
        mr.reduce_batch(self._reduce)
        if phases is not None:
            self.output_ready()
        tick("Reduce")
        return self.nurls

    def output_bytes(self) -> bytes:
        if self.output is None:
            return b""
        if self._gen is not None and pools.generation("ii_out") - self._gen >= 2:
            raise RuntimeError("InvertedIndex.output was overwritten by a later job (two-slot pinned pool); "
                               "read it sooner or construct with own_output=True")
        self.output_ready()
        return bytes(self.output.cpu().numpy())

    def output_lines(self):
        return self.output_bytes().decode("utf-8", "replace").splitlines()


class _Ticker:
    def __init__(self, phases, comm):
        self.phases = phases
        self.comm = comm
        if phases is not None:
            self.t = comm.wtime()

    def __call__(self, name):
        if self.phases is None:
            return
        t = self.comm.wtime()
        self.phases[name] = self.phases.get(name, 0.0) + (t - self.t)
        self.t = t


def reference_inverted_index(files):
    """Pure-Python oracle: {url: sorted list of file names} over all files."""
    import re
    idx = {}
    pat = re.compile(rb'<a href="')
    for name, t in files:
        b = bytes(t.cpu().numpy())
        for m in pat.finditer(b):
            s = m.end()
            e = b.find(b'"', s)
            e = len(b) if e < 0 else e
            idx.setdefault(b[s:e], []).append(name)
    return {k: sorted(v) for k, v in idx.items()}
