"""Streaming part-file input for device jobs (the MI355X analog of the
reference's per-task fread, examples/wordfreq.cpp:104-130 and
cuda/InvertedIndex.cu:170-190).

RingReader reads the part files of consecutive jobs into a ring of pinned
host buffers with a pool of threads (os.preadv releases the GIL; 32 MiB
pieces spread one file over several cores). A job gets its files as
(pinned view, ready) entries — ready.result() blocks until that file is read
— plus an on_copied(i, event) callback the job calls once file i's
host->device copy is issued. A ring slot is refilled only after the copy out
of it has completed, so host memory stays at `slots` buffers however long the
job, and the reads of file i + slots overlap the copy and map of file i.
"""
from __future__ import annotations

import os
import threading
from concurrent.futures import ThreadPoolExecutor

import torch


class _AllDone:
    """ready.result() over the piece reads of one file"""

    def __init__(self, futs):
        self.futs = futs

    def result(self):
        for f in self.futs:
            f.result()


class RingReader:
    def __init__(self, paths, slots=8, threads=8, piece=32 << 20, pin=True):
        """paths: list of (path, nbytes) part files, read in this order by
        every job"""
        self.paths = list(paths)
        self.R = max(1, int(slots))
        self.piece = int(piece)
        maxlen = max((n for _, n in self.paths), default=1)
        self.bufs = [torch.empty(max(maxlen, 1), dtype=torch.uint8, pin_memory=pin) for _ in range(self.R)]
        self.views = [memoryview(b.numpy()) for b in self.bufs]
        self.fds = [os.open(p, os.O_RDONLY) for p, _ in self.paths]
        self.pool = ThreadPoolExecutor(max_workers=max(1, int(threads)), thread_name_prefix="mrh-read")
        self.cv = threading.Condition()
        self.copied = [-1] * self.R   # per slot: the last global file index whose copy out of it was issued
        self.events = [None] * self.R
        self.next_g = 0
        self.closed = False

    def _gate(self, g):
        """block until slot g % R is free: the copy of file g - R out of it is done"""
        if g < self.R:
            return
        slot, want = g % self.R, g - self.R
        with self.cv:
            self.cv.wait_for(lambda: self.copied[slot] >= want or self.closed)
            ev = self.events[slot]
        if ev is not None:
            ev.synchronize()

    def _read(self, g, i, o, n):
        self._gate(g)
        got = os.preadv(self.fds[i], [self.views[g % self.R][o:o + n]], o)
        if got != n:
            raise OSError(f"short read of {self.paths[i][0]} at {o}: {got} of {n} bytes")

    def job(self):
        """the next job's input: ([(pinned view, ready)] in file order,
        on_copied(i, event)); its reads are queued now (behind any earlier
        job's) and start as ring slots free up"""
        base = self.next_g
        self.next_g += len(self.paths)
        entries = []
        for i, (_, n) in enumerate(self.paths):
            g = base + i
            futs = [self.pool.submit(self._read, g, i, o, min(self.piece, n - o)) for o in range(0, n, self.piece)]
            entries.append((self.bufs[g % self.R][:n], _AllDone(futs)))

        def on_copied(i, event):
            g = base + i
            with self.cv:
                self.events[g % self.R] = event
                self.copied[g % self.R] = g
                self.cv.notify_all()
        return entries, on_copied

    def close(self):
        with self.cv:
            self.closed = True
            self.cv.notify_all()
        self.pool.shutdown(wait=True)
        for fd in self.fds:
            os.close(fd)
        self.fds = []
