"""OINK, the MapReduce scripting layer (reference oink/), from Python.

The interpreter, variables, MR-object registry, MR-method dispatcher, named
commands and callback library are native C++ (csrc/oink, in libmrhip.so —
the same code behind the `oink` executable and the oink_* C API). This
module only adapts Python arguments: a Comm, screen output to any object
with .write(), and `-partition` worlds for host (gloo) communicators, which
are split through torch.distributed.
"""
from __future__ import annotations

import sys

from .._ext import C
from ..parallel.comm import Comm, world
from ..runtime.mapreduce import MapReduce

# errors of the native interpreter (variables, evaluator, commands:
# csrc/oink/variable.cpp, oink.cpp)
OinkError = C.OinkError


def _world_of(ucomm: Comm, partitions):
    sizes = []
    for p in partitions or []:
        if "x" in p:
            n, m = p.split("x")
            sizes += [int(m)] * int(n)
        else:
            sizes.append(int(p))
    if len(sizes) <= 1 or ucomm.size == 1:
        return None
    acc = 0
    for i, s in enumerate(sizes):
        if ucomm.rank < acc + s:
            return ucomm.split(i)
        acc += s
    return None


class OINK:
    """Script interpreter. Create with a Comm (or None for the default world)."""

    def __init__(self, comm: Comm | None = None, partitions=None, screen=sys.stdout, logfile="log.oink",
                 variables=None, echo=None):
        ucomm = comm if comm is not None else world()
        w = _world_of(ucomm, partitions)
        self.comm = w if w is not None else ucomm
        write = None
        if screen is not None:
            write = screen.write
        vars_ = [(str(n), [str(v) for v in vals]) for n, vals in (variables or [])]
        self._o = C.Oink(ucomm.native, [str(p) for p in (partitions or [])], write,
                         logfile if logfile else "none", vars_, echo or "",
                         w.native if w is not None else None)

    def file(self, path=None, text=None):
        """Run a script from a path, a string, or stdin."""
        if text is not None:
            self._o.text(text)
        else:
            self._o.file(path or "")

    def one(self, line):
        return self._o.one(line)

    @property
    def deltatime(self):
        return self._o.deltatime

    def mr(self, name) -> MapReduce:
        """A named MR object of the script, as a Python MapReduce."""
        return MapReduce(self.comm, _native=self._o.mr(name))

    def close(self):
        self._o.close()


def main(argv=None):
    """oink [-in file] [-var name v1 v2 ...] [-partition NxM ...] [-screen file|none]
    [-log file|none] [-echo style]"""
    argv = list(sys.argv[1:] if argv is None else argv)
    from ..parallel import comm as pcomm
    comm = pcomm.init()
    infile = None
    variables, partitions = [], []
    screen, logfile, echo = sys.stdout, "log.oink", None
    i = 0
    while i < len(argv):
        a = argv[i]
        if a in ("-in", "-i"):
            infile = argv[i + 1]
            i += 2
        elif a in ("-var", "-v"):
            j = i + 2
            while j < len(argv) and not argv[j].startswith("-"):
                j += 1
            variables.append((argv[i + 1], argv[i + 2:j]))
            i = j
        elif a in ("-partition", "-p"):
            j = i + 1
            while j < len(argv) and not argv[j].startswith("-"):
                partitions.append(argv[j])
                j += 1
            i = j
        elif a in ("-screen", "-sc"):
            screen = None if argv[i + 1] == "none" else open(argv[i + 1], "w")
            i += 2
        elif a in ("-log", "-l"):
            logfile = argv[i + 1]
            i += 2
        elif a in ("-echo", "-e"):
            echo = argv[i + 1]
            i += 2
        else:
            raise SystemExit(f"Invalid command-line argument {a}")
    oink = OINK(comm, partitions=partitions, screen=screen, logfile=logfile, variables=variables, echo=echo)
    oink.file(infile)
    oink.close()
    return 0
