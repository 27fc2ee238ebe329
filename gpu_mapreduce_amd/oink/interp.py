"""OINK: the MapReduce scripting front-end (reference oink/oink.cpp, input.cpp,
object.cpp, mrmpi.cpp, universe.cpp), on top of the MI355X MapReduce engine.

Script semantics follow the reference: rank 0 reads lines (with `&`
continuation) and broadcasts them; `#` comments; `$x` / `${name}` variable
substitution; quoted arguments; built-ins (clear echo if include jump label
log next print shell variable input mr output set); named commands with
`-i` / `-o` descriptors; `<mrname> <method> args` drives any MapReduce method
on a named MR object. Named commands and callbacks come from a static
registry (commands.py, callbacks.py) — no code generation step (the
reference's Make.py/style_*.h).
"""
from __future__ import annotations

import os
import shlex
import sys
import time

from ..parallel.comm import Comm, world
from ..runtime.mapreduce import MapReduce
from .variable import OinkError, Variable

MAXLINE = 8192


class Universe:
    """-partition NxM: split the world into sub-communicators (oink/universe.cpp)."""

    def __init__(self, comm: Comm, partitions=None):
        self.ucomm = comm
        self.me = comm.rank
        self.nprocs = comm.size
        sizes = []
        for p in (partitions or []):
            if "x" in p:
                n, m = p.split("x")
                sizes += [int(m)] * int(n)
            else:
                sizes.append(int(p))
        if not sizes:
            sizes = [self.nprocs]
        if sum(sizes) != self.nprocs:
            raise OinkError("Processor partitions are inconsistent")
        self.sizes = sizes
        self.nworlds = len(sizes)
        acc = 0
        for i, s in enumerate(sizes):
            if self.me < acc + s:
                self.iworld = i
                break
            acc += s
        self.world = comm if self.nworlds == 1 else comm.split(self.iworld)
        self.world_me = self.world.rank


class MRWrap:
    def __init__(self, mr, name=None):
        self.mr = mr
        self.name = name
        self.permanent = name is not None


class InputDesc:
    def __init__(self):
        self.index = -1
        self.prepend = None
        self.pflag = 0
        self.suflag = 0
        self.substitute = 0
        self.multi = 1
        self.strings = []
        self.mmode = 0
        self.recurse = 0
        self.self = 0
        self.readfile = 0
        self.nmap = 0
        self.sepchar = "\n"
        self.sepstr = "\n"
        self.delta = 80
        self.mode = None      # "mr" | "path"
        self.mrwrap = None


class OutputDesc:
    def __init__(self):
        self.index = -1
        self.name = None
        self.prepend = None
        self.pflag = 0
        self.suflag = 0
        self.substitute = 0
        self.procfile = None
        self.mode = "neither"


class Object:
    """Registry of named/temporary MR objects + command I/O descriptors (oink/object.cpp)."""

    def __init__(self, oink):
        self.oink = oink
        self.mrs: list[MRWrap] = []
        self.inputs = []
        self.outputs = []
        self.userinputs = {}
        self.useroutputs = {}
        self.g = dict(verbosity=0, timer=0, memsize=64, outofcore=0, minpage=0, maxpage=0, freepage=1,
                      zeropage=0, scratch=None, prepend=None, substitute=0)

    @property
    def me(self):
        return self.oink.comm.rank

    # ---------------------------------------------------------------- MR registry
    def allocate_mr(self, verbosity=None, timer=None, memsize=None, outofcore=None):
        g = self.g
        mr = MapReduce(self.oink.comm)
        mr.verbosity = g["verbosity"] if verbosity is None else verbosity
        mr.timer = g["timer"] if timer is None else timer
        mr.memsize = g["memsize"] if memsize is None else memsize
        mr.outofcore = g["outofcore"] if outofcore is None else outofcore
        mr.minpage, mr.maxpage = g["minpage"], g["maxpage"]
        mr.freepage, mr.zeropage = g["freepage"], g["zeropage"]
        if g["scratch"]:
            mr.set_fpath(g["scratch"])
        return mr

    def create_mr(self):
        mr = self.allocate_mr()
        self.mrs.append(MRWrap(mr))
        return mr

    def copy_mr(self, mr):
        c = mr.copy()
        self.mrs.append(MRWrap(c))
        return c

    def find_mr(self, name):
        for i, w in enumerate(self.mrs):
            if w.permanent and w.name == name:
                return i
        return -1

    def permanent(self, mr):
        return any(w.mr is mr and w.permanent for w in self.mrs)

    def add_mr_named(self, args):
        if not 1 <= len(args) <= 5:
            raise OinkError("Illegal mr command")
        name = args[0]
        if not all(c.isalnum() or c == "_" for c in name):
            raise OinkError("MR ID must be alphanumeric or underscore characters")
        if self.find_mr(name) >= 0:
            raise OinkError("ID in mr command is already in use")
        vals = [int(a) for a in args[1:]] + [None] * (5 - len(args))
        mr = self.allocate_mr(*vals[:4])
        self.mrs.append(MRWrap(mr, name))

    def delete_mr(self, index):
        self.mrs[index].mr.destroy()
        del self.mrs[index]

    def cleanup(self):
        """delete temporary MRs and descriptors after a command"""
        keep = []
        for w in self.mrs:
            if w.permanent:
                keep.append(w)
            else:
                w.mr.destroy()
        self.mrs = keep
        self.inputs, self.outputs = [], []

    # ---------------------------------------------------------------- descriptors
    def _default_input(self):
        return InputDesc()

    def add_input(self, index, s):
        d = self.userinputs.pop(index, None) or self._default_input()
        d.index = index
        while len(self.inputs) <= index:
            self.inputs.append(None)
        self.inputs[index] = d
        imr = self.find_mr(s)
        if imr >= 0:
            d.mode = "mr"
            d.mrwrap = self.mrs[imr]
            return
        d.mode = "path"
        if s.startswith("v_"):
            var = self.oink.variable
            if not var.find(s[2:]):
                raise OinkError("Command input variable is unknown")
            items = var.retrieve_all(s[2:])
        else:
            items = [s]
        g = self.g
        pre = d.prepend if d.pflag else g["prepend"]
        sub = d.substitute if d.suflag else g["substitute"]
        d.strings = [self.expandpath(one, pre, 0, sub, j + 1) for one in items for j in range(d.multi)]

    def add_output(self, index, file, name):
        d = self.useroutputs.pop(index, None) or OutputDesc()
        d.index = index
        while len(self.outputs) <= index:
            self.outputs.append(None)
        self.outputs[index] = d
        if name != "NULL":
            if not all(c.isalnum() or c == "_" for c in name):
                raise OinkError("Ouptut MR ID must be alphanumeric or underscore characters")
            d.name = name
        if file != "NULL":
            g = self.g
            pre = d.prepend if d.pflag else g["prepend"]
            sub = d.substitute if d.suflag else g["substitute"]
            d.procfile = self.expandpath(file, pre, 1, sub, 0)
            self.createdir(d.procfile)
        d.mode = "both" if (d.procfile and d.name) else "path" if d.procfile else "mr" if d.name else "neither"

    def expandpath(self, inpath, prepend, postpend, substitute, multi):
        me = self.me
        if prepend and postpend:
            p = f"{prepend}/{inpath}.{me}"
        elif prepend:
            p = f"{prepend}/{inpath}"
        elif postpend:
            p = f"{inpath}.{me}"
        else:
            p = inpath
        if "%" in p:
            p = p.replace("%", str(me if substitute == 0 else (me % substitute) + 1), 1)
        if "*" in p:
            p = p.replace("*", str(multi), 1)
        return p

    @staticmethod
    def createdir(path):
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)

    def user_input(self, args):
        if len(args) < 3:
            raise OinkError("Illegal input command")
        index = int(args[0]) - 1
        d = self.userinputs.setdefault(index, self._default_input())
        it = iter(args[1:])
        for k in it:
            v = next(it, None)
            if v is None:
                raise OinkError("Illegal input command")
            if k == "prepend":
                d.pflag, d.prepend = 1, v
            elif k == "substitute":
                d.suflag, d.substitute = 1, int(v)
            elif k in ("multi", "mmode", "recurse", "self", "readfile", "nmap", "delta"):
                setattr(d, k, int(v))
            elif k == "sepchar":
                d.sepchar = v[0]
            elif k == "sepstr":
                d.sepstr = v
            else:
                raise OinkError("Illegal input command")

    def user_output(self, args):
        if len(args) < 3:
            raise OinkError("Illegal output command")
        index = int(args[0]) - 1
        d = self.useroutputs.setdefault(index, OutputDesc())
        it = iter(args[1:])
        for k in it:
            v = next(it, None)
            if k == "prepend":
                d.pflag, d.prepend = 1, v
            elif k == "substitute":
                d.suflag, d.substitute = 1, int(v)
            else:
                raise OinkError("Illegal output command")

    def set(self, args):
        if len(args) % 2:
            raise OinkError("Illegal set command")
        for k, v in zip(args[0::2], args[1::2]):
            if k in ("scratch", "prepend"):
                self.g[k] = v
            elif k in self.g:
                self.g[k] = int(v)
            else:
                raise OinkError("Illegal set command")

    # ---------------------------------------------------------------- command-side I/O
    def input(self, index, map_file=None, map_str=None, ptr=None):
        """MR for input #index (1-based): the named MR itself, or a new temporary MR
        filled from the file(s) by map_file (mmode 0) or map_str (mmode 1/2)."""
        if index < 1 or index > len(self.inputs) or self.inputs[index - 1] is None:
            raise OinkError("Command input invoked with invalid index")
        d = self.inputs[index - 1]
        if d.mode == "mr":
            return d.mrwrap.mr
        mr = self.create_mr()
        if map_file is None and map_str is None:
            raise OinkError("Command input not allowed from file")
        if d.mmode == 0:
            if map_file is None:
                raise OinkError("Comand input map function does not match input mode")
            mr.map_file(d.strings, d.self, d.recurse, d.readfile, map_file, ptr)
        else:
            if map_str is None:
                raise OinkError("Command input map function does not match input mode")
            if d.mmode == 1:
                mr.map_file_char(d.nmap, d.strings, d.self, d.recurse, d.readfile, d.sepchar, d.delta, map_str, ptr)
            else:
                mr.map_file_str(d.nmap, d.strings, d.self, d.recurse, d.readfile, d.sepstr, d.delta, map_str, ptr)
        return mr

    def output(self, index, mr, printer=None, ptr=None, disallow=0):
        """Name mr (if -o ... name) and/or write it to the per-rank file via
        printer(mr, fp[, ptr]) (the reference's scan/map/reduce-to-file)."""
        if index < 1 or index > len(self.outputs) or self.outputs[index - 1] is None:
            raise OinkError("Command output invoked with invalid index")
        d = self.outputs[index - 1]
        if d.mode in ("mr", "both"):
            if disallow:
                raise OinkError("Command output as MR object not allowed")
            w = next((w for w in self.mrs if w.mr is mr), None)
            if w is None:
                raise OinkError("Command output called with unknown MR object")
            for o in self.mrs:
                if o is not w and o.permanent and o.name == d.name:
                    o.permanent, o.name = False, None
            w.name, w.permanent = d.name, True
        if d.mode in ("path", "both"):
            if printer is None:
                raise OinkError("Command input not allowed to file")
            with open(d.procfile, "w") as fp:
                printer(mr, fp) if ptr is None else printer(mr, fp, ptr)


class OINK:
    """Script interpreter. Create with a Comm (or None for the default world)."""

    def __init__(self, comm: Comm | None = None, partitions=None, screen=sys.stdout, logfile="log.oink",
                 variables=None, echo=None):
        ucomm = comm if comm is not None else world()
        self.universe = Universe(ucomm, partitions)
        self.comm = self.universe.world
        self.me = self.comm.rank
        self.screen = screen if self.me == 0 else None
        self.logfile = None
        if self.me == 0 and logfile and logfile != "none":
            self.logfile = open(logfile, "w")
        self.variable = Variable(self)
        self.obj = Object(self)
        self.deltatime = 0.0
        self.echo_screen, self.echo_log = 0, 1
        if echo:
            self._echo([echo])
        self.label_active = False
        self.labelstr = None
        self.jump_skip = 0
        self.files = []     # stack of open script iterators (rank 0)
        for name, vals in (variables or []):
            self.variable.set([name, "index"] + list(vals))
        from . import commands  # noqa: F401  (registers commands)

    # ---------------------------------------------------------------- output helpers
    def message(self, s):
        if self.me == 0:
            if self.screen:
                print(s, file=self.screen)
            if self.logfile:
                print(s, file=self.logfile)
                self.logfile.flush()

    def _emit_echo(self, line):
        if self.me == 0 and not self.label_active:
            if self.echo_screen and self.screen:
                self.screen.write(line if line.endswith("\n") else line + "\n")
            if self.echo_log and self.logfile:
                self.logfile.write(line if line.endswith("\n") else line + "\n")

    # ---------------------------------------------------------------- reading
    def file(self, path=None, text=None):
        """Run a script from a path, a string, or stdin."""
        if self.me == 0:
            if text is not None:
                self.files.append(iter(text.splitlines(keepends=True)))
            elif path is not None:
                self.files.append(iter(open(path).readlines()))
                self._self_path = path
            else:
                self.files.append(iter(sys.stdin.readlines()))
        while True:
            line = None
            if self.me == 0:
                line = self._readline()
            line = self.comm.bcast_object(line, 0)
            if line is None:
                if self.label_active:
                    raise OinkError("Label wasn't found in input script")
                break
            self._emit_echo(line)
            self.one(line, echo=False)

    def _readline(self):
        while self.files:
            buf = ""
            for ln in self.files[-1]:
                stripped = ln.rstrip()
                if stripped.endswith("&"):
                    buf += stripped[:-1] + " "
                    continue
                return buf + ln
            if buf:
                return buf
            self.files.pop()
        return None

    def one(self, line, echo=True):
        if echo:
            self._emit_echo(line)
        cmd, args = self.parse(line)
        if cmd is None:
            return None
        if self.label_active and cmd != "label":
            return None
        if not self.execute(cmd, args):
            raise OinkError(f"Unknown command: {line.strip()}")
        return cmd

    def parse(self, line):
        # strip comments outside quotes
        out, q = [], None
        for ch in line:
            if ch == "#" and not q:
                break
            if ch == q:
                q = None
            elif ch in "\"'" and not q:
                q = ch
            out.append(ch)
        s = "".join(out)
        if not self.label_active:
            s = self.substitute(s)
        try:
            toks = shlex.split(s, posix=True)
        except ValueError:
            raise OinkError("Unbalanced quotes in input line")
        if not toks:
            return None, []
        return toks[0], toks[1:]

    def substitute(self, s):
        out, i, q = [], 0, None
        while i < len(s):
            ch = s[i]
            if ch == "$" and not q and i + 1 < len(s):
                if s[i + 1] == "{":
                    j = s.find("}", i + 2)
                    if j < 0:
                        raise OinkError("Invalid variable name")
                    name = s[i + 2:j]
                    i = j + 1
                else:
                    name = s[i + 1]
                    i += 2
                val = self.variable.retrieve(name)
                if val is None:
                    raise OinkError("Substitution for illegal variable")
                out.append(val)
                continue
            if ch == q:
                q = None
            elif ch in "\"'" and not q:
                q = ch
            out.append(ch)
            i += 1
        return "".join(out)

    # ---------------------------------------------------------------- dispatch
    def execute(self, cmd, args):
        builtin = {"clear": self._clear, "echo": self._echo, "if": self._if, "include": self._include,
                   "jump": self._jump, "label": self._label, "log": self._log, "next": self._next,
                   "print": self._print, "shell": self._shell, "variable": self.variable.set,
                   "input": self.obj.user_input, "mr": self.obj.add_mr_named, "output": self.obj.user_output,
                   "set": self.obj.set}
        if cmd in builtin:
            builtin[cmd](args)
            return True
        from .commands import COMMANDS
        if cmd in COMMANDS:
            c = COMMANDS[cmd](self)
            i = 0
            while i < len(args) and args[i] not in ("-i", "-o"):
                i += 1
            c.params(args[:i])
            isw = osw = False
            while i < len(args):
                sw = args[i]
                j = i + 1
                other = "-o" if sw == "-i" else "-i"
                while j < len(args) and args[j] != other:
                    j += 1
                if sw == "-i":
                    c.inputs(args[i + 1:j])
                    isw = True
                elif sw == "-o":
                    c.outputs(args[i + 1:j])
                    osw = True
                else:
                    raise OinkError("Invalid command switch")
                i = j
            if not isw:
                c.inputs([])
            if not osw:
                c.outputs([])
            self.comm.barrier()
            t0 = time.perf_counter()
            c.run()
            self.comm.barrier()
            self.deltatime = time.perf_counter() - t0
            return True
        idx = self.obj.find_mr(cmd)
        if idx >= 0:
            from .mrmpi import run_method
            self.comm.barrier()
            t0 = time.perf_counter()
            run_method(self, idx, args)
            self.comm.barrier()
            self.deltatime = time.perf_counter() - t0
            return True
        return False

    # ---------------------------------------------------------------- built-ins
    def _clear(self, args):
        if args:
            raise OinkError("Illegal clear command")
        for w in self.obj.mrs:
            w.mr.destroy()
        self.obj = Object(self)
        self.variable = Variable(self)

    def _echo(self, args):
        if len(args) != 1 or args[0] not in ("none", "screen", "log", "both"):
            raise OinkError("Illegal echo command")
        self.echo_screen = int(args[0] in ("screen", "both"))
        self.echo_log = int(args[0] in ("log", "both"))

    def _if(self, args):
        if len(args) < 3 or args[1] != "then":
            raise OinkError("Illegal if command")
        conds = [(args[0], 2)]
        blocks = []
        i = 2
        cur_cond, start = args[0], 2
        while True:
            j = start
            while j < len(args) and args[j] not in ("elif", "else"):
                j += 1
            blocks.append((cur_cond, args[start:j]))
            if j >= len(args):
                break
            if args[j] == "elif":
                if j + 2 > len(args):
                    raise OinkError("Illegal if command")
                cur_cond, start = args[j + 1], j + 2
            else:
                cur_cond, start = None, j + 1
        del conds, i
        for cond, cmds in blocks:
            ok = True if cond is None else self.variable.evaluate_boolean(self.substitute(cond))
            if ok:
                if not cmds:
                    raise OinkError("Illegal if command")
                for c in cmds:
                    self.one(c)
                return

    def _include(self, args):
        if len(args) != 1:
            raise OinkError("Illegal include command")
        if self.me == 0:
            if not os.path.exists(args[0]):
                raise OinkError(f"Cannot open input script {args[0]}")
            self.files.append(iter(open(args[0]).readlines()))

    def _jump(self, args):
        if not 1 <= len(args) <= 2:
            raise OinkError("Illegal jump command")
        if self.jump_skip:
            self.jump_skip = 0
            return
        if self.me == 0:
            if args[0] == "SELF":
                src = getattr(self, "_self_path", None)
                if src is None:
                    raise OinkError("Cannot jump SELF on stdin/text input")
                self.files[-1] = iter(open(src).readlines())
            else:
                self.files[-1] = iter(open(args[0]).readlines())
                self._self_path = args[0]
        if len(args) == 2:
            self.label_active = True
            self.labelstr = args[1]

    def _label(self, args):
        if len(args) != 1:
            raise OinkError("Illegal label command")
        if self.label_active and self.labelstr == args[0]:
            self.label_active = False

    def _log(self, args):
        if len(args) != 1:
            raise OinkError("Illegal log command")
        if self.me == 0:
            if self.logfile:
                self.logfile.close()
            self.logfile = None if args[0] == "none" else open(args[0], "w")

    def _next(self, args):
        if self.variable.next(args):
            self.jump_skip = 1

    def _print(self, args):
        if len(args) != 1:
            raise OinkError("Illegal print command")
        self.message(self.substitute(args[0]))

    def _shell(self, args):
        if not args:
            raise OinkError("Illegal shell command")
        op, rest = args[0], args[1:]
        if op == "cd":
            os.chdir(rest[0])
        elif self.me != 0:
            return
        elif op == "mkdir":
            for d in rest:
                os.makedirs(d, exist_ok=True)
        elif op == "mv":
            os.rename(rest[0], rest[1])
        elif op == "rm":
            for f in rest:
                if os.path.exists(f):
                    os.unlink(f)
        elif op == "rmdir":
            for d in rest:
                os.rmdir(d)
        else:
            raise OinkError("Illegal shell command")

    def close(self):
        self.obj.cleanup()
        if self.logfile:
            self.logfile.close()
            self.logfile = None


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
