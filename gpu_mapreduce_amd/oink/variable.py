"""OINK variables (reference oink/variable.cpp): styles index, loop, world,
universe, uloop, string, equal; `next` iteration; equal-style formula
evaluator with the reference's operator precedence
(| < & < ==,!= < <,<=,>,>= < +,- < *,/ < ^ < unary -,!), math functions
(sqrt exp ln log sin cos tan asin acos atan atan2 random normal ceil floor
round), the constant PI and the keywords nprocs and time."""
from __future__ import annotations

import math
import os
import random
import time

PREC = {"DONE": 0, "|": 1, "&": 2, "==": 3, "!=": 3, "<": 4, "<=": 4, ">": 4, ">=": 4, "+": 5, "-": 5,
        "*": 6, "/": 6, "^": 7, "NEG": 8, "!": 8}


class OinkError(RuntimeError):
    pass


class Variable:
    def __init__(self, oink):
        self.oink = oink
        self.vars = {}   # name -> dict(style, data(list), which, offset, pad)
        self.rng = None

    # ------------------------------------------------------------------ set / next
    def set(self, args):
        if len(args) < 2:
            raise OinkError("Illegal variable command")
        name, style = args[0], args[1]
        if not all(c.isalnum() or c == "_" for c in name):
            raise OinkError("Variable name must be alphanumeric or underscore characters")
        if style == "delete":
            self.vars.pop(name, None)
            return
        if style in ("index", "loop", "world", "universe", "uloop") and name in self.vars:
            return
        uni = self.oink.universe
        if style == "index":
            if len(args) < 3:
                raise OinkError("Illegal variable command")
            v = dict(style=style, data=list(args[2:]), which=0, offset=0, pad=0)
        elif style == "loop":
            pad = 0
            rest = args[2:]
            if rest and rest[-1] == "pad":
                rest = rest[:-1]
                pad = 1
            if len(rest) == 1:
                first, last = 1, int(rest[0])
            elif len(rest) == 2:
                first, last = int(rest[0]), int(rest[1])
            else:
                raise OinkError("Illegal variable command")
            if last <= 0 or first > last:
                raise OinkError("Illegal variable command")
            v = dict(style=style, data=[None] * (last - first + 1), which=0, offset=first,
                     pad=len(str(last)) if pad else 0)
        elif style == "world":
            if len(args) - 2 != uni.nworlds:
                raise OinkError("World variable count doesn't match # of partitions")
            v = dict(style=style, data=list(args[2:]), which=uni.iworld, offset=0, pad=0)
        elif style in ("universe", "uloop"):
            if style == "universe":
                data = list(args[2:])
                pad = 0
            else:
                n = int(args[2])
                data = [None] * n
                pad = len(str(n)) if len(args) == 4 and args[3] == "pad" else 0
            if len(data) < uni.nworlds:
                raise OinkError("Universe/uloop variable count < # of partitions")
            v = dict(style=style, data=data, which=uni.iworld, offset=0 if style == "universe" else 1, pad=pad)
            if uni.me == 0:
                with open("tmp.oink.variable", "w") as f:
                    f.write(f"{uni.nworlds}\n")
        elif style in ("string", "equal"):
            if len(args) != 3:
                raise OinkError("Illegal variable command")
            if name in self.vars and self.vars[name]["style"] != style:
                raise OinkError("Cannot redefine variable as a different style")
            v = dict(style=style, data=[args[2]], which=0, offset=0, pad=0)
        else:
            raise OinkError("Illegal variable command")
        self.vars[name] = v

    def next(self, names):
        if not names:
            raise OinkError("Illegal next command")
        for n in names:
            if n not in self.vars:
                raise OinkError("Invalid variable in next command")
        style = self.vars[names[0]]["style"]
        if style in ("string", "equal", "world"):
            raise OinkError("Invalid variable style with next command")
        flag = 0
        if style in ("index", "loop"):
            for n in names:
                v = self.vars[n]
                v["which"] += 1
                if v["which"] >= len(v["data"]):
                    flag = 1
                    del self.vars[n]
        else:
            uni = self.oink.universe
            nxt = None
            if uni.world_me == 0:
                while True:
                    try:
                        os.rename("tmp.oink.variable", "tmp.oink.variable.lock")
                        break
                    except OSError:
                        time.sleep(0.1)
                with open("tmp.oink.variable.lock") as f:
                    nxt = int(f.read().split()[0])
                with open("tmp.oink.variable.lock", "w") as f:
                    f.write(f"{nxt + 1}\n")
                os.rename("tmp.oink.variable.lock", "tmp.oink.variable")
            nxt = self.oink.comm.bcast_object(nxt, 0)
            for n in names:
                v = self.vars[n]
                v["which"] = nxt
                if v["which"] >= len(v["data"]):
                    flag = 1
                    del self.vars[n]
        return flag

    # ------------------------------------------------------------------ retrieval
    def find(self, name):
        return name in self.vars

    def retrieve(self, name):
        v = self.vars.get(name)
        if v is None or v["which"] >= len(v["data"]):
            return None
        st = v["style"]
        if st in ("index", "world", "universe", "string"):
            return v["data"][v["which"]]
        if st in ("loop", "uloop"):
            val = v["which"] + v["offset"]
            return str(val).zfill(v["pad"]) if v["pad"] else str(val)
        # equal
        return "%.10g" % self.evaluate(v["data"][0])

    def retrieve_all(self, name):
        """every value of an index-style variable (used by -i v_name)"""
        v = self.vars[name]
        if v["style"] == "equal":
            raise OinkError("Command input is equal-style variable")
        if v["style"] in ("loop", "uloop"):
            return [str(i + v["offset"]) for i in range(len(v["data"]))]
        return list(v["data"])

    # ------------------------------------------------------------------ evaluator
    def evaluate(self, s: str) -> float:
        toks = self._tokenize(s)
        pos = [0]

        def peek():
            return toks[pos[0]] if pos[0] < len(toks) else ("END", None)

        def take():
            t = peek()
            pos[0] += 1
            return t

        argstack, opstack = [], []

        def apply(op):
            b = argstack.pop()
            if op == "NEG":
                argstack.append(-b)
                return
            if op == "!":
                argstack.append(1.0 if b == 0.0 else 0.0)
                return
            a = argstack.pop()
            r = {"+": lambda: a + b, "-": lambda: a - b, "*": lambda: a * b,
                 "/": lambda: a / b if b != 0 else self._err("Divide by 0 in variable formula"),
                 "^": lambda: (a ** b) if not (b == 0 and a == 0) else self._err("Power by 0 in variable formula"),
                 "==": lambda: float(a == b), "!=": lambda: float(a != b), "<": lambda: float(a < b),
                 "<=": lambda: float(a <= b), ">": lambda: float(a > b), ">=": lambda: float(a >= b),
                 "&": lambda: float(a != 0 and b != 0), "|": lambda: float(a != 0 or b != 0)}[op]()
            argstack.append(float(r))

        expect_arg = True
        while True:
            kind, val = take()
            if kind == "END":
                if expect_arg:
                    raise OinkError("Invalid syntax in variable formula")
                while opstack:
                    apply(opstack.pop())
                break
            if kind in ("NUM", "PAREN", "WORD"):
                if not expect_arg:
                    raise OinkError("Invalid syntax in variable formula")
                expect_arg = False
                if kind == "NUM":
                    argstack.append(val)
                elif kind == "PAREN":
                    argstack.append(self.evaluate(val))
                else:
                    argstack.append(self._word(val, toks, pos))
                continue
            op = val
            if expect_arg:
                if op == "-":
                    opstack.append("NEG")
                    continue
                if op == "!":
                    opstack.append("!")
                    continue
                raise OinkError("Invalid syntax in variable formula")
            while opstack and PREC[opstack[-1]] >= PREC[op] and not (op == "^" and opstack[-1] == "^" and False):
                apply(opstack.pop())
            opstack.append(op)
            expect_arg = True
        if len(argstack) != 1:
            raise OinkError("Invalid syntax in variable formula")
        return argstack[0]

    def _err(self, m):
        raise OinkError(m)

    def _tokenize(self, s):
        toks = []
        i, n = 0, len(s)
        while i < n:
            c = s[i]
            if c.isspace():
                i += 1
            elif c == "(":
                depth, j = 1, i + 1
                while j < n and depth:
                    depth += {"(": 1, ")": -1}.get(s[j], 0)
                    j += 1
                if depth:
                    raise OinkError("Invalid syntax in variable formula")
                toks.append(("PAREN", s[i + 1:j - 1]))
                i = j
            elif c.isdigit() or c == ".":
                j = i
                while j < n and (s[j].isdigit() or s[j] == "."):
                    j += 1
                if j < n and s[j] in "eE":
                    j += 1
                    if j < n and s[j] in "+-":
                        j += 1
                    while j < n and s[j].isdigit():
                        j += 1
                toks.append(("NUM", float(s[i:j])))
                i = j
            elif c.isalpha():
                j = i
                while j < n and (s[j].isalnum() or s[j] == "_"):
                    j += 1
                toks.append(("WORD", s[i:j]))
                i = j
            else:
                two = s[i:i + 2]
                if two in ("==", "!=", "<=", ">=", "&&", "||"):
                    toks.append(("OP", {"&&": "&", "||": "|"}.get(two, two)))
                    i += 2
                elif c in "+-*/^<>!&|":
                    toks.append(("OP", c))
                    i += 1
                elif c == "=":
                    toks.append(("OP", "=="))
                    i += 1
                else:
                    raise OinkError("Invalid syntax in variable formula")
        return toks

    def _word(self, w, toks, pos):
        if w.startswith("v_"):
            val = self.retrieve(w[2:])
            if val is None:
                raise OinkError("Invalid variable evaluation in variable formula")
            return float(val)
        if pos[0] < len(toks) and toks[pos[0]][0] == "PAREN":
            args = [self.evaluate(a) for a in _split_args(toks[pos[0]][1])]
            pos[0] += 1
            return self._math(w, args)
        if w == "PI":
            return math.pi
        if w == "nprocs":
            return float(self.oink.comm.size)
        if w == "time":
            return float(self.oink.deltatime)
        raise OinkError("Invalid math/group/special function in variable formula")

    def _math(self, w, a):
        def need(k):
            if len(a) != k:
                raise OinkError("Invalid math function in variable formula")
        if w in ("random", "normal"):
            need(3)
            if self.rng is None:
                seed = int(a[2])
                if seed <= 0:
                    raise OinkError("Invalid math function in variable formula")
                self.rng = random.Random(seed)
            if w == "random":
                return self.rng.random() * (a[1] - a[0]) + a[0]
            return a[0] + a[1] * self.rng.gauss(0.0, 1.0)
        if w == "atan2":
            need(2)
            return math.atan2(a[0], a[1])
        need(1)
        x = a[0]
        f = {"sqrt": math.sqrt, "exp": math.exp, "ln": math.log, "log": math.log10, "sin": math.sin,
             "cos": math.cos, "tan": math.tan, "asin": math.asin, "acos": math.acos, "atan": math.atan,
             "ceil": math.ceil, "floor": math.floor,
             "round": lambda v: math.ceil(v) if v - math.floor(v) >= 0.5 else math.floor(v)}.get(w)
        if f is None:
            raise OinkError("Invalid math function in variable formula")
        if (w == "sqrt" and x < 0) or (w in ("ln", "log") and x <= 0) or (w in ("asin", "acos") and abs(x) > 1):
            raise OinkError("Invalid math function in variable formula")
        return float(f(x))

    def evaluate_boolean(self, s: str) -> bool:
        """if-command conditions: numbers compared numerically, otherwise as strings"""
        for op in ("==", "!=", "<=", ">=", "<", ">"):
            if op in s:
                a, b = s.split(op, 1)
                a, b = a.strip(), b.strip()
                try:
                    x, y = float(a), float(b)
                except ValueError:
                    x, y = a, b
                return {"==": x == y, "!=": x != y, "<=": x <= y, ">=": x >= y, "<": x < y, ">": x > y}[op]
        return self.evaluate(s) != 0.0


def _split_args(s):
    out, depth, cur = [], 0, ""
    for c in s:
        if c == "," and depth == 0:
            out.append(cur)
            cur = ""
            continue
        depth += {"(": 1, ")": -1}.get(c, 0)
        cur += c
    out.append(cur)
    return out
