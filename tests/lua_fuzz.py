"""Random Lua 4 programs for the differential test of the native interpreter
(tests/test_lua_interp.py::test_lua_random_programs): a seeded generator of
expressions and statement blocks over numbers (complex included), strings,
tables, closures and the libraries, each program run as a MagDirFctn through
call(function() ... end, {}) by both the reference's liblua and xfk_lua.cpp.
Run directly (python tests/lua_fuzz.py N SEED) for a longer search."""
import random

NUMS = ["0", "1", "2", "3", "-1", "0.5", "-2.5", "1e3", "7", "x", "y", "theta", "R", "I", "PI", "pi", "(x+I*y)",
        "Complex(1, -2)", "-0", "1/3"]
STRS = ['"a"', '"abc"', '"10"', '"2.5"', '"x=1"', '""', '"hello world"', '" 12 "', '"AbC"', '"%d"']
UN = ["abs", "sin", "cos", "sqrt", "floor", "ceil", "exp", "deg", "rad", "arg", "re", "im", "conj", "tanh",
      "atan", "log10"]


class Gen:
    def __init__(self, rng):
        self.r = rng
        self.locals = []

    def num(self, d=0):
        r = self.r.random()
        if d > 3 or r < 0.3:
            c = self.r.choice(NUMS + self.locals) if self.locals and self.r.random() < 0.3 else self.r.choice(NUMS)
            return c
        if r < 0.55:
            op = self.r.choice(["+", "-", "*", "/", "^"])
            b = self.num(d + 1) if op != "^" else self.r.choice(["2", "3", "0.5", "-1", "2"])
            return "(%s %s %s)" % (self.num(d + 1), op, b)
        if r < 0.7:
            return "%s(%s)" % (self.r.choice(UN), self.num(d + 1))
        if r < 0.75:
            return "-%s" % self.num(d + 1)
        if r < 0.8:
            return "strlen(%s)" % self.str_(d + 1)
        if r < 0.85:
            return "tonumber(%s) or 0" % self.r.choice(STRS)
        if r < 0.9:
            return "getn(%s)" % self.table(d + 1)
        if r < 0.95:
            return "(%s %s %s and %s or %s)" % (self.num(d + 1), self.r.choice(["<", ">", "<=", ">=", "==", "~="]),
                                                 self.num(d + 1), self.num(d + 1), self.num(d + 1))
        return "mod(%s, %s)" % (self.num(d + 1), self.r.choice(["3", "7", "2.5"]))

    def str_(self, d=0):
        r = self.r.random()
        if d > 3 or r < 0.35:
            return self.r.choice(STRS)
        if r < 0.55:
            return "(%s .. %s)" % (self.str_(d + 1), self.r.choice([self.str_(d + 1), self.num(d + 1)]))
        if r < 0.65:
            return "strsub(%s, %s, %s)" % (self.str_(d + 1), self.r.choice(["1", "2", "-2", "0"]),
                                           self.r.choice(["-1", "3", "1", "10"]))
        if r < 0.72:
            return "strupper(%s)" % self.str_(d + 1)
        if r < 0.8:
            return 'format("%s", %s)' % (self.r.choice(["%5.2f", "%g", "%d", "%.3e", "%x", "%05.1f"]), self.num(d + 1))
        if r < 0.88:
            return "gsub(%s, %s, %s)" % (self.str_(d + 1), self.r.choice(['"a"', '"%d"', '"(%w)"', '"l+"', '""']),
                                         self.r.choice(['"<%1>"', '"-"', '"%0%0"', '"X"']))
        if r < 0.94:
            return "tostring(%s)" % self.num(d + 1)
        return "strrep(%s, %s)" % (self.str_(d + 1), self.r.choice(["0", "1", "3"]))

    def table(self, d=0):
        r = self.r.random()
        if r < 0.4:
            return "{%s}" % ", ".join(self.num(d + 1) for _ in range(self.r.randint(0, 5)))
        if r < 0.7:
            keys = self.r.sample(["a", "b", "c", "k1", "k2", "theta", "n", "x", "zz"], self.r.randint(1, 5))
            return "{%s}" % ", ".join("%s = %s" % (k, self.num(d + 1)) for k in keys)
        return "{%s; %s}" % (", ".join(self.num(d + 1) for _ in range(self.r.randint(1, 3))),
                             ", ".join("[%s] = %s" % (self.r.choice(['"p"', "10", "2.5", '"q"']), self.num(d + 1))
                                       for _ in range(self.r.randint(1, 3))))

    def block(self, depth=0, n=None):
        out = []
        for _ in range(n or self.r.randint(1, 4)):
            r = self.r.random()
            if r < 0.25 or not self.locals:
                v = "v%d" % len(self.locals)
                out.append("local %s = %s" % (v, self.num()))
                self.locals.append(v)
            elif r < 0.4:
                out.append("%s = %s" % (self.r.choice(self.locals), self.num()))
            elif r < 0.5 and depth < 2:
                i = "i%d" % depth
                out.append("for %s = %s, %s, %s do %s = %s + %s end" % (
                    i, self.r.choice(["1", "x", "-2"]), self.r.choice(["3", "5", "0", "y"]),
                    self.r.choice(["1", "2", "-1", "0.5"]), self.r.choice(self.locals), self.r.choice(self.locals),
                    i))
            elif r < 0.6 and depth < 2:
                t = self.table()
                acc = self.r.choice(self.locals)
                out.append("for kk, vv in %s do %s = %s * 1.5 + vv end" % (t, acc, acc))
            elif r < 0.7:
                out.append("if %s < %s then %s = %s else %s = %s end" % (
                    self.num(), self.num(), self.r.choice(self.locals), self.num(), self.r.choice(self.locals),
                    self.num()))
            elif r < 0.8:
                t = "t%d" % len(self.locals)
                out.append("local %s = %s tinsert(%s, %s) sort(%s, function(a, b) return re(a) < re(b) end)" % (
                    t, "{%s}" % ", ".join(self.num() for _ in range(self.r.randint(1, 6))), t, self.num(), t))
                acc = self.r.choice(self.locals)
                out.append("%s = %s[1] + getn(%s)" % (acc, t, t))
            elif r < 0.9:
                s = self.r.choice(self.locals)
                out.append("local f%d = function(a, b) return a * %%%s + (b or 1) end %s = f%d(%s)" % (
                    len(self.locals), s, s, len(self.locals), self.num()))
            else:
                v = self.r.choice(self.locals)
                out.append("local s_ = %s %s = %s + strlen(s_)" % (self.str_(), v, v))
        return " ".join(out)

    def program(self):
        self.locals = []
        body = self.block(n=self.r.randint(2, 6))
        ret = self.r.choice(self.locals) if self.locals else self.num()
        if self.r.random() < 0.3:
            ret = "%s + %s" % (ret, self.num())
        return "call(function() %s return %s end, {})" % (body, ret)


def programs(n, seed):
    g = Gen(random.Random(seed))
    return [g.program() for _ in range(n)]


if __name__ == "__main__":
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import numpy as np
    from oracle import oracle
    from test_lua_interp import same_bits
    from test_magdir import evaluate, mesh_sample
    from xfemm_amd import kernels
    n, seed = int(sys.argv[1]), int(sys.argv[2])
    p, x, y = mesh_sample(6, 3)
    bad = 0
    for e in programs(n, seed):
        ref = evaluate(oracle.ref_magdir, e, p, x, y, 0, 7.0)
        got = evaluate(kernels.magdir_eval, e, p, x, y, 0, 7.0)
        if isinstance(ref, str):
            ok = isinstance(got, str) and ref in got
        else:
            ok = not isinstance(got, str) and same_bits(ref, got)
        if not ok:
            bad += 1
            print("MISMATCH", e, "\n  ref", ref, "\n  got", got)
    print("%d programs, %d mismatches" % (n, bad))
