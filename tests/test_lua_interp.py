"""MagDirFctn beyond expressions: the native Lua 4 interpreter (xfk_lua.cpp)
against the reference's own liblua (oracle/_ref/libreflua.so, driven as
static2d.cpp:509-583 drives it: one interpreter for all elements, globals
persisting from element to element).  Host only, no GPU.

The bar is the same as tests/test_magdir.py: bit-identical angles for every
element.  The programs run statements through call() / dostring() (the chunk
itself is "return <MagDirFctn>"), build and traverse tables (traversal order is
the reference's hash-table order: floating sums in that order, key strings
concatenated in that order, the whole table of globals walked), close over
upvalues, take varargs, sort with and without comparators, match patterns,
format numbers, and carry state from one element to the next.  What the
interpreter refuses must be refused with a message naming the construct."""
import numpy as np
import pytest

from oracle import oracle
from xfemm_amd import kernels

from test_magdir import evaluate, mesh_sample

needs_lua = pytest.mark.skipif(not oracle.ref_lua_available(), reason="oracle/_ref/libreflua.so not built")

PROGRAMS = [
    # library functions the expression evaluator used to refuse
    'tonumber("5")*x', 'strlen("abc")*10', "getn({1,2})*x", 'tonumber("ff", 16) + x', 'tonumber("  12  ")',
    'tonumber("1e2") * y', 'tonumber("z") and 1 or 2', "type(x) == 'number' and theta or -theta",
    'strsub("hello", 2, -2) == "ell" and 1 or 0', 'strbyte("A") + strbyte("abc", -1)', 'strlen(strrep("ab", 3))',
    'strupper("abc") == "ABC" and strlower("XY") == "xy" and 5', 'strbyte(strchar(65, 66), 2)',
    'tostring(x)', 'tostring(theta) .. "0"', 'strlen(tostring(nil))', 'tostring("7") + 1',
    # patterns
    'strfind("hello world", "o w")', 'strfind("abc123def", "(%d+)")', 'strfind("abc", "b", 1, 1)',
    'strfind("  key = 42", "^%s*(%w+)%s*=%s*(%d+)")', 'strfind("(a(b)c)", "%b()")', 'strfind("aaa", "a-b")',
    'gsub("hello", "l", "L")', 'strlen(gsub("a,b,,c", ",", ";"))', 'gsub("abc", "%w", "%0%0")',
    'strlen(gsub("hello world", "(%w+)", "<%1>"))', 'gsub("x=1, y=2", "(%w+)=(%w+)", "%2=%1")',
    'gsub("abc", "", "-")', 'gsub("hello", "l+", function(s) return strlen(s) end)', 'strfind("a.b", ".", 1, 1)',
    'strfind("[x]", "[%[]")', 'strfind("f(1)", "%((%d)%)")', 'strfind("aXb", "%u")', 'strfind(" x", "%S")',
    'strfind("abcabc", "(abc)%1")', 'strfind("123", "^%d+$")', 'strfind("a1", "[^%a]")', 'strfind("z", "[a-y]")',
    # format
    'format("%5.2f", x)', 'format("%d", theta)', 'format("%x", 255) == "ff" and 1 or 0', 'format("%g", R)',
    'strlen(format("%q", "a\\"b\\n"))', 'format("%e", y)', 'format("%s%%", 12)', 'format("%3$s", 1, 2, 3)',
    'format("%-6.1f|", x)', 'strlen(format("%c", 66))', 'format("%.3s", "12345")', 'format("%05d", -3)',
    # tables, traversal order, getn / tinsert / tremove
    'call(function() local t = {} for i = 1, 20 do t[i] = i * x end local s = 0 for k, v in t do s = s + v end '
    'return s end, {})',
    'call(function() local t = {a = 1, b = 2, c = 3, theta = theta, [10] = y} local s = "" '
    'for k, v in t do s = s .. type(k) .. "." end return strbyte(s, 1) * 1000 + strlen(s) end, {})',
    'call(function() local t = {x, y, theta; n = 2} return getn(t) + t[3] end, {})',
    'call(function() local t = {1, 2, 3} tinsert(t, x) tinsert(t, 1, y) return t[1] + t[5] * getn(t) end, {})',
    'call(function() local t = {x, y, 3} local r = tremove(t, 1) return r + getn(t) + t.n end, {})',
    'call(function() local t = {} t[1.5] = x t[-3] = y t["k"] = 1 t[theta] = 2 local s = 0 '
    'for k, v in t do s = s * 3 + v end return s end, {})',
    'call(function() local t = {} for i = 1, 100 do t[i * 7 - 3] = i end for i = 1, 100, 3 do t[i * 7 - 3] = nil end '
    'local s = 0 local m = 1 for k, v in t do s = s + v * m m = m + 1 end return s end, {})',
    'call(function() local t = {} for i = 1, 70 do t[i] = i end local s = 0 for k, v in t do s = s * 1.01 + v end '
    'return s end, {})',
    'call(function() local t = {} for i = 1, 40 do t["k" .. i] = i end local s = 0 for k, v in t do '
    's = s * 1.01 + v end return s end, {})',
    'call(function() local s = 0 local k, v = next({a = 1}) return v + s end, {})',
    'call(function() local t = {10, 20, 30} local r = 0 foreachi(t, function(i, v) %t[i] = nil end) '
    'return getn(t) end, {})',
    'call(function() local t = {x, y, theta} return foreachi(t, function(i, v) if v > 0 then return i end end) '
    'or 0 end, {})',
    'call(function() local n = 0 foreach({a = 1, b = 2, c = 3}, function(k, v) n = (n or 0) + v end) return 1 end, {})',
    'rawget({5}, 1) + getn(rawset({}, 1, x))',
    # another table of globals (lua_setglobals), for the call and for the elements after it
    'call(function() local gl = globals local old = gl({x = 5, y = 2}) local v = x + y gl(old) return v end, {})',
    'call(function() if not done_ then local gl = globals local t = {} for k, v in gl() do t[k] = v end '
    't.done_ = 1 gl(t) end return x + (rawget(globals(), "done_") or 0) end, {})',
    "dofile('/nonexistent/xfemm/defs.lua') == nil and 3 or 4",
    "call(function() local a, b = dofile('/nonexistent/xfemm/defs.lua') return strlen(b) end, {})",
    # the whole table of globals, in the reference's hash order
    'call(function() acc = "" foreach(globals(), function(k, v) if type(v) == "function" then '
    'acc = acc .. strsub(k, 1, 1) end end) local h = 0 for i = 1, strlen(acc) do h = mod(h * 31 + strbyte(acc, i), '
    '1000003) end return h end, {})',
    'call(function() local n = 0 local k = nil repeat k = next(globals(), k) n = n + 1 until k == nil return n end, {})',
    # sort
    'call(function() local t = {5, 3, 8, 1, x, y, theta, -2, 9, 0, 4} sort(t) return t[1] + t[2] * 2 + t[11] * 3 end, {})',
    'call(function() local t = {x, y, theta, R, 1, 2, 3} sort(t, function(a, b) return a > b end) '
    'return t[1] * 10 + t[7] end, {})',
    'call(function() local t = {"pear", "apple", "fig", "kiwi"} sort(t) return strbyte(t[1]) + strbyte(t[4]) end, {})',
    'call(function() local t = {} for i = 1, 50 do t[i] = mod(i * 37, 17) + x end sort(t) local s = 0 '
    'for i = 1, 50 do s = s * 1.1 + t[i] end return s end, {})',
    'call(function() local t = {{k = 3}, {k = 1}, {k = 2}, {k = 1}} sort(t, function(a, b) return a.k < b.k end) '
    'return t[1].k + t[4].k * 10 end, {})',
    # closures, upvalues, varargs, methods, recursion
    'call(function() local a = x local f = function(b) return %a + b end return f(y) end, {})',
    'call(function() local f = function() return %theta end return f() end, {})',
    "call(function() return %y end, {})",
    'call(function(...) return arg.n + arg[1] * 2 end, {x, y, 3})',
    'call(function(a, b, ...) return a + b + arg.n end, {x, y})',
    'call(function() local o = {v = x} function o:get(k) return self.v * k end return o:get(2) end, {})',
    'call(function() local o = {v = y} function o.f(s, k) return s.v - k end return o:f(1) end, {})',
    'call(function() local function_ = nil fact = function(n) if n <= 1 then return 1 end return n * fact(n - 1) end '
    'return fact(10) + x end, {})',
    'call(function() local t = {1, 2} local a, b, c = unpack_(t) return a end, {}, "x") or 7',
    # control flow
    'call(function() local i = 0 repeat i = i + 1 until i > 5 while 1 do i = i + 1 if i > 10 then break end end '
    'return i * x end, {})',
    'call(function() local s = 0 for i = 10, 1, -2 do s = s + i end for i = 1, 0 do s = s + 100 end return s end, {})',
    'call(function() local s = 0 for i = x, x + 3 do s = s + i end return s end, {})',
    'call(function() local s = 0 for i = 1, 3, 0.5 do s = s + i end return s end, {})',
    'call(function() local s = "" for i = 1, 3 do s = s .. i end return s end, {})',
    'call(function() local a, b = 1 if b then return 1 elseif a then return 2 else return 3 end end, {})',
    'call(function() local a, b, c = 1, 2 return (c and 0 or 10) + a + b end, {})',
    'call(function() local a, b = x, y a, b = b, a return a - b end, {})',
    'call(function() local t = {1, 2} local i = 1 i, t[i] = i + 1, 20 return t[1] * 10 + t[2] + i end, {})',
    'call(function() local s = 0 for i = 1, 5 do if mod(i, 2) == 0 then s = s + i end end do local s = 99 end '
    'return s end, {})',
    'call(function() local t = {n = 0} local i = 0 while i < 30 do i = i + 1 tinsert(t, i * i) end return t.n end, {})',
    # complex numbers, the LuaInstance globals
    'Complex(1, 2) * x', 'im(Complex(x, y) * I)', 'pi * theta / 180', 'getcompatibilitymode() + 1',
    'arg(Complex(-1, -0) * x)', 're(sqrt(Complex(x, y)))', '"2" ^ 3 + x', '2 ^ "3"', 'abs(Complex(3, 4))',
    # the C library's generator (a fresh process: seed 1), reseeded
    "random()", "random(6)", "random(-3, 3) * theta", "call(function() randomseed(7) return random() end, {})",
    "call(function() if not s0 then randomseed(12345) s0 = 1 end return random(100) + random() end, {})",
    # state carried from element to element
    'call(function() cnt = (cnt or 0) + 1 return cnt end, {})',
    'call(function() last = (last or 0) * 0.5 + theta return last end, {})',
    'call(function() if not seen then seen = {} end tinsert(seen, x) return getn(seen) end, {})',
    'dostring("return " .. x .. " + 1")', 'dostring("k = (k or 0) + 1 return k")',
    'dostring("syntax error here")', 'dostring("error(\'boom\')")',
    'call(function() error("x") end, {}, "x") or 5', 'call(function() return nil + 1 end, {}, "x") or 6',
    'call(function() local a = {} return a.b.c end, {}, "x") or 8',
    # multiple values and their leak (the last value counts)
    'x, y, theta', 'strfind("abc", "b")', 'frexp(R)',
]


TAGM = [
    # tag methods (ltm.cpp, lvm.cpp): operator overloading on tagged tables,
    # `a - k` reaching the "add" method with -k (the ADDI peephole), index /
    # gettable / settable / function methods, getglobal / setglobal on nil,
    # numbers' pow replaced, the tag-0 fallback, copytagmethods
    'call(function() local tg = newtag() settagmethod(tg, "add", function(a, b, e) '
    'return (type(a) == "table" and a.v or a) * 1000 + (type(b) == "table" and b.v or b) + strlen(e) end) '
    'local t = settag({v = x}, tg) return (t + y) + (y + t) + (t - 1) + (t + 2) end, {})',
    'call(function() local tg = newtag() settagmethod(tg, "sub", function(a, b, e) return a.v - b * 3 end) '
    'settagmethod(tg, "mul", function(a, b) return 5 end) settagmethod(tg, "div", function(a, b) return b.v end) '
    'local t = settag({v = theta}, tg) return (t - y) + t * 2 + x / t end, {})',
    'call(function() local tg = newtag() settagmethod(tg, "unm", function(a, b, e) return a.v * 2 + (b and 1 or 0) end) '
    'return -settag({v = x}, tg) end, {})',
    'call(function() local tg = newtag() settagmethod(tg, "concat", function(a, b, e) '
    'return (type(a) == "string" and strlen(a) or 0) + (type(b) == "table" and b.v or 0) + strlen(e) end) '
    'local t = settag({v = y}, tg) return ("ab" .. t) + (t .. 5) end, {})',
    'call(function() local tg = newtag() settagmethod(tg, "lt", function(a, b) return a.v < b.v end) '
    'local p, q = settag({v = x}, tg), settag({v = y}, tg) '
    'return (p < q and 1 or 0) + (p > q and 2 or 0) + (p <= q and 4 or 0) + (p >= q and 8 or 0) end, {})',
    'call(function() local tg = newtag() settagmethod(tg, "index", function(t, k) return strlen(k) * 10 end) '
    'local t = settag({a = x}, tg) return t.abc + t.q + t.a end, {})',
    'call(function() settagmethod(tag({}), "index", function(t, k) return 7 end) local t = {} return t.zz + x end, {})',
    'call(function() local tg = newtag() settagmethod(tg, "gettable", function(t, k) return (rawget(t, k) or 99) + 1 end) '
    'settagmethod(tg, "settable", function(t, k, v) rawset(t, k, v * 2) end) '
    'local t = settag({}, tg) t.a = x t[3] = y return t.a + t[3] + t.nothing end, {})',
    'call(function() local tg = newtag() settagmethod(tg, "function", function(self, a, b) return a + b * self.v end) '
    'local t = settag({v = 3}, tg) return t(x, y) end, {})',
    'call(function() settagmethod(tag(nil), "getglobal", function(name, v) return strlen(name) end) '
    'return undefined_name_xyz + 1 end, {})',
    'call(function() settagmethod(tag(nil), "setglobal", function(name, old, new) rawset(globals(), name, new * 2) end) '
    'newglob_q = x return newglob_q end, {})',
    'call(function() settagmethod(tag(1), "pow", function(a, b, e) return a * 100 + b end) return x ^ 2 end, {})',
    'call(function() settagmethod(0, "add", function(a, b) return 42 end) return {} + {} end, {})',
    'call(function() local t1 = newtag() settagmethod(t1, "add", function(a, b) return b * 7 end) '
    'local t2 = copytagmethods(newtag(), t1) return settag({}, t2) + x end, {})',
    'call(function() return (gettagmethod(tag(1), "pow") == gettagmethod(tag(2), "pow") and 1 or 0) + '
    '(gettagmethod(newtag(), "add") == nil and 2 or 0) end, {})',
    'tag(x) + tag({}) * 10 + tag(print) * 100 + tag(nil) * 1000 + tag("s") * 10000 + tag(_STDOUT) * 100000',
    'call(function() tnew = tnew or newtag() return tnew end, {})',
    'call(function() local tg = newtag() local old = settagmethod(tg, "add", function() return 1 end) '
    'local old2 = settagmethod(tg, "add", nil) return (old == nil and 1 or 0) + (type(old2) == "function" and 2 or 0) '
    '+ (gettagmethod(tg, "add") == nil and 4 or 0) end, {})',
]
PROGRAMS = PROGRAMS + TAGM

# Lua errors (the reference's message) and non-numeric results
BAD = ['call(function() error("x") end, {})', 'dostring("return")', 'call(function() return {} end, {})',
       "getn(5)", 'strsub("a")', 'format("%y", 1)', 'strrep("a")', 'sort({1, "a"})', "{1, a = 2}",
       'call(function() local t = {} t[nil] = 1 end, {})', "nil .. 1", 'tonumber("1", 99)', "%x",
       "function() end", 'call(function() for i = 1, "a" do end end, {})',
       'call(function() for k, v in 5 do end end, {})', "next({}, 1)", "tinsert(nil, 1)", 'strfind("a", "(")',
       'strfind("a", "%")', 'gsub("a", "a", {})', "foreach({}, 5)", "call(5, {})", "assert(nil)",
       'format("%d", "z")', "x = 1", "return 1", "1 1",
       'settagmethod(tag(1), "add", print)', "settag({}, 3)", 'settagmethod(tag({}), "gc", print)',
       'settagmethod(newtag(), "le", print)', 'gettagmethod(99, "add")', 'settagmethod(newtag(), "foo", print)',
       'settagmethod(newtag(), "add")', 'settagmethod(newtag(), "add", 5)', "settag(5, newtag())",
       "call(function() local t = {} return t + 1 end, {})"]

UNSUPPORTED = ['dofile()', 'openfile("x", "r")',
               "femmVersion()", 'call(function() return 1 end, {}, "", print)', "gcinfo()",
               'call(function() g = function(n) return g(n + 1) end return g(1) end, {})',
               'writeto("x")', 'date()']


def same_bits(ref, got):
    """Bit-identical, except that a NaN matches any NaN: which operand's NaN
    an SSE instruction propagates follows the compiler's operand order, so
    the sign of a NaN (the text "nan" / "-nan") is not pinned."""
    ref, got = np.asarray(ref), np.asarray(got)
    if ref.shape != got.shape:
        return False
    nan = np.isnan(ref)
    return bool((nan == np.isnan(got)).all() and np.array_equal(ref[~nan].view(np.int64), got[~nan].view(np.int64)))


def compare(e, lu=0, n=400, seed=1):
    p, x, y = mesh_sample(n, seed)
    ref = evaluate(oracle.ref_magdir, e, p, x, y, lu, 7.0)
    got = evaluate(kernels.magdir_eval, e, p, x, y, lu, 7.0)
    return ref, got


@needs_lua
@pytest.mark.parametrize("lu", [0, 3])
def test_lua_programs_bit_identical_to_reference(lu):
    bad = []
    for e in PROGRAMS:
        ref, got = compare(e, lu)
        if isinstance(ref, str):
            if not (isinstance(got, str) and ref in got):
                bad.append((e, ref, got))
            continue
        if isinstance(got, str) or not same_bits(ref, got):
            bad.append((e, ref[:3], got if isinstance(got, str) else got[:3]))
    assert not bad, bad


@needs_lua
def test_lua_errors_carry_the_reference_message():
    for e in BAD:
        ref, got = compare(e, 0, 20)
        assert isinstance(ref, str) and isinstance(got, str), (e, ref, got)
        assert ref in got, (e, ref, got)


@needs_lua
@pytest.mark.parametrize("e", UNSUPPORTED)
def test_lua_unsupported_is_named(e):
    """What the interpreter refuses (xfk_lua.h): a message naming it, never a
    Lua error or a silent value."""
    got = evaluate(kernels.magdir_eval, e, *mesh_sample(4), 0, 0.0)
    assert isinstance(got, str) and "not supported by the native Lua interpreter" in got, (e, got)
    assert "Lua error occurred" not in got


@needs_lua
def test_lua_state_persists_across_many_elements():
    """A counter and a growing table over 5000 elements: the globals carry
    from element to element as in the reference's one interpreter (and the
    collector between elements keeps what is reachable)."""
    e = ('call(function() cnt = (cnt or 0) + 1 if not acc then acc = {} end acc[mod(cnt, 97)] = '
         'strrep("x", mod(cnt, 7)) local s = 0 for k, v in acc do s = s + strlen(v) * k end return s + cnt end, {})')
    ref, got = compare(e, 0, 5000, 3)
    assert not isinstance(ref, str) and not isinstance(got, str), (ref, got)
    assert same_bits(ref, got)


@needs_lua
def test_lua_leaked_values_within_the_stack():
    """A chunk returning two values leaves one on the reference's stack per
    element: fine up to 3000 (the reference's 4096-slot stack holds them),
    refused beyond (it overflows near 4096)."""
    ref, got = compare("theta, R", 0, 2500, 5)
    assert same_bits(ref, got)
    got = evaluate(kernels.magdir_eval, "theta, R", *mesh_sample(3500, 5), 0, 0.0)
    assert isinstance(got, str) and "not supported" in got


GLOBAL_WALK = ('call(function() local h = 0 local k = nil repeat k = next(globals(), k) if type(k) == "string" then '
               'h = mod(h * 31 + strbyte(k, 1), 1000003) end until k == nil return h end, {})')


@needs_lua
@pytest.mark.parametrize("axi", [False, True])
def test_lua_problem_loop_shares_one_interpreter(axi):
    """A problem's element loop (xfk_magdir_eval_labels, what problem
    creation runs): three labels interleaved, one interpreter -- label 2 reads
    the counter label 0 keeps, label 1 has no function; the axisymmetric chunk
    sets r and z first, which the walk over the table of globals sees."""
    p, x, y = mesh_sample(600, 7)
    n = len(p)
    lbl = (np.arange(n) % 4).astype(np.int32)
    fctns = ['call(function() cnt = (cnt or 0) + 1 return cnt + theta end, {})', None, "cnt * 2 + r", GLOBAL_WALK]
    md = [1.0, 2.0, 3.0, 4.0]
    ref = oracle.ref_magdir_labels(fctns, md, p, lbl, x, y, 2, axi)
    got = kernels.magdir_eval_labels(fctns, md, p, lbl, x, y, 2, axi)
    assert same_bits(ref, got)
    assert (got[lbl == 1] == 2.0).all()


@needs_lua
def test_lua_nonlinear_problem_refuses_stateful_chunks():
    """A nonlinear problem re-runs the element loop every Newton pass: a
    chunk that changes state, or leaves values on the stack, would give other
    angles (or a stack overflow) in later passes -- refused, not silently
    evaluated once; a pure chunk is the same every pass and runs."""
    p, x, y = mesh_sample(50, 2)
    lbl = np.zeros(len(p), np.int32)
    for f in ['call(function() cnt = (cnt or 0) + 1 return cnt end, {})', "theta, R",
              'call(function() setcompatibilitymode(1) return 1 end, {})', "random() * 360"]:
        with pytest.raises(kernels.XfkError, match="not supported"):
            kernels.magdir_eval_labels([f], [0.0], p, lbl, x, y, 0, False, True)
        kernels.magdir_eval_labels([f], [0.0], p, lbl, x, y, 0, False, False)
    pure = 'call(function() local t = {x, y} local s = 0 for k, v in t do s = s + v end return s end, {})'
    ref = oracle.ref_magdir_labels([pure], [0.0], p, lbl, x, y, 0)
    got = kernels.magdir_eval_labels([pure], [0.0], p, lbl, x, y, 0, False, True)
    assert same_bits(ref, got)


@needs_lua
@pytest.mark.parametrize("seed", [11, 12])
def test_lua_random_programs(seed):
    """Seeded random programs (tests/lua_fuzz.py: locals, loops over ranges
    and tables, closures with upvalues, sort with a comparator, string and
    format functions, complex arithmetic) -- the same angles, or the same
    error, as the reference's liblua."""
    import lua_fuzz
    p, x, y = mesh_sample(6, 3)
    bad = []
    for e in lua_fuzz.programs(300, seed):
        ref = evaluate(oracle.ref_magdir, e, p, x, y, 0, 7.0)
        got = evaluate(kernels.magdir_eval, e, p, x, y, 0, 7.0)
        if isinstance(ref, str):
            ok = isinstance(got, str) and ref in got
        else:
            ok = not isinstance(got, str) and same_bits(ref, got)
        if not ok:
            bad.append((e, ref, got))
    assert not bad, bad[:3]


@needs_lua
def test_lua_dofile_runs_a_file(tmp_path):
    """dofile: the chunk in the file runs on the same interpreter (its globals
    stay), its results are dofile's; a syntax error in it gives nil and
    "syntax error"; a missing file nil and "file error"."""
    defs = tmp_path / "defs.lua"
    defs.write_text("k_ = (k_ or 0) + 1\nfunction ang(t) return t * 2 + k_ end\nreturn 7, 8\n")
    bad = tmp_path / "bad.lua"
    bad.write_text("x = = 1\n")
    for e in ['call(function() dofile("%s") return ang(theta) end, {})' % defs,
              'call(function() local a, b = dofile("%s") return a * 10 + b end, {})' % defs,
              'call(function() local a, b = dofile("%s") return (a == nil and 1 or 0) + strlen(b) end, {})' % bad]:
        ref, got = compare(e, 0, 50, 4)
        assert not isinstance(ref, str) and not isinstance(got, str), (e, ref, got)
        assert same_bits(ref, got), e
