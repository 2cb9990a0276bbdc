// xfk_lua.cpp -- Lua 4.0 with xfemm's complex numbers, restated for the
// magnetisation-direction functions (see xfk_lua.h for what and why).
//
// Sources restated (temudschin/xfemm @ 2025-02-04, cfemm/libfemm/liblua):
// llex.cpp (tokens), lparser.cpp (grammar, scoping, upvalues, constructors),
// lcode.cpp (the numeric peepholes that change a value: PUSHINT / PUSHNEGNUM
// constants, `-k` folding, `a - k` as ADDI), lvm.cpp (operations, for loops,
// SETLIST / SETMAP order), ldo.cpp (calls, varargs), ltable.cpp (the hash
// table), lstring.cpp (string hash), lobject.cpp (number <-> text),
// lapi.cpp (lua_getn), lbaselib.cpp, lstrlib.cpp, lmathlib.cpp,
// femmcomplex.cpp, LuaInstance.cpp.  Line numbers below are of those files.
#include "xfk_lua.h"

#include <cctype>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

namespace xfk {
namespace lua {

// ===========================================================================
// CComplex arithmetic (femmcomplex.cpp; line numbers of that file)
// ===========================================================================
namespace {

const double kPi = 3.141592653589793238462643383;            // femmconstants.h
const double kRadPerDeg = 3.14159265358979323846 / 180.0;    // lmathlib.cpp:18-19

inline Cx add(Cx a, Cx b) { return {a.re + b.re, a.im + b.im}; }                                  // :249-252
inline Cx sub(Cx a, Cx b) { return {a.re - b.re, a.im - b.im}; }                                  // :302-305
inline Cx mul(Cx a, Cx b) { return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }      // :355-358
inline Cx neg(Cx a) { return {-a.re, -a.im}; }                                                    // :256-259
inline Cx scale(Cx a, double d) { return {a.re * d, a.im * d}; }                                  // :323-326
inline Cx divd(Cx a, double d) { return {a.re / d, a.im / d}; }                                   // :388-391
inline Cx ipart(double l) { return {0.0 * l, 1.0 * l}; }                 // I * double (:323 on I)
inline Cx dminus(double d, Cx y) { return {d - y.re, -y.im}; }                                    // :297-300
inline Cx dplus(double d, Cx y) { return {d + y.re, y.im}; }                                      // :244-247

inline Cx recip(Cx z)   // the factor y of operator/ (:461-471)
{
    Cx y;
    if (std::fabs(z.re) > std::fabs(z.im)) {
        const double c = z.im / z.re;
        y.re = 1. / (z.re * (1. + c * c));
        y.im = (-c) * y.re;
    } else {
        const double c = z.re / z.im;
        y.im = (-1.) / (z.im * (1. + c * c));
        y.re = (-c) * y.im;
    }
    return y;
}
inline Cx cdiv(Cx x, Cx z) { return mul(x, recip(z)); }                                           // :456-474

double cabs_(Cx x)   // :749-757
{
    if (x.re == 0 && x.im == 0) return 0.;
    if (std::fabs(x.re) > std::fabs(x.im)) return std::fabs(x.re) * std::sqrt(1. + (x.im / x.re) * (x.im / x.re));
    return std::fabs(x.im) * std::sqrt(1. + (x.re / x.im) * (x.re / x.im));
}

double carg(Cx x)   // :764-769
{
    if (x.re == 0 && x.im == 0) return 0.;
    return std::atan2(x.im, x.re);
}

Cx cexp(Cx x)   // :622-634
{
    const double e = std::exp(x.re);
    double s, c;
    sincos(x.im, &s, &c);
    return {c * e, s * e};
}

Cx csqrt(Cx x)   // :636-673
{
    double w, z;
    if (x.re == 0 && x.im == 0) w = 0;
    else if (std::fabs(x.re) > std::fabs(x.im)) {
        z = x.im / x.re;
        w = std::sqrt(std::fabs(x.re)) * std::sqrt((1. + std::sqrt(1. + z * z)) / 2.);
    } else {
        z = x.re / x.im;
        w = std::sqrt(std::fabs(x.im)) * std::sqrt((std::fabs(z) + std::sqrt(1. + z * z)) / 2.);
    }
    if (w == 0) return {0, 0};
    if (x.re >= 0) return {w, x.im / (2. * w)};
    if (x.im >= 0) return {std::fabs(x.im) / (2. * w), w};
    return {std::fabs(x.im) / (2. * w), -w};
}

Cx clog(Cx x) { return {std::log(cabs_(x)), carg(x)}; }   // :771-779

const Cx kI = {0, 1};
const Cx kMinusI = {-0.0, -1};   // -I (member unary minus on I)

Cx csin(Cx x) { return cdiv(sub(cexp(mul(kI, x)), cexp(mul(kMinusI, x))), Cx{0., 2.}); }   // :715-718
Cx ccos(Cx x) { return divd(add(cexp(mul(kI, x)), cexp(mul(kMinusI, x))), 2.); }         // :700-703
Cx ctan(Cx x) { return cdiv(csin(x), ccos(x)); }                                          // :730-733

Cx asin_w(Cx x) { return add(mul(kI, x), csqrt(Cx{1.0 - mul(x, x).re, -mul(x, x).im})); }   // I x + sqrt(1 - x x)

Cx casin(Cx x)   // :720-728
{
    const Cx w = asin_w(x);
    if (x.im == 0 && x.re <= 1 && x.re >= -1) return {carg(w), 0.};
    return dminus(carg(w), ipart(std::log(cabs_(w))));
}

Cx cacos(Cx x)   // :705-713
{
    const Cx w = asin_w(x);
    if (x.im == 0 && x.re <= 1 && x.re >= -1) return {kPi / 2. - carg(w), 0.};
    return dplus(kPi / 2. - carg(w), ipart(std::log(cabs_(w))));
}

Cx catan(Cx x)   // :735-740
{
    if (x.im == 0) return {std::atan(x.re), 0.};
    const Cx ix = mul(kI, x);
    const Cx a = {1.0 + ix.re, ix.im}, b = {1.0 - ix.re, -ix.im};
    const double d = carg(a) - carg(b);
    return divd(dminus(d, ipart(std::log(cabs_(a) / cabs_(b)))), 2.);
}

Cx catan2(Cx y, Cx x)   // :742-747
{
    if (y.im == 0 && x.im == 0) return {std::atan2(y.re, x.re), 0.};
    const Cx xy = add(x, mul(kI, y));
    const Cx s = add(mul(x, x), mul(y, y));
    const double a = carg(cdiv(xy, csqrt(s)));
    return dminus(a, ipart(std::log(cabs_(xy) / std::sqrt(cabs_(s)))));
}

Cx csinh(Cx x) { return divd(sub(cexp(x), cexp(neg(x))), 2.); }   // :689-692
Cx ccosh(Cx x) { return divd(add(cexp(x), cexp(neg(x))), 2.); }   // :694-697

Cx ctanh(Cx x)   // :675-687
{
    if (x.re > 0) {
        const Cx e = cexp(scale(x, -2.0));
        return cdiv(Cx{1.0 - e.re, -e.im}, Cx{1.0 + e.re, e.im});
    }
    const Cx e = cexp(scale(x, 2.0));
    return cdiv(Cx{e.re - 1.0, e.im}, Cx{e.re + 1.0, e.im});
}

Cx cpow_int(Cx x, long long y)   // :781-799
{
    if (y == 0) return {1, 0};
    Cx z;
    if (y > 0) {
        z = x;
        for (long long i = 1; i < y; ++i) z = mul(z, x);
    } else {
        z = scale(recip(x), 1.0);
        const Cx w = z;
        for (long long i = 1; i < -y; ++i) z = mul(z, w);
    }
    return z;
}

// double -> long / int as x86-64's cvttsd2si (the reference's `(long)` and
// `(int)` casts): out of range and NaN give the minimum
inline long to_long(double d)
{
    if (!(d > -9223372036854775808.0 - 1.0 && d < 9223372036854775808.0)) return LONG_MIN;
    return (long)d;
}
inline int to_int(double d)
{
    if (!(d > -2147483649.0 && d < 2147483648.0)) return INT_MIN;
    return (int)d;
}

// ===========================================================================
// numbers <-> text (lobject.cpp, femmcomplex.cpp)
// ===========================================================================
// lua_number2str (lobject.cpp:228-232) = CComplex::ToString (femmcomplex.cpp:150-176)
std::string number2str(Cx n)
{
    char s[256];
    const double re = n.re, im = n.im;
    if (im == 0) std::snprintf(s, sizeof s, "%.16g", re);
    else if (im == 1) {
        if (re == 0) std::snprintf(s, sizeof s, "I");
        else std::snprintf(s, sizeof s, "%.16g+I", re);
    } else if (im == -1) {
        if (re == 0) std::snprintf(s, sizeof s, "-I");
        else std::snprintf(s, sizeof s, "%.16g-I", re);
    } else if (im < 0) {
        if (re != 0) std::snprintf(s, sizeof s, "%.16g-I*%.16g", re, std::fabs(im));
        else std::snprintf(s, sizeof s, "-I*%.16g", std::fabs(im));
    } else if (im > 0) {
        if (re != 0) std::snprintf(s, sizeof s, "%.16g+I*%.16g", re, im);
        else std::snprintf(s, sizeof s, "I*%.16g", im);
    } else s[0] = '\0';   // a NaN imaginary part: ToString leaves the text empty
    return s;
}

// luaO_str2d (lobject.cpp:138-147) over lua_str2number (:78-136), which also
// reads the "a+I*b" forms
bool str2d(const char *s, Cx *out)
{
    char *q;
    Cx x{0., 0.};
    x.re = std::strtod(s, &q);
    const char *end = q;
    if (q[0] != '\0') {
        char *e2;
        if (std::strcmp(q, "I") == 0) { x.im = 1; end = q + 1; }
        else if (std::strcmp(q, "+I") == 0) { x.im = 1; end = q + 2; }
        else if (std::strcmp(q, "-I") == 0) { x.im = -1; end = q + 2; }
        else if (std::strncmp(q, "I*", 2) == 0) { x.im = std::strtod(q + 2, &e2); end = e2; }
        else if (std::strncmp(q, "+I*", 3) == 0) { x.im = std::strtod(q + 3, &e2); end = e2; }
        else if (std::strncmp(q, "-I*", 3) == 0) { x.im = -std::strtod(q + 3, &e2); end = e2; }
    }
    if (end == s) return false;
    while (std::isspace((unsigned char)*end)) ++end;
    if (*end != '\0') return false;
    *out = x;
    return true;
}

// ===========================================================================
// values and objects
// ===========================================================================
enum Tag : uint8_t { TUD = 0, TNIL = 1, TNUM = 2, TSTR = 3, TTAB = 4, TFUN = 5 };   // lua.h:76-81
const char *const kTypeName[] = {"userdata", "nil", "number", "string", "table", "function"};   // ltm.cpp

struct Obj {
    Obj *gcnext = nullptr;
    bool mark = false;
    bool fixed = false;   // a compiled constant: never collected
    virtual ~Obj() {}
};

struct StrObj : Obj {
    std::string s;
    unsigned long hash = 0;
};

struct Value {
    Tag t = TNIL;
    Cx n{0., 0.};
    Obj *o = nullptr;
};

struct Node {
    Value key, val;
    int next = -1;
};

struct TableObj : Obj {
    std::vector<Node> node;
    int firstfree = 0;
    int htag = TTAB;        // settag()
    long long epoch = 0;   // the element whose run created it
};

struct Proto;
typedef void (*Builtin)(Interp &, std::vector<Value> &, std::vector<Value> &);

struct FuncObj : Obj {
    const Proto *p = nullptr;   // a Lua function, or
    Builtin c = nullptr;        // a library function
    const char *name = "";      // (library functions: for messages)
    std::vector<Value> up;      // Lua 4 upvalues: values captured at closure time
};

struct UdObj : Obj {
    const void *ptr = nullptr;
    int tag = 0;
};

inline Value nil() { return Value(); }
inline Value num(Cx c) { Value v; v.t = TNUM; v.n = c; return v; }
inline Value num(double d) { return num(Cx{d, 0.}); }
inline const std::string &sv(const Value &v) { return static_cast<StrObj *>(v.o)->s; }
inline TableObj *tv(const Value &v) { return static_cast<TableObj *>(v.o); }
inline FuncObj *fv(const Value &v) { return static_cast<FuncObj *>(v.o); }

// lstring.cpp:51-58
unsigned long hash_s(const char *s, size_t l)
{
    unsigned long h = l;
    const size_t step = (l >> 5) | 1;
    for (; l >= step; l -= step) h = h ^ ((h << 5) + (h >> 2) + (unsigned char)*(s++));
    return h;
}

// luaO_equalObj (lobject.cpp:45-63)
bool raweq(const Value &a, const Value &b)
{
    if (a.t != b.t) return false;
    switch (a.t) {
    case TNIL: return true;
    case TNUM: return a.n.re == b.n.re && a.n.im == b.n.im;
    case TSTR: return a.o == b.o || sv(a) == sv(b);
    case TUD: {
        const UdObj *x = static_cast<const UdObj *>(a.o), *y = static_cast<const UdObj *>(b.o);
        return x == y || (x->ptr == y->ptr && x->tag == y->tag);
    }
    default: return a.o == b.o;
    }
}

// run-time and syntax errors (what lua_dostring / call / dostring see)
struct LuaError {
    int status;   // 1 LUA_ERRRUN, 3 LUA_ERRSYNTAX
    std::string msg;
};
[[noreturn]] void rt_error(const std::string &m) { throw LuaError{1, m}; }

// tag-method events (ltm.h ORDER TM; ltm.cpp:14-20)
enum TMS { TM_GETTABLE, TM_SETTABLE, TM_INDEX, TM_GETGLOBAL, TM_SETGLOBAL, TM_ADD, TM_SUB, TM_MUL, TM_DIV, TM_POW,
           TM_UNM, TM_LT, TM_CONCAT, TM_GC, TM_FUNCTION, TM_N };
const char *const kEventName[] = {"gettable", "settable", "index", "getglobal", "setglobal", "add", "sub", "mul",
                                  "div", "pow", "unm", "lt", "concat", "gc", "function", "le", "gt", "ge"};
const int kNumTags = 6;   // NUM_TAGS
// luaT_validevents (ltm.cpp:52-60), ORDER LUA_T x ORDER TM
const char kValidEvents[kNumTags][TM_N] = {
    {1, 1, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 0, 1},   // userdata
    {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1},   // nil
    {1, 1, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1},   // number
    {1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1},   // string
    {0, 0, 1, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 0, 1},   // table
    {1, 1, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0}};  // function
inline bool valid_event(int t, int e) { return t >= kNumTags || kValidEvents[t][e]; }

// ===========================================================================
// tables: the chained scatter table of ltable.cpp
// ===========================================================================
// luaH_mainposition (ltable.cpp:42-67); -1 for a nil key
int mainpos(const TableObj *t, const Value &k)
{
    uintptr_t h;
    switch (k.t) {
    case TNUM: h = (uintptr_t)to_long(k.n.re); break;
    case TSTR: h = static_cast<const StrObj *>(k.o)->hash; break;
    case TUD: case TTAB: case TFUN: h = (unsigned int)((size_t)k.o & UINT_MAX); break;   // IntPoint (llimits.h:64)
    default: return -1;
    }
    return (int)(h & (uintptr_t)(t->node.size() - 1));
}

// luaH_get (ltable.cpp:70-125): the node of key k, or -1 (not present)
int tfind(const TableObj *t, const Value &k)
{
    const int mp = mainpos(t, k);
    if (mp < 0) rt_error("table index is nil");
    int n = mp;
    do {
        if (raweq(k, t->node[n].key)) return n;
        n = t->node[n].next;
    } while (n >= 0);
    return -1;
}
Value *tget(TableObj *t, const Value &k)
{
    const int n = tfind(t, k);
    return n < 0 ? nullptr : &t->node[n].val;
}

void setnodevector(TableObj *t, long long size)   // ltable.cpp:184-198
{
    if (size > INT_MAX) rt_error("table overflow");
    t->node.assign((size_t)size, Node());
    t->firstfree = (int)size - 1;
}

int power2(long long n)   // luaO_power2 (lobject.cpp:37-42)
{
    long long p = 4;   // MINPOWER2
    while (p <= n) p <<= 1;
    return (int)p;
}

Value *tset(TableObj *t, const Value &k);

void rehash(TableObj *t)   // ltable.cpp:237-262
{
    const int oldsize = (int)t->node.size();
    std::vector<Node> nold;
    nold.swap(t->node);
    int nelems = 0;
    for (const Node &n : nold)
        if (n.val.t != TNIL) ++nelems;
    if (nelems >= oldsize - oldsize / 4) setnodevector(t, (long long)oldsize * 2);
    else if (nelems <= oldsize / 4 && oldsize > 4) setnodevector(t, oldsize / 2);
    else setnodevector(t, oldsize);
    for (int i = 0; i < oldsize; ++i)
        if (nold[i].val.t != TNIL) *tset(t, nold[i].key) = nold[i].val;
}

// luaH_set (ltable.cpp:273-316): the value slot of k, inserted if absent
Value *tset(TableObj *t, const Value &k)
{
    int mp = mainpos(t, k);
    if (mp < 0) rt_error("table index is nil");
    int n = mp;
    do {
        if (raweq(k, t->node[n].key)) return &t->node[n].val;
        n = t->node[n].next;
    } while (n >= 0);
    std::vector<Node> &N = t->node;
    if (N[mp].key.t != TNIL) {   // main position taken
        n = t->firstfree;
        int othern;
        if (mp > n && (othern = mainpos(t, N[mp].key)) != mp) {
            // the colliding node is out of its main position: move it
            while (N[othern].next != mp) othern = N[othern].next;
            N[othern].next = n;
            N[n] = N[mp];
            N[mp].next = -1;
        } else {   // the new key goes to the free position
            N[n].next = N[mp].next;
            N[mp].next = n;
            mp = n;
        }
    }
    N[mp].key = k;
    for (;;) {   // correct firstfree
        if (N[t->firstfree].key.t == TNIL) return &N[mp].val;
        if (t->firstfree == 0) break;
        --t->firstfree;
    }
    rehash(t);
    return tset(t, k);
}

// luaH_next (ltable.cpp:128-150): the next node with a value, or -1
int tnext(TableObj *t, const Value &k)
{
    int i = 0;
    if (k.t != TNIL) {
        const int n = tfind(t, k);
        if (n < 0) rt_error("invalid key for `next'");
        i = n + 1;
    }
    for (; i < (int)t->node.size(); ++i)
        if (t->node[i].val.t != TNIL) return i;
    return -1;
}

// ===========================================================================
// syntax tree
// ===========================================================================
enum ExprKind {
    X_NIL, X_INT, X_NUM, X_NEGNUM, X_STR, X_LOCAL, X_GLOBAL, X_UPVAL, X_INDEX, X_CALL, X_METHOD, X_FUNC,
    X_TABLE, X_UNM, X_NOT, X_BIN, X_AND, X_OR
};
enum BinOp { B_ADD, B_SUB, B_MUL, B_DIV, B_POW, B_CONCAT, B_NE, B_EQ, B_LT, B_LE, B_GT, B_GE, B_AND, B_OR, B_NONE };

struct Expr {
    ExprKind k;
    int op = 0;             // X_INT constant; X_LOCAL slot; X_UPVAL index; X_BIN operator; X_FUNC proto
    double v = 0;           // X_NUM / X_NEGNUM constant
    Value s;                // X_STR constant; X_GLOBAL / X_METHOD name
    Expr *a = nullptr, *b = nullptr;   // operands; X_INDEX table / key; X_CALL function; X_METHOD object
    std::vector<Expr *> list;          // call arguments; constructor list items
    std::vector<std::pair<Expr *, Expr *>> rec;   // constructor record items
    bool rec_first = false;            // constructor: the record part is written first
    int nelems = 0;                    // constructor: CREATETABLE's size
};

enum StatKind { S_LOCAL, S_ASSIGN, S_CALL, S_IF, S_WHILE, S_REPEAT, S_FORNUM, S_FORIN, S_DO, S_RETURN, S_BREAK };

struct Target {
    int kind = 0;   // 0 local, 1 global, 2 indexed
    int slot = 0;
    Value name;
    Expr *obj = nullptr, *key = nullptr;
};

struct Block;
struct Stat {
    StatKind k;
    int slot = 0, nvars = 0;
    std::vector<Expr *> exprs;       // right-hand sides / return list / call
    std::vector<Target> targets;
    std::vector<Expr *> conds;       // if / elseif conditions; while / repeat condition
    std::vector<Block *> blocks;     // their blocks (+ else); loop body
};

struct Block {
    std::vector<Stat *> stats;
};

struct UpDesc {
    bool global;
    int slot;
    Value name;
};

struct Chunk;
struct Proto {
    const Chunk *owner = nullptr;
    int nparams = 0;
    bool vararg = false;
    int maxslots = 0;
    std::vector<UpDesc> ups;
    Block *body = nullptr;
};

// everything one compiled chunk owns
struct Chunk {
    std::vector<std::unique_ptr<Expr>> exprs;
    std::vector<std::unique_ptr<Stat>> stats;
    std::vector<std::unique_ptr<Block>> blocks;
    std::vector<std::unique_ptr<Proto>> protos;   // [0]: the main function
    std::vector<std::unique_ptr<StrObj>> consts;
    std::map<std::string, StrObj *> const_index;
};

}  // namespace

// ===========================================================================
// the interpreter state
// ===========================================================================
struct Interp {
    bool axi;
    Obj *gclist = nullptr;
    long long nobjs = 0, gc_at = 200000;
    TableObj *G = nullptr;                 // the table of globals
    std::vector<Value> leaked;             // values left on the reference's stack
    std::map<std::string, std::unique_ptr<Chunk>> chunks;   // compiled texts
    Value errormessage_fn, alert_fn, tostring_name;          // the library's own _ERRORMESSAGE / _ALERT
    UdObj *null_ud = nullptr;
    long long epoch = 0;                   // the running element (tables record it)
    bool changed = false;                  // see Session::state_changed
    bool compat = false;                   // LuaInstance compatibility mode
    // the C library's rand() (glibc's TYPE_3 additive feedback generator,
    // state as after srand(1): what a fresh reference process starts from)
    uint32_t rng[34];
    int rng_i = 0;
    void srand_(unsigned seed)
    {
        int32_t r[34];
        r[0] = (int32_t)(seed == 0 ? 1 : seed);
        for (int i = 1; i < 31; ++i) {   // 16807 r mod (2^31 - 1), Schrage's method
            const int32_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
            int32_t w = 16807 * lo - 2836 * hi;
            if (w < 0) w += 2147483647;
            r[i] = w;
        }
        for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
        for (int i = 0; i < 34; ++i) rng[i] = (uint32_t)r[i];
        rng_i = 0;   // rng holds r[k .. k+33] as a ring; k = 0
        for (int i = 0; i < 310; ++i) rand_();   // outputs 0 .. 309 are discarded
    }
    int rand_()   // r[i] = r[i-31] + r[i-3] (i >= 34), output r[i] >> 1
    {
        const uint32_t v = rng[(rng_i + 3) % 34] + rng[(rng_i + 31) % 34];
        rng[rng_i] = v;   // r[i] replaces r[i-34]
        rng_i = (rng_i + 1) % 34;
        return (int)(v >> 1);
    }
    int depth = 0;                         // Lua calls active
    const char *stack_top = nullptr;       // the C stack at the run's entry (see check_stack)
    // deep recursion in the evaluator (nested calls of nested expressions)
    // stops before the thread's C stack would: at 2 MB below the entry
    void check_stack()
    {
        char here;
        if (stack_top && stack_top - &here > (2 << 20))
            throw Unsupported("nesting of calls and expressions beyond 2 MB of the evaluator's stack");
    }
    long long units = 0;                   // estimated stack slots of the active calls
    long long steps = 0;                   // statements + calls in this element
    bool in_prelude = false;
    // tag methods (ltm.cpp): per tag, per event; tags 0..5 the basic types,
    // 6 and 7 the io library's (liolib.cpp:775-776), then newtag()'s
    std::vector<std::vector<Value>> tms;
    int last_tag = kNumTags - 1;
    int newtag()
    {
        tms.emplace_back(TM_N, Value());
        return ++last_tag;
    }
    static int tag_of(const Value &v)   // luaT_tag (ltm.cpp:124-136)
    {
        if (v.t == TUD) return static_cast<const UdObj *>(v.o)->tag;
        if (v.t == TTAB) return static_cast<const TableObj *>(v.o)->htag;
        return v.t;
    }
    const Value &gettm(int tag, int e) const { return tms[(size_t)tag][(size_t)e]; }
    // a tag method's call (luaD_callTM): its first result (or none)
    Value call_tm(const Value &tm, std::vector<Value> args)
    {
        std::vector<Value> res;
        call(tm, args, res);
        return res.empty() ? Value() : res[0];
    }
    // call_binTM (lvm.cpp:262-280): the first operand's method, the second's,
    // then tag 0's (the "global" method); false if none
    bool bin_tm(const Value &a, const Value &b, int e, Value *out)
    {
        Value tm = gettm(tag_of(a), e);
        if (tm.t == TNIL) tm = gettm(tag_of(b), e);
        if (tm.t == TNIL) tm = gettm(0, e);
        if (tm.t == TNIL) return false;
        *out = call_tm(tm, {a, b, str(kEventName[e])});
        return true;
    }
    bool lessthan(const Value &l, const Value &r);
    std::string *capture = nullptr;        // stdout of print / write (nullptr: the process's stdout)
    void out(int fd, const std::string &t)
    {
        if (fd == 1 && capture) capture->append(t);
        else std::fwrite(t.data(), 1, t.size(), fd == 2 ? stderr : stdout);
    }
    Value nm[7];                           // "x" "y" "r" "z" "theta" "R" "n" (fixed)
    std::string last_text;                 // the last element's function (one-entry cache)
    Chunk *last_chunk = nullptr;           // ... compiled (nullptr: no entry)

    explicit Interp(bool axisymmetric);
    ~Interp();

    template <class T> T *alloc()
    {
        // (collected only between elements: one element's garbage is bounded)
        if (nobjs > 50000000LL) throw Unsupported("more than 5 * 10^7 Lua objects alive within one element");
        T *o = new T();
        o->gcnext = gclist;
        gclist = o;
        ++nobjs;
        return o;
    }
    Value str(const std::string &s)
    {
        StrObj *o = alloc<StrObj>();
        o->s = s;
        o->hash = hash_s(s.data(), s.size());
        Value v;
        v.t = TSTR;
        v.o = o;
        return v;
    }
    Value table(int size)
    {
        TableObj *t = alloc<TableObj>();
        t->epoch = epoch;
        setnodevector(t, power2(size));
        Value v;
        v.t = TTAB;
        v.o = t;
        return v;
    }
    Value builtin(Builtin f, const char *name)
    {
        FuncObj *c = alloc<FuncObj>();
        c->c = f;
        c->name = name;
        Value v;
        v.t = TFUN;
        v.o = c;
        return v;
    }
    Value udata(const void *p, int tag)
    {
        UdObj *u = alloc<UdObj>();
        u->ptr = p;
        u->tag = tag;
        Value v;
        v.t = TUD;
        v.o = u;
        return v;
    }

    // -- the state a second Newton pass would see --------------------------
    void note_write(TableObj *t, const Value &k)
    {
        if (in_prelude || t->epoch == epoch) return;
        if (t == G && k.t == TSTR) {   // the prelude's six globals are rewritten per element anyway
            static const char *const pre[] = {"x", "y", "r", "z", "theta", "R"};
            for (const char *p : pre)
                if (sv(k) == p) return;
        }
        changed = true;
    }

    // -- primitive table access (lua_rawget / lua_rawset) ------------------
    Value rawget(TableObj *t, const Value &k)
    {
        Value *v = tget(t, k);
        return v ? *v : Value();
    }
    void rawset(TableObj *t, const Value &k, const Value &v)
    {
        note_write(t, k);
        *tset(t, k) = v;
    }
    Value rawgeti(TableObj *t, int i) { return rawget(t, num((double)i)); }
    void rawseti(TableObj *t, int i, const Value &v) { rawset(t, num((double)i), v); }

    // luaV_gettable (lvm.cpp:125-163): a table with the default tag or no
    // "gettable" method reads primitively, then its "index" method on nil;
    // anything else goes to its "gettable" method
    Value gettable(const Value &t, const Value &k)
    {
        Value tm;
        if (t.t == TTAB && (tv(t)->htag == TTAB || gettm(tv(t)->htag, TM_GETTABLE).t == TNIL)) {
            const Value v = rawget(tv(t), k);
            if (v.t != TNIL || (tm = gettm(tv(t)->htag, TM_INDEX)).t == TNIL) return v;
        } else {
            tm = gettm(tag_of(t), TM_GETTABLE);
        }
        if (tm.t == TNIL) rt_error(std::string("attempt to index a ") + kTypeName[t.t] + " value");
        return call_tm(tm, {t, k});
    }
    // luaV_settable (lvm.cpp:169-197)
    void settable(const Value &t, const Value &k, const Value &v)
    {
        if (t.t == TTAB && (tv(t)->htag == TTAB || gettm(tv(t)->htag, TM_SETTABLE).t == TNIL)) {
            rawset(tv(t), k, v);
            return;
        }
        const Value tm = gettm(tag_of(t), TM_SETTABLE);
        if (tm.t == TNIL) rt_error(std::string("attempt to index a ") + kTypeName[t.t] + " value");
        std::vector<Value> res;
        call(tm, {t, k, v}, res);
    }
    // luaV_getglobal / luaV_setglobal (lvm.cpp:200-257): the method of the
    // value's (the old value's) tag
    Value getglobal(const Value &name)
    {
        const Value v = rawget(G, name);
        const Value tm = gettm(tag_of(v), TM_GETGLOBAL);
        if (tm.t == TNIL) return v;
        return call_tm(tm, {name, v});
    }
    Value getglobal(const char *name) { return getglobal(str(name)); }
    void setglobal(const Value &name, const Value &v)
    {
        const Value old = rawget(G, name);
        const Value tm = gettm(tag_of(old), TM_SETGLOBAL);
        if (tm.t == TNIL) {
            rawset(G, name, v);
            return;
        }
        std::vector<Value> res;
        call(tm, {name, old, v}, res);
    }
    void setglobal(const char *name, const Value &v) { setglobal(str(name), v); }

    // -- conversions (lvm.cpp:42-68, lapi.cpp) -----------------------------
    static bool tonumber(Value &a)   // in place, as luaV_tonumber
    {
        if (a.t == TNUM) return true;
        if (a.t != TSTR) return false;
        Cx c;
        if (!str2d(sv(a).c_str(), &c)) return false;
        a = num(c);
        return true;
    }
    bool tostring(const Value &a, std::string *out)   // lua_tostring: numbers and strings
    {
        if (a.t == TSTR) { *out = sv(a); return true; }
        if (a.t != TNUM) return false;
        *out = number2str(a.n);
        return true;
    }

    // -- calls ---------------------------------------------------------------
    void call(const Value &f, std::vector<Value> &args, std::vector<Value> &res);
    void call(const Value &f, std::vector<Value> &&args, std::vector<Value> &res) { call(f, args, res); }
    void run_proto(const FuncObj *cl, std::vector<Value> &args, std::vector<Value> &res);
    int protected_call(const Value &f, std::vector<Value> &args, std::vector<Value> &res);
    int dostring(const std::string &text, std::vector<Value> &res);
    Chunk *compile(const std::string &text);   // throws LuaError (syntax)

    void gc();
};

namespace {

// ===========================================================================
// lexer (llex.cpp)
// ===========================================================================
enum Tok {
    T_AND = 257, T_BREAK, T_DO, T_ELSE, T_ELSEIF, T_END, T_FOR, T_FUNCTION, T_IF, T_LOCAL, T_NIL, T_NOT, T_OR,
    T_REPEAT, T_RETURN, T_THEN, T_UNTIL, T_WHILE, T_NAME, T_CONCAT, T_DOTS, T_EQ, T_GE, T_LE, T_NE, T_NUMBER,
    T_STRING, T_EOS
};
const char *const kReserved[] = {"and", "break", "do", "else", "elseif", "end", "for", "function", "if", "local",
                                 "nil", "not", "or", "repeat", "return", "then", "until", "while"};

struct Lexer {
    const std::string &src;
    size_t pos = 0;
    int tok = 0;
    double numval = 0;
    std::string sval;
    // one token of lookahead (constructor: NAME '=')
    bool have_ahead = false;
    int ahead_tok = 0;
    double ahead_num = 0;
    std::string ahead_s;

    explicit Lexer(const std::string &s) : src(s) {}

    [[noreturn]] void error(const char *m) { throw LuaError{3, m}; }
    int cur() const { return pos < src.size() ? (unsigned char)src[pos] : -1; }

    void read_number(bool comma)   // llex.cpp:167-208
    {
        std::string b;
        if (comma) b += '.';
        while (std::isdigit(cur())) b += (char)src[pos++];
        if (cur() == '.') {
            b += src[pos++];
            if (cur() == '.') error("ambiguous syntax (decimal point x string concatenation)");
        }
        while (std::isdigit(cur())) b += (char)src[pos++];
        if (cur() == 'e' || cur() == 'E') {
            b += src[pos++];
            if (cur() == '+' || cur() == '-') b += src[pos++];
            while (std::isdigit(cur())) b += (char)src[pos++];
        }
        Cx c;
        if (!str2d(b.c_str(), &c)) error("malformed number");
        numval = c.re;
    }

    void read_long_string()   // llex.cpp:211-258
    {
        int cont = 0;
        sval.clear();
        pos += 2;   // "[["
        for (;;) {
            const int c = cur();
            if (c < 0) error("unfinished long string");
            if (c == '[' && pos + 1 < src.size() && src[pos + 1] == '[') {
                ++cont;
                sval += "[[";
                pos += 2;
                continue;
            }
            if (c == ']' && pos + 1 < src.size() && src[pos + 1] == ']') {
                if (cont == 0) { pos += 2; return; }
                --cont;
                sval += "]]";
                pos += 2;
                continue;
            }
            if (c == ']' || c == '[') { sval += (char)c; ++pos; continue; }
            sval += (char)c;
            ++pos;
        }
    }

    void read_string(int del)   // llex.cpp:261-352
    {
        sval.clear();
        ++pos;
        while (cur() != del) {
            int c = cur();
            if (c < 0 || c == '\n') error("unfinished string");
            if (c != '\\') { sval += (char)c; ++pos; continue; }
            ++pos;
            c = cur();
            switch (c) {
            case 'a': sval += '\a'; ++pos; break;
            case 'b': sval += '\b'; ++pos; break;
            case 'f': sval += '\f'; ++pos; break;
            case 'n': sval += '\n'; ++pos; break;
            case 'r': sval += '\r'; ++pos; break;
            case 't': sval += '\t'; ++pos; break;
            case 'v': sval += '\v'; ++pos; break;
            case '\n': sval += '\n'; ++pos; break;
            default:
                if (c >= '0' && c <= '9') {
                    int v = 0, i = 0;
                    do {
                        v = 10 * v + (cur() - '0');
                        ++pos;
                    } while (++i < 3 && std::isdigit(cur()));
                    if (v != (unsigned char)v) error("escape sequence too large");
                    sval += (char)v;
                } else {
                    if (c < 0) error("unfinished string");   // (EOZ after the backslash)
                    sval += (char)c;
                    ++pos;
                }
            }
        }
        ++pos;   // the delimiter
    }

    int lex()   // luaX_lex (llex.cpp:355-493)
    {
        for (;;) {
            const int c = cur();
            switch (c) {
            case ' ': case '\t': case '\r': case '\n': ++pos; continue;
            case '$': error("unexpected `$' (pragmas are no longer supported)");
            case '-':
                ++pos;
                if (cur() != '-') return '-';
                while (cur() != '\n' && cur() >= 0) ++pos;
                continue;
            case '[':
                if (pos + 1 < src.size() && src[pos + 1] == '[') {
                    read_long_string();
                    return T_STRING;
                }
                ++pos;
                return '[';
            case '=': ++pos; if (cur() != '=') return '='; ++pos; return T_EQ;
            case '<': ++pos; if (cur() != '=') return '<'; ++pos; return T_LE;
            case '>': ++pos; if (cur() != '=') return '>'; ++pos; return T_GE;
            case '~': ++pos; if (cur() != '=') return '~'; ++pos; return T_NE;
            case '"': case '\'': read_string(c); return T_STRING;
            case '.':
                ++pos;
                if (cur() == '.') {
                    ++pos;
                    if (cur() == '.') { ++pos; return T_DOTS; }
                    return T_CONCAT;
                }
                if (!std::isdigit(cur())) return '.';
                read_number(true);
                return T_NUMBER;
            case -1: return T_EOS;
            default:
                if (std::isdigit(c)) { read_number(false); return T_NUMBER; }
                if (c != '_' && !std::isalpha(c)) {
                    if (std::iscntrl(c)) error("invalid control char");
                    ++pos;
                    return c;
                }
                sval.clear();
                while (std::isalnum(cur()) || cur() == '_') sval += src[pos++];
                for (int r = 0; r < 18; ++r)
                    if (sval == kReserved[r]) return T_AND + r;
                return T_NAME;
            }
        }
    }

    void next()
    {
        if (have_ahead) {
            have_ahead = false;
            tok = ahead_tok;
            numval = ahead_num;
            sval = ahead_s;
            return;
        }
        tok = lex();
    }
    int lookahead()
    {
        if (!have_ahead) {
            const int t0 = tok;
            const double n0 = numval;
            const std::string s0 = sval;
            ahead_tok = lex();
            ahead_num = numval;
            ahead_s = sval;
            have_ahead = true;
            tok = t0;
            numval = n0;
            sval = s0;
        }
        return ahead_tok;
    }
};

// ===========================================================================
// parser (lparser.cpp) -> syntax tree
// ===========================================================================
const int kMaxArgS = ((1 << 26) - 1) >> 1;   // MAXARG_S (llimits.h:101-119)
const int kLFields = 62, kRFields = 31;      // LFIELDS_PER_FLUSH, RFIELDS_PER_FLUSH (llimits.h:190-198)

struct FuncState {
    FuncState *prev = nullptr;
    Proto *f = nullptr;
    std::vector<std::string> actloc;   // active locals, innermost last (slot = index)
    std::vector<UpDesc> ups;
    int loops = 0;                     // enclosing loops (for break)
};

struct Parser {
    Lexer L;
    Interp &I;
    Chunk &C;
    FuncState *fs = nullptr;

    Parser(const std::string &text, Interp &in, Chunk &c) : L(text), I(in), C(c) {}

    [[noreturn]] void error(const char *m) { throw LuaError{3, m}; }
    void check(int t)
    {
        if (L.tok != t) error("unexpected token");
        L.next();
    }
    bool optional(int t)
    {
        if (L.tok != t) return false;
        L.next();
        return true;
    }
    std::string checkname()
    {
        if (L.tok != T_NAME) error("<name> expected");
        std::string s = L.sval;
        L.next();
        return s;
    }
    Value konst(const std::string &s)
    {
        auto it = C.const_index.find(s);
        StrObj *o;
        if (it != C.const_index.end()) o = it->second;
        else {
            C.consts.emplace_back(new StrObj());
            o = C.consts.back().get();
            o->s = s;
            o->hash = hash_s(s.data(), s.size());
            o->fixed = true;
            C.const_index[s] = o;
        }
        Value v;
        v.t = TSTR;
        v.o = o;
        return v;
    }
    Expr *ex(ExprKind k)
    {
        C.exprs.emplace_back(new Expr());
        C.exprs.back()->k = k;
        return C.exprs.back().get();
    }
    Stat *st(StatKind k)
    {
        C.stats.emplace_back(new Stat());
        C.stats.back()->k = k;
        return C.stats.back().get();
    }
    Block *blk()
    {
        C.blocks.emplace_back(new Block());
        return C.blocks.back().get();
    }

    // -- scopes --------------------------------------------------------------
    void open_func(FuncState &n)
    {
        C.protos.emplace_back(new Proto());
        n.f = C.protos.back().get();
        n.f->owner = &C;
        n.prev = fs;
        fs = &n;
    }
    int new_local(const std::string &name)   // new_localvar + adjustlocalvars, in one
    {
        if ((int)fs->actloc.size() + 1 > 200) error("too many local variables");   // MAXLOCALS
        fs->actloc.push_back(name);
        fs->f->maxslots = std::max(fs->f->maxslots, (int)fs->actloc.size());
        return (int)fs->actloc.size() - 1;
    }
    // search_local (lparser.cpp:210-230): level 0 here, 1 the enclosing function, -1 global
    int search_local(const std::string &n, int *slot)
    {
        int level = 0;
        for (FuncState *f = fs; f; f = f->prev, ++level)
            for (int i = (int)f->actloc.size() - 1; i >= 0; --i)
                if (f->actloc[i] == n) {
                    *slot = i;
                    return level;
                }
        return -1;
    }
    // singlevar (lparser.cpp:233-240)
    Expr *singlevar(const std::string &n)
    {
        int slot = 0;
        const int level = search_local(n, &slot);
        if (level >= 1) error("cannot access a variable in outer scope");
        if (level == 0) {
            Expr *e = ex(X_LOCAL);
            e->op = slot;
            return e;
        }
        Expr *e = ex(X_GLOBAL);
        e->s = konst(n);
        return e;
    }
    // pushupvalue (lparser.cpp:259-274) + indexupvalue (:243-256)
    Expr *upvalue(const std::string &n)
    {
        int slot = 0;
        const int level = search_local(n, &slot);
        UpDesc d;
        if (level == -1) {
            if (!fs->prev) error("cannot access upvalue in main");
            d.global = true;
            d.slot = 0;
            d.name = konst(n);
        } else if (level != 1) {
            error("upvalue must be global or local to immediately outer scope");
        } else {
            d.global = false;
            d.slot = slot;
        }
        int idx = -1;
        for (int i = 0; i < (int)fs->ups.size(); ++i) {
            const UpDesc &u = fs->ups[i];
            if (u.global == d.global && (d.global ? sv(u.name) == sv(d.name) : u.slot == d.slot)) idx = i;
        }
        if (idx < 0) {
            if ((int)fs->ups.size() + 1 > 32) error("too many upvalues");   // MAXUPVALUES
            fs->ups.push_back(d);
            idx = (int)fs->ups.size() - 1;
        }
        Expr *e = ex(X_UPVAL);
        e->op = idx;
        return e;
    }

    // -- expressions -----------------------------------------------------------
    Expr *number(double f)   // luaK_number (lcode.cpp:131-137)
    {
        if (f <= (double)kMaxArgS && (double)(int)f == f) {
            Expr *e = ex(X_INT);
            e->op = (int)f;
            return e;
        }
        Expr *e = ex(X_NUM);
        e->v = f;
        return e;
    }

    void explist1(std::vector<Expr *> &out)
    {
        out.push_back(expr());
        while (L.tok == ',') {
            L.next();
            out.push_back(expr());
        }
    }

    void funcargs(Expr *call)   // lparser.cpp:429-470
    {
        switch (L.tok) {
        case '(':
            L.next();
            if (L.tok != ')') explist1(call->list);
            check(')');
            break;
        case '{': call->list.push_back(constructor()); break;
        case T_STRING: {
            Expr *e = ex(X_STR);
            e->s = konst(L.sval);
            L.next();
            call->list.push_back(e);
            break;
        }
        default: error("function arguments expected");
        }
    }

    // var_or_func (lparser.cpp:473-545); *is_call: the result is a call
    Expr *var_or_func(bool *is_call)
    {
        Expr *v;
        *is_call = false;
        if (optional('%')) {
            v = upvalue(checkname());
        } else {
            v = singlevar(checkname());
        }
        for (;;) {
            switch (L.tok) {
            case '.': {
                L.next();
                Expr *e = ex(X_INDEX);
                e->a = v;
                Expr *k = ex(X_STR);
                k->s = konst(checkname());
                e->b = k;
                v = e;
                *is_call = false;
                break;
            }
            case '[': {
                L.next();
                Expr *e = ex(X_INDEX);
                e->a = v;
                e->b = expr();
                check(']');
                v = e;
                *is_call = false;
                break;
            }
            case ':': {
                L.next();
                Expr *e = ex(X_METHOD);
                e->a = v;
                e->s = konst(checkname());
                funcargs(e);
                v = e;
                *is_call = true;
                break;
            }
            case '(': case T_STRING: case '{': {
                Expr *e = ex(X_CALL);
                e->a = v;
                funcargs(e);
                v = e;
                *is_call = true;
                break;
            }
            default: return v;
            }
        }
    }

    Expr *constructor()   // lparser.cpp:548-683
    {
        Expr *t = ex(X_TABLE);
        check('{');
        const int k1 = part(t);
        if (optional(';')) {
            const int k2 = part(t);
            if (k1 == k2) error("invalid constructor syntax");
        }
        const int n = (int)t->list.size() + (int)t->rec.size();
        check('}');
        t->nelems = n;
        return t;
    }
    // constructor_part (lparser.cpp:618-651): 0 list, 1 record, an empty part its token
    int part(Expr *t)
    {
        if (L.tok == ';' || L.tok == '}') return L.tok;
        bool rec = L.tok == '[';
        if (L.tok == T_NAME && L.lookahead() == '=') rec = true;
        if (rec) {
            if (t->list.empty()) t->rec_first = true;
            for (;;) {
                Expr *key;
                if (L.tok == T_NAME) {
                    key = ex(X_STR);
                    key->s = konst(checkname());
                } else if (L.tok == '[') {
                    L.next();
                    key = expr();
                    check(']');
                } else {
                    error("<name> or `[' expected");
                }
                check('=');
                t->rec.emplace_back(key, expr());
                if (L.tok != ',') break;
                L.next();
                if (L.tok == ';' || L.tok == '}') break;
            }
            return 1;
        }
        for (;;) {
            t->list.push_back(expr());
            if (L.tok != ',') break;
            L.next();
            if (L.tok == ';' || L.tok == '}') break;
        }
        return 0;
    }

    Expr *simpleexp()   // lparser.cpp:689-745
    {
        switch (L.tok) {
        case T_NUMBER: {
            const double f = L.numval;
            L.next();
            return number(f);
        }
        case T_STRING: {
            Expr *e = ex(X_STR);
            e->s = konst(L.sval);
            L.next();
            return e;
        }
        case T_NIL: L.next(); return ex(X_NIL);
        case '{': return constructor();
        case T_FUNCTION: {
            L.next();
            Expr *e = ex(X_FUNC);
            e->op = body(false);
            return e;
        }
        case '(': {
            L.next();
            Expr *e = expr();
            check(')');
            return e;
        }
        case T_NAME: case '%': {
            bool call;
            return var_or_func(&call);
        }
        default: error("<expression> expected");
        }
    }

    static BinOp binop(int t)
    {
        switch (t) {
        case '+': return B_ADD;
        case '-': return B_SUB;
        case '*': return B_MUL;
        case '/': return B_DIV;
        case '^': return B_POW;
        case T_CONCAT: return B_CONCAT;
        case T_NE: return B_NE;
        case T_EQ: return B_EQ;
        case '<': return B_LT;
        case T_LE: return B_LE;
        case '>': return B_GT;
        case T_GE: return B_GE;
        case T_AND: return B_AND;
        case T_OR: return B_OR;
        default: return B_NONE;
        }
    }
    // priority[] (lparser.cpp:808-821), ORDER of BinOp
    static int left(BinOp o) { static const int p[] = {5, 5, 6, 6, 9, 4, 2, 2, 2, 2, 2, 2, 1, 1}; return p[o]; }
    static int right(BinOp o) { static const int p[] = {5, 5, 6, 6, 8, 3, 2, 2, 2, 2, 2, 2, 1, 1}; return p[o]; }

    // nesting of expressions and blocks (the reference's recursive-descent
    // parser has no limit but the C stack's; this one stops loudly)
    int nest = 0;
    struct Nest {
        Parser &P;
        explicit Nest(Parser &p) : P(p)
        {
            if (++P.nest > 1000) throw Unsupported("expressions or blocks nested more than 1000 deep");
        }
        ~Nest() { --P.nest; }
    };

    Expr *subexpr(int limit, BinOp *stop)   // lparser.cpp:828-853
    {
        Nest guard(*this);
        Expr *v;
        if (L.tok == '-' || L.tok == T_NOT) {
            const bool minus = L.tok == '-';
            L.next();
            BinOp dummy;
            Expr *e = subexpr(7, &dummy);   // UNARY_PRIORITY
            if (minus && e->k == X_INT) {           // PUSHINT -> PUSHINT -k (lcode.cpp:653-656)
                e->op = -e->op;
                v = e;
            } else if (minus && e->k == X_NUM) {    // PUSHNUM -> PUSHNEGNUM (:657-660)
                e->k = X_NEGNUM;
                v = e;
            } else {
                v = ex(minus ? X_UNM : X_NOT);
                v->a = e;
            }
        } else {
            v = simpleexp();
        }
        BinOp op = binop(L.tok);
        while (op != B_NONE && left(op) > limit) {
            L.next();
            BinOp nextop;
            Expr *r = subexpr(right(op), &nextop);
            Expr *n = ex(op == B_AND ? X_AND : op == B_OR ? X_OR : X_BIN);
            n->op = op;
            n->a = v;
            n->b = r;
            v = n;
            op = nextop;
        }
        *stop = op;
        return v;
    }
    Expr *expr()
    {
        BinOp stop;
        return subexpr(-1, &stop);
    }

    // -- statements ------------------------------------------------------------
    static bool block_follow(int t) { return t == T_ELSE || t == T_ELSEIF || t == T_END || t == T_UNTIL || t == T_EOS; }

    Block *block()   // lparser.cpp:887-895: the block's locals end with it
    {
        const size_t n0 = fs->actloc.size();
        Block *b = chunk();
        fs->actloc.resize(n0);
        return b;
    }

    Block *chunk()   // lparser.cpp:1302-1313
    {
        Nest guard(*this);
        Block *b = blk();
        bool last = false;
        while (!last && !block_follow(L.tok)) {
            last = stat(b);
            optional(';');
        }
        return b;
    }

    void check_match(int what) { check(what); }

    Target target_of(Expr *v)
    {
        Target t;
        if (v->k == X_LOCAL) { t.kind = 0; t.slot = v->op; }
        else if (v->k == X_GLOBAL) { t.kind = 1; t.name = v->s; }
        else if (v->k == X_INDEX) { t.kind = 2; t.obj = v->a; t.key = v->b; }
        else error("syntax error");
        return t;
    }

    bool stat(Block *b)   // lparser.cpp:1183-1247; true: must be the last statement
    {
        switch (L.tok) {
        case T_IF: {   // ifstat (:1060-1084)
            Stat *s = st(S_IF);
            L.next();
            s->conds.push_back(expr());
            check(T_THEN);
            s->blocks.push_back(block());
            while (L.tok == T_ELSEIF) {
                L.next();
                s->conds.push_back(expr());
                check(T_THEN);
                s->blocks.push_back(block());
            }
            if (L.tok == T_ELSE) {
                L.next();
                s->blocks.push_back(block());
            }
            check_match(T_END);
            b->stats.push_back(s);
            return false;
        }
        case T_WHILE: {   // whilestat (:936-952)
            Stat *s = st(S_WHILE);
            L.next();
            s->conds.push_back(expr());
            check(T_DO);
            ++fs->loops;
            s->blocks.push_back(block());
            --fs->loops;
            check_match(T_END);
            b->stats.push_back(s);
            return false;
        }
        case T_DO: {
            Stat *s = st(S_DO);
            L.next();
            s->blocks.push_back(block());
            check_match(T_END);
            b->stats.push_back(s);
            return false;
        }
        case T_FOR: {   // forstat (:1025-1047)
            L.next();
            ++fs->loops;
            const std::string var = checkname();
            Stat *s;
            if (L.tok == '=') {   // fornum (:987-1003)
                s = st(S_FORNUM);
                L.next();
                s->exprs.push_back(expr());
                check(',');
                s->exprs.push_back(expr());
                if (optional(',')) s->exprs.push_back(expr());
                s->slot = (int)fs->actloc.size();
                check(T_DO);
                new_local(var);
                new_local("(limit)");
                new_local("(step)");
            } else if (L.tok == ',') {   // forlist (:1006-1022)
                s = st(S_FORIN);
                L.next();
                const std::string val = checkname();
                if (L.tok != T_NAME || L.sval != "in") error("`in' expected");
                L.next();
                s->exprs.push_back(expr());
                s->slot = (int)fs->actloc.size();
                check(T_DO);
                new_local("(table)");
                new_local(var);
                new_local(val);
            } else {
                error("`=' or `,' expected");
            }
            s->blocks.push_back(block());
            fs->actloc.resize(s->slot);
            --fs->loops;
            check_match(T_END);
            b->stats.push_back(s);
            return false;
        }
        case T_REPEAT: {   // repeatstat (:955-969): `until' sees no local of the block
            Stat *s = st(S_REPEAT);
            L.next();
            ++fs->loops;
            s->blocks.push_back(block());
            --fs->loops;
            check_match(T_UNTIL);
            s->conds.push_back(expr());
            b->stats.push_back(s);
            return false;
        }
        case T_FUNCTION: {   // funcstat (:1107-1133): NAME [('.' | ':') NAME]
            L.next();
            Expr *v = singlevar(checkname());
            bool self = false;
            if (L.tok == ':' || L.tok == '.') {
                self = L.tok == ':';
                L.next();
                Expr *e = ex(X_INDEX);
                e->a = v;
                Expr *k = ex(X_STR);
                k->s = konst(checkname());
                e->b = k;
                v = e;
            }
            Stat *s = st(S_ASSIGN);
            s->targets.push_back(target_of(v));
            Expr *f = ex(X_FUNC);
            f->op = body(self);
            s->exprs.push_back(f);
            b->stats.push_back(s);
            return false;
        }
        case T_LOCAL: {   // localstat (:1087-1104): the names are in scope after the list
            Stat *s = st(S_LOCAL);
            std::vector<std::string> names;
            do {
                L.next();
                names.push_back(checkname());
            } while (L.tok == ',');
            if (optional('=')) explist1(s->exprs);
            s->slot = (int)fs->actloc.size();
            s->nvars = (int)names.size();
            for (const std::string &n : names) new_local(n);
            b->stats.push_back(s);
            return false;
        }
        case T_NAME: case '%': {   // namestat (:1136-1152)
            bool is_call;
            Expr *v = var_or_func(&is_call);
            if (is_call) {
                Stat *s = st(S_CALL);
                s->exprs.push_back(v);
                b->stats.push_back(s);
                return false;
            }
            if (v->k == X_UPVAL) error("syntax error");
            Stat *s = st(S_ASSIGN);
            s->targets.push_back(target_of(v));
            while (L.tok == ',') {   // assignment (:898-925)
                L.next();
                Expr *w = var_or_func(&is_call);
                if (is_call || w->k == X_UPVAL) error("syntax error");
                s->targets.push_back(target_of(w));
                if ((int)s->targets.size() > 100) error("too many variables in a multiple assignment");   // MAXVARSLH
            }
            check('=');
            explist1(s->exprs);
            b->stats.push_back(s);
            return false;
        }
        case T_RETURN: {   // retstat (:1155-1164)
            Stat *s = st(S_RETURN);
            L.next();
            if (!block_follow(L.tok)) explist1(s->exprs);
            b->stats.push_back(s);
            return true;
        }
        case T_BREAK: {   // breakstat (:1167-1180)
            if (fs->loops == 0) error("no loop to break");
            L.next();
            b->stats.push_back(st(S_BREAK));
            return true;
        }
        default: error("<statement> expected");
        }
    }

    int body(bool needself)   // lparser.cpp:1250-1299; the index of the new proto
    {
        FuncState nfs;
        open_func(nfs);
        const int idx = (int)C.protos.size() - 1;
        check('(');
        if (needself) new_local("self");
        int nparams = needself ? 1 : 0;
        bool dots = false;
        if (L.tok != ')') {
            do {
                if (L.tok == T_DOTS) {
                    L.next();
                    dots = true;
                } else if (L.tok == T_NAME) {
                    new_local(checkname());
                    ++nparams;
                } else {
                    error("<name> or `...' expected");
                }
            } while (!dots && optional(','));
        }
        if (nparams > 100) error("too many parameters");   // MAXPARAMS
        nfs.f->nparams = nparams;
        nfs.f->vararg = dots;
        if (dots) new_local("arg");
        check(')');
        nfs.f->body = chunk();
        check_match(T_END);
        nfs.f->ups = nfs.ups;
        fs = nfs.prev;
        return idx;
    }

    void main_chunk()   // luaY_parser (lparser.cpp:389-408)
    {
        FuncState mfs;
        open_func(mfs);
        L.next();
        mfs.f->body = chunk();
        if (L.tok != T_EOS) error("<eof> expected");
        fs = nullptr;
    }
};

// ===========================================================================
// evaluation (lvm.cpp, ldo.cpp)
// ===========================================================================
enum Flow { F_NORMAL, F_BREAK, F_RETURN };

}  // namespace

bool Interp::lessthan(const Value &l, const Value &r)   // luaV_lessthan (lvm.cpp:306-323)
{
    if (l.t == TNUM && r.t == TNUM) return l.n.re < r.n.re;
    if (l.t == TSTR && r.t == TSTR) {   // luaV_strcomp: strcoll over the '\0'-separated pieces
        const std::string &a = sv(l), &b = sv(r);
        const char *p = a.c_str(), *q = b.c_str();
        size_t la = a.size(), lb = b.size();
        for (;;) {
            const int c = std::strcoll(p, q);
            if (c != 0) return c < 0;
            size_t len = std::strlen(p);
            if (len == la) return len != lb;
            if (len == lb) return false;
            ++len;
            p += len;
            la -= len;
            q += len;
            lb -= len;
        }
    }
    Value v;
    if (!bin_tm(l, r, TM_LT, &v)) rt_error("attempt to compare");
    return v.t != TNIL;
}

namespace {

const long long kMaxSteps = 1000000000LL;
const int kMaxDepth = 200;
const long long kMaxUnits = 3500, kMaxLeaked = 3000;

struct Frame {
    std::vector<Value> slots;
    const FuncObj *cl;
    const Chunk *chunk;
};

struct Exec {
    Interp &I;
    Frame &F;

    const Proto &proto(int i) const { return *F.chunk->protos[i]; }

    void step()
    {
        if (++I.steps > kMaxSteps)
            throw Unsupported("more than 10^9 steps for one element (the reference's Lua would not return either)");
    }

    // -- arithmetic (lvm.cpp:575-660) ------------------------------------------
    Value arith(int op, Value a, Value b, const Expr *rhs)
    {
        Value v;
        if (op == B_POW) {   // OP_POW: always the "pow" method (the math library's on numbers, lmathlib.cpp:319-320)
            if (!I.bin_tm(a, b, TM_POW, &v)) rt_error("undefined operation");
            return v;
        }
        // `a + k` / `a - k` with an integer literal k are ADDI +-k (lcode.cpp:609-634):
        // on a non-number the "add" method sees the literal, negated for `-`
        const bool addi = (op == B_ADD || op == B_SUB) && rhs->k == X_INT;
        if (!Interp::tonumber(a) || !Interp::tonumber(b)) {   // (in place, the left operand first)
            static const int ev[] = {TM_ADD, TM_SUB, TM_MUL, TM_DIV};
            if (addi) {
                b = num((double)(op == B_SUB ? -rhs->op : rhs->op));
                op = B_ADD;
            }
            if (!I.bin_tm(a, b, ev[op], &v)) rt_error("attempt to perform arithmetic");
            return v;
        }
        const Cx x = a.n, y = b.n;
        switch (op) {
        case B_ADD: return num(add(x, y));
        case B_SUB:
            // `a - k` with an integer literal k is ADDI -k (lcode.cpp:622-634): re + (-k), im + 0
            if (rhs->k == X_INT) return num(Cx{x.re + (double)(-rhs->op), x.im + 0.0});
            return num(sub(x, y));
        case B_MUL: return num(mul(x, y));
        case B_DIV: return num(cdiv(x, y));
        default: rt_error("bad operator");
        }
    }

    bool lessthan(const Value &l, const Value &r) { return I.lessthan(l, r); }

    Value concat(Value a, const Value &b)   // luaV_strconc (lvm.cpp:326-362)
    {
        std::string sa, sb;
        const bool oka = I.tostring(a, &sa);
        if (oka && a.t == TNUM) a = I.str(sa);   // (converted in place before the other is tried)
        if (!oka || !I.tostring(b, &sb)) {
            Value v;
            if (!I.bin_tm(a, b, TM_CONCAT, &v)) rt_error("attempt to concat");
            return v;
        }
        return I.str(sa + sb);
    }

    // -- expressions -------------------------------------------------------------
    Value eval(const Expr *e)
    {
        if (e->a && e->a->a) I.check_stack();   // (nested operands only: the leaves stay cheap)
        switch (e->k) {
        case X_NIL: return Value();
        case X_INT: return num((double)e->op);
        case X_NUM: return num(e->v);
        case X_NEGNUM: return num(Cx{-e->v, -0.0});
        case X_STR: return e->s;
        case X_LOCAL: return F.slots[e->op];
        case X_GLOBAL: return I.getglobal(e->s);
        case X_UPVAL: return F.cl->up[e->op];
        case X_INDEX: {
            const Value t = eval(e->a);
            const Value k = eval(e->b);
            return I.gettable(t, k);
        }
        case X_CALL: case X_METHOD: {
            std::vector<Value> r;
            call(e, r);
            return r.empty() ? Value() : r[0];
        }
        case X_FUNC: return closure(e->op);
        case X_TABLE: return constructor(e);
        case X_UNM: {   // OP_MINUS (lvm.cpp:651-660); constants were folded by the parser
            Value a = eval(e->a);
            if (!Interp::tonumber(a)) {
                Value v;
                if (!I.bin_tm(a, Value(), TM_UNM, &v)) rt_error("attempt to perform arithmetic");
                return v;
            }
            return num(neg(a.n));
        }
        case X_NOT: {
            const Value a = eval(e->a);
            return a.t == TNIL ? num(1.0) : Value();
        }
        case X_AND: {
            const Value a = eval(e->a);
            if (a.t == TNIL) return a;
            return eval(e->b);
        }
        case X_OR: {
            const Value a = eval(e->a);
            if (a.t != TNIL) return a;
            return eval(e->b);
        }
        case X_BIN: break;
        }
        const Value a = eval(e->a);
        const Value b = eval(e->b);
        switch (e->op) {
        case B_EQ: return raweq(a, b) ? num(1.0) : Value();
        case B_NE: return raweq(a, b) ? Value() : num(1.0);
        case B_LT: return lessthan(a, b) ? num(1.0) : Value();
        case B_GT: return lessthan(b, a) ? num(1.0) : Value();
        case B_LE: return lessthan(b, a) ? Value() : num(1.0);
        case B_GE: return lessthan(a, b) ? Value() : num(1.0);
        case B_CONCAT: return concat(a, b);
        default: return arith(e->op, a, b, e->b);
        }
    }

    // an expression list adjusted to `want` values (-1: all of them)
    void explist(const std::vector<Expr *> &es, int want, std::vector<Value> &out)
    {
        out.clear();
        for (size_t i = 0; i < es.size(); ++i) {
            const Expr *e = es[i];
            if (i + 1 == es.size() && (e->k == X_CALL || e->k == X_METHOD)) {
                std::vector<Value> r;
                call(e, r);
                out.insert(out.end(), r.begin(), r.end());
            } else {
                out.push_back(eval(e));
            }
        }
        if (want >= 0) out.resize((size_t)want);
    }

    void call(const Expr *e, std::vector<Value> &res)
    {
        Value f;
        std::vector<Value> args;
        if (e->k == X_METHOD) {   // OP_PUSHSELF (lvm.cpp:488-497)
            const Value o = eval(e->a);
            f = I.gettable(o, e->s);
            args.push_back(o);
            std::vector<Value> rest;
            explist(e->list, -1, rest);
            args.insert(args.end(), rest.begin(), rest.end());
        } else {
            f = eval(e->a);
            explist(e->list, -1, args);
        }
        I.call(f, args, res);
    }

    Value closure(int pi)   // OP_CLOSURE (lvm.cpp:795-803): upvalues by value, now
    {
        const Proto &p = proto(pi);
        FuncObj *c = I.alloc<FuncObj>();
        c->p = &p;
        for (const UpDesc &u : p.ups) c->up.push_back(u.global ? I.getglobal(u.name) : F.slots[u.slot]);
        Value v;
        v.t = TFUN;
        v.o = c;
        return v;
    }

    Value constructor(const Expr *e)   // OP_CREATETABLE, SETLIST, SETMAP (lvm.cpp:498-555)
    {
        Value tv_ = I.table(e->nelems);
        TableObj *t = tv(tv_);
        auto do_list = [&]() {
            std::vector<Value> vals;
            for (size_t i = 0; i < e->list.size(); ++i) {
                vals.push_back(eval(e->list[i]));
                const size_t n = vals.size();
                if (n % kLFields == 0 || i + 1 == e->list.size()) {   // a flush: the group written last first
                    const size_t g0 = (n - 1) / kLFields * kLFields;
                    for (size_t j = n; j > g0; --j) *tset(t, num((double)j)) = vals[j - 1];
                }
            }
        };
        auto do_rec = [&]() {
            std::vector<std::pair<Value, Value>> kv;
            for (size_t i = 0; i < e->rec.size(); ++i) {
                const Value k = eval(e->rec[i].first);
                const Value v = eval(e->rec[i].second);
                kv.emplace_back(k, v);
                const size_t n = kv.size();
                if (n % kRFields == 0 || i + 1 == e->rec.size()) {
                    const size_t g0 = (n - 1) / kRFields * kRFields;
                    for (size_t j = n; j > g0; --j) *tset(t, kv[j - 1].first) = kv[j - 1].second;
                }
            }
        };
        if (e->rec_first) {
            do_rec();
            do_list();
        } else {
            do_list();
            do_rec();
        }
        return tv_;
    }

    // -- statements --------------------------------------------------------------
    void store(const Target &t, const Value &obj, const Value &key, const Value &v)
    {
        switch (t.kind) {
        case 0: F.slots[t.slot] = v; break;
        case 1: I.setglobal(t.name, v); break;
        default: I.settable(obj, key, v); break;
        }
    }

    Flow block(const Block *b, std::vector<Value> &ret)
    {
        for (const Stat *s : b->stats) {
            step();
            const Flow f = stat(s, ret);
            if (f != F_NORMAL) return f;
        }
        return F_NORMAL;
    }

    bool truth(const Expr *e) { return eval(e).t != TNIL; }

    Flow stat(const Stat *s, std::vector<Value> &ret)
    {
        switch (s->k) {
        case S_LOCAL: {
            std::vector<Value> v;
            explist(s->exprs, s->nvars, v);
            for (int i = 0; i < s->nvars; ++i) F.slots[s->slot + i] = v[i];
            return F_NORMAL;
        }
        case S_ASSIGN: {   // targets' tables and keys, then the values, then the stores right to left
            const size_t n = s->targets.size();
            std::vector<Value> obj(n), key(n);
            for (size_t i = 0; i < n; ++i)
                if (s->targets[i].kind == 2) {
                    obj[i] = eval(s->targets[i].obj);
                    key[i] = eval(s->targets[i].key);
                }
            std::vector<Value> v;
            explist(s->exprs, (int)n, v);
            for (size_t i = n; i-- > 0;) store(s->targets[i], obj[i], key[i], v[i]);
            return F_NORMAL;
        }
        case S_CALL: {
            std::vector<Value> r;
            call(s->exprs[0], r);
            return F_NORMAL;
        }
        case S_IF: {
            for (size_t i = 0; i < s->conds.size(); ++i)
                if (truth(s->conds[i])) return block(s->blocks[i], ret);
            if (s->blocks.size() > s->conds.size()) return block(s->blocks.back(), ret);
            return F_NORMAL;
        }
        case S_WHILE: {
            while (truth(s->conds[0])) {
                step();
                const Flow f = block(s->blocks[0], ret);
                if (f == F_BREAK) break;
                if (f == F_RETURN) return f;
            }
            return F_NORMAL;
        }
        case S_REPEAT: {
            for (;;) {
                step();
                const Flow f = block(s->blocks[0], ret);
                if (f == F_BREAK) break;
                if (f == F_RETURN) return f;
                if (truth(s->conds[0])) break;
            }
            return F_NORMAL;
        }
        case S_DO: return block(s->blocks[0], ret);
        case S_FORNUM: {   // OP_FORPREP / OP_FORLOOP (lvm.cpp:722-754)
            Value a = eval(s->exprs[0]);
            Value l = eval(s->exprs[1]);
            Value st_ = s->exprs.size() > 2 ? eval(s->exprs[2]) : num(1.0);
            if (!Interp::tonumber(st_)) rt_error("`for' step must be a number");
            if (!Interp::tonumber(l)) rt_error("`for' limit must be a number");
            if (!Interp::tonumber(a)) rt_error("`for' initial value must be a number");
            const int i0 = s->slot;
            F.slots[i0] = a;
            F.slots[i0 + 1] = l;
            F.slots[i0 + 2] = st_;
            auto out = [&]() {
                const Cx idx = F.slots[i0].n, lim = F.slots[i0 + 1].n, stp = F.slots[i0 + 2].n;
                return stp.re > 0 ? idx.re > lim.re : idx.re < lim.re;
            };
            if (out()) return F_NORMAL;
            for (;;) {
                step();
                const Flow f = block(s->blocks[0], ret);
                if (f == F_BREAK) break;
                if (f == F_RETURN) return f;
                if (F.slots[i0].t != TNUM) rt_error("`for' index must be a number");
                F.slots[i0].n = add(F.slots[i0].n, F.slots[i0 + 2].n);
                if (out()) break;
            }
            return F_NORMAL;
        }
        case S_FORIN: {   // OP_LFORPREP / OP_LFORLOOP (lvm.cpp:756-793)
            const Value t = eval(s->exprs[0]);
            if (t.t != TTAB) rt_error("`for' table must be a table");
            const int i0 = s->slot;
            F.slots[i0] = t;
            int nd = tnext(tv(t), Value());
            if (nd < 0) return F_NORMAL;
            F.slots[i0 + 1] = tv(t)->node[nd].key;
            F.slots[i0 + 2] = tv(t)->node[nd].val;
            for (;;) {
                step();
                const Flow f = block(s->blocks[0], ret);
                if (f == F_BREAK) break;
                if (f == F_RETURN) return f;
                TableObj *tt = tv(F.slots[i0]);
                nd = tnext(tt, F.slots[i0 + 1]);
                if (nd < 0) break;
                F.slots[i0 + 1] = tt->node[nd].key;
                F.slots[i0 + 2] = tt->node[nd].val;
            }
            return F_NORMAL;
        }
        case S_RETURN: explist(s->exprs, -1, ret); return F_RETURN;
        case S_BREAK: return F_BREAK;
        }
        return F_NORMAL;
    }
};

}  // namespace

// ===========================================================================
// calls (ldo.cpp, lvm.cpp:365-385 varargs)
// ===========================================================================
void Interp::run_proto(const FuncObj *cl, std::vector<Value> &args, std::vector<Value> &res)
{
    const Proto &p = *cl->p;
    Frame F;
    F.cl = cl;
    F.chunk = p.owner;
    F.slots.assign((size_t)std::max(p.maxslots, 1), Value());
    for (int i = 0; i < p.nparams && i < (int)args.size(); ++i) F.slots[i] = args[i];
    if (p.vararg) {   // luaV_pack: arg = {extra...; n = count}
        Value t = table(0);
        int n = 0;
        for (size_t i = (size_t)p.nparams; i < args.size(); ++i) *tset(tv(t), num((double)(++n))) = args[i];
        *tset(tv(t), nm[6]) = num((double)n);
        F.slots[p.nparams] = t;
    }
    const long long u = 1 + p.maxslots + 10;
    check_stack();
    if (++depth > kMaxDepth) throw Unsupported("recursion deeper than 200 calls");
    units += u;
    if (units + (long long)leaked.size() > kMaxUnits)
        throw Unsupported("more Lua stack than the reference's 4096 slots are sure to hold");
    Exec X{*this, F};
    res.clear();
    const Flow fl = X.block(p.body, res);
    if (fl != F_RETURN) res.clear();
    units -= u;
    --depth;
}

void Interp::call(const Value &f, std::vector<Value> &args, std::vector<Value> &res)
{
    if (++steps > kMaxSteps)
        throw Unsupported("more than 10^9 steps for one element (the reference's Lua would not return either)");
    if (f.t != TFUN) {   // luaD_call (ldo.cpp:178-187): the "function" method, with f first
        const Value tm = gettm(tag_of(f), TM_FUNCTION);
        if (tm.t == TNIL) rt_error(std::string("attempt to call a ") + kTypeName[f.t] + " value");
        args.insert(args.begin(), f);
        call(tm, args, res);
        return;
    }
    const FuncObj *c = fv(f);
    res.clear();
    if (c->c) {
        if (++depth > kMaxDepth) throw Unsupported("recursion deeper than 200 calls");
        c->c(*this, args, res);
        --depth;
        return;
    }
    run_proto(c, args, res);
}

// an error caught inside the chunk (call with "x", dostring): the reference
// hands the message to _ERRORMESSAGE first (ldo.cpp), which a chunk may have
// replaced
static void check_error_handlers(Interp &I)
{
    // (luaH_getglobal: raw, in the current table of globals; a non-function
    // is not called -- ldo.cpp:368-380)
    const Value em = I.rawget(I.G, I.str("_ERRORMESSAGE")), al = I.rawget(I.G, I.str("_ALERT"));
    if ((em.t == TFUN && !raweq(em, I.errormessage_fn)) || (al.t == TFUN && !raweq(al, I.alert_fn)))
        throw Unsupported("an error caught while _ERRORMESSAGE or _ALERT is not the library's");
}

int Interp::protected_call(const Value &f, std::vector<Value> &args, std::vector<Value> &res)
{
    const int d0 = depth;
    const long long u0 = units;
    try {
        call(f, args, res);
        return 0;
    } catch (const LuaError &e) {
        depth = d0;
        units = u0;
        res.clear();
        check_error_handlers(*this);
        return e.status;
    }
}

Chunk *Interp::compile(const std::string &text)
{
    auto it = chunks.find(text);
    if (it != chunks.end()) return it->second.get();
    if (chunks.size() >= 100000) throw Unsupported("more than 10^5 distinct chunks compiled (dostring)");
    std::unique_ptr<Chunk> c(new Chunk());
    Parser P(text, *this, *c);
    P.main_chunk();   // throws LuaError{3}
    Chunk *raw = c.get();
    chunks[text] = std::move(c);
    return raw;
}

int Interp::dostring(const std::string &text, std::vector<Value> &res)   // lua_dobuffer
{
    Chunk *c;
    try {
        c = compile(text);
    } catch (const LuaError &e) {
        res.clear();
        check_error_handlers(*this);
        return e.status;
    }
    FuncObj *main = alloc<FuncObj>();
    main->p = c->protos[0].get();
    Value f;
    f.t = TFUN;
    f.o = main;
    std::vector<Value> none;
    return protected_call(f, none, res);
}

// ===========================================================================
// the libraries
// ===========================================================================
namespace {

// lua_isnull: no argument at `i` (1-based)
inline bool isnull(const std::vector<Value> &a, int i) { return i > (int)a.size(); }
inline Value arg(const std::vector<Value> &a, int i) { return isnull(a, i) ? Value() : a[i - 1]; }

[[noreturn]] void argerror(int i, const char *what)
{
    char b[128];
    std::snprintf(b, sizeof b, "bad argument #%d (%s)", i, what);
    rt_error(b);
}
// luaL_check_number (lauxlib.cpp:96-104): a number or a numeric string
Cx check_number(std::vector<Value> &a, int i)
{
    if (isnull(a, i)) argerror(i, "number expected, got no value");
    Value v = a[i - 1];
    if (!Interp::tonumber(v)) argerror(i, "number expected");
    return v.n;
}
Cx opt_number(std::vector<Value> &a, int i, double def) { return isnull(a, i) ? Cx{def, 0.} : check_number(a, i); }
int check_int(std::vector<Value> &a, int i) { return to_int(check_number(a, i).re); }
int opt_int(std::vector<Value> &a, int i, int def) { return to_int(opt_number(a, i, (double)def).re); }
long check_long(std::vector<Value> &a, int i) { return to_long(check_number(a, i).re); }
long opt_long(std::vector<Value> &a, int i, long def) { return to_long(opt_number(a, i, (double)def).re); }
// luaL_check_lstr (lauxlib.cpp:75-81): a string, or a number's text
std::string check_str(Interp &I, std::vector<Value> &a, int i)
{
    std::string s;
    if (isnull(a, i) || !I.tostring(a[i - 1], &s)) argerror(i, "string expected");
    return s;
}
void check_any(std::vector<Value> &a, int i)
{
    if (isnull(a, i)) argerror(i, "value expected");
}
TableObj *check_table(std::vector<Value> &a, int i)
{
    if (isnull(a, i) || a[i - 1].t != TTAB) argerror(i, "table expected");
    return tv(a[i - 1]);
}

// lua_getn (lapi.cpp:534-556)
int getn(Interp &I, TableObj *t)
{
    const Value n = I.rawget(t, I.nm[6]);
    if (n.t == TNUM) return to_int(n.n.re);
    Cx mx{0., 0.};
    for (const Node &nd : t->node)
        if (nd.key.t == TNUM && nd.val.t != TNIL && nd.key.n.re > mx.re) mx = nd.key.n;
    return to_int(mx.re);
}

[[noreturn]] void unsupported_fn(const char *name)
{
    throw Unsupported(std::string("the library function ") + name + "()");
}

// -- base library (lbaselib.cpp) ------------------------------------------------
void b_alert(Interp &I, std::vector<Value> &a, std::vector<Value> &)
{
    const std::string s = check_str(I, a, 1);
    std::fputs(s.c_str(), stderr);
}
void b_errormessage(Interp &I, std::vector<Value> &a, std::vector<Value> &)   // liolib errorfb: to stderr
{
    const std::string s = check_str(I, a, 1);
    std::fprintf(stderr, "error: %s\n", s.c_str());
}
void b_call(Interp &I, std::vector<Value> &a, std::vector<Value> &r)   // lbaselib.cpp:311-351
{
    const std::string options = isnull(a, 3) ? std::string() : check_str(I, a, 3);
    TableObj *t = check_table(a, 2);
    const int n = getn(I, t);
    if (!isnull(a, 4)) throw Unsupported("call() with an error method");
    std::vector<Value> args;
    for (int i = 0; i < n; ++i) args.push_back(I.rawgeti(t, i + 1));
    const int status = I.protected_call(arg(a, 1), args, r);
    if (status != 0) {
        if (options.find('x') != std::string::npos) {
            r.assign(1, Value());
            return;
        }
        rt_error("error in call");   // (propagated)
    }
    if (options.find('p') != std::string::npos) rt_error("deprecated option `p' in `call'");
}
void b_collectgarbage(Interp &, std::vector<Value> &a, std::vector<Value> &) { (void)opt_int(a, 1, 0); }
void b_dostring(Interp &I, std::vector<Value> &a, std::vector<Value> &r)   // lbaselib.cpp:286-294
{
    const std::string s = check_str(I, a, 1);
    if (!s.empty() && s[0] == '\27') rt_error("`dostring' cannot run pre-compiled code");
    if (!isnull(a, 2)) (void)check_str(I, a, 2);
    const int status = I.dostring(s, r);
    if (status == 0) {
        if (r.empty()) {   // at least one result to signal no errors: userdata NULL
            Value u;
            u.t = TUD;
            u.o = I.null_ud;
            r.push_back(u);
        }
        return;
    }
    static const char *const names[] = {"ok", "run-time error", "file error", "syntax error", "memory error",
                                        "error in error handling"};
    r.assign(1, Value());
    r.push_back(I.str(names[status]));
}
void b_error(Interp &I, std::vector<Value> &a, std::vector<Value> &)
{
    rt_error(isnull(a, 1) ? std::string("error") : check_str(I, a, 1));
}
void b_foreach(Interp &I, std::vector<Value> &a, std::vector<Value> &r)   // lbaselib.cpp:387-403
{
    TableObj *t = check_table(a, 1);
    if (isnull(a, 2) || a[1].t != TFUN) argerror(2, "function expected");
    const Value f = a[1];
    Value k;
    for (;;) {
        const int nd = tnext(t, k);
        if (nd < 0) return;
        k = t->node[nd].key;
        std::vector<Value> args{k, t->node[nd].val}, res;
        I.call(f, args, res);
        if (!res.empty() && res[0].t != TNIL) {
            r.assign(1, res[0]);
            return;
        }
    }
}
void b_foreachi(Interp &I, std::vector<Value> &a, std::vector<Value> &r)   // lbaselib.cpp:368-384
{
    TableObj *t = check_table(a, 1);
    if (isnull(a, 2) || a[1].t != TFUN) argerror(2, "function expected");
    const Value f = a[1];
    const int n = getn(I, t);
    for (int i = 1; i <= n; ++i) {
        std::vector<Value> args{num((double)i), I.rawgeti(t, i)}, res;
        I.call(f, args, res);
        if (!res.empty() && res[0].t != TNIL) {
            r.assign(1, res[0]);
            return;
        }
    }
}
void b_getglobal(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    r.assign(1, I.getglobal(I.str(check_str(I, a, 1))));
}
void b_globals(Interp &I, std::vector<Value> &a, std::vector<Value> &r)   // lbaselib.cpp:175-185
{
    Value g;
    g.t = TTAB;
    g.o = I.G;
    if (!isnull(a, 1)) {   // lua_setglobals: the new table of globals
        TableObj *t = check_table(a, 1);
        if (t != I.G) I.changed = true;
        I.G = t;
    }
    r.assign(1, g);
}
void b_next(Interp &, std::vector<Value> &a, std::vector<Value> &r)   // lbaselib.cpp:242-253
{
    TableObj *t = check_table(a, 1);
    const int nd = tnext(t, arg(a, 2));
    if (nd < 0) {
        r.assign(1, Value());
        return;
    }
    r = {t->node[nd].key, t->node[nd].val};
}
void b_print(Interp &I, std::vector<Value> &a, std::vector<Value> &)   // lbaselib.cpp:69-87
{
    const Value ts = I.getglobal("tostring");
    for (size_t i = 0; i < a.size(); ++i) {
        std::vector<Value> args{a[i]}, res;
        I.call(ts, args, res);
        std::string s;
        if (res.empty() || !I.tostring(res[0], &s)) rt_error("`tostring' must return a string to `print'");
        if (i > 0) I.out(1, "\t");
        I.out(1, s.substr(0, std::strlen(s.c_str())));   // (fputs: up to a '\0')
    }
    I.out(1, "\n");
}
void b_rawget(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    TableObj *t = check_table(a, 1);
    check_any(a, 2);
    r.assign(1, I.rawget(t, a[1]));
}
void b_rawset(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    TableObj *t = check_table(a, 1);
    check_any(a, 2);
    check_any(a, 3);
    I.rawset(t, a[1], a[2]);
    r.assign(1, a[0]);
}
void b_setglobal(Interp &I, std::vector<Value> &a, std::vector<Value> &)   // the value at the top
{
    check_any(a, 2);
    const std::string n = check_str(I, a, 1);
    I.setglobal(I.str(n), a.back());
}
void b_tag(Interp &, std::vector<Value> &a, std::vector<Value> &r)
{
    check_any(a, 1);
    r.assign(1, num((double)Interp::tag_of(a[0])));
}
void b_tonumber(Interp &I, std::vector<Value> &a, std::vector<Value> &r)   // lbaselib.cpp:90-122
{
    const int base = opt_int(a, 2, 10);
    if (base == 10) {
        check_any(a, 1);
        Value v = a[0];
        if (Interp::tonumber(v)) {
            r.assign(1, v);
            return;
        }
    } else {
        const std::string s = check_str(I, a, 1);
        if (!(2 <= base && base <= 36)) argerror(2, "base out of range");
        const char *s1 = s.c_str();
        char *s2;
        const unsigned long n = std::strtoul(s1, &s2, base);
        if (s1 != s2) {
            while (std::isspace((unsigned char)*s2)) ++s2;
            if (*s2 == '\0') {
                r.assign(1, num((double)n));
                return;
            }
        }
    }
    r.assign(1, Value());
}
void b_tostring(Interp &I, std::vector<Value> &a, std::vector<Value> &r)   // lbaselib.cpp:354-385
{
    if (isnull(a, 1)) argerror(1, "value expected");
    const Value &v = a[0];
    char buf[64];
    switch (v.t) {
    case TNUM: r.assign(1, I.str(number2str(v.n))); return;
    case TSTR: r.assign(1, v); return;
    case TTAB: std::snprintf(buf, sizeof buf, "table: %p", (void *)v.o); break;
    case TFUN: std::snprintf(buf, sizeof buf, "function: %p", (void *)v.o); break;
    case TUD: {
        const UdObj *u = static_cast<const UdObj *>(v.o);
        std::snprintf(buf, sizeof buf, "userdata(%d): %p", u->tag, u->ptr);
        break;
    }
    default: r.assign(1, I.str("nil")); return;
    }
    r.assign(1, I.str(buf));
}
void b_type(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    check_any(a, 1);
    r.assign(1, I.str(kTypeName[a[0].t]));
}
void b_assert(Interp &I, std::vector<Value> &a, std::vector<Value> &)
{
    check_any(a, 1);
    if (a[0].t == TNIL) rt_error("assertion failed!  " + (isnull(a, 2) ? std::string() : check_str(I, a, 2)));
}
void b_getn(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    r.assign(1, num((double)getn(I, check_table(a, 1))));
}
void b_tinsert(Interp &I, std::vector<Value> &a, std::vector<Value> &)   // lbaselib.cpp:414-434
{
    const int v = (int)a.size();
    TableObj *t = check_table(a, 1);
    int n = getn(I, t);
    const int pos = v == 2 ? n + 1 : check_int(a, 2);
    I.rawset(t, I.nm[6], num((double)(n + 1)));
    for (; n >= pos; --n) I.rawseti(t, n + 1, I.rawgeti(t, n));
    I.rawseti(t, pos, a[v - 1]);
}
void b_tremove(Interp &I, std::vector<Value> &a, std::vector<Value> &r)   // lbaselib.cpp:437-455
{
    TableObj *t = check_table(a, 1);
    const int n = getn(I, t);
    int pos = opt_int(a, 2, n);
    if (n <= 0) return;
    const Value res = I.rawgeti(t, pos);
    for (; pos < n; ++pos) I.rawseti(t, pos, I.rawgeti(t, pos + 1));
    I.rawset(t, I.nm[6], num((double)(n - 1)));
    I.rawseti(t, n, Value());
    r.assign(1, res);
}

// sort (lbaselib.cpp:468-576): the same comparisons in the same order
struct Sorter {
    Interp &I;
    TableObj *t;
    Value f;
    bool comp(const Value &a, const Value &b)
    {
        if (f.t != TNIL) {
            std::vector<Value> args{a, b}, res;
            I.call(f, args, res);
            return !res.empty() && res[0].t != TNIL;
        }
        return I.lessthan(a, b);
    }
    Value get(int i) { return I.rawgeti(t, i); }
    void set(int i, const Value &v) { I.rawseti(t, i, v); }
    void aux(int l, int u)
    {
        while (l < u) {
            {
                const Value al = get(l), au = get(u);
                if (comp(au, al)) {
                    set(l, au);
                    set(u, al);
                }
            }
            if (u - l == 1) break;
            int i = (l + u) / 2;
            {
                const Value ai = get(i), al = get(l);
                if (comp(ai, al)) {
                    set(i, al);
                    set(l, ai);
                } else {
                    const Value au = get(u);
                    if (comp(au, ai)) {
                        set(i, au);
                        set(u, ai);
                    }
                }
            }
            if (u - l == 2) break;
            const Value P = get(i);
            {
                const Value au1 = get(u - 1);
                set(i, au1);
                set(u - 1, P);
            }
            i = l;
            int j = u - 1;
            for (;;) {
                Value ai, aj;
                while (ai = get(++i), comp(ai, P))
                    if (i > u) rt_error("invalid order function for sorting");
                while (aj = get(--j), comp(P, aj))
                    if (j < l) rt_error("invalid order function for sorting");
                if (j < i) break;
                set(i, aj);
                set(j, ai);
            }
            {
                const Value au1 = get(u - 1), ai = get(i);
                set(u - 1, ai);
                set(i, au1);
            }
            if (i - l < u - i) {
                j = l;
                i = i - 1;
                l = i + 2;
            } else {
                j = i + 1;
                i = u;
                u = j - 2;
            }
            aux(j, i);
        }
    }
};
void b_sort(Interp &I, std::vector<Value> &a, std::vector<Value> &)
{
    TableObj *t = check_table(a, 1);
    const int n = getn(I, t);
    if (!isnull(a, 2) && a[1].t != TFUN) argerror(2, "function expected");
    Sorter S{I, t, arg(a, 2)};
    S.aux(1, n);
}
void b_deprecated(Interp &, std::vector<Value> &, std::vector<Value> &) { rt_error("function is deprecated"); }

// dofile (lbaselib.cpp:297-304 over lua_dofile, ldo.cpp:290-325): a text
// chunk read from the file, run as dostring runs its string
void b_dofile(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    if (isnull(a, 1)) throw Unsupported("dofile() of the standard input");
    const std::string name = check_str(I, a, 1);
    std::string text;
    FILE *f = std::fopen(name.c_str(), "r");
    int status = 0;
    if (!f) {
        status = 2;   // LUA_ERRFILE
    } else {
        char buf[65536];
        size_t n;
        while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) text.append(buf, n);
        std::fclose(f);
        if (!text.empty() && text[0] == '\27') throw Unsupported("dofile() of a precompiled chunk");
    }
    if (status == 0) status = I.dostring(text, r);
    else r.clear();
    if (status == 0) {
        if (r.empty()) {
            Value u;
            u.t = TUD;
            u.o = I.null_ud;
            r.push_back(u);
        }
        return;
    }
    static const char *const names[] = {"ok", "run-time error", "file error", "syntax error", "memory error",
                                        "error in error handling"};
    r.assign(1, Value());
    r.push_back(I.str(names[status]));
}
void u_gcinfo(Interp &, std::vector<Value> &, std::vector<Value> &) { unsupported_fn("gcinfo"); }

// tag methods from Lua (lbaselib.cpp:140-230, lapi.cpp:484-499, ltm.cpp:22-184)
int check_event(const std::string &name, int t)   // luaI_checkevent
{
    int e = -1;
    for (int i = 0; i < 18; ++i)
        if (name == kEventName[i]) e = i;
    if (e >= TM_N) rt_error("event `" + name + "' is deprecated");
    if (e == TM_GC && t == TTAB) rt_error("event `gc' for tables is deprecated");
    if (e < 0) rt_error("`" + name + "' is not a valid event name");
    return e;
}
void check_tag(Interp &I, int t)
{
    if (!(0 <= t && t <= I.last_tag)) rt_error("not a valid tag");
}
Value get_tag_method(Interp &I, int t, const std::string &event)   // lua_gettagmethod
{
    const int e = check_event(event, t);
    check_tag(I, t);
    return valid_event(t, e) ? I.gettm(t, e) : Value();
}
void b_newtag(Interp &I, std::vector<Value> &, std::vector<Value> &r)
{
    I.changed = true;
    r.assign(1, num((double)I.newtag()));
}
void b_settag(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    TableObj *t = check_table(a, 1);
    const int tg = check_int(a, 2);
    if (!(kNumTags <= tg && tg <= I.last_tag)) rt_error("tag was not created by `newtag'");   // luaT_realtag
    if (t->htag != tg) I.changed = true;
    t->htag = tg;
    r.assign(1, a[0]);
}
void b_settagmethod(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    const int t = check_int(a, 1);
    const std::string event = check_str(I, a, 2);
    if (isnull(a, 3) || !(a[2].t == TFUN || a[2].t == TNIL)) argerror(3, "function or nil expected");
    if (event == "gc") rt_error("deprecated use: cannot set the `gc' tag method from Lua");
    const Value old = get_tag_method(I, t, event);
    const int e = check_event(event, t);   // lua_settagmethod
    check_tag(I, t);
    if (!valid_event(t, e)) rt_error("cannot change tag method for this type");
    I.tms[(size_t)t][(size_t)e] = arg(a, 3);
    I.changed = true;
    r.assign(1, old);
}
void b_gettagmethod(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    const int t = check_int(a, 1);
    const std::string event = check_str(I, a, 2);
    if (event == "gc") rt_error("deprecated use: cannot get the `gc' tag method from Lua");
    r.assign(1, get_tag_method(I, t, event));
}
void b_copytagmethods(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    const int to = check_int(a, 1), from = check_int(a, 2);
    check_tag(I, to);
    check_tag(I, from);
    for (int e = 0; e < TM_N; ++e)
        if (valid_event(to, e)) I.tms[(size_t)to][(size_t)e] = I.gettm(from, e);
    I.changed = true;
    r.assign(1, num((double)to));
}
void u_io(Interp &, std::vector<Value> &, std::vector<Value> &) { throw Unsupported("the io library"); }
// io_write (liolib.cpp:504-532) on the predefined handles: the first argument
// if it is one, else _OUTPUT; numbers as CComplex::ToString
void io_write(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    auto handle = [](const Value &v, int *fd) {
        if (v.t != TUD) return false;
        const UdObj *u = static_cast<const UdObj *>(v.o);
        if (!u->ptr || u->tag != 6) return false;
        *fd = *static_cast<const int *>(u->ptr);
        return true;
    };
    int fd = 1;
    size_t k = 0;
    if (!a.empty() && handle(a[0], &fd)) k = 1;
    else if (!handle(I.getglobal("_OUTPUT"), &fd)) rt_error("global variable `_OUTPUT' is not a file handle");
    if (fd == 0) throw Unsupported("write() to the standard input");
    for (; k < a.size(); ++k) {
        std::string t;
        if (a[k].t == TNUM) {
            t = number2str(a[k].n);
            if (t.empty()) throw Unsupported("write() of a number with a NaN imaginary part");
        } else {
            t = check_str(I, a, (int)k + 1);
        }
        I.out(fd, t);
    }
    Value u;
    u.t = TUD;
    u.o = I.null_ud;
    r.assign(1, u);
}
// math_random / math_randomseed (lmathlib.cpp:196-234) over the C library's rand()
void m_random(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    I.changed = true;   // (the generator's state moves)
    const double x = (double)(I.rand_() % 2147483647) / (double)2147483647;
    switch (a.size()) {
    case 0: r.assign(1, num(x)); return;
    case 1: {
        const int u = check_int(a, 1);
        if (!(1 <= u)) argerror(1, "interval is empty");
        r.assign(1, num((double)((int)(x * u) + 1)));
        return;
    }
    case 2: {
        const int l = check_int(a, 1), u = check_int(a, 2);
        if (!(l <= u)) argerror(2, "interval is empty");
        r.assign(1, num((double)((int)(x * (u - l + 1)) + l)));
        return;
    }
    default: rt_error("wrong number of arguments");
    }
}
void m_randomseed(Interp &I, std::vector<Value> &a, std::vector<Value> &)
{
    I.changed = true;
    I.srand_((unsigned)check_int(a, 1));
}
void u_femmversion(Interp &, std::vector<Value> &, std::vector<Value> &) { unsupported_fn("femmVersion"); }

// -- string library (lstrlib.cpp) ---------------------------------------------
long posrelat(long pos, size_t len) { return pos >= 0 ? pos : (long)len + pos + 1; }

void s_len(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    r.assign(1, num((double)check_str(I, a, 1).size()));
}
void s_sub(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    const std::string s = check_str(I, a, 1);
    const size_t l = s.size();
    long start = posrelat(check_long(a, 2), l);
    long end = posrelat(opt_long(a, 3, -1), l);
    if (start < 1) start = 1;
    if (end > (long)l) end = (long)l;
    r.assign(1, start <= end ? I.str(s.substr((size_t)start - 1, (size_t)(end - start + 1))) : I.str(""));
}
void s_lower(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    std::string s = check_str(I, a, 1);
    for (char &c : s) c = (char)std::tolower((unsigned char)c);
    r.assign(1, I.str(s));
}
void s_upper(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    std::string s = check_str(I, a, 1);
    for (char &c : s) c = (char)std::toupper((unsigned char)c);
    r.assign(1, I.str(s));
}
void s_rep(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    const std::string s = check_str(I, a, 1);
    int n = check_int(a, 2);
    if ((long long)s.size() * std::max(n, 0) > (1LL << 30)) throw Unsupported("strrep() beyond 1 GiB");
    std::string o;
    while (n-- > 0) o += s;
    r.assign(1, I.str(o));
}
void s_byte(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    const std::string s = check_str(I, a, 1);
    const long pos = posrelat(opt_long(a, 2, 1), s.size());
    if (!(0 < pos && (size_t)pos <= s.size())) argerror(2, "out of range");
    r.assign(1, num((double)(unsigned char)s[(size_t)pos - 1]));
}
void s_char(Interp &I, std::vector<Value> &a, std::vector<Value> &r)
{
    std::string o;
    for (int i = 1; i <= (int)a.size(); ++i) {
        const int c = check_int(a, i);
        if ((unsigned char)c != c) argerror(i, "invalid value");
        o += (char)(unsigned char)c;
    }
    r.assign(1, I.str(o));
}

// pattern matching (lstrlib.cpp:125-450)
struct Capture {
    const char *src_end;
    int level;
    struct {
        const char *init;
        long len;
    } capture[32];   // MAX_CAPTURES
};

int check_capture(int l, Capture *cap)
{
    l -= '1';
    if (!(0 <= l && l < cap->level && cap->capture[l].len != -1)) rt_error("invalid capture index");
    return l;
}
int capture_to_close(Capture *cap)
{
    int level = cap->level;
    for (level--; level >= 0; level--)
        if (cap->capture[level].len == -1) return level;
    rt_error("invalid pattern capture");
}
const char *classend(const char *p)
{
    switch (*p++) {
    case '%':
        if (*p == '\0') rt_error("malformed pattern (ends with `%')");
        return p + 1;
    case '[':
        if (*p == '^') p++;
        do {
            if (*p == '\0') rt_error("malformed pattern (missing `]')");
            if (*(p++) == '%' && *p != '\0') p++;
        } while (*p != ']');
        return p + 1;
    default: return p;
    }
}
int match_class(int c, int cl)
{
    int res;
    switch (std::tolower(cl)) {
    case 'a': res = std::isalpha(c); break;
    case 'c': res = std::iscntrl(c); break;
    case 'd': res = std::isdigit(c); break;
    case 'l': res = std::islower(c); break;
    case 'p': res = std::ispunct(c); break;
    case 's': res = std::isspace(c); break;
    case 'u': res = std::isupper(c); break;
    case 'w': res = std::isalnum(c); break;
    case 'x': res = std::isxdigit(c); break;
    case 'z': res = (c == '\0'); break;
    default: return cl == c;
    }
    return std::islower(cl) ? res : !res;
}
int matchbracketclass(int c, const char *p, const char *endclass)
{
    int sig = 1;
    if (*(p + 1) == '^') {
        sig = 0;
        p++;
    }
    while (++p < endclass) {
        if (*p == '%') {
            p++;
            if (match_class(c, (unsigned char)*p)) return sig;
        } else if (*(p + 1) == '-' && p + 2 < endclass) {
            p += 2;
            if ((int)(unsigned char)*(p - 2) <= c && c <= (int)(unsigned char)*p) return sig;
        } else if ((int)(unsigned char)*p == c) {
            return sig;
        }
    }
    return !sig;
}
int singlematch(int c, const char *p, const char *ep)
{
    switch (*p) {
    case '.': return 1;
    case '%': return match_class(c, (unsigned char)*(p + 1));
    case '[': return matchbracketclass(c, p, ep - 1);
    default: return (unsigned char)*p == c;
    }
}

struct Matcher {
    Interp &I;
    long long calls = 0;
    int depth = 0;   // recursion of match (the reference's: the C stack's only)
    const char *match(const char *s, const char *p, Capture *cap);

    const char *matchbalance(const char *s, const char *p, Capture *cap)
    {
        if (*p == 0 || *(p + 1) == 0) rt_error("unbalanced pattern");
        if (*s != *p) return nullptr;
        const int b = *p, e = *(p + 1);
        int cont = 1;
        while (++s < cap->src_end) {
            if (*s == e) {
                if (--cont == 0) return s + 1;
            } else if (*s == b) {
                cont++;
            }
        }
        return nullptr;
    }
    const char *max_expand(const char *s, const char *p, const char *ep, Capture *cap)
    {
        long i = 0;
        while ((s + i) < cap->src_end && singlematch((unsigned char)*(s + i), p, ep)) i++;
        while (i >= 0) {
            const char *res = match(s + i, ep + 1, cap);
            if (res) return res;
            i--;
        }
        return nullptr;
    }
    const char *min_expand(const char *s, const char *p, const char *ep, Capture *cap)
    {
        for (;;) {
            const char *res = match(s, ep + 1, cap);
            if (res != nullptr) return res;
            if (s < cap->src_end && singlematch((unsigned char)*s, p, ep)) s++;
            else return nullptr;
        }
    }
    const char *start_capture(const char *s, const char *p, Capture *cap)
    {
        const int level = cap->level;
        if (level >= 32) rt_error("too many captures");
        cap->capture[level].init = s;
        cap->capture[level].len = -1;
        cap->level = level + 1;
        const char *res = match(s, p + 1, cap);
        if (res == nullptr) cap->level--;
        return res;
    }
    const char *end_capture(const char *s, const char *p, Capture *cap)
    {
        const int l = capture_to_close(cap);
        cap->capture[l].len = s - cap->capture[l].init;
        const char *res = match(s, p + 1, cap);
        if (res == nullptr) cap->capture[l].len = -1;
        return res;
    }
    const char *match_capture(const char *s, int level, Capture *cap)
    {
        const int l = check_capture(level, cap);
        const size_t len = (size_t)cap->capture[l].len;
        if ((size_t)(cap->src_end - s) >= len && std::memcmp(cap->capture[l].init, s, len) == 0) return s + len;
        return nullptr;
    }
};

const char *Matcher::match(const char *s, const char *p, Capture *cap)
{
    if (++calls > 100000000LL) throw Unsupported("a pattern match of more than 10^8 steps");
    struct Depth {
        int &d;
        explicit Depth(int &x) : d(x)
        {
            if (++d > 5000) throw Unsupported("a pattern match recursing more than 5000 deep");
        }
        ~Depth() { --d; }
    } guard(depth);
init:
    switch (*p) {
    case '(': return start_capture(s, p, cap);
    case ')': return end_capture(s, p, cap);
    case '%':
        if (std::isdigit((unsigned char)*(p + 1))) {
            s = match_capture(s, *(p + 1), cap);
            if (s == nullptr) return nullptr;
            p += 2;
            goto init;
        } else if (*(p + 1) == 'b') {
            s = matchbalance(s, p + 2, cap);
            if (s == nullptr) return nullptr;
            p += 4;
            goto init;
        }
        goto dflt;
    case '\0': return s;
    case '$':
        if (*(p + 1) == '\0') return s == cap->src_end ? s : nullptr;
        goto dflt;
    default:
    dflt: {
        const char *ep = classend(p);
        const int m = s < cap->src_end && singlematch((unsigned char)*s, p, ep);
        switch (*ep) {
        case '?': {
            const char *res;
            if (m && (res = match(s + 1, ep + 1, cap)) != nullptr) return res;
            p = ep + 1;
            goto init;
        }
        case '*': return max_expand(s, p, ep, cap);
        case '+': return m ? max_expand(s + 1, p, ep, cap) : nullptr;
        case '-': return min_expand(s, p, ep, cap);
        default:
            if (!m) return nullptr;
            s++;
            p = ep;
            goto init;
        }
    }
    }
}

const char *lmemfind(const char *s1, size_t l1, const char *s2, size_t l2)
{
    if (l2 == 0) return s1;
    if (l2 > l1) return nullptr;
    const char *init;
    l2--;
    l1 = l1 - l2;
    while (l1 > 0 && (init = (const char *)std::memchr(s1, *s2, l1)) != nullptr) {
        init++;
        if (std::memcmp(init, s2 + 1, l2) == 0) return init - 1;
        l1 -= init - s1;
        s1 = init;
    }
    return nullptr;
}

void push_captures(Interp &I, Capture *cap, std::vector<Value> &r)
{
    for (int i = 0; i < cap->level; i++) {
        const long l = cap->capture[i].len;
        if (l == -1) rt_error("unfinished capture");
        r.push_back(I.str(std::string(cap->capture[i].init, (size_t)l)));
    }
}

void s_find(Interp &I, std::vector<Value> &a, std::vector<Value> &r)   // lstrlib.cpp:487-521
{
    const std::string S = check_str(I, a, 1);
    const std::string Pt = check_str(I, a, 2);
    const char *s = S.c_str(), *p = Pt.c_str();
    const size_t l1 = S.size(), l2 = Pt.size();
    const long init = posrelat(opt_long(a, 3, 1), l1) - 1;
    if (!(0 <= init && (size_t)init <= l1)) argerror(3, "out of range");
    if (a.size() > 3 || std::strpbrk(p, "^$*+?.([%-") == nullptr) {
        const char *s2 = lmemfind(s + init, l1 - (size_t)init, p, l2);
        if (s2) {
            r = {num((double)(s2 - s + 1)), num((double)(s2 - s + (long)l2))};
            return;
        }
    } else {
        const int anchor = *p == '^' ? (p++, 1) : 0;
        const char *s1 = s + init;
        Capture cap;
        cap.src_end = s + l1;
        Matcher M{I};
        do {
            cap.level = 0;
            const char *res = M.match(s1, p, &cap);
            if (res != nullptr) {
                r = {num((double)(int)(s1 - s + 1)), num((double)(int)(res - s))};
                push_captures(I, &cap, r);
                return;
            }
        } while (s1++ < cap.src_end && !anchor);
    }
    r.assign(1, Value());
}

void s_gsub(Interp &I, std::vector<Value> &a, std::vector<Value> &r)   // lstrlib.cpp:562-597
{
    const std::string Src = check_str(I, a, 1);
    const std::string Pt = check_str(I, a, 2);
    const char *src = Src.c_str();
    const char *p = Pt.c_str();
    const size_t srcl = Src.size();
    const int max_s = opt_int(a, 4, (int)srcl + 1);
    const int anchor = *p == '^' ? (p++, 1) : 0;
    std::string repl_text;
    bool repl_is_text = false;
    if (!(a.size() >= 3 && (a[2].t == TSTR || a[2].t == TNUM || a[2].t == TFUN))) argerror(3, "string or function expected");
    if (a[2].t != TFUN) {
        repl_is_text = true;
        I.tostring(a[2], &repl_text);
    }
    int n = 0;
    Capture cap;
    cap.src_end = src + srcl;
    Matcher M{I};
    std::string b;
    while (n < max_s) {
        cap.level = 0;
        const char *e = M.match(src, p, &cap);
        if (e) {
            n++;
            if (repl_is_text) {   // add_s (lstrlib.cpp:524-559)
                for (size_t i = 0; i < repl_text.size(); i++) {
                    if (repl_text[i] != '%') b += repl_text[i];
                    else {
                        i++;
                        if (!std::isdigit((unsigned char)repl_text[i])) b += repl_text[i];
                        else {
                            const int level = check_capture(repl_text[i], &cap);
                            b.append(cap.capture[level].init, (size_t)cap.capture[level].len);
                        }
                    }
                }
            } else {
                std::vector<Value> args, res;
                push_captures(I, &cap, args);
                I.call(a[2], args, res);
                std::string t;
                if (!res.empty() && I.tostring(res[0], &t)) b += t;
            }
        }
        if (e && e > src) src = e;
        else if (src < cap.src_end) b += *src++;
        else break;
        if (anchor) break;
    }
    b.append(src, (size_t)(cap.src_end - src));
    r = {I.str(b), num((double)n)};
}

void s_format(Interp &I, std::vector<Value> &a, std::vector<Value> &r)   // lstrlib.cpp:627-716
{
    int argi = 1;
    const std::string F = check_str(I, a, argi);
    const char *strfrmt = F.c_str();
    std::string b;
    Matcher M{I};
    while (*strfrmt) {
        if (*strfrmt != '%') b += *strfrmt++;
        else if (*++strfrmt == '%') b += *strfrmt++;
        else {
            Capture cap;
            char form[20];
            char buff[512];
            const char *initf = strfrmt;
            form[0] = '%';
            if (std::isdigit((unsigned char)*initf) && *(initf + 1) == '$') {
                argi = *initf - '0';
                initf += 2;
            }
            argi++;
            cap.src_end = strfrmt + std::strlen(strfrmt) + 1;
            cap.level = 0;
            strfrmt = M.match(initf, "[-+ #0]*(%d*)%.?(%d*)", &cap);
            if (cap.capture[0].len > 2 || cap.capture[1].len > 2 || strfrmt - initf > 20 - 2)
                rt_error("invalid format (width or precision too long)");
            std::strncpy(form + 1, initf, (size_t)(strfrmt - initf + 1));
            form[strfrmt - initf + 2] = 0;
            switch (*strfrmt++) {
            case 'c': case 'd': case 'i':
                std::snprintf(buff, sizeof buff, form, check_int(a, argi));
                break;
            case 'o': case 'u': case 'x': case 'X':
                std::snprintf(buff, sizeof buff, form, (unsigned int)check_number(a, argi).re);
                break;
            case 'e': case 'E': case 'f': case 'g': case 'G':
                // (the reference passes the CComplex through `...`; on x86-64
                // the conversion reads its real part)
                std::snprintf(buff, sizeof buff, form, check_number(a, argi).re);
                break;
            case 'q': {   // luaI_addquoted (lstrlib.cpp:602-623)
                const std::string s = check_str(I, a, argi);
                b += '"';
                for (char c : s) {
                    if (c == '"' || c == '\\' || c == '\n') { b += '\\'; b += c; }
                    else if (c == '\0') b += "\\000";
                    else b += c;
                }
                b += '"';
                continue;
            }
            case 's': {
                const std::string s = check_str(I, a, argi);
                if (cap.capture[1].len == 0 && s.size() >= 100) {
                    b += s;
                    continue;
                }
                std::snprintf(buff, sizeof buff, form, s.c_str());
                break;
            }
            default: rt_error("invalid option in `format'");
            }
            b.append(buff, std::strlen(buff));
        }
    }
    r.assign(1, I.str(b));
}

// -- math library (lmathlib.cpp), complex as femmcomplex.cpp ----------------------
#define MATH1(NAME, EXPR)                                                    \
    void NAME(Interp &, std::vector<Value> &a, std::vector<Value> &r)       \
    {                                                                        \
        const Cx x = check_number(a, 1);                                     \
        r.assign(1, num(EXPR));                                              \
    }
MATH1(m_abs, Cx({cabs_(x), 0.}))
MATH1(m_sin, csin(x))
MATH1(m_cos, ccos(x))
MATH1(m_tan, ctan(x))
MATH1(m_asin, casin(x))
MATH1(m_acos, cacos(x))
MATH1(m_atan, catan(x))
MATH1(m_ceil, Cx({std::ceil(x.re), 0.}))
MATH1(m_floor, Cx({std::floor(x.re), 0.}))
MATH1(m_sqrt, csqrt(x))
MATH1(m_log, clog(x))
MATH1(m_log10, divd(clog(x), std::log(10.)))
MATH1(m_exp, cexp(x))
MATH1(m_deg, divd(x, kRadPerDeg))
MATH1(m_rad, scale(x, kRadPerDeg))
MATH1(m_arg, Cx({carg(x), 0.}))
MATH1(m_re, Cx({x.re, 0.}))
MATH1(m_im, Cx({x.im, 0.}))
MATH1(m_conj, Cx({x.re, -x.im}))
MATH1(m_tanh, ctanh(x))
MATH1(m_cosh, ccosh(x))
MATH1(m_sinh, csinh(x))
#undef MATH1
void m_pow(Interp &, std::vector<Value> &a, std::vector<Value> &r)   // math_pow (lmathlib.cpp:114-118)
{
    const Cx x = check_number(a, 1), y = check_number(a, 2);
    if (y.im == 0 && y.re == std::floor(y.re)) {   // pow(CComplex, CComplex) (femmcomplex.cpp:807-812)
        if (std::fabs(y.re) > 1048576.0)
            throw Unsupported("an integral exponent beyond 2^20 (the reference multiplies that many times)");
        r.assign(1, num(cpow_int(x, (long long)(int)y.re)));
        return;
    }
    r.assign(1, num(cexp(mul(y, clog(x)))));
}
void m_atan2(Interp &, std::vector<Value> &a, std::vector<Value> &r)
{
    const Cx y = check_number(a, 1), x = check_number(a, 2);
    r.assign(1, num(catan2(y, x)));
}
void m_mod(Interp &, std::vector<Value> &a, std::vector<Value> &r)
{
    const Cx x = check_number(a, 1), y = check_number(a, 2);
    r.assign(1, num(std::fmod(x.re, y.re)));
}
void m_frexp(Interp &, std::vector<Value> &a, std::vector<Value> &r)
{
    int e;
    const double m = std::frexp(check_number(a, 1).re, &e);
    r = {num(m), num((double)e)};
}
void m_ldexp(Interp &, std::vector<Value> &a, std::vector<Value> &r)
{
    const Cx x = check_number(a, 1);
    const int e = check_int(a, 2);
    r.assign(1, num(std::ldexp(x.re, e)));
}
void m_min(Interp &, std::vector<Value> &a, std::vector<Value> &r)
{
    double d = check_number(a, 1).re;
    for (int i = 2; i <= (int)a.size(); ++i) {
        const double y = check_number(a, i).re;
        if (y < d) d = y;
    }
    r.assign(1, num(d));
}
void m_max(Interp &, std::vector<Value> &a, std::vector<Value> &r)
{
    double d = check_number(a, 1).re;
    for (int i = 2; i <= (int)a.size(); ++i) {
        const double y = check_number(a, i).re;
        if (y > d) d = y;
    }
    r.assign(1, num(d));
}

// -- LuaInstance (LuaInstance.cpp:228-312) ------------------------------------------
void l_complex(Interp &, std::vector<Value> &a, std::vector<Value> &r)
{
    auto tonum = [&](int i) {   // lua_tonumber: 0 for what is not a number
        Value v = a[i - 1];
        return Interp::tonumber(v) ? v.n : Cx{0., 0.};
    };
    Cx y{0., 0.};
    if (a.size() == 2) y = add(tonum(1), mul(kI, tonum(2)));
    else if (a.size() == 1) y = tonum(1);
    r.assign(1, num(y));
}
void l_setcompat(Interp &I, std::vector<Value> &a, std::vector<Value> &)
{
    if (a.empty()) return;
    Value v = a[0];
    const bool m = Interp::tonumber(v) ? (v.n.re == 1) : false;
    if (m != I.compat) I.changed = true;
    I.compat = m;
}
void l_getcompat(Interp &I, std::vector<Value> &, std::vector<Value> &r) { r.assign(1, num(I.compat ? 1.0 : 0.0)); }
void l_trace(Interp &, std::vector<Value> &, std::vector<Value> &) {}

}  // namespace

// ===========================================================================
// state
// ===========================================================================
Interp::Interp(bool axisymmetric) : axi(axisymmetric)
{
    srand_(1);
    tms.assign(kNumTags, std::vector<Value>(TM_N));   // luaT_init
    Value g = table(10);   // lstate.cpp:58
    G = tv(g);
    G->fixed = true;
    UdObj *nu = alloc<UdObj>();
    nu->fixed = true;
    null_ud = nu;
    // the globals in the order the reference defines them: lua_open
    // (lstate.cpp:64), lua_baselibopen, lua_strlibopen, lua_mathlibopen,
    // lua_iolibopen, LuaInstance::initializeLua (LuaInstance.cpp:194-207)
    auto reg = [&](const char *name, Builtin f) { setglobal(name, builtin(f, name)); };
    reg("_ERRORMESSAGE", b_errormessage);
    const struct {
        const char *n;
        Builtin f;
    } base[] = {{"_ALERT", b_alert}, {"_ERRORMESSAGE", b_errormessage}, {"call", b_call},
                {"collectgarbage", b_collectgarbage}, {"copytagmethods", b_copytagmethods}, {"dofile", b_dofile},
                {"dostring", b_dostring}, {"error", b_error}, {"foreach", b_foreach}, {"foreachi", b_foreachi},
                {"gcinfo", u_gcinfo}, {"getglobal", b_getglobal}, {"gettagmethod", b_gettagmethod},
                {"globals", b_globals}, {"newtag", b_newtag}, {"next", b_next}, {"print", b_print},
                {"rawget", b_rawget}, {"rawset", b_rawset}, {"rawgettable", b_rawget}, {"rawsettable", b_rawset},
                {"setglobal", b_setglobal}, {"settag", b_settag}, {"settagmethod", b_settagmethod}, {"tag", b_tag},
                {"tonumber", b_tonumber}, {"tostring", b_tostring}, {"type", b_type}, {"assert", b_assert},
                {"getn", b_getn}, {"sort", b_sort}, {"tinsert", b_tinsert}, {"tremove", b_tremove}};
    for (const auto &b : base) reg(b.n, b.f);
    setglobal("_VERSION", str("Lua 4.0"));
    for (const char *d : {"foreachvar", "nextvar", "rawgetglobal", "rawsetglobal"}) reg(d, b_deprecated);
    const struct {
        const char *n;
        Builtin f;
    } strl[] = {{"strlen", s_len}, {"strsub", s_sub}, {"strlower", s_lower}, {"strupper", s_upper},
                {"strchar", s_char}, {"strrep", s_rep}, {"ascii", s_byte}, {"strbyte", s_byte},
                {"format", s_format}, {"strfind", s_find}, {"gsub", s_gsub}};
    for (const auto &b : strl) reg(b.n, b.f);
    const struct {
        const char *n;
        Builtin f;
    } math[] = {{"abs", m_abs}, {"sin", m_sin}, {"cos", m_cos}, {"tan", m_tan}, {"asin", m_asin},
                {"acos", m_acos}, {"atan", m_atan}, {"atan2", m_atan2}, {"ceil", m_ceil}, {"floor", m_floor},
                {"mod", m_mod}, {"frexp", m_frexp}, {"ldexp", m_ldexp}, {"sqrt", m_sqrt}, {"min", m_min},
                {"max", m_max}, {"log", m_log}, {"log10", m_log10}, {"exp", m_exp}, {"deg", m_deg},
                {"rad", m_rad}, {"random", m_random}, {"randomseed", m_randomseed}, {"arg", m_arg},
                {"re", m_re}, {"im", m_im}, {"conj", m_conj}, {"tanh", m_tanh}, {"cosh", m_cosh},
                {"sinh", m_sinh}};
    for (const auto &b : math) reg(b.n, b.f);
    tms[TNUM][TM_POW] = builtin(m_pow, "pow");   // lmathlib.cpp:319-320
    setglobal("PI", num(kPi));
    setglobal("I", num(Cx{0., 1.}));
    reg("_ERRORMESSAGE", b_errormessage);   // liolib.cpp's errorfb replaces it
    for (const char *n : {"clock", "date", "debug", "execute", "exit", "getenv", "remove", "rename", "setlocale",
                          "tmpname", "appendto", "closefile", "flush", "openfile", "read", "readfrom", "seek"})
        reg(n, u_io);
    reg("write", io_write);
    reg("writeto", u_io);
    newtag();   // the io library's iotag (6) and closedtag (7), liolib.cpp:775-776
    newtag();
    // the predefined file handles (liolib.cpp:129-137, 785-790): userdata of the io tag
    static const int kStdin = 0, kStdout = 1, kStderr = 2;
    setglobal("_INPUT", udata(&kStdin, 6));
    setglobal("_OUTPUT", udata(&kStdout, 6));
    setglobal("_STDIN", udata(&kStdin, 6));
    setglobal("_STDOUT", udata(&kStdout, 6));
    setglobal("_STDERR", udata(&kStderr, 6));
    reg("Complex", l_complex);
    reg("setcompatibilitymode", l_setcompat);
    reg("getcompatibilitymode", l_getcompat);
    reg("femmVersion", u_femmversion);
    reg("trace", l_trace);
    setglobal("pi", num(kPi));
    static const char *const names[7] = {"x", "y", "r", "z", "theta", "R", "n"};
    for (int k = 0; k < 7; ++k) {
        nm[k] = str(names[k]);
        nm[k].o->fixed = true;
    }
    errormessage_fn = getglobal("_ERRORMESSAGE");
    alert_fn = getglobal("_ALERT");
}

Interp::~Interp()
{
    while (gclist) {
        Obj *n = gclist->gcnext;
        delete gclist;
        gclist = n;
    }
}

// mark from the roots (the globals, the values left on the stack, the
// library's handlers), sweep the rest; only between elements
void Interp::gc()
{
    std::vector<Obj *> work;
    auto push = [&](const Value &v) {
        if (v.o && !v.o->mark) {
            v.o->mark = true;
            work.push_back(v.o);
        }
    };
    G->mark = true;
    work.push_back(G);
    null_ud->mark = true;
    for (const Value &v : leaked) push(v);
    push(errormessage_fn);
    push(alert_fn);
    for (const auto &per_tag : tms)
        for (const Value &v : per_tag) push(v);
    while (!work.empty()) {
        Obj *o = work.back();
        work.pop_back();
        if (TableObj *t = dynamic_cast<TableObj *>(o)) {
            for (const Node &n : t->node) {
                push(n.key);
                push(n.val);
            }
        } else if (FuncObj *f = dynamic_cast<FuncObj *>(o)) {
            for (const Value &u : f->up) push(u);
        }
    }
    Obj **pp = &gclist;
    long long n = 0;
    while (*pp) {
        Obj *o = *pp;
        if (o->mark || o->fixed) {
            o->mark = false;
            pp = &o->gcnext;
            ++n;
        } else {
            *pp = o->gcnext;
            delete o;
        }
    }
    nobjs = n;
    gc_at = std::max<long long>(200000, 2 * n);
}

// ===========================================================================
// Session: one element of static2d.cpp:509-583 / staticaxi.cpp:350-406
// ===========================================================================
bool text_to_number(const char *s, Cx *out) { return str2d(s, out); }

int Session::run_chunk(const std::string &text, std::string *output)
{
    char top;
    I->stack_top = &top;
    I->capture = output;
    I->steps = 0;
    I->depth = 0;
    I->units = 0;
    ++I->epoch;
    std::vector<Value> res;
    int status;
    try {
        status = I->dostring(text, res);
    } catch (...) {
        I->capture = nullptr;
        throw;
    }
    I->capture = nullptr;
    return status;
}

Session::Session(bool axisymmetric) : I(new Interp(axisymmetric)) {}
Session::~Session() = default;
bool Session::state_changed() const { return I->changed; }
long long Session::leaked() const { return (long long)I->leaked.size(); }

namespace {
// the value "name=%.17g" leaves in a global: the literal read back by the
// lexer, a leading '-' the unary minus of lcode.cpp:649-664; "inf" / "nan"
// are names (globals, nil unless a chunk defined them)
Value literal(Interp &I, double v)
{
    const bool minus = std::signbit(v);   // (%.17g prints the sign of -0 too)
    if (!std::isfinite(v)) {   // "inf" / "nan": names
        Value g = I.getglobal(std::isnan(v) ? "nan" : "inf");
        if (!minus) return g;
        if (!Interp::tonumber(g)) rt_error("attempt to perform arithmetic");
        return num(neg(g.n));
    }
    // %.17g and the lexer's strtod give the double back exactly
    const double f = std::fabs(v);
    if (f <= (double)kMaxArgS && (double)(int)f == f) return num(Cx{(double)(minus ? -(int)f : (int)f), 0.});
    return num(minus ? Cx{-f, -0.0} : Cx{f, 0.});
}
}  // namespace

ElementResult Session::run_element(const std::string &fctn, Cx X)
{
    Interp &S = *I;
    char top;
    S.stack_top = &top;
    ElementResult R;
    ++S.epoch;
    S.steps = 0;
    S.depth = 0;
    S.units = 0;
    const double theta = carg(X) * 180 / kPi, RR = cabs_(X);
    try {
        Chunk *c;
        if (S.last_chunk && S.last_text == fctn) {
            c = S.last_chunk;
        } else {
            // the 4096-byte buffer (static2d.cpp:517, 530): a longer chunk is
            // cut (the prelude is at most ~130 bytes)
            std::string body = fctn.substr(0, std::strlen(fctn.c_str()));   // (a C string)
            bool cut = false;
            if (body.size() + 160 > 4095) {
                char pre[512];
                const int np = std::snprintf(pre, sizeof pre, "x=%.17g\ny=%.17g\nr=x\nz=y\ntheta=%.17g\nR=%.17g\nreturn ",
                                             X.re, X.im, theta, RR);
                if (np + body.size() > 4095) {
                    body.resize(np > 4095 ? 0 : 4095 - (size_t)np);
                    cut = true;
                }
            }
            c = S.compile("return " + body);
            S.last_text = fctn;
            S.last_chunk = cut ? nullptr : c;   // (a cut chunk depends on this element's digits)
        }
        // the prelude: six global assignments
        S.in_prelude = true;
        const Value *n = S.nm;   // x y r z theta R
        if (S.axi) {
            S.setglobal(n[2], literal(S, X.re));
            S.setglobal(n[3], literal(S, X.im));
            S.setglobal(n[0], S.getglobal(n[2]));
            S.setglobal(n[1], S.getglobal(n[3]));
        } else {
            S.setglobal(n[0], literal(S, X.re));
            S.setglobal(n[1], literal(S, X.im));
            S.setglobal(n[2], S.getglobal(n[0]));
            S.setglobal(n[3], S.getglobal(n[1]));
        }
        S.setglobal(n[4], literal(S, theta));
        S.setglobal(n[5], literal(S, RR));
        S.in_prelude = false;
        FuncObj main;
        main.p = c->protos[0].get();
        std::vector<Value> none, res;
        S.run_proto(&main, none, res);
        R.nresults = (int)res.size();
        if (!res.empty()) {
            R.text = S.tostring(res.back(), &R.str);
            for (size_t k = 0; k + 1 < res.size(); ++k) S.leaked.push_back(res[k]);   // Unsafe: one popped
            if ((long long)S.leaked.size() > kMaxLeaked)
                throw Unsupported("more than 3000 values left on the reference's Lua stack (a chunk returning "
                                  "several values; the reference's 4096-slot stack overflows near there)");
        }
    } catch (const LuaError &) {
        S.in_prelude = false;
        R = ElementResult();
        R.error = true;
    }
    if (S.nobjs > S.gc_at) S.gc();
    return R;
}

}  // namespace lua
}  // namespace xfk
