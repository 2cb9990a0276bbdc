// xfk_magdir.cpp -- evaluator of MagDirFctn expressions (see xfk_magdir.h).
//
// What is restated, and from where (temudschin/xfemm @ 2025-02-04):
//   * the chunk static2d.cpp:530-531 builds: the element centroid X (CComplex
//     sum of the three nodes, / units[LengthUnits] / 3), x = Re X, y = Im X,
//     r = x, z = y, theta = arg(X) 180 / PI, R = abs(X), each printed with
//     %.17g and read back by the Lua lexer -- so a negative non-integral
//     value arrives as the negated literal (imaginary part -0) and an integral
//     one as a PUSHINT constant (lcode.cpp:131-137, 649-664, lvm.cpp:460-486);
//   * Lua 4.0's expression grammar and priorities (lparser.cpp:689-858:
//     + - 5/5, * / 6/6, ^ 9/8 right-assoc, comparisons 2/2, and / or 1/1,
//     unary - and not at 7), the `a + k` / `a - k` integer peephole (ADDI,
//     lcode.cpp:609-634) and the value semantics of lvm.cpp (arithmetic on
//     non-numbers is a run-time error; comparisons give 1 or nil; a <= b is
//     not (b < a); and / or return an operand);
//   * the complex number of the xfemm Lua (femmcomplex.cpp), operation by
//     operation as the C++ overloads resolve there, and the math library
//     lmathlib.cpp registers (radians; PI, I globals; pow as the ^ tag method).
// Not supported (refused with a message naming the construct, not a Lua
// error): tables, field access and indexing, anonymous functions, upvalues,
// method calls, '...', and the base / string / I/O library functions,
// random / randomseed included (not reproducible).
#include "xfk_magdir.h"

#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace xfk {
namespace {

// ---------------------------------------------------------------------------
// CComplex arithmetic (femmcomplex.cpp); line numbers of that file
// ---------------------------------------------------------------------------
struct Cx {
    double re, im;
};

const double kPi = 3.141592653589793238462643383;            // femmcomplex.cpp:26, femmconstants.h
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

bool cpow(Cx x, Cx y, Cx *out)   // :807-812 (the integer loop is capped: an exponent beyond 2^20 is refused)
{
    if (y.im == 0 && y.re == std::floor(y.re)) {
        if (std::fabs(y.re) > 1048576.0) return false;
        *out = cpow_int(x, (long long)(int)y.re);
        return true;
    }
    *out = cexp(mul(y, clog(x)));
    return true;
}

// ---------------------------------------------------------------------------
// numbers <-> strings as the xfemm Lua converts them
// ---------------------------------------------------------------------------
// lua_number2str (lobject.cpp:228-232) = CComplex::ToString (femmcomplex.cpp:150-176);
// false for the empty text ToString gives a NaN imaginary part
bool number2str(Cx n, char *s, size_t len)
{
    const double re = n.re, im = n.im;
    if (im == 0) std::snprintf(s, len, "%.16g", re);
    else if (im == 1) {
        if (re == 0) std::snprintf(s, len, "I");
        else std::snprintf(s, len, "%.16g+I", re);
    } else if (im == -1) {
        if (re == 0) std::snprintf(s, len, "-I");
        else std::snprintf(s, len, "%.16g-I", re);
    } else if (im < 0) {
        if (re != 0) std::snprintf(s, len, "%.16g-I*%.16g", re, std::fabs(im));
        else std::snprintf(s, len, "-I*%.16g", std::fabs(im));
    } else if (im > 0) {
        if (re != 0) std::snprintf(s, len, "%.16g+I*%.16g", re, im);
        else std::snprintf(s, len, "I*%.16g", im);
    } else s[0] = '\0';
    return s[0] != '\0';
}

// string -> number: luaO_str2d (lobject.cpp:138-147) over lua_str2number
// (:78-136), which also reads "a+I*b" forms
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

// ---------------------------------------------------------------------------
// values and the parsed expression
// ---------------------------------------------------------------------------
enum VType { V_NIL = 0, V_NUM = 1, V_FN = 2, V_STR = 3 };

struct Val {
    int t = V_NIL;
    Cx v{0, 0};
    int fn = -1;
    std::string s;   // V_STR
};

// tonumber (lvm.cpp:42-53): a number, or a string luaO_str2d reads
bool coerce(Val &a)
{
    if (a.t == V_NUM) return true;
    if (a.t != V_STR || !str2d(a.s.c_str(), &a.v)) return false;
    a.t = V_NUM;
    return true;
}

// tostring (lvm.cpp:56-68): a string, or a number's ToString text
bool to_str(const Val &a, std::string *out)
{
    if (a.t == V_STR) { *out = a.s; return true; }
    if (a.t != V_NUM) return false;
    char buf[256];
    number2str(a.v, buf, sizeof buf);
    *out = buf;
    return true;
}

enum Builtin {
    F_ABS, F_SIN, F_COS, F_TAN, F_ASIN, F_ACOS, F_ATAN, F_ATAN2, F_CEIL, F_FLOOR, F_MOD, F_FREXP, F_LDEXP,
    F_SQRT, F_MIN, F_MAX, F_LOG, F_LOG10, F_EXP, F_DEG, F_RAD, F_ARG, F_RE, F_IM, F_CONJ, F_TANH, F_COSH,
    F_SINH, F_COUNT
};
const char *const kBuiltinNames[F_COUNT] = {
    "abs", "sin", "cos", "tan", "asin", "acos", "atan", "atan2", "ceil", "floor", "mod", "frexp", "ldexp",
    "sqrt", "min", "max", "log", "log10", "exp", "deg", "rad", "arg", "re", "im", "conj", "tanh", "cosh", "sinh"};

// the chunk's globals: x y r z theta R (static2d.cpp:530), PI and I (lmathlib.cpp:321-325)
enum Global { G_X, G_Y, G_R, G_Z, G_THETA, G_RR, G_PI, G_I, G_COUNT };

enum Kind { K_INT, K_NUM, K_NEGNUM, K_STR, K_NIL, K_GLOBAL, K_FN, K_UNDEF, K_CALL, K_UNM, K_NOT, K_BIN, K_AND, K_OR };
enum BinOp { B_ADD, B_SUB, B_MUL, B_DIV, B_POW, B_EQ, B_NE, B_LT, B_LE, B_GT, B_GE, B_AND, B_OR, B_CONCAT, B_NONE };

struct Node {
    Kind k;
    int op = 0;             // BinOp, global index or builtin id; K_INT: the constant; K_STR: string index
    double v = 0;           // K_NUM / K_NEGNUM constant
    std::vector<int> kids;  // operands / call arguments
};

}  // namespace

struct MagDirExpr {
    std::string text;       // MagDirFctn as given (for the messages)
    std::vector<Node> nodes;
    std::vector<std::string> strs;   // string literals
    std::vector<int> ret;   // the return list (empty: the chunk returns nothing)
};

namespace {

// ---------------------------------------------------------------------------
// lexer (llex.cpp) and parser (lparser.cpp), expressions only
// ---------------------------------------------------------------------------
enum Tok { T_EOS = 256, T_NUM, T_STR, T_CONCAT, T_NAME, T_EQ, T_NE, T_LE, T_GE, T_AND, T_OR, T_NOT, T_NIL, T_KEYWORD, T_BAD };

const int kMaxArgS = ((1 << 26) - 1) >> 1;   // MAXARG_S (llimits.h:101-119)

struct Parser {
    const char *s;
    size_t pos = 0;
    int tok = T_EOS;
    double num = 0;
    std::string name, str;
    bool ok = true;
    std::string unsup;   // a construct the reference's Lua accepts and this evaluator does not
    MagDirExpr *E;

    explicit Parser(const char *text, MagDirExpr *e) : s(text), E(e) { next(); }

    void fail() { ok = false; tok = T_BAD; }
    void unsupported(const std::string &what)
    {
        if (unsup.empty()) unsup = what;
        fail();
    }

    void next()
    {
        if (!ok) return;
        for (;;) {
            const char c = s[pos];
            if (c == '\0') { tok = T_EOS; return; }
            if (std::isspace((unsigned char)c)) { ++pos; continue; }
            if (c == '-' && s[pos + 1] == '-') {   // comment to the end of the line (llex.cpp:375-383)
                while (s[pos] && s[pos] != '\n') ++pos;
                continue;
            }
            break;
        }
        const char c = s[pos];
        if (std::isdigit((unsigned char)c) || (c == '.' && std::isdigit((unsigned char)s[pos + 1]))) {
            // read_number (llex.cpp:168-208) + luaO_str2d / lua_str2number
            std::string buf;
            while (std::isdigit((unsigned char)s[pos])) buf += s[pos++];
            if (s[pos] == '.') {
                buf += s[pos++];
                if (s[pos] == '.') { fail(); return; }   // "ambiguous syntax"
            }
            while (std::isdigit((unsigned char)s[pos])) buf += s[pos++];
            if (s[pos] == 'e' || s[pos] == 'E') {
                buf += s[pos++];
                if (s[pos] == '+' || s[pos] == '-') buf += s[pos++];
                while (std::isdigit((unsigned char)s[pos])) buf += s[pos++];
            }
            char *end = nullptr;
            num = std::strtod(buf.c_str(), &end);
            while (end && std::isspace((unsigned char)*end)) ++end;
            if (!end || end == buf.c_str() || *end != '\0') { fail(); return; }   // "malformed number"
            tok = T_NUM;
            return;
        }
        if (std::isalpha((unsigned char)c) || c == '_') {
            name.clear();
            while (std::isalnum((unsigned char)s[pos]) || s[pos] == '_') name += s[pos++];
            static const char *const kw[] = {"break", "do", "else", "elseif", "end", "for", "function", "if",
                                             "in", "local", "repeat", "return", "then", "until", "while"};
            if (name == "and") tok = T_AND;
            else if (name == "or") tok = T_OR;
            else if (name == "not") tok = T_NOT;
            else if (name == "nil") tok = T_NIL;
            else {
                tok = T_NAME;
                for (const char *k : kw)
                    if (name == k) tok = T_KEYWORD;
            }
            return;
        }
        ++pos;
        const char d = s[pos];
        switch (c) {
        case '=': if (d == '=') { ++pos; tok = T_EQ; } else tok = '='; return;
        case '<': if (d == '=') { ++pos; tok = T_LE; } else tok = '<'; return;
        case '>': if (d == '=') { ++pos; tok = T_GE; } else tok = '>'; return;
        case '~': if (d == '=') { ++pos; tok = T_NE; } else fail(); return;
        case '+': case '-': case '*': case '/': case '^': case '(': case ')': case ',': case ';':
            tok = c;
            return;
        case '.':   // '..' (a lone '.', field access, and '...' are not supported)
            if (d == '.' && s[pos + 1] != '.') { ++pos; tok = T_CONCAT; }
            else unsupported(d == '.' ? "'...' (variable arguments)" : "field access ('.')");
            return;
        case '"':
        case '\'':   // read_string (llex.cpp:261-352)
            str.clear();
            for (;;) {
                char ch = s[pos];
                if (ch == c) { ++pos; break; }
                if (ch == '\0' || ch == '\n') { fail(); return; }   // "unfinished string"
                if (ch != '\\') { str += ch; ++pos; continue; }
                ch = s[++pos];
                switch (ch) {
                case 'a': str += '\a'; ++pos; break;
                case 'b': str += '\b'; ++pos; break;
                case 'f': str += '\f'; ++pos; break;
                case 'n': str += '\n'; ++pos; break;
                case 'r': str += '\r'; ++pos; break;
                case 't': str += '\t'; ++pos; break;
                case 'v': str += '\v'; ++pos; break;
                case '\0': fail(); return;
                default:
                    if (std::isdigit((unsigned char)ch)) {
                        int v = 0, k = 0;
                        do { v = 10 * v + (s[pos] - '0'); ++pos; } while (++k < 3 && std::isdigit((unsigned char)s[pos]));
                        if (v != (unsigned char)v) { fail(); return; }   // "escape sequence too large"
                        str += (char)v;
                    } else {
                        str += ch;   // \\, \", \', \newline, ...
                        ++pos;
                    }
                }
            }
            tok = T_STR;
            return;
        case '[':   // [[long string]] (llex.cpp:212-258)
            if (d != '[') { unsupported("table indexing ('[')"); return; }
            {
                ++pos;
                int cont = 0;
                str.clear();
                for (;;) {
                    const char ch = s[pos];
                    if (ch == '\0') { fail(); return; }   // "unfinished long string"
                    if (ch == '[' && s[pos + 1] == '[') { ++cont; str += "[["; pos += 2; continue; }
                    if (ch == ']' && s[pos + 1] == ']') {
                        if (cont == 0) { pos += 2; break; }
                        --cont;
                        str += "]]";
                        pos += 2;
                        continue;
                    }
                    str += ch;
                    ++pos;
                }
            }
            tok = T_STR;
            return;
        case '{': case '}': unsupported("tables ('{ }')"); return;
        case '%': unsupported("upvalues ('%')"); return;
        case ':': unsupported("method calls (':')"); return;
        default:   // not a Lua 4 token either: the reference's lexer refuses it too
            fail();
            return;
        }
    }

    int add(Node n)
    {
        E->nodes.push_back(std::move(n));
        return (int)E->nodes.size() - 1;
    }

    static BinOp binop(int t)
    {
        switch (t) {
        case '+': return B_ADD;
        case '-': return B_SUB;
        case '*': return B_MUL;
        case '/': return B_DIV;
        case '^': return B_POW;
        case T_EQ: return B_EQ;
        case T_NE: return B_NE;
        case '<': return B_LT;
        case T_LE: return B_LE;
        case '>': return B_GT;
        case T_GE: return B_GE;
        case T_AND: return B_AND;
        case T_OR: return B_OR;
        case T_CONCAT: return B_CONCAT;
        default: return B_NONE;
        }
    }
    // priority[] of lparser.cpp:808-821
    static int left(BinOp o) { static const int p[] = {5, 5, 6, 6, 9, 2, 2, 2, 2, 2, 2, 1, 1, 4}; return p[o]; }
    static int right(BinOp o) { static const int p[] = {5, 5, 6, 6, 8, 2, 2, 2, 2, 2, 2, 1, 1, 3}; return p[o]; }

    int number_node(double f)   // luaK_number (lcode.cpp:131-137)
    {
        Node n;
        if (f <= (double)kMaxArgS && (double)(int)f == f) {
            n.k = K_INT;
            n.op = (int)f;
        } else {
            n.k = K_NUM;
            n.v = f;
        }
        return add(n);
    }

    int primary()   // simpleexp (lparser.cpp:689-745)
    {
        if (!ok) return -1;
        if (tok == T_NUM) {
            const double f = num;
            next();
            return number_node(f);
        }
        if (tok == T_NIL) {
            next();
            Node n;
            n.k = K_NIL;
            return add(n);
        }
        if (tok == T_STR) {
            Node n;
            n.k = K_STR;
            n.op = (int)E->strs.size();
            E->strs.push_back(str);
            next();
            return add(n);
        }
        if (tok == '(') {
            next();
            const int e = expr();
            if (!ok || tok != ')') { fail(); return -1; }
            next();
            return e;
        }
        if (tok == T_NAME) {
            const std::string nm = name;
            next();
            Node n;
            static const char *const gl[G_COUNT] = {"x", "y", "r", "z", "theta", "R", "PI", "I"};
            n.k = K_UNDEF;
            for (int g = 0; g < G_COUNT; ++g)
                if (nm == gl[g]) { n.k = K_GLOBAL; n.op = g; }
            for (int f = 0; f < F_COUNT && n.k == K_UNDEF; ++f)
                if (nm == kBuiltinNames[f]) { n.k = K_FN; n.op = f; }
            if (n.k == K_UNDEF && tok == '(') {
                // functions of the reference Lua's base, string and math
                // libraries this evaluator does not restate (lbaselib.cpp,
                // lstrlib.cpp, lmathlib.cpp random / randomseed)
                static const char *const lib[] = {
                    "assert", "call", "collectgarbage", "copytagmethods", "dofile", "dostring", "error", "foreach",
                    "foreachi", "getglobal", "getn", "gettagmethod", "globals", "newtag", "next", "print", "rawget",
                    "rawset", "setglobal", "settag", "settagmethod", "sort", "tag", "tinsert", "tonumber",
                    "tostring", "tremove", "type", "strlen", "strsub", "strlower", "strupper", "strchar", "strrep",
                    "ascii", "strbyte", "format", "strfind", "gsub", "random", "randomseed", "rawgettable",
                    "rawsettable", "read", "write", "date", "clock", "getenv", "execute", "remove", "rename",
                    "tmpname", "exit", "openfile", "closefile", "readfrom", "writeto", "appendto", "flush", "seek"};
                for (const char *f : lib)
                    if (nm == f) {
                        unsupported("the library function " + nm + "()");
                        return -1;
                    }
            }
            int id = add(n);
            while (ok && tok == '(') {   // call suffix: f(args)
                next();
                Node c;
                c.k = K_CALL;
                c.kids.push_back(id);
                if (tok != ')') {
                    for (;;) {
                        const int a = expr();
                        if (!ok) return -1;
                        c.kids.push_back(a);
                        if (tok != ',') break;
                        next();
                    }
                }
                if (tok != ')') { fail(); return -1; }
                next();
                id = add(c);
            }
            return id;
        }
        if (tok == T_KEYWORD && name == "function") unsupported("anonymous functions");
        else fail();   // "<expression> expected"
        return -1;
    }

    int subexpr(int limit, int *stop)   // lparser.cpp:828-853
    {
        int v;
        if (tok == '-' || tok == T_NOT) {
            const bool minus = tok == '-';
            next();
            int dummy;
            const int e = subexpr(7, &dummy);   // UNARY_PRIORITY
            if (!ok) return -1;
            if (minus && E->nodes[e].k == K_INT) {          // PUSHINT -> PUSHINT -k (lcode.cpp:653-656)
                E->nodes[e].op = -E->nodes[e].op;
                v = e;
            } else if (minus && E->nodes[e].k == K_NUM) {   // PUSHNUM -> PUSHNEGNUM (:657-660)
                E->nodes[e].k = K_NEGNUM;
                v = e;
            } else {
                Node n;
                n.k = minus ? K_UNM : K_NOT;
                n.kids.push_back(e);
                v = add(n);
            }
        } else {
            v = primary();
        }
        if (!ok) return -1;
        BinOp op = binop(tok);
        while (op != B_NONE && left(op) > limit) {
            next();
            BinOp nextop;
            int nx = 0;
            const int r = subexpr(right(op), &nx);
            if (!ok) return -1;
            nextop = (BinOp)nx;
            Node n;
            n.k = op == B_AND ? K_AND : op == B_OR ? K_OR : K_BIN;
            n.op = op;
            n.kids = {v, r};
            v = add(n);
            op = nextop;
        }
        *stop = op;
        return v;
    }

    int expr()
    {
        int stop;
        return subexpr(-1, &stop);
    }
};

// ---------------------------------------------------------------------------
// evaluation (lvm.cpp semantics)
// ---------------------------------------------------------------------------
struct Eval {
    const MagDirExpr &E;
    Val g[G_COUNT];
    bool ok = true;

    Val num(Cx c) { Val v; v.t = V_NUM; v.v = c; return v; }
    Val num(double d) { return num(Cx{d, 0.}); }
    Val err() { ok = false; return Val(); }

    // a builtin (lmathlib.cpp:36-277): args checked as luaL_check_number does
    std::vector<Val> call(int f, const std::vector<Val> &a)
    {
        auto arg = [&](size_t k, Cx *c) {   // luaL_check_number: a number or a numeric string
            if (k >= a.size()) return false;
            Val v = a[k];
            if (!coerce(v)) return false;
            *c = v.v;
            return true;
        };
        Cx x, y;
        if (!arg(0, &x)) { ok = false; return {}; }
        switch (f) {
        case F_ABS: return {num(cabs_(x))};
        case F_SIN: return {num(csin(x))};
        case F_COS: return {num(ccos(x))};
        case F_TAN: return {num(ctan(x))};
        case F_ASIN: return {num(casin(x))};
        case F_ACOS: return {num(cacos(x))};
        case F_ATAN: return {num(catan(x))};
        case F_ATAN2:
            if (!arg(1, &y)) { ok = false; return {}; }
            return {num(catan2(x, y))};
        case F_CEIL: return {num(std::ceil(x.re))};
        case F_FLOOR: return {num(std::floor(x.re))};
        case F_MOD:
            if (!arg(1, &y)) { ok = false; return {}; }
            return {num(std::fmod(x.re, y.re))};
        case F_FREXP: {
            int e;
            const double m = std::frexp(x.re, &e);
            return {num(m), num((double)e)};
        }
        case F_LDEXP:
            if (!arg(1, &y)) { ok = false; return {}; }
            return {num(std::ldexp(x.re, (int)y.re))};
        case F_SQRT: return {num(csqrt(x))};
        case F_MIN:
        case F_MAX: {
            double d = x.re;
            for (size_t k = 1; k < a.size(); ++k) {
                if (!arg(k, &y)) { ok = false; return {}; }
                if (f == F_MIN ? y.re < d : y.re > d) d = y.re;
            }
            return {num(d)};
        }
        case F_LOG: return {num(clog(x))};
        case F_LOG10: return {num(divd(clog(x), std::log(10.)))};
        case F_EXP: return {num(cexp(x))};
        case F_DEG: return {num(divd(x, kRadPerDeg))};
        case F_RAD: return {num(scale(x, kRadPerDeg))};
        case F_ARG: return {num(carg(x))};
        case F_RE: return {num(x.re)};
        case F_IM: return {num(x.im)};
        case F_CONJ: return {num(Cx{x.re, -x.im})};
        case F_TANH: return {num(ctanh(x))};
        case F_COSH: return {num(ccosh(x))};
        case F_SINH: return {num(csinh(x))};
        default: ok = false; return {};
        }
    }

    // every value of node i (a call may give several); expressions use the first
    std::vector<Val> multi(int i)
    {
        const Node &n = E.nodes[i];
        if (n.k != K_CALL) return {one(i)};
        const Val fv = one(n.kids[0]);
        if (!ok) return {};
        if (fv.t != V_FN) { ok = false; return {}; }   // "attempt to call a nil / number value"
        std::vector<Val> args;
        for (size_t k = 1; k < n.kids.size(); ++k) {
            if (k + 1 == n.kids.size()) {
                for (const Val &v : multi(n.kids[k])) args.push_back(v);   // the last argument expands
            } else {
                args.push_back(one(n.kids[k]));
            }
            if (!ok) return {};
        }
        return call(fv.fn, args);
    }

    Val one(int i)
    {
        if (!ok) return Val();
        const Node &n = E.nodes[i];
        switch (n.k) {
        case K_INT: return num((double)n.op);
        case K_NUM: return num(n.v);
        case K_NEGNUM: return num(Cx{-n.v, -0.0});
        case K_STR: { Val v; v.t = V_STR; v.s = E.strs[n.op]; return v; }
        case K_NIL: return Val();
        case K_GLOBAL: return g[n.op];
        case K_FN: { Val v; v.t = V_FN; v.fn = n.op; return v; }
        case K_UNDEF: return Val();
        case K_CALL: {
            std::vector<Val> r = multi(i);
            if (!ok) return Val();
            return r.empty() ? Val() : r[0];
        }
        case K_UNM: {
            Val a = one(n.kids[0]);
            if (!ok || !coerce(a)) return err();
            return num(neg(a.v));
        }
        case K_NOT: {
            const Val a = one(n.kids[0]);
            if (!ok) return Val();
            return a.t == V_NIL ? num(1.0) : Val();
        }
        case K_AND: {
            const Val a = one(n.kids[0]);
            if (!ok || a.t == V_NIL) return a;
            return one(n.kids[1]);
        }
        case K_OR: {
            const Val a = one(n.kids[0]);
            if (!ok || a.t != V_NIL) return a;
            return one(n.kids[1]);
        }
        case K_BIN: break;
        }
        Val a = one(n.kids[0]);
        Val b = one(n.kids[1]);
        if (!ok) return Val();
        const int op = n.op;
        if (op == B_EQ || op == B_NE) {   // luaO_equalObj: same type, same value
            bool eq = a.t == b.t &&
                      (a.t == V_NIL || (a.t == V_NUM ? a.v.re == b.v.re && a.v.im == b.v.im
                                                     : a.t == V_STR ? a.s == b.s : a.fn == b.fn));
            if (op == B_NE) eq = !eq;
            return eq ? num(1.0) : Val();
        }
        if (op == B_CONCAT) {   // luaV_strconc: strings and numbers (ToString text)
            std::string sa, sb;
            if (!to_str(a, &sa) || !to_str(b, &sb)) return err();
            Val v;
            v.t = V_STR;
            v.s = sa + sb;
            return v;
        }
        if (op >= B_LT && op <= B_GE) {   // luaV_lessthan: two numbers or two strings, no coercion
            bool lt;
            const bool swap = op == B_GT || op == B_LE;   // a > b is b < a; a <= b is not (b < a)
            const Val &l = swap ? b : a, &r = swap ? a : b;
            if (l.t == V_NUM && r.t == V_NUM) lt = l.v.re < r.v.re;   // CComplex::operator< (:539-543)
            else if (l.t == V_STR && r.t == V_STR) lt = std::strcoll(l.s.c_str(), r.s.c_str()) < 0;
            else return err();
            if (op == B_LE || op == B_GE) lt = !lt;
            return lt ? num(1.0) : Val();
        }
        // arithmetic: tonumber of the left operand, then of the right (lvm.cpp:590-637)
        if (!coerce(a) || !coerce(b)) return err();   // no tag method for nil / functions / text
        const Cx x = a.v, y = b.v;
        switch (op) {
        case B_ADD: return num(add(x, y));
        case B_SUB:
            // `a - k` with an integer literal k is ADDI -k (lcode.cpp:622-634): re + (-k), im + 0
            if (E.nodes[n.kids[1]].k == K_INT) return num(Cx{x.re + (double)(-E.nodes[n.kids[1]].op), x.im + 0.0});
            return num(sub(x, y));
        case B_MUL: return num(mul(x, y));
        case B_DIV: return num(cdiv(x, y));
        case B_POW: {
            Cx r;
            if (!cpow(x, y, &r)) return err();
            return num(r);
        }
        default: return err();
        }
    }
};

// the value the chunk's "x=%.17g" (etc.) leaves in a global: the literal read
// back by the lexer (a leading '-' is the unary minus of lcode.cpp:649-664)
Val literal_global(double v)
{
    char buf[64];
    std::snprintf(buf, sizeof buf, "%.17g", v);
    const bool minus = buf[0] == '-';
    const double f = std::strtod(buf + (minus ? 1 : 0), nullptr);
    Val r;
    if (!std::isfinite(f)) return r;   // "inf" / "nan" read as undefined names: nil
    r.t = V_NUM;
    if (f <= (double)kMaxArgS && (double)(int)f == f) r.v = {(double)(minus ? -(int)f : (int)f), 0.};
    else r.v = minus ? Cx{-f, -0.0} : Cx{f, 0.};
    return r;
}

std::string quoted(const char *fmt, const std::string &fctn)
{
    std::vector<char> buf(fctn.size() + 128);
    std::snprintf(buf.data(), buf.size(), fmt, fctn.c_str());
    return std::string(buf.data());
}

}  // namespace

std::shared_ptr<const MagDirExpr> magdir_parse(const std::string &fctn, std::string &err)
{
    auto E = std::make_shared<MagDirExpr>();
    E->text = fctn;
    Parser P(fctn.c_str(), E.get());
    // retstat (lparser.cpp): an optional expression list unless the block ends
    // or ';' follows, then an optional ';' and the end of the chunk
    if (P.tok == T_KEYWORD && P.name == "function") P.unsupported("anonymous functions");
    if (P.ok && P.tok != T_EOS && P.tok != ';' && P.tok != T_KEYWORD) {
        for (;;) {
            const int e = P.expr();
            if (!P.ok) break;
            E->ret.push_back(e);
            if (P.tok != ',') break;
            P.next();
        }
    }
    if (P.ok && P.tok == ';') P.next();
    if (!P.unsup.empty()) {   // valid Lua the native evaluator does not restate: say so
        err = "MagDirFctn \"" + fctn + "\": " + P.unsup +
              " not supported by the native expression evaluator (the reference's Lua would evaluate it)";
        return nullptr;
    }
    if (!P.ok || P.tok != T_EOS) {
        err = quoted("Lua error occurred when evaluating:\n\"%s\"", fctn);   // static2d.cpp:550-552
        return nullptr;
    }
    return E;
}

bool magdir_eval(const MagDirExpr &e, const double x[3], const double y[3], int length_units, double mag_dir,
                 double *t, std::string &err)
{
    static const double units[] = {2.54, 0.1, 1., 100., 0.00254, 1.e-04};   // femm::LengthUnit in cm
    // X = sum (x + I y) / units / 3 (static2d.cpp:521-525)
    Cx X{0., 0.};
    for (int j = 0; j < 3; ++j) {
        const Cx node = dplus(x[j], ipart(y[j]));   // x + I*y
        X = add(X, node);
    }
    X = divd(divd(X, units[length_units]), 3.);
    Eval ev{e};
    ev.g[G_X] = literal_global(X.re);
    ev.g[G_Y] = literal_global(X.im);
    ev.g[G_R] = ev.g[G_X];
    ev.g[G_Z] = ev.g[G_Y];
    ev.g[G_THETA] = literal_global(carg(X) * 180 / kPi);
    ev.g[G_RR] = literal_global(cabs_(X));
    ev.g[G_PI] = ev.num(3.14159265358979323846);   // lmathlib.cpp:321-322
    ev.g[G_I] = ev.num(Cx{0., 1.});
    if (e.ret.empty()) {   // nothing returned: the label's MagDir stays (static2d.cpp:559-561)
        *t = mag_dir;
        return true;
    }
    Val last;
    for (size_t k = 0; k < e.ret.size() && ev.ok; ++k) {
        if (k + 1 == e.ret.size()) {
            std::vector<Val> vs = ev.multi(e.ret[k]);
            if (ev.ok && !vs.empty()) last = vs.back();
        } else {
            ev.one(e.ret[k]);
        }
    }
    if (!ev.ok) {   // LUA_ERRRUN (static2d.cpp:539-556)
        err = quoted("Lua error occurred when evaluating:\n\"%s\"", e.text);
        return false;
    }
    // The reference reads the result back through lua_tostring and then
    // lua_tonumber (static2d.cpp:563-577): the number becomes the text of
    // CComplex::ToString (16 significant digits), which is parsed again.
    std::string str;
    if (!to_str(last, &str) || str.empty()) {
        err = quoted("\"%s\" does not evaluate to a numerical value", e.text);
        return false;
    }
    Cx v{0., 0.};   // lua_tonumber of a text luaO_str2d rejects is 0
    if (!str2d(str.c_str(), &v)) v = Cx{0., 0.};
    *t = v.re;
    return true;
}

}  // namespace xfk

namespace xfk {
void set_error(const std::string &msg);   // xfk_api.hip
}

extern "C" int xfk_magdir_eval(const char *fctn, int n_elems, const int *p, const double *x, const double *y,
                               int length_units, double mag_dir, double *t)
{
    if (!fctn || n_elems < 0 || (n_elems > 0 && (!p || !x || !y || !t)) || length_units < 0 || length_units > 5) {
        xfk::set_error("xfk_magdir_eval: bad arguments");
        return -1;   // XFK_ERR_ARG
    }
    std::string err;
    auto e = xfk::magdir_parse(fctn, err);
    if (!e) {
        xfk::set_error(err);
        return -1;
    }
    for (int i = 0; i < n_elems; ++i) {
        const double X[3] = {x[p[3LL * i]], x[p[3LL * i + 1]], x[p[3LL * i + 2]]};
        const double Y[3] = {y[p[3LL * i]], y[p[3LL * i + 1]], y[p[3LL * i + 2]]};
        if (!xfk::magdir_eval(*e, X, Y, length_units, mag_dir, t + i, err)) {
            xfk::set_error(err);
            return -1;
        }
    }
    return 0;
}
