// Exact fast paths for the number conversions of the mesh files and the .ans.
//
// parse_double: the value strtod gives, bit for bit (fscanf "%lf" is strtod,
// FSolver::LoadMesh reads every coordinate with it, fsolver.cpp:350-718 of
// the reference).  A decimal token [-]digits[.digits][(e|E)[+-]digits] with
// at most 19 significant digits (an integer m < 2^64, exact in the x87 64-bit
// significand) and a decimal exponent |k| <= 27 (10^|k| exact there) is
// m * 10^k or m / 10^-k, rounded once to 64 bits; rounding that to a double
// is the correctly rounded value unless the 64-bit result lies within one of
// its own ulps of a double midpoint (its low 11 bits 0x3ff / 0x400 / 0x401):
// then, and for every other token (hex floats, inf / nan, a leading '+',
// more digits, larger exponents), strtod itself runs.  %.17g output of
// Triangle / fmesher (17 significant digits, exponents near 0) takes the
// fast path.
//
// put_g17: the characters printf("%.17g") writes (the .ans columns,
// static2d.cpp:1038-1195 of the reference).  For |v| in [1e-11, 1e17) the 17
// significant digits are formed exactly: v = m 2^e, m < 2^53, so
// v 10^s = m 5^s 2^(e+s) with s = 16 - floor(log10 |v|) <= 27 is an
// unsigned 128-bit product shifted, rounded half-to-even on the exact
// remainder -- printf's correctly rounded digits -- then laid out in %g's
// fixed / exponential form without trailing zeros.  Other values (zero
// aside) go through std::to_chars, which gives printf's %.17g characters.
#pragma once

#include <charconv>
#include <cstdint>
#include <cstdlib>
#include <cstring>

namespace xfemm {
namespace fastnum {

inline long double pow10_ld(int k)
{
    static const long double t[28] = {1e0L,  1e1L,  1e2L,  1e3L,  1e4L,  1e5L,  1e6L,  1e7L,  1e8L,  1e9L,
                                      1e10L, 1e11L, 1e12L, 1e13L, 1e14L, 1e15L, 1e16L, 1e17L, 1e18L, 1e19L,
                                      1e20L, 1e21L, 1e22L, 1e23L, 1e24L, 1e25L, 1e26L, 1e27L};
    return t[k];
}

// the 64-bit significand of a positive, finite, normal long double
inline uint64_t ld_mant(long double v)
{
    uint64_t m;
    std::memcpy(&m, &v, sizeof m);   // (x87 extended: the first 8 bytes are the explicit significand)
    return m;
}

// p at a token (no leading white space); on success *end after it
inline bool parse_double(const char *p, double &v, const char **end)
{
    const char *s = p;
    const bool neg = (*s == '-');
    s += neg;
    uint64_t m = 0;
    int nd = 0, dexp = 0;
    bool any = false;
    while (*s == '0') {   // leading zeros: no significant digit yet
        ++s;
        any = true;
    }
    if ((*s == 'x' || *s == 'X') && s - p - neg == 1) goto slow;   // "0x..": hexadecimal, strtod's
    while (*s >= '0' && *s <= '9') {
        if (nd < 19) m = 10 * m + (uint64_t)(*s - '0');
        else if (*s != '0') goto slow;
        else ++dexp;   // (trailing integer zeros beyond 19 digits scale the exponent)
        ++nd;
        ++s;
        any = true;
    }
    if (*s == '.') {
        ++s;
        if (nd == 0)
            while (*s == '0') {
                ++s;
                --dexp;
                any = true;
            }
        while (*s >= '0' && *s <= '9') {
            if (nd < 19) {
                m = 10 * m + (uint64_t)(*s - '0');
                --dexp;
            } else if (*s != '0') {
                goto slow;
            }
            ++nd;
            ++s;
            any = true;
        }
    }
    if (!any) goto slow;
    if (*s == 'e' || *s == 'E') {
        const char *e = s + 1;
        const bool eneg = (*e == '-');
        if (*e == '-' || *e == '+') ++e;
        if (*e >= '0' && *e <= '9') {
            int x = 0;
            while (*e >= '0' && *e <= '9') {
                if (x > 100000) goto slow;
                x = 10 * x + (*e - '0');
                ++e;
            }
            dexp += eneg ? -x : x;
            s = e;
        }
    }
    if ((*s >= '0' && *s <= '9') || *s == '.' || *s == 'x' || *s == 'X' || *s == 'p' || *s == 'P') goto slow;
    if (m == 0) {
        v = neg ? -0.0 : 0.0;
        *end = s;
        return true;
    }
    if (dexp < -27 || dexp > 27) goto slow;
    {
        const long double r = dexp >= 0 ? (long double)m * pow10_ld(dexp) : (long double)m / pow10_ld(-dexp);
        const uint64_t low = ld_mant(r) & 0x7ffu;
        if (low >= 0x3ffu && low <= 0x401u) goto slow;   // within an ulp of a double midpoint
        const double d = (double)r;
        v = neg ? -d : d;
        *end = s;
        return true;
    }
slow:
    char *q = nullptr;
    v = std::strtod(p, &q);
    *end = q;
    return q != p;
}

inline char *put_g17_slow(char *p, double v)
{
    return std::to_chars(p, p + 32, v, std::chars_format::general, 17).ptr;
}

inline char *put_g17(char *p, double v)
{
    uint64_t bits;
    std::memcpy(&bits, &v, sizeof bits);
    const bool neg = (bits >> 63) != 0;
    const int be = (int)((bits >> 52) & 0x7ff);
    const uint64_t frac = bits & ((1ULL << 52) - 1);
    if (be == 0 && frac == 0) {   // +-0
        if (neg) *p++ = '-';
        *p++ = '0';
        return p;
    }
    if (be == 0 || be == 0x7ff) return put_g17_slow(p, v);   // subnormal, inf, nan
    const uint64_t m = frac | (1ULL << 52);
    const int e2 = be - 1075;                                 // v = m 2^e2
    // floor(log10 |v|), possibly one too small: corrected below
    int E = (int)(((long long)(e2 + 52) * 78913) >> 18);       // floor((e2 + 52) log10 2)
    static const uint64_t p5[28] = {1ULL,
                                    5ULL,
                                    25ULL,
                                    125ULL,
                                    625ULL,
                                    3125ULL,
                                    15625ULL,
                                    78125ULL,
                                    390625ULL,
                                    1953125ULL,
                                    9765625ULL,
                                    48828125ULL,
                                    244140625ULL,
                                    1220703125ULL,
                                    6103515625ULL,
                                    30517578125ULL,
                                    152587890625ULL,
                                    762939453125ULL,
                                    3814697265625ULL,
                                    19073486328125ULL,
                                    95367431640625ULL,
                                    476837158203125ULL,
                                    2384185791015625ULL,
                                    11920928955078125ULL,
                                    59604644775390625ULL,
                                    298023223876953125ULL,
                                    1490116119384765625ULL,
                                    7450580596923828125ULL};
    const uint64_t P16 = 10000000000000000ULL, P17 = 100000000000000000ULL;
    uint64_t D = 0;
    for (int pass = 0;; ++pass) {
        const int sh10 = 16 - E;
        if (sh10 < 0 || sh10 > 27 || pass > 2) return put_g17_slow(p, v);
        const unsigned __int128 N = (unsigned __int128)m * p5[sh10];
        const int sh = e2 + sh10;   // v 10^sh10 = N 2^sh
        unsigned __int128 q;
        bool up = false;
        if (sh >= 0) {
            if (sh > 10) return put_g17_slow(p, v);
            q = N << sh;
        } else {
            const int r = -sh;
            if (r >= 120) return put_g17_slow(p, v);
            q = N >> r;
            const unsigned __int128 rem = N - (q << r), half = (unsigned __int128)1 << (r - 1);
            up = rem > half || (rem == half && (q & 1));
        }
        if (q >= P17) {   // E one too small
            ++E;
            continue;
        }
        if (q < P16) return put_g17_slow(p, v);   // (cannot happen: the estimate is never too large)
        D = (uint64_t)q + (up ? 1 : 0);
        if (D == P17) {   // rounded up to 10^17
            D = P16;
            ++E;
        }
        break;
    }
    char dg[17];
    {
        uint64_t hi = D / 1000000000ULL, lo = D % 1000000000ULL;
        for (int k = 16; k >= 8; --k) {
            dg[k] = (char)('0' + lo % 10);
            lo /= 10;
        }
        for (int k = 7; k >= 0; --k) {
            dg[k] = (char)('0' + hi % 10);
            hi /= 10;
        }
    }
    int nd = 17;   // significant digits after dropping trailing zeros
    while (nd > 1 && dg[nd - 1] == '0') --nd;
    if (neg) *p++ = '-';
    if (E >= -4 && E < 17) {   // %g fixed form
        if (E >= 0) {
            for (int k = 0; k <= E; ++k) *p++ = dg[k];
            if (nd > E + 1) {
                *p++ = '.';
                for (int k = E + 1; k < nd; ++k) *p++ = dg[k];
            }
        } else {
            *p++ = '0';
            *p++ = '.';
            for (int k = 0; k < -E - 1; ++k) *p++ = '0';
            for (int k = 0; k < nd; ++k) *p++ = dg[k];
        }
    } else {   // exponential form: d[.ddd]e+XX
        *p++ = dg[0];
        if (nd > 1) {
            *p++ = '.';
            for (int k = 1; k < nd; ++k) *p++ = dg[k];
        }
        *p++ = 'e';
        int x = E;
        if (x < 0) {
            *p++ = '-';
            x = -x;
        } else {
            *p++ = '+';
        }
        if (x >= 100) {
            *p++ = (char)('0' + x / 100);
            x %= 100;
        }
        *p++ = (char)('0' + x / 10);
        *p++ = (char)('0' + x % 10);
    }
    return p;
}

}  // namespace fastnum
}  // namespace xfemm
