// Checks xfemm::fastnum::parse_double against strtod, bit for bit and in the
// characters consumed, on every whitespace-separated token of the input
// files, then on a sweep of generated %.17g / %.Ng / %e strings.
// Prints "checked N fast F" on success, the first mismatch otherwise.
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../xfemm_amd/csrc/fsolver/fastnum.h"

static long long n_checked = 0;

static bool check(const char *tok)
{
    char *qe = nullptr;
    const double a = std::strtod(tok, &qe);
    const char *fe = nullptr;
    double b = 0;
    const bool ok = xfemm::fastnum::parse_double(tok, b, &fe);
    ++n_checked;
    if ((qe != tok) != ok || (ok && (fe != qe || std::memcmp(&a, &b, sizeof a) != 0))) {
        std::printf("MISMATCH '%s': strtod %.17g (+%d) fast %.17g (+%d) ok %d\n", tok, a, (int)(qe - tok), b,
                    fe ? (int)(fe - tok) : -1, ok);
        return false;
    }
    return true;
}

int main(int argc, char **argv)
{
    for (int i = 1; i < argc; ++i) {
        FILE *fp = std::fopen(argv[i], "rb");
        if (!fp) return 2;
        char buf[256];
        while (std::fscanf(fp, "%255s", buf) == 1)
            if (!check(buf)) return 1;
        std::fclose(fp);
    }
    std::mt19937_64 rng(12345);
    char buf[128];
    const char *fmts[] = {"%.17g", "%.16g", "%.15g", "%.19g", "%.20g", "%.6g", "%.17e", "%.3f", "%.10f", "%.25g"};
    for (int k = 0; k < 3000000; ++k) {
        double v;
        switch (k % 5) {
        case 0: v = std::ldexp((double)(rng() >> 11), -53) * 10.0; break;                        // [0, 10)
        case 1: v = ((double)(int64_t)(rng() % 2000001) - 1000000) * 0.01; break;                 // grid coordinates
        case 2: v = std::ldexp((double)(rng() >> 11), (int)(rng() % 120) - 113); break;          // wide exponents
        case 3: { uint64_t u = rng(); std::memcpy(&v, &u, sizeof v); if (!std::isfinite(v)) v = 1.5; } break;
        default: v = (double)(int64_t)(rng() % 100000) / 1000.0; break;
        }
        std::snprintf(buf, sizeof buf, fmts[k % 10], (k & 64) ? -v : v);
        if (!check(buf)) return 1;
    }
    // near-midpoint decimal strings: a double's neighbours' midpoint written out to 19-25 digits
    for (int k = 0; k < 200000; ++k) {
        double v = std::ldexp((double)(rng() >> 11), -52) * (1 + (int)(rng() % 1000));
        const double w = std::nextafter(v, 1e300);
        std::snprintf(buf, sizeof buf, "%.*g", 17 + (int)(rng() % 9), 0.5 * v + 0.5 * w);
        if (!check(buf)) return 1;
    }
    const char *odd[] = {"0", "-0", "0.0", "00012.5", ".5", "-.5", "5.", "1e5", "1E+05", "1e-5", "1e", "1e+", "1.5e",
                         "+1.5", "0x1p3", "0X10", "inf", "-inf", "nan", "infinity", "1e400", "1e-400", "2.2250738585072014e-308",
                         "123456789012345678901234567890", "0.000000000000000000000000000001234", "9007199254740993",
                         "18446744073709551615", "18446744073709551616", "1234567890123456789", "12345678901234567890",
                         "1.00000000000000000000000000000001", "4.9406564584124654e-324", "1e22", "1e23", "1e27",
                         "1e28", "-", ".", "e5", "-e", "1..2", "1.2.3", "7e-27", "7e-28", "00x5", "0.5x"};
    for (const char *t : odd)
        if (!check(t)) return 1;
    // %.17g formatting against snprintf
    long long n_fmt = 0;
    auto fcheck = [&](double v) {
        char a[64], b[64];
        std::snprintf(a, sizeof a, "%.17g", v);
        char *e = xfemm::fastnum::put_g17(b, v);
        *e = 0;
        ++n_fmt;
        if (std::strcmp(a, b) != 0) {
            std::printf("FORMAT MISMATCH %a: printf '%s' fast '%s'\n", v, a, b);
            return false;
        }
        return true;
    };
    for (int k = 0; k < 4000000; ++k) {
        double v;
        switch (k % 6) {
        case 0: v = std::ldexp((double)(rng() >> 11), -53) * 10.0; break;
        case 1: v = ((double)(int64_t)(rng() % 2000001) - 1000000) * 0.01; break;
        case 2: v = std::ldexp((double)(rng() >> 11), (int)(rng() % 140) - 130); break;
        case 3: { uint64_t u = rng(); std::memcpy(&v, &u, sizeof v); } break;
        case 4: v = std::ldexp(1.0, (int)(rng() % 200) - 100) * (double)(1 + rng() % 7); break;   // dyadic: exact ties
        default: v = std::pow(10.0, (double)((int)(rng() % 60) - 30)) * ((rng() & 1) ? 1 : std::nextafter(1.0, 2.0)); break;
        }
        if (k & 1) v = -v;
        if (!fcheck(v)) return 1;
    }
    const double sp[] = {0.0, -0.0, 1.0, -1.0, 0.1, 1e-5, 1e-4, 9.9999999999999995e-5, 1e16, 1e17, 9.9999999999999998e16,
                         123456789012345678.0, 1e-11, 1e-12, 0.5, 2.5, 1e300, 1e-300, 4.9406564584124654e-324, 1.0 / 0.0,
                         -1.0 / 0.0, std::nan(""), 5e-324, 2.2250738585072014e-308, 99999999999999999.0, 0.30000000000000004};
    for (double v : sp)
        if (!fcheck(v)) return 1;
    for (int e = -1074; e < 1024; ++e)   // every power of two and its neighbours
        for (double v : {std::ldexp(1.0, e), std::nextafter(std::ldexp(1.0, e), 0.0), std::nextafter(std::ldexp(1.0, e), 1e308)})
            if (!fcheck(v)) return 1;
    std::printf("checked %lld formatted %lld\n", n_checked, n_fmt);
    return 0;
}
