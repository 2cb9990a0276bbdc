// .fem parser and B-H curve preprocessing (see femm_problem.h).
#include "femm_problem.h"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace xfemm {

namespace {

std::string lower(std::string s)
{
    for (auto &c : s) c = (char)std::tolower((unsigned char)c);
    return s;
}

std::string trim(const std::string &s)
{
    size_t a = s.find_first_not_of(" \t\r\n");
    if (a == std::string::npos) return "";
    size_t b = s.find_last_not_of(" \t\r\n");
    return s.substr(a, b - a + 1);
}

std::string first_token(const std::string &line)
{
    std::istringstream is(line);
    std::string t;
    is >> t;
    return lower(t);
}

// text after the first '=' (fparse.cpp expectChar + rest of line)
bool rest_after_eq(const std::string &line, std::string &rest)
{
    size_t k = line.find('=');
    if (k == std::string::npos) return false;
    rest = trim(line.substr(k + 1));
    return true;
}

// fparse.cpp parseString: '"' ... last '"' of the line
bool parse_string(const std::string &rest, std::string &out)
{
    std::string r = trim(rest);
    if (r.empty() || r[0] != '"') return false;
    size_t pos = r.find_last_of('"');
    if (pos == 0) return false;
    out = r.substr(1, pos - 1);
    return true;
}

bool parse_double(const std::string &rest, double &v)
{
    try {
        size_t sz = 0;
        v = std::stod(rest, &sz);
        return true;
    } catch (const std::exception &) {
        return false;
    }
}

bool parse_int(const std::string &rest, int &v)
{
    try {
        size_t sz = 0;
        v = std::stoi(rest, &sz);
        return true;
    } catch (const std::exception &) {
        return false;
    }
}

struct LineReader {
    std::vector<std::string> lines;
    size_t i = 0;
    bool good() const { return i < lines.size(); }
    std::string next() { return lines[i++]; }
};

// iterate over the (token, line) pairs of one <BeginX> ... <EndX> block
template <class F>
bool read_block(LineReader &in, const char *begin, const char *end, std::string &err, F &&f)
{
    while (in.good()) {
        std::string ln = trim(in.next());
        if (ln.empty()) continue;
        if (first_token(ln) != begin) {
            err = std::string("expected ") + begin + ", got: " + ln;
            return false;
        }
        break;
    }
    while (in.good()) {
        std::string ln = trim(in.next());
        if (ln.empty()) continue;
        std::string tok = first_token(ln);
        if (tok == end) return true;
        std::string rest;
        if (!rest_after_eq(ln, rest)) {
            err = "missing '=' in: " + ln;
            return false;
        }
        if (!f(tok, rest, in)) {
            err = "bad value in: " + ln;
            return false;
        }
    }
    err = std::string("unterminated block, expected ") + end;
    return false;
}

// femmcomplex.cpp:367-372 on the real axis: a / z == a * (1 / z)
inline double recip(double z) { return 1. / (z * (1. + 0.0 * 0.0)); }

}  // namespace

bool CMSolverMaterialProp::GetSlopes()
{
    // CMMaterialProp::GetSlopes(omega == 0), CMaterialProp.cpp:127-348
    if (BHpoints == 0 || !slope.empty()) return true;
    const int n = BHpoints;
    if (n < 2) return false;
    std::vector<double> &B = Bdata, &H = Hdata;
    mu_x = B[1] / (kMuo * std::fabs(H[1]));
    mu_y = mu_x;
    Theta_hx = Theta_hn;
    Theta_hy = Theta_hn;
    bool CurveOK = false, ProcessedLams = false;
    std::vector<double> bn(n, 0.0), hn(n, 0.0);
    std::vector<std::vector<double>> M;
    std::vector<double> b;
    while (!CurveOK) {
        M.assign(n, std::vector<double>(n, 0.0));
        b.assign(n, 0.0);
        double l1 = B[1] - B[0];
        M[0][0] = 4. / l1;
        M[0][1] = 2. / l1;
        b[0] = 6. * (H[1] - H[0]) / (l1 * l1);
        l1 = B[n - 1] - B[n - 2];
        M[n - 1][n - 1] = 4. / l1;
        M[n - 1][n - 2] = 2. / l1;
        b[n - 1] = 6. * (H[n - 1] - H[n - 2]) / (l1 * l1);
        for (int i = 1; i < n - 1; i++) {
            l1 = B[i] - B[i - 1];
            double l2 = B[i + 1] - B[i];
            M[i][i - 1] = 2. / l1;
            M[i][i] = 4. * (l1 + l2) / (l1 * l2);
            M[i][i + 1] = 2. / l2;
            b[i] = 6. * (H[i] - H[i - 1]) / (l1 * l1) + 6. * (H[i + 1] - H[i]) / (l2 * l2);
        }
        // CComplexFullMatrix::GaussSolve (fullmatrix.cpp:183-218)
        int q = 0;
        for (int i = 0; i < n; i++) {
            double mx = 0;
            for (int j = i; j < n; j++)
                if (std::fabs(M[j][i]) > std::fabs(mx)) {
                    mx = M[j][i];
                    q = j;
                }
            if (mx == 0) return false;
            std::swap(M[i], M[q]);
            std::swap(b[i], b[q]);
            for (int j = i + 1; j < n; j++) {
                double f = M[j][i] * recip(M[i][i]);
                b[j] = b[j] - f * b[i];
                for (int k = i; k < n; k++) M[j][k] -= (f * M[i][k]);
            }
        }
        for (int i = n - 1; i >= 0; i--) {
            double f = 0;
            for (int j = n - 1; j > i; j--) f += M[i][j] * b[j];
            b[i] = (b[i] - f) * recip(M[i][i]);
        }
        slope = b;
        CurveOK = true;
        for (int i = 1; i < n; i++) {
            double d0 = slope[i - 1], d1 = slope[i], u0 = H[i - 1], u1 = H[i];
            double L = B[i] - B[i - 1];
            double c0 = d0;
            double c1 = -(2. * (2. * d0 * L + d1 * L + 3. * u0 - 3. * u1)) / (L * L);
            double c2 = (3. * (d0 * L + d1 * L + 2. * u0 - 2. * u1)) / (L * L * L);
            double X0 = -1., X1 = -1.;
            u0 = c1 * c1 - 4. * c0 * c2;
            if (c2 == 0) {
                if (c1 != 0) X0 = -c0 / c1;
            } else if (u0 > 0) {
                u0 = std::sqrt(u0);
                X0 = -(c1 + u0) / (2. * c2);
                X1 = (-c1 + u0) / (2. * c2);
            }
            if (((X0 >= 0.) && (X0 <= L)) || ((X1 >= 0.) && (X1 <= L))) CurveOK = false;
        }
        if (!CurveOK) {
            for (int i = 1; i < n - 1; i++) {
                bn[i] = (B[i - 1] + B[i] + B[i + 1]) / 3.;
                hn[i] = (H[i - 1] + H[i] + H[i + 1]) / 3.;
            }
            for (int i = 1; i < n - 1; i++) {
                H[i] = hn[i];
                B[i] = bn[i];
            }
        }
        if (CurveOK && !ProcessedLams) {
            if ((LamType == 0) && (LamFill != 1)) {
                for (int i = 1; i < n; i++) {
                    double mu = (recip(H[i]) * (LamFill * B[i])) + (1. - LamFill) * kMuo;
                    B[i] = std::fabs(mu * H[i]);
                    H[i] = B[i] * recip(mu);
                }
                CurveOK = false;
            }
            ProcessedLams = true;
        }
    }
    return true;
}

namespace {

// femmcomplex.cpp arithmetic: products as written, quotients through the
// scaled reciprocal, the scaled modulus
struct Fc {
    double re = 0, im = 0;
    Fc() = default;
    Fc(double r, double i = 0) : re(r), im(i) {}
};
inline Fc operator+(Fc a, Fc b) { return Fc(a.re + b.re, a.im + b.im); }
inline Fc operator-(Fc a, Fc b) { return Fc(a.re - b.re, a.im - b.im); }
inline Fc operator*(Fc a, Fc b) { return Fc(a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re); }
inline Fc operator*(double s, Fc a) { return Fc(s * a.re, s * a.im); }
inline Fc operator*(Fc a, double s) { return Fc(a.re * s, a.im * s); }
inline Fc operator/(Fc a, double s) { return Fc(a.re / s, a.im / s); }
inline Fc frecip(Fc z)
{
    Fc y;
    if (std::fabs(z.re) > std::fabs(z.im)) {
        double c = z.im / z.re;
        y.re = 1. / (z.re * (1. + c * c));
        y.im = (-c) * y.re;
    } else {
        double c = z.re / z.im;
        y.im = (-1.) / (z.im * (1. + c * c));
        y.re = (-c) * y.im;
    }
    return y;
}
inline Fc operator/(Fc a, Fc b) { return a * frecip(b); }
inline Fc operator/(double a, Fc b)
{
    Fc y = frecip(b);
    return Fc(y.re * a, y.im * a);
}
inline double fabs_(Fc x)
{
    if (x.re == 0 && x.im == 0) return 0.;
    if (std::fabs(x.re) > std::fabs(x.im)) return std::fabs(x.re) * std::sqrt(1. + (x.im / x.re) * (x.im / x.re));
    return std::fabs(x.im) * std::sqrt(1. + (x.re / x.im) * (x.re / x.im));
}
inline Fc fexp(Fc x)
{
    const double e = std::exp(x.re);
    return Fc(std::cos(x.im) * e, std::sin(x.im) * e);
}

// Hermite pieces on a complex curve: H(b) (CMSolverMaterialProp::GetH,
// CMaterialProp.cpp:960-990) and dH/dB (CMMaterialProp::GetdHdB, :461-486)
struct CCurve {
    const std::vector<double> &B;
    const std::vector<Fc> &H, &S;
    Fc h(double x) const
    {
        const int n = (int)B.size();
        const double b = std::fabs(x);
        if (b > B[n - 1]) return H[n - 1] + S[n - 1] * (b - B[n - 1]);
        for (int i = 0; i < n - 1; i++)
            if (b >= B[i] && b <= B[i + 1]) {
                const double l = B[i + 1] - B[i], z = (b - B[i]) / l, z2 = z * z;
                return (1. - 3. * z2 + 2. * z2 * z) * H[i] + z * (1. - 2. * z + z2) * l * S[i] +
                       z2 * (3. - 2. * z) * H[i + 1] + z2 * (z - 1.) * l * S[i + 1];
            }
        return Fc(0);
    }
    Fc dhdb(double x) const
    {
        const int n = (int)B.size();
        const double b = std::fabs(x);
        if (b > B[n - 1]) return S[n - 1];
        for (int i = 0; i < n - 1; i++)
            if (b >= B[i] && b <= B[i + 1]) {
                const double l = B[i + 1] - B[i], z = (b - B[i]) / l;
                return 6. * z * (z - 1.) * H[i] / l + (1. - 4. * z + 3. * z * z) * S[i] +
                       6. * z * (1. - z) * H[i + 1] / l + z * (3. * z - 2.) * S[i + 1];
            }
        return Fc(0);
    }
};


// the effective permeability of lamination-curve point i (1-D nonlinear
// eddy-current problem across half a lamination, CMaterialProp.cpp:1060-1160)
Fc laminated_mu(const CMSolverMaterialProp &m, const std::vector<Fc> &H, const std::vector<Fc> &S, double w, int i)
{
    const CCurve cv{m.Bdata, H, S};
    Fc mu = m.Bdata[i] / H[i];
    const double o = m.Cduct * 1.e6, d = (m.Lam_d * 0.001) / 2.;
    const double ds = std::sqrt(2 / (w * o * fabs_(mu)));
    const int n = 10 * (int)std::ceil(d / ds);
    const double L = d / (double)n;
    std::vector<Fc> x(n + 1), b(n + 1), m0(n + 1), m1(n + 1);
    int iter = 0;
    double res = 0, lastres, Relax = 1;
    for (;;) {
        std::fill(m0.begin(), m0.end(), Fc(0));
        std::fill(m1.begin(), m1.end(), Fc(0));
        std::fill(b.begin(), b.end(), Fc(0));
        for (int k = 0; k < n; k++) {
            Fc vo, vi;
            if (iter != 0) {
                const double Bk = fabs_(x[k + 1] - x[k]) / L;
                vi = cv.dhdb(Bk);
                vo = cv.h(Bk) / Bk;
            } else {
                vo = 1. / mu;
                vi = 1. / mu;
            }
            const Fc jw = Fc(0, 1) * w * o * L / 4.;
            Fc Md = (vi + vo) / (2. * L) + jw, Mo = (-1. * (vi + vo)) / (2. * L) + jw;
            m0[k] = m0[k] + Md;
            m1[k] = m1[k] + Mo;
            m0[k + 1] = m0[k + 1] + Md;
            Md = (vi - vo) / (2. * L);
            Mo = (-1. * (vi - vo)) / (2. * L);
            b[k] = b[k] + (Md * x[k] + Mo * x[k + 1]);
            b[k + 1] = b[k + 1] + (Mo * x[k] + Md * x[k + 1]);
        }
        m1[0] = Fc(0);
        b[0] = Fc(0);
        b[n] = b[n] + H[i];
        for (int k = 0; k < n; k++) {   // tridiagonal elimination
            const Fc c = m1[k] / m0[k];
            m0[k + 1] = m0[k + 1] - m1[k] * c;
            b[k + 1] = b[k + 1] - b[k] * c;
        }
        b[n] = b[n] / m0[n];
        for (int k = n - 1; k >= 0; k--) b[k] = (b[k] - m1[k] * b[k + 1]) / m0[k];
        iter++;
        lastres = res;
        res = fabs_(b[n] - x[n]) / d;
        const bool conv = res < 1.e-8;
        if (iter > 5) {
            if ((res > lastres) && (Relax > 0.1)) Relax /= 2.;
            else Relax += 0.1 * (1. - Relax);
        }
        for (int k = 0; k <= n; k++) x[k] = Relax * b[k] + (1.0 - Relax) * x[k];
        if (conv) break;
        if (iter > 100000) break;   // the reference loops until converged
    }
    return x[n] / (H[i] * d);
}

}  // namespace

bool CMSolverMaterialProp::GetSlopesAC(double omega)
{
    if (BHpoints == 0) return true;
    const int n = BHpoints;
    if (n < 2 || (int)Bdata.size() != n || (int)Hdata.size() != n) return false;
    std::vector<double> &B = Bdata;
    std::vector<Fc> H(n), S(n), hn(n);
    for (int i = 0; i < n; i++) H[i] = Fc(Hdata[i]);
    mu_x = B[1] / (kMuo * fabs_(H[1]));
    mu_y = mu_x;
    Theta_hx = Theta_hn;
    Theta_hy = Theta_hn;
    std::vector<double> bn(n, 0.0);
    if (omega != 0) {
        // effective amplitude of B for a sinusoidal H of amplitude H_i
        double mumax = 0;
        for (int i = 1; i < n; i++) {
            const double Hi = H[i].re;
            hn[i] = H[i];
            bn[i] = 0;
            for (int k = 1; k <= i; k++) {
                const double h0 = H[k - 1].re, h1 = H[k].re;
                const double num = 4. * (h1 * B[k - 1] - h0 * B[k]) *
                                       (-std::cos((h0 * kPi) * (1. / (2. * Hi))) +
                                        std::cos((h1 * kPi) * (1. / (2. * Hi)))) +
                                   (-B[k - 1] + B[k]) * ((h0 - h1) * kPi +
                                                         Hi * (-std::sin((h0 * kPi) * (1. / Hi)) +
                                                               std::sin((h1 * kPi) * (1. / Hi))));
                bn[i] += num * (1. / ((h0 - h1) * kPi));
            }
        }
        for (int i = 1; i < n; i++) {
            B[i] = bn[i];
            H[i] = hn[i];
            const double munow = (B[i] / H[i]).re;
            if (munow > mumax) mumax = munow;
        }
        // hysteresis lag proportional to permeability (O'Kelly)
        for (int i = 1; i < n; i++) H[i] = H[i] * fexp(Fc(0, 1) * (B[i] * Theta_hn * kDeg) / (H[i] * mumax));
        MuMax = mumax / kMuo;
    }
    bool CurveOK = false, ProcessedLams = false;
    std::vector<std::vector<double>> M;
    std::vector<Fc> rhs;
    int guard = 0;
    while (!CurveOK) {
        if (++guard > 10000) return false;
        // slopes: natural end conditions; the matrix is real, so its complex
        // Gauss elimination (fullmatrix.cpp) acts on the real and imaginary
        // parts of the right-hand side alike
        M.assign(n, std::vector<double>(n, 0.0));
        rhs.assign(n, Fc(0));
        double l1 = B[1] - B[0];
        M[0][0] = 4. / l1;
        M[0][1] = 2. / l1;
        rhs[0] = 6. * (H[1] - H[0]) / (l1 * l1);
        l1 = B[n - 1] - B[n - 2];
        M[n - 1][n - 1] = 4. / l1;
        M[n - 1][n - 2] = 2. / l1;
        rhs[n - 1] = 6. * (H[n - 1] - H[n - 2]) / (l1 * l1);
        for (int i = 1; i < n - 1; i++) {
            l1 = B[i] - B[i - 1];
            const double l2 = B[i + 1] - B[i];
            M[i][i - 1] = 2. / l1;
            M[i][i] = 4. * (l1 + l2) / (l1 * l2);
            M[i][i + 1] = 2. / l2;
            rhs[i] = 6. * (H[i] - H[i - 1]) / (l1 * l1) + 6. * (H[i + 1] - H[i]) / (l2 * l2);
        }
        int q = 0;
        for (int i = 0; i < n; i++) {
            double mx = 0;
            for (int j = i; j < n; j++)
                if (std::fabs(M[j][i]) > std::fabs(mx)) {
                    mx = M[j][i];
                    q = j;
                }
            if (mx == 0) return false;
            std::swap(M[i], M[q]);
            std::swap(rhs[i], rhs[q]);
            for (int j = i + 1; j < n; j++) {
                const double f = M[j][i] * recip(M[i][i]);
                rhs[j] = rhs[j] - f * rhs[i];
                for (int k = i; k < n; k++) M[j][k] -= (f * M[i][k]);
            }
        }
        for (int i = n - 1; i >= 0; i--) {
            Fc f(0);
            for (int j = n - 1; j > i; j--) f = f + M[i][j] * rhs[j];
            rhs[i] = (rhs[i] - f) * recip(M[i][i]);
        }
        S = rhs;
        // monotonicity test on the real parts
        CurveOK = true;
        for (int i = 1; i < n; i++) {
            double d0 = S[i - 1].re, d1 = S[i].re, u0 = H[i - 1].re, u1 = H[i].re;
            const double L = B[i] - B[i - 1];
            const double c0 = d0;
            const double c1 = -(2. * (2. * d0 * L + d1 * L + 3. * u0 - 3. * u1)) / (L * L);
            const double c2 = (3. * (d0 * L + d1 * L + 2. * u0 - 2. * u1)) / (L * L * L);
            double X0 = -1., X1 = -1.;
            u0 = c1 * c1 - 4. * c0 * c2;
            if (c2 == 0) {
                if (c1 != 0) X0 = -c0 / c1;
            } else if (u0 > 0) {
                u0 = std::sqrt(u0);
                X0 = -(c1 + u0) / (2. * c2);
                X1 = (-c1 + u0) / (2. * c2);
            }
            if (((X0 >= 0.) && (X0 <= L)) || ((X1 >= 0.) && (X1 <= L))) CurveOK = false;
        }
        if (!CurveOK) {   // 3-point moving average
            for (int i = 1; i < n - 1; i++) {
                bn[i] = (B[i - 1] + B[i] + B[i + 1]) / 3.;
                hn[i] = (H[i - 1] + H[i] + H[i + 1]) / 3.;
            }
            for (int i = 1; i < n - 1; i++) {
                H[i] = hn[i];
                B[i] = bn[i];
            }
        }
        if (CurveOK && !ProcessedLams) {
            if ((omega > 0) && (Lam_d != 0) && (Cduct != 0)) {
                for (int i = 1; i < n; i++) {
                    const Fc mu = laminated_mu(*this, H, S, omega, i);
                    bn[i] = fabs_(mu * H[i]);
                    hn[i] = bn[i] / mu;
                }
                for (int i = 1; i < n; i++) {
                    B[i] = bn[i];
                    H[i] = hn[i];
                }
                CurveOK = false;
            }
            if ((LamType == 0) && (LamFill != 1)) {
                for (int i = 1; i < n; i++) {
                    const Fc mu = (LamFill * B[i]) / H[i] + Fc((1. - LamFill) * kMuo);
                    B[i] = fabs_(mu * H[i]);
                    H[i] = B[i] / mu;
                }
                CurveOK = false;
            }
            ProcessedLams = true;
        }
    }
    Hdata.assign(n, 0.0);
    Hdata_im.assign(n, 0.0);
    slope.assign(n, 0.0);
    slope_im.assign(n, 0.0);
    for (int i = 0; i < n; i++) {
        Hdata[i] = H[i].re;
        Hdata_im[i] = H[i].im;
        slope[i] = S[i].re;
        slope_im[i] = S[i].im;
    }
    return true;
}

bool ParseFemFile(const std::string &path, FemmProblemData &pr, std::string &err)
{
    std::ifstream f(path);
    if (!f.is_open()) {
        err = "Couldn't read from specified .fem file: " + path;
        return false;
    }
    LineReader in;
    std::string line;
    while (std::getline(f, line)) in.lines.push_back(line);
    pr = FemmProblemData();
    while (in.good()) {
        std::string ln = trim(in.next());
        if (ln.empty()) continue;
        std::string tok = first_token(ln), rest;
        if (tok == "[numpoints]" || tok == "[numsegments]" || tok == "[numarcsegments]" || tok == "[numholes]") {
            int n = 0;
            if (!rest_after_eq(ln, rest) || !parse_int(rest, n)) {
                err = "bad count: " + ln;
                return false;
            }
            for (int k = 0; k < n && in.good(); ++k) in.next();
            continue;
        }
        if (!rest_after_eq(ln, rest)) {
            err = "Unknown token: " + tok;
            return false;
        }
        bool ok = true;
        if (tok == "[format]") ok = parse_double(rest, pr.FileFormat);
        else if (tok == "[frequency]") ok = parse_double(rest, pr.Frequency);
        else if (tok == "[precision]") ok = parse_double(rest, pr.Precision);
        else if (tok == "[minangle]") ok = parse_double(rest, pr.MinAngle);
        else if (tok == "[depth]") ok = parse_double(rest, pr.Depth);
        else if (tok == "[lengthunits]") {
            std::string u = first_token(rest);
            if (u == "inches") pr.LengthUnits = LengthInches;
            else if (u == "millimeters") pr.LengthUnits = LengthMillimeters;
            else if (u == "centimeters") pr.LengthUnits = LengthCentimeters;
            else if (u == "mils") pr.LengthUnits = LengthMils;
            else if (u == "microns") pr.LengthUnits = LengthMicrometers;
            else if (u == "meters") pr.LengthUnits = LengthMeters;
        } else if (tok == "[coordinates]") {
            std::string u = first_token(rest);
            if (u == "cartesian") pr.Coords = CART;
            if (u == "polar") pr.Coords = POLAR;
        } else if (tok == "[problemtype]") {
            std::string u = first_token(rest);
            if (u == "planar") pr.ProblemTypeV = PLANAR;
            if (u == "axisymmetric") pr.ProblemTypeV = AXISYMMETRIC;
        } else if (tok == "[extzo]") ok = parse_double(rest, pr.extZo);   // feasolver.cpp:306-326
        else if (tok == "[extro]") ok = parse_double(rest, pr.extRo);
        else if (tok == "[extri]") ok = parse_double(rest, pr.extRi);
        else if (tok == "[forcemaxmesh]" || tok == "[dosmartmesh]") {
            // meshing options, unused by the solver
        } else if (tok == "[comment]") ok = parse_string(rest, pr.comment);
        else if (tok == "[acsolver]") ok = parse_int(rest, pr.ACSolver);
        else if (tok == "[prevtype]") ok = parse_int(rest, pr.PrevType);
        else if (tok == "[prevsoln]") {
            ok = parse_string(rest, pr.previousSolutionFile);
            pr.prevSolnInFile = true;
        }
        else if (tok == "[pointprops]") {
            int k = 0;
            ok = parse_int(rest, k);
            for (int i = 0; ok && i < k; ++i) {
                CMPointProp p;
                ok = read_block(in, "<beginpoint>", "<endpoint>", err, [&](const std::string &t, const std::string &r, LineReader &) {
                    if (t == "<pointname>") return parse_string(r, p.PointName);
                    if (t == "<a_re>") return parse_double(r, p.A_re);
                    if (t == "<a_im>") return parse_double(r, p.A_im);
                    if (t == "<i_re>") return parse_double(r, p.J_re);
                    if (t == "<i_im>") return parse_double(r, p.J_im);
                    return true;
                });
                pr.nodeproplist.push_back(p);
            }
        } else if (tok == "[bdryprops]") {
            int k = 0;
            ok = parse_int(rest, k);
            for (int i = 0; ok && i < k; ++i) {
                CMBoundaryProp b;
                ok = read_block(in, "<beginbdry>", "<endbdry>", err, [&](const std::string &t, const std::string &r, LineReader &) {
                    if (t == "<bdryname>") return parse_string(r, b.BdryName);
                    if (t == "<bdrytype>") return parse_int(r, b.BdryFormat);
                    if (t == "<mu_ssd>") return parse_double(r, b.Mu);
                    if (t == "<sigma_ssd>") return parse_double(r, b.Sig);
                    if (t == "<a_0>") return parse_double(r, b.A0);
                    if (t == "<a_1>") return parse_double(r, b.A1);
                    if (t == "<a_2>") return parse_double(r, b.A2);
                    if (t == "<phi>") return parse_double(r, b.phi);
                    if (t == "<c0>") return parse_double(r, b.c0_re);
                    if (t == "<c1>") return parse_double(r, b.c1_re);
                    if (t == "<c0i>") return parse_double(r, b.c0_im);
                    if (t == "<c1i>") return parse_double(r, b.c1_im);
                    if (t == "<innerangle>") return parse_double(r, b.InnerAngle);
                    if (t == "<outerangle>") return parse_double(r, b.OuterAngle);
                    return true;
                });
                pr.lineproplist.push_back(b);
            }
        } else if (tok == "[blockprops]") {
            int k = 0;
            ok = parse_int(rest, k);
            for (int i = 0; ok && i < k; ++i) {
                CMSolverMaterialProp m;
                ok = read_block(in, "<beginblock>", "<endblock>", err, [&](const std::string &t, const std::string &r, LineReader &ls) {
                    if (t == "<blockname>") return parse_string(r, m.BlockName);
                    if (t == "<mu_x>") return parse_double(r, m.mu_x);
                    if (t == "<mu_y>") return parse_double(r, m.mu_y);
                    if (t == "<h_c>") return parse_double(r, m.H_c);
                    if (t == "<h_cangle>") return parse_double(r, m.Theta_m);
                    if (t == "<j_re>") return parse_double(r, m.J_re);
                    if (t == "<j_im>") return parse_double(r, m.J_im);
                    if (t == "<sigma>") return parse_double(r, m.Cduct);
                    if (t == "<phi_h>") return parse_double(r, m.Theta_hn);
                    if (t == "<phi_hx>") return parse_double(r, m.Theta_hx);
                    if (t == "<phi_hy>") return parse_double(r, m.Theta_hy);
                    if (t == "<d_lam>") return parse_double(r, m.Lam_d);
                    if (t == "<lamfill>") return parse_double(r, m.LamFill);
                    if (t == "<wired>") return parse_double(r, m.WireD);
                    if (t == "<lamtype>") return parse_int(r, m.LamType);
                    if (t == "<nstrands>") return parse_int(r, m.NStrands);
                    if (t == "<bhpoints>") {
                        if (!parse_int(r, m.BHpoints)) return false;
                        std::vector<double> vals;
                        while ((int)vals.size() < 2 * m.BHpoints && ls.good()) {
                            std::istringstream is(ls.next());
                            double v;
                            while (is >> v) vals.push_back(v);
                        }
                        if ((int)vals.size() < 2 * m.BHpoints) return false;
                        for (int q = 0; q < m.BHpoints; ++q) {
                            m.Bdata.push_back(vals[2 * q]);
                            m.Hdata.push_back(vals[2 * q + 1]);
                        }
                        return true;
                    }
                    return true;
                });
                pr.blockproplist.push_back(m);
            }
        } else if (tok == "[circuitprops]" || tok == "[conductorprops]") {
            int k = 0;
            ok = parse_int(rest, k);
            for (int i = 0; ok && i < k; ++i) {
                CMCircuit c;
                ok = read_block(in, "<begincircuit>", "<endcircuit>", err, [&](const std::string &t, const std::string &r, LineReader &) {
                    if (t == "<circuitname>") return parse_string(r, c.CircName);
                    if (t == "<voltgradient_re>") return parse_double(r, c.dVolts_re);
                    if (t == "<voltgradient_im>") return parse_double(r, c.dVolts_im);
                    if (t == "<totalamps_re>") return parse_double(r, c.Amps_re);
                    if (t == "<totalamps_im>") return parse_double(r, c.Amps_im);
                    if (t == "<circuittype>") return parse_int(r, c.CircType);
                    return true;
                });
                pr.circproplist.push_back(c);
            }
        } else if (tok == "[numblocklabels]") {
            int k = 0;
            ok = parse_int(rest, k);
            for (int i = 0; ok && i < k && in.good(); ++i) {
                // CMBlockLabel::fromStream (CBlockLabel.cpp:110-154)
                std::string l = trim(in.next());
                CMBlockLabel lb;
                size_t qpos = l.find('"');
                std::string head = (qpos == std::string::npos) ? l : l.substr(0, qpos);
                std::istringstream is(head);
                double maxarea = 0;
                int extDefault = 0;
                if (is >> lb.x >> lb.y >> lb.BlockType) {
                    lb.BlockType--;
                    if (is >> maxarea) lb.MaxArea = (maxarea <= 0) ? 0 : maxarea * (kPi * maxarea / 4.);
                    if (is >> lb.InCircuit) lb.InCircuit--;
                    else lb.InCircuit = -1;
                    is >> lb.MagDir >> lb.InGroup >> lb.Turns >> extDefault;
                }
                lb.IsDefault = extDefault & 2;
                lb.IsExternal = extDefault & 1;
                if (qpos != std::string::npos) parse_string(l.substr(qpos), lb.MagDirFctn);
                pr.labellist.push_back(lb);
            }
        } else {
            err = "Unknown token: " + tok + "\nContext line:\n" + ln;
            return false;
        }
        if (!ok) {
            if (err.empty()) err = "Parse error in line: " + ln;
            err = "Parse error while reading input file " + path + "!\n" + err;
            return false;
        }
    }
    return true;
}

}  // namespace xfemm
