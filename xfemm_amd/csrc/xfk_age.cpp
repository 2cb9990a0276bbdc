// Air-gap element contributions, reduced once per problem on the host
// (see xfk_age.h).  Reference: cfemm/fsolver/static2d.cpp:191-344.
#include "xfk_age.h"

#include <cmath>
#include <map>
#include <string>

#include "xfk_age_table.h"

namespace xfk {
void set_error(const std::string &msg);

void age_matrix(double ci, double co, double K, double Ki, double MG[10][10])
{
    // monomial tables of the reference's closed form (tools/gen_age_table.py)
    double pi[8], po[8];
    pi[0] = po[0] = 1.0;
    for (int k = 1; k < 8; ++k) {
        pi[k] = pi[k - 1] * ci;
        po[k] = po[k - 1] * co;
    }
    for (int a = 0; a < 10; ++a)
        for (int b = 0; b < 10; ++b) MG[a][b] = 0.0;
    for (int t = 0; t < k_age_nterms; ++t) {
        const int *r = k_age_terms[t];
        MG[r[0]][r[1]] += (r[4] * K + r[5] * Ki) * pi[r[2]] * po[r[3]];
    }
    for (int a = 0; a < 10; ++a)
        for (int b = a; b < 10; ++b) {
            MG[a][b] /= 48.;
            MG[b][a] = MG[a][b];
        }
}

int age_entries(const xfk_problem_desc *d, double sign, std::vector<long long> &key, std::vector<double> &val)
{
    key.clear();
    val.clear();
    if (d->n_ages <= 0 || d->problem_type != XFK_PLANAR) return XFK_OK;
    if (!d->ages) {
        set_error("missing air-gap element table");
        return XFK_ERR_ARG;
    }
    const double kPi = 3.141592653589793238462643383;
    std::map<long long, double> acc;
    for (int g = 0; g < d->n_ages; ++g) {
        const xfk_age_desc &A = d->ages[g];
        const int n = A.n_arc;
        if (n < 2 || !A.qn || !A.qw || !(A.ro > A.ri) || !(A.total_arc_length > 0)) {
            set_error("malformed air-gap element " + std::to_string(g));
            return XFK_ERR_ARG;
        }
        for (int k = 0; k < 4 * (n + 1); ++k)
            if (A.qn[k] < 0 || A.qn[k] >= d->n_nodes) {
                set_error("air-gap element node index out of range");
                return XFK_ERR_ARG;
            }
        // K = dr / (R dtheta) of one arc element (static2d.cpp:199-204)
        const double dt = (kPi / 180.) * (A.total_arc_length / n);
        const double K = 2. * (A.ro - A.ri) / (dt * (A.ro + A.ri));
        // shift of the inner ring relative to the outer one, in [0, 1]
        double ci = A.inner_shift, co = A.outer_shift;
        if (ci > co) {
            ci -= co;
            co = 0;
        } else {
            ci = 1 - co + ci;
            co = 1;
        }
        double MG[10][10];
        age_matrix(ci, co, K, 1. / K, MG);

        // quadNode k holds the ring nodes either side of arc position k:
        // (n0, n1) inner, (n2, n3) outer.  Element k reads positions k-1 .. k+2
        // of both rings, wrapping over the arc (static2d.cpp:277-330).
        auto q = [&](int k) { return k < 0 ? n - 1 : (k > n ? 1 : k); };
        for (int k = 0; k < n; ++k) {
            int nn[10];
            double ww[10];
            for (int ring = 0; ring < 2; ++ring) {
                const int o = 5 * ring, lo = 2 * ring, hi = 2 * ring + 1;   // n0/n1 or n2/n3
                const int km = q(k - 1), kp = q(k + 2);
                nn[o + 0] = A.qn[4 * km + lo];      ww[o + 0] = A.qw[4 * km + lo];
                nn[o + 1] = A.qn[4 * k + lo];       ww[o + 1] = A.qw[4 * k + lo];
                nn[o + 2] = A.qn[4 * k + hi];       ww[o + 2] = A.qw[4 * k + hi];
                nn[o + 3] = A.qn[4 * (k + 1) + hi]; ww[o + 3] = A.qw[4 * (k + 1) + hi];
                nn[o + 4] = A.qn[4 * kp + hi];      ww[o + 4] = A.qw[4 * kp + hi];
            }
            if (A.format == 1) {   // antiperiodic copies change sign across the slice ends
                if (k == 0) { ww[0] = -ww[0]; ww[5] = -ww[5]; }
                // Static2D flips the wrap-around of the last element too
                // (static2d.cpp:333); Harmonic2D (sign < 0) tests
                // k == totalArcElements (harmonic2d.cpp:373), never true: the
                // reference's answers are reproduced, flip omitted
                if (k + 1 == n && sign > 0) { ww[4] = -ww[4]; ww[9] = -ww[9]; }
            }
            for (int a = 0; a < 10; ++a)
                for (int b = a; b < 10; ++b) {
                    int r = nn[a], c = nn[b];
                    if (c < r) std::swap(r, c);
                    acc[((long long)r << 32) | (unsigned)c] += sign * MG[a][b] * ww[a] * ww[b];
                }
        }
    }
    for (auto &kv : acc) {
        if (kv.second == 0.0) continue;   // e.g. ring positions an aligned ring does not reach
        key.push_back(kv.first);
        val.push_back(kv.second);
    }
    return XFK_OK;
}

}  // namespace xfk

extern "C" int xfk_age_element_matrix(double ci, double co, double K, double Ki, double *MG)
{
    if (!MG) return XFK_ERR_ARG;
    double M[10][10];
    xfk::age_matrix(ci, co, K, Ki, M);
    for (int a = 0; a < 10; ++a)
        for (int b = 0; b < 10; ++b) MG[10 * a + b] = M[a][b];
    return XFK_OK;
}
