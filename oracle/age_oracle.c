/* Air-gap element contributions (CPU oracle).
 *
 * TEST INFRASTRUCTURE ONLY: the checker, never the thing measured or shipped.
 *
 * Restates the "tack in air gap element contributions" loop that opens every
 * assembly of FSolver::Static2D (cfemm/fsolver/static2d.cpp:191-344) and
 * FSolver::Harmonic2D (cfemm/fsolver/harmonic2d.cpp:227-380): per AGE, the
 * ring-shift reduction and K = dr / (R dtheta) (static2d.cpp:199-215), the
 * 10x10 serendipity-derived matrix (static2d.cpp:209-263; evaluated here from
 * the monomial table oracle/age_table.h, generated from that closed form by
 * tools/gen_age_table.py and pinned by tests/golden/age_mg.json), the
 * ten-node gather with wrap-around and antiperiodic sign fixes
 * (static2d.cpp:277-337), and the AddTo of the upper triangle weighted by
 * ww[ii] ww[jj] (static2d.cpp:340-342), in the reference's order.
 */
#include "static2d_oracle.h"

#include "age_table.h"

#define AGE_PI 3.141592653589793238462643383

void ora_age_matrix(double ci, double co, double K, double Ki, double *MG)
{
    double pi[8], po[8];
    pi[0] = po[0] = 1.0;
    for (int k = 1; k < 8; k++) {
        pi[k] = pi[k - 1] * ci;
        po[k] = po[k - 1] * co;
    }
    for (int k = 0; k < 100; k++) MG[k] = 0.0;
    for (int t = 0; t < k_age_nterms; t++) {
        const int *r = k_age_terms[t];
        MG[10 * r[0] + r[1]] += (r[4] * K + r[5] * Ki) * pi[r[2]] * po[r[3]];
    }
    for (int a = 0; a < 10; a++)
        for (int b = a; b < 10; b++) {
            MG[10 * a + b] /= 48.;
            MG[10 * b + a] = MG[10 * a + b];
        }
}

void ora_age_assemble(int n_ages, const ora_age *ages, ora_age_emit emit, void *ctx)
{
    for (int i = 0; i < n_ages; i++) {
        const ora_age *ag = &ages[i];
        const int M = ag->totalArcElements;
        double MG[100], ww[10], ci, co, dt, K;
        int nn[10];

        dt = (AGE_PI / 180.) * (ag->totalArcLength / M);
        K = 2. * (ag->ro - ag->ri) / (dt * (ag->ro + ag->ri));
        ci = ag->InnerShift;
        co = ag->OuterShift;
        if (ci > co) {
            ci = ci - co;
            co = 0;
        } else {
            ci = 1 - co + ci;
            co = 1;
        }
        ora_age_matrix(ci, co, K, 1. / K, MG);

        for (int k = 0; k < M; k++) {
            /* quadNode[j].{n,w}{0,1,2,3} live at qn/qw[4 j + 0..3] */
            const int prev = (k - 1 < 0) ? M - 1 : k - 1;
            const int next2 = (k + 2 > M) ? 1 : k + 2;
            for (int side = 0; side < 2; side++) {
                const int lo = 2 * side, hi = lo + 1, o = 5 * side;
                nn[o + 0] = ag->qn[4 * prev + lo];
                ww[o + 0] = ag->qw[4 * prev + lo];
                nn[o + 1] = ag->qn[4 * k + lo];
                ww[o + 1] = ag->qw[4 * k + lo];
                nn[o + 2] = ag->qn[4 * k + hi];
                ww[o + 2] = ag->qw[4 * k + hi];
                nn[o + 3] = ag->qn[4 * (k + 1) + hi];
                ww[o + 3] = ag->qw[4 * (k + 1) + hi];
                nn[o + 4] = ag->qn[4 * next2 + hi];
                ww[o + 4] = ag->qw[4 * next2 + hi];
            }
            if (k == 0 && ag->BdryFormat == 1) {
                ww[0] = -ww[0];
                ww[5] = -ww[5];
            }
            if (k + 1 == M && ag->BdryFormat == 1) {
                ww[4] = -ww[4];
                ww[9] = -ww[9];
            }
            for (int ii = 0; ii < 10; ii++)
                for (int jj = ii; jj < 10; jj++)
                    emit(ctx, MG[10 * ii + jj] * ww[ii] * ww[jj], nn[ii], nn[jj]);
        }
    }
}
