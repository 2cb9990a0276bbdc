/* Air-gap element contributions (CPU oracle).
 *
 * TEST INFRASTRUCTURE ONLY: the checker, never the thing measured or shipped.
 *
 * Restates the "tack in air gap element contributions" loop that opens every
 * assembly of FSolver::Static2D (cfemm/fsolver/static2d.cpp:191-344) and
 * FSolver::Harmonic2D (cfemm/fsolver/harmonic2d.cpp:227-382): per AGE, the
 * ring-shift reduction and K = dr / (R dtheta) (static2d.cpp:199-215), the
 * 10x10 element matrix, the ten-node gather with wrap-around and antiperiodic
 * sign fixes (static2d.cpp:277-337; harmonic2d.cpp:367-377 tests
 * k == totalArcElements for the last-element fix, which never holds, so the
 * reference's Harmonic2D never applies it -- reproduced, see `harmonic`), and
 * the AddTo of the upper triangle weighted by ww[ii] ww[jj]
 * (static2d.cpp:340-342), in the reference's order.
 *
 * The element matrix is NOT taken from the reference's closed form
 * (static2d.cpp:218-268, a machine-generated polynomial in ci, co) nor from the
 * product's monomial table (xfemm_amd/csrc/xfk_age_table.h, generated from
 * that text): it is built here from the element it describes,
 *
 *     MG = T(ci, co)^T  (K Ktheta + Ki Kr)  T(ci, co),
 *
 * a rectangle of the annulus (theta x r, aspect K = dr / (R dtheta)) whose four
 * corner values are Catmull-Rom interpolants, at parameter 1 - shift, of four
 * consecutive nodes of the ring they lie on (T, 4 x 10), and whose stiffness
 * is the mean of the bilinear quadrilateral's and the two-triangle
 * split's (Ktheta = [20 -20 4 -4] / 48 pattern, Kr its transpose in r).
 * This reproduces the reference's closed form to rounding (8e-16 relative at
 * random shifts), so it pins both the closed form's transcription into the
 * product table and the table itself (tests/test_oracle_age.py).
 */
#include "static2d_oracle.h"

#define AGE_PI 3.141592653589793238462643383

/* Catmull-Rom weights of p0..p3 at t in [0, 1] (between p1 and p2) */
static void catmull_rom(double t, double *w)
{
    const double t2 = t * t, t3 = t2 * t;
    w[0] = 0.5 * (-t + 2. * t2 - t3);
    w[1] = 0.5 * (2. - 5. * t2 + 3. * t3);
    w[2] = 0.5 * (t + 4. * t2 - 3. * t3);
    w[3] = 0.5 * (-t2 + t3);
}

void ora_age_matrix(double ci, double co, double K, double Ki, double *MG)
{
    /* corners: 0 inner/left, 1 inner/right, 2 outer/left, 3 outer/right; ring
       nodes 0..4 inner (k-2 .. k+2), 5..9 outer */
    double T[4][10] = {{0}}, wi[4], wo[4];
    catmull_rom(1. - ci, wi);
    catmull_rom(1. - co, wo);
    for (int m = 0; m < 4; m++) {
        T[0][m] = wi[m];
        T[1][m + 1] = wi[m];
        T[2][m + 5] = wo[m];
        T[3][m + 6] = wo[m];
    }
    /* rectangle stiffness: theta-derivative part couples left/right corners,
       r-derivative part inner/outer ones; mean of bilinear quad and
       two-triangle split: diagonal 20, same-edge partner -20 / 4, opposite 4 / -20 */
    static const double Kt[4][4] = {{20, -20, 4, -4}, {-20, 20, -4, 4}, {4, -4, 20, -20}, {-4, 4, -20, 20}};
    static const double Kr[4][4] = {{20, 4, -20, -4}, {4, 20, -4, -20}, {-20, -4, 20, 4}, {-4, -20, 4, 20}};
    double Q[4][4];
    for (int a = 0; a < 4; a++)
        for (int b = 0; b < 4; b++) Q[a][b] = (K * Kt[a][b] + Ki * Kr[a][b]) / 48.;
    for (int a = 0; a < 10; a++)
        for (int b = 0; b < 10; b++) {
            double s = 0.;
            for (int u = 0; u < 4; u++) {
                if (T[u][a] == 0.) continue;
                for (int v = 0; v < 4; v++) s += T[u][a] * Q[u][v] * T[v][b];
            }
            MG[10 * a + b] = s;
        }
}

void ora_age_assemble(int n_ages, const ora_age *ages, int harmonic, ora_age_emit emit, void *ctx)
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
            /* Static2D: (k+1) == totalArcElements (static2d.cpp:333); Harmonic2D
               tests k == totalArcElements (harmonic2d.cpp:373): never true */
            if (!harmonic && k + 1 == M && ag->BdryFormat == 1) {
                ww[4] = -ww[4];
                ww[9] = -ww[9];
            }
            for (int ii = 0; ii < 10; ii++)
                for (int jj = ii; jj < 10; jj++)
                    emit(ctx, MG[10 * ii + jj] * ww[ii] * ww[jj], nn[ii], nn[jj]);
        }
    }
}
