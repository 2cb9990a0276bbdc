/* CPU oracle for the fsolver static-2D hot path -- TEST INFRASTRUCTURE ONLY.
 * See static2d_oracle.h for scope and the reference lines each part follows.
 *
 * Storage restates CBigLinProb's per-row linked lists (spars.cpp:105-160):
 * row i keeps its diagonal first, then the upper-triangular entries (c > i)
 * in increasing column order.  Here a row is a small growable array instead
 * of a list; the arithmetic order of every loop is kept so that results are
 * bit-identical with the reference's spars.cpp.
 */
#include "static2d_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ORA_PI 3.141592653589793238462643383
#define ORA_DEG 0.01745329251994329576923690768
#define ORA_MUO 1.2566370614359173e-6

/* ------------------------------------------------------------------------ */
/* CBigLinProb restatement                                                  */
/* ------------------------------------------------------------------------ */

typedef struct {
    int len, cap;
    int *c;
    double *x;
} ora_row;

typedef struct {
    int n, bdw;
    double precision, lambda;
    ora_row *M;
    double *V, *P, *R, *U, *Z, *b;
} ora_lp;

static void row_reserve(ora_row *r, int cap)
{
    if (cap <= r->cap) return;
    int nc = r->cap ? r->cap * 2 : 8;
    while (nc < cap) nc *= 2;
    r->c = (int *)realloc(r->c, sizeof(int) * nc);
    r->x = (double *)realloc(r->x, sizeof(double) * nc);
    r->cap = nc;
}

void *ora_lp_create(int n, int bw, double precision)
{   /* spars.cpp:80-103 */
    ora_lp *L = (ora_lp *)calloc(1, sizeof(ora_lp));
    L->n = n;
    L->bdw = bw;
    L->precision = precision;
    L->lambda = 1.5; /* spars.cpp:46 */
    L->M = (ora_row *)calloc(n, sizeof(ora_row));
    L->V = (double *)calloc(n, sizeof(double));
    L->P = (double *)calloc(n, sizeof(double));
    L->R = (double *)calloc(n, sizeof(double));
    L->U = (double *)calloc(n, sizeof(double));
    L->Z = (double *)calloc(n, sizeof(double));
    L->b = (double *)calloc(n, sizeof(double));
    for (int i = 0; i < n; i++) {
        row_reserve(&L->M[i], 8);
        L->M[i].len = 1;
        L->M[i].c[0] = i;
        L->M[i].x[0] = 0.0;
    }
    return L;
}

void ora_lp_destroy(void *lp)
{
    ora_lp *L = (ora_lp *)lp;
    if (!L) return;
    for (int i = 0; i < L->n; i++) {
        free(L->M[i].c);
        free(L->M[i].x);
    }
    free(L->M);
    free(L->V); free(L->P); free(L->R); free(L->U); free(L->Z); free(L->b);
    free(L);
}

/* spars.cpp:105-142: create/set entry (p,q), p<=q after the swap */
static void lp_put(ora_lp *L, double v, int p, int q)
{
    if (q < p) { int t = p; p = q; q = t; }
    ora_row *r = &L->M[p];
    int k = 0;
    while (k < r->len && r->c[k] < q) k++;
    if (k < r->len && r->c[k] == q) { r->x[k] = v; return; }
    row_reserve(r, r->len + 1);
    memmove(r->c + k + 1, r->c + k, sizeof(int) * (r->len - k));
    memmove(r->x + k + 1, r->x + k, sizeof(double) * (r->len - k));
    r->c[k] = q;
    r->x[k] = v;
    r->len++;
}

static double lp_get(ora_lp *L, int p, int q)
{   /* spars.cpp:144-160 */
    if (q < p) { int t = p; p = q; q = t; }
    const ora_row *r = &L->M[p];
    for (int k = 0; k < r->len; k++) {
        if (r->c[k] == q) return r->x[k];
        if (r->c[k] > q) break;
    }
    return 0.0;
}

double ora_lp_get(void *L, int p, int q) { return lp_get((ora_lp *)L, p, q); }

void ora_lp_addto(void *lp, double v, int p, int q)
{   /* spars.cpp:162-165 */
    ora_lp *L = (ora_lp *)lp;
    lp_put(L, lp_get(L, p, q) + v, p, q);
}

double *ora_lp_b(void *L) { return ((ora_lp *)L)->b; }
double *ora_lp_V(void *L) { return ((ora_lp *)L)->V; }

void ora_lp_multA(void *lp, const double *X, double *Y)
{   /* spars.cpp:167-185 */
    ora_lp *L = (ora_lp *)lp;
    int n = L->n;
    for (int i = 0; i < n; i++) Y[i] = 0;
    for (int i = 0; i < n; i++) {
        const ora_row *r = &L->M[i];
        Y[i] += r->x[0] * X[i];
        for (int k = 1; k < r->len; k++) {
            int c = r->c[k];
            Y[i] += r->x[k] * X[c];
            Y[c] += r->x[k] * X[i];
        }
    }
}

static double lp_dot(const double *X, const double *Y, int n)
{   /* spars.cpp:187-195 */
    double z = 0;
    for (int i = 0; i < n; i++) z += X[i] * Y[i];
    return z;
}

static void lp_multpc(ora_lp *L, const double *X, double *Y)
{   /* spars.cpp:197-236: SSOR preconditioner */
    int n = L->n;
    double lam = L->lambda;
    double c = lam * (2. - lam);
    for (int i = 0; i < n; i++) Y[i] = X[i] * c;
    for (int i = 0; i < n; i++) {
        const ora_row *r = &L->M[i];
        Y[i] /= r->x[0];
        for (int k = 1; k < r->len; k++)
            Y[r->c[k]] -= r->x[k] * Y[i] * lam;
    }
    for (int i = 0; i < n; i++) Y[i] *= L->M[i].x[0];
    for (int i = n - 1; i >= 0; i--) {
        const ora_row *r = &L->M[i];
        for (int k = 1; k < r->len; k++)
            Y[i] -= r->x[k] * Y[r->c[k]] * lam;
        Y[i] /= r->x[0];
    }
}

int ora_lp_pcgsolve(void *lp, int flag, long long *iters)
{   /* spars.cpp:238-316 */
    ora_lp *L = (ora_lp *)lp;
    int n = L->n;
    double res, res_o, res_new, er, del, rho, pAp;
    long long it = 0;
    for (int i = 0; i < n; i++)
        if (L->M[i].x[0] == 0) {
            fprintf(stderr, "singular flag tripped at %i of %i\n", i, n);
            if (iters) *iters = 0;
            return 0;
        }
    lp_multpc(L, L->b, L->Z);
    res_o = lp_dot(L->Z, L->b, n);
    if (res_o == 0) { if (iters) *iters = 0; return 1; }
    if (flag == 0) for (int i = 0; i < n; i++) L->V[i] = 0;
    ora_lp_multA(L, L->V, L->R);
    for (int i = 0; i < n; i++) L->R[i] = L->b[i] - L->R[i];
    lp_multpc(L, L->R, L->Z);
    for (int i = 0; i < n; i++) L->P[i] = L->Z[i];
    res = lp_dot(L->Z, L->R, n);
    do {
        ora_lp_multA(L, L->P, L->U);
        pAp = lp_dot(L->P, L->U, n);
        del = res / pAp;
        for (int i = 0; i < n; i++) {
            L->V[i] += (del * L->P[i]);
            L->R[i] -= (del * L->U[i]);
        }
        lp_multpc(L, L->R, L->Z);
        res_new = lp_dot(L->Z, L->R, n);
        rho = res_new / res;
        res = res_new;
        for (int i = 0; i < n; i++) L->P[i] = L->Z[i] + (rho * L->P[i]);
        er = sqrt(res / res_o);
        it++;
    } while (er > L->precision);
    if (iters) *iters = it;
    return 1;
}

void ora_lp_setvalue(void *lp, int i, double x)
{   /* spars.cpp:318-346 */
    ora_lp *L = (ora_lp *)lp;
    int fst, lst;
    if (L->bdw == 0) { fst = 0; lst = L->n; }
    else {
        fst = i - L->bdw; if (fst < 0) fst = 0;
        lst = i + L->bdw; if (lst > L->n) lst = L->n;
    }
    for (int k = fst; k < lst; k++) {
        double z = lp_get(L, k, i);
        if (z != 0) {
            L->b[k] = L->b[k] - (z * x);
            if (i != k) lp_put(L, 0., k, i);
        }
    }
    L->b[i] = lp_get(L, i, i) * x;
}

static void lp_wipe(void *lp)
{   /* spars.cpp:348-364 */
    ora_lp *L = (ora_lp *)lp;
    for (int i = 0; i < L->n; i++) {
        L->b[i] = 0.;
        for (int k = 0; k < L->M[i].len; k++) L->M[i].x[k] = 0;
    }
}

static void lp_pbc(ora_lp *L, int i, int j, double sgn)
{   /* spars.cpp:366-474 (KLUDGE: bdw forced to 0 -> full scan) */
    if (j < i) { int t = j; j = i; i = t; }
    for (int k = 0; k < L->n; k++) {
        if ((k != i) && (k != j)) {
            double v1 = lp_get(L, k, i);
            double v2 = lp_get(L, k, j);
            if ((v1 != 0) || (v2 != 0)) {
                double c = (sgn > 0) ? (v1 + v2) / 2. : (v1 - v2) / 2.;
                lp_put(L, c, k, i);
                lp_put(L, sgn > 0 ? c : -c, k, j);
            }
        }
    }
    double c;
    if (sgn > 0) c = (lp_get(L, i, i) + lp_get(L, j, j)) / 2.;
    else c = 0.5 * (lp_get(L, i, i) + lp_get(L, j, j));
    lp_put(L, c, i, i);
    lp_put(L, c, j, j);
    if (sgn > 0) {
        c = 0.5 * (L->b[i] + L->b[j]);
        L->b[i] = c;
        L->b[j] = c;
    } else {
        c = 0.5 * (L->b[i] - L->b[j]);
        L->b[i] = c;
        L->b[j] = -c;
    }
}

void ora_lp_periodicity(void *L, int i, int j) { lp_pbc((ora_lp *)L, i, j, 1.0); }
void ora_lp_antiperiodicity(void *L, int i, int j) { lp_pbc((ora_lp *)L, i, j, -1.0); }

long long ora_lp_export_upper(void *lp, int *rows, int *cols, double *vals, long long cap)
{
    ora_lp *L = (ora_lp *)lp;
    long long k = 0;
    for (int i = 0; i < L->n; i++)
        for (int m = 0; m < L->M[i].len; m++) {
            if (k < cap) { rows[k] = i; cols[k] = L->M[i].c[m]; vals[k] = L->M[i].x[m]; }
            k++;
        }
    return k;
}

static int lp_pcg_ops(void *L, int flag, long long *iters) { return ora_lp_pcgsolve(L, flag, iters); }

static const ora_linprob_ops k_builtin = {
    ora_lp_create, ora_lp_destroy, ora_lp_addto, ora_lp_b, ora_lp_V, ora_lp_setvalue,
    ora_lp_periodicity, ora_lp_antiperiodicity, lp_wipe, lp_pcg_ops,
};

const ora_linprob_ops *ora_builtin_linprob(void) { return &k_builtin; }

/* ------------------------------------------------------------------------ */
/* CMSolverMaterialProp::GetBHProps (CMaterialProp.cpp:997-1057)            */
/* ------------------------------------------------------------------------ */

void ora_get_bh_props(const ora_block *m, double B, double *v, double *dv)
{
    double b = fabs(B);
    int n = m->BHpoints;
    if (n == 0) { *v = m->mu_x; *dv = 0; return; }
    if (b == 0) { *v = m->slope[0]; *dv = 0; return; }
    if (b > m->Bdata[n - 1]) {
        double h = (m->Hdata[n - 1] + m->slope[n - 1] * (b - m->Bdata[n - 1]));
        double dh = m->slope[n - 1];
        *v = h / b;
        *dv = 0.5 * (dh / (b * b) - h / (b * b * b));
        return;
    }
    for (int i = 0; i < n - 1; i++)
        if ((b >= m->Bdata[i]) && (b <= m->Bdata[i + 1])) {
            double l = (m->Bdata[i + 1] - m->Bdata[i]);
            double z = (b - m->Bdata[i]) / l;
            double z2 = z * z;
            double h = (1. - 3. * z2 + 2. * z2 * z) * m->Hdata[i] +
                       z * (1. - 2. * z + z2) * l * m->slope[i] +
                       z2 * (3. - 2. * z) * m->Hdata[i + 1] +
                       z2 * (z - 1.) * l * m->slope[i + 1];
            double dh = 6. * z * (z - 1.) * m->Hdata[i] / l +
                        (1. - 4. * z + 3. * z * z) * m->slope[i] +
                        6. * z * (1. - z) * m->Hdata[i + 1] / l +
                        z * (3. * z - 2.) * m->slope[i + 1];
            *v = h / b;
            *dv = 0.5 * (dh / (b * b) - h / (b * b * b));
            return;
        }
    /* unreachable for a monotone table; the reference leaves v, dv untouched */
}

/* ------------------------------------------------------------------------ */
/* FSolver::Static2D (static2d.cpp:53-1033)                                 */
/* ------------------------------------------------------------------------ */

static void ora_circuits(ora_problem *pr)
{
    const int NE = pr->n_elems;
    /* circuits (static2d.cpp:84-167) */
    if (pr->n_circs > 0) {
        double *CI1 = (double *)calloc(pr->n_circs, sizeof(double));
        double *CI2 = (double *)calloc(pr->n_circs, sizeof(double));
        double *CI3 = (double *)calloc(pr->n_circs, sizeof(double));
        for (int i = 0; i < NE; i++) {
            int lb = pr->lbl[i];
            if (lb >= 0 && pr->labels[lb].InCircuit != -1) {
                const int *n = pr->p + 3 * i;
                double p0 = pr->y[n[1]] - pr->y[n[2]];
                double p1 = pr->y[n[2]] - pr->y[n[0]];
                double q0 = pr->x[n[2]] - pr->x[n[1]];
                double q1 = pr->x[n[0]] - pr->x[n[2]];
                double a = (p0 * q1 - p1 * q0) / 2.;
                const ora_block *bp = &pr->blocks[pr->blk[i]];
                double Cduct = bp->Cduct;
                if (pr->labels[lb].bIsWound) Cduct = 0;
                int ic = pr->labels[lb].InCircuit;
                CI1[ic] += a;
                if (pr->axisymmetric) {   /* staticaxi.cpp:96-104 */
                    double r = (pr->x[n[0]] + pr->x[n[1]] + pr->x[n[2]]) / 3.;
                    CI2[ic] += 100. * a * Cduct / r;
                } else {
                    CI2[ic] += a * Cduct;
                }
                CI3[ic] += bp->J_re * a * 100.;
            }
        }
        for (int i = 0; i < pr->n_circs; i++) {
            ora_circ *cp = &pr->circs[i];
            if (cp->CircType == 0) {
                if (CI2[i] == 0) {
                    cp->Case = 1;
                    if (CI1[i] == 0.) cp->J = 0.;
                    else cp->J = 0.01 * (cp->Amps_re - CI3[i]) / CI1[i];
                } else {
                    cp->Case = 0;
                    cp->dV = -0.01 * (cp->Amps_re - CI3[i]) / CI2[i];
                }
            } else {
                cp->Case = 0;
                cp->dV = cp->dVolts_re;
            }
        }
        free(CI1); free(CI2); free(CI3);
    }

}

/* one Newton iteration's assembly + boundary conditions (static2d.cpp:186-940) */
static void age_emit(void *ctx, double v, int p, int q)
{
    struct age_ctx { const ora_linprob_ops *ops; void *L; } *a = ctx;
    a->ops->addto(a->L, v, p, q);
}

static void ora_assemble(ora_problem *pr, const ora_linprob_ops *ops, void *L, int Iter,
                         double *mu1, double *mu2, double *v12, int *LinearFlag_io)
{
    const double c = ORA_PI * 4.e-05;
    const double units[] = {2.54, 0.1, 1., 100., 0.00254, 1.e-04};
    const int NN = pr->n_nodes, NE = pr->n_elems;
    int LinearFlag = *LinearFlag_io;
        double *b = ops->b(L);
        double *Vv = ops->V(L);

        /* air-gap elements first (static2d.cpp:191-344) */
        struct age_ctx { const ora_linprob_ops *ops; void *L; } actx = {ops, L};
        ora_age_assemble(pr->n_ages, pr->ages, 0, age_emit, &actx);

        for (int i = 0; i < NE; i++) {
            double Me[3][3], be[3], Mx[3][3], My[3][3], Mxy[3][3], Mn[3][3];
            double l[3], p[3], q[3], v[3], u[3];
            int n[3];
            double a, K, t, B1, B2, B, mu, dv;
            for (int j = 0; j < 3; j++) {
                for (int k = 0; k < 3; k++) {
                    Me[j][k] = 0.; Mx[j][k] = 0.; My[j][k] = 0.; Mn[j][k] = 0.; Mxy[j][k] = 0.;
                }
                be[j] = 0.;
            }
            for (int k = 0; k < 3; k++) n[k] = pr->p[3 * i + k];
            const double *X = pr->x, *Y = pr->y;
            p[0] = Y[n[1]] - Y[n[2]];
            p[1] = Y[n[2]] - Y[n[0]];
            p[2] = Y[n[0]] - Y[n[1]];
            q[0] = X[n[2]] - X[n[1]];
            q[1] = X[n[0]] - X[n[2]];
            q[2] = X[n[1]] - X[n[0]];
            for (int j = 0, k = 1; j < 3; k++, j++) {
                if (k == 3) k = 0;
                l[j] = sqrt(pow(X[n[k]] - X[n[j]], 2.) + pow(Y[n[k]] - Y[n[j]], 2.));
            }
            a = (p[0] * q[1] - p[1] * q[0]) / 2.;

            K = (-1. / (4. * a));
            for (int j = 0; j < 3; j++)
                for (int k = j; k < 3; k++) {
                    Mx[j][k] += K * p[j] * p[k];
                    if (j != k) Mx[k][j] += K * p[j] * p[k];
                }
            for (int j = 0; j < 3; j++)
                for (int k = j; k < 3; k++) {
                    My[j][k] += K * q[j] * q[k];
                    if (j != k) My[k][j] += K * q[j] * q[k];
                }
            for (int j = 0; j < 3; j++)
                for (int k = j; k < 3; k++) {
                    Mxy[j][k] += K * (p[j] * q[k] + p[k] * q[j]);
                    if (j != k) Mxy[k][j] += K * (p[j] * q[k] + p[k] * q[j]);
                }

            /* mixed (derivative) boundary conditions */
            for (int j = 0; j < 3; j++) {
                int ej = pr->e[3 * i + j];
                if (ej >= 0 && pr->lines[ej].BdryFormat == 2) {
                    K = -0.0001 * c * pr->lines[ej].c0 * l[j] / 6.;
                    int k = j + 1;
                    if (k == 3) k = 0;
                    Me[j][j] += K * 2.;
                    Me[k][k] += K * 2.;
                    Me[j][k] += K;
                    Me[k][j] += K;
                    K = (pr->lines[ej].c1 * l[j] / 2.) * 0.0001;
                    be[j] += K;
                    be[k] += K;
                }
            }

            const ora_label *lab = &pr->labels[pr->lbl[i]];
            const ora_block *bp = &pr->blocks[pr->blk[i]];
            /* source current density */
            for (int j = 0; j < 3; j++) {
                t = 0;
                if (lab->InCircuit >= 0) {
                    const ora_circ *cp = &pr->circs[lab->InCircuit];
                    if (cp->Case == 1) t = cp->J;
                    if (cp->Case == 0) t = -cp->dV * bp->Cduct;
                }
                K = -(bp->J_re + t) * a / 3.;
                be[j] += K;
            }
            /* magnetization (static2d.cpp:509-598; a MagDirFctn label's direction per element) */
            t = pr->elem_magdir ? pr->elem_magdir[i] : lab->MagDir;
            for (int j = 0; j < 3; j++) {
                int k = j + 1;
                if (k == 3) k = 0;
                K = 0.0001 * bp->H_c * (cos(t * ORA_PI / 180.) * (X[n[k]] - X[n[j]]) +
                                        sin(t * ORA_PI / 180.) * (Y[n[k]] - Y[n[j]])) / 2.;
                be[j] += K;
                be[k] += K;
            }

            /* nonlinear part */
            if (Iter == 0) {
                if (bp->LamType == 0) {
                    t = bp->LamFill;
                    mu1[i] = bp->mu_x * t + (1. - t);
                    mu2[i] = bp->mu_y * t + (1. - t);
                }
                if (bp->LamType == 1) {
                    t = bp->LamFill;
                    mu = bp->mu_x;
                    mu1[i] = mu * t + (1. - t);
                    mu2[i] = mu / (t + mu * (1. - t));
                }
                if (bp->LamType == 2) {
                    t = bp->LamFill;
                    mu = bp->mu_y;
                    mu2[i] = mu * t + (1. - t);
                    mu1[i] = mu / (t + mu * (1. - t));
                }
                if (bp->LamType > 2) { mu1[i] = 1; mu2[i] = 1; }
                if (bp->BHpoints != 0) LinearFlag = 0;
            } else {
                if ((bp->LamType == 0) && (mu1[i] == mu2[i]) && (bp->BHpoints > 0)) {
                    B1 = 0.; B2 = 0.;
                    for (int j = 0; j < 3; j++) {
                        B1 += Vv[n[j]] * q[j];
                        B2 += Vv[n[j]] * p[j];
                    }
                    B = c * sqrt(B1 * B1 + B2 * B2) / (0.02 * a);
                    ora_get_bh_props(bp, B, &mu, &dv);
                    mu = 1. / (ORA_MUO * mu);
                    mu1[i] = mu;
                    mu2[i] = mu;
                    for (int j = 0; j < 3; j++) {
                        v[j] = 0;
                        for (int w = 0; w < 3; w++) v[j] += (Mx[j][w] + My[j][w]) * Vv[n[w]];
                    }
                    K = -200. * c * c * c * dv / a;
                    for (int j = 0; j < 3; j++)
                        for (int w = 0; w < 3; w++) Mn[j][w] = K * v[j] * v[w];
                }
                if ((bp->LamType == 1) && (bp->BHpoints > 0)) {
                    t = bp->LamFill;
                    B1 = 0.; B2 = 0.;
                    for (int j = 0; j < 3; j++) {
                        B1 += Vv[n[j]] * q[j];
                        B2 += Vv[n[j]] * p[j] / t;
                    }
                    B = c * sqrt(B1 * B1 + B2 * B2) / (0.02 * a);
                    ora_get_bh_props(bp, B, &mu, &dv);
                    mu = 1. / (ORA_MUO * mu);
                    mu1[i] = mu * t;
                    mu2[i] = mu / (t + mu * (1. - t));
                    for (int j = 0; j < 3; j++) {
                        v[j] = 0; u[j] = 0;
                        for (int w = 0; w < 3; w++) {
                            v[j] += (My[j][w] / t + Mx[j][w]) * Vv[n[w]];
                            u[j] += (My[j][w] / t + t * Mx[j][w]) * Vv[n[w]];
                        }
                    }
                    K = -100. * c * c * c * dv / (a);
                    for (int j = 0; j < 3; j++)
                        for (int w = 0; w < 3; w++) Mn[j][w] = K * (v[j] * u[w] + v[w] * u[j]);
                }
                if ((bp->LamType == 2) && (bp->BHpoints > 0)) {
                    t = bp->LamFill;
                    B1 = 0.; B2 = 0.;
                    for (int j = 0; j < 3; j++) {
                        B1 += (Vv[n[j]] * q[j]) / t;
                        B2 += Vv[n[j]] * p[j];
                    }
                    B = c * sqrt(B1 * B1 + B2 * B2) / (0.02 * a);
                    ora_get_bh_props(bp, B, &mu, &dv);
                    mu = 1. / (ORA_MUO * mu);
                    mu2[i] = mu * t;
                    mu1[i] = mu / (t + mu * (1. - t));
                    for (int j = 0; j < 3; j++) {
                        v[j] = 0; u[j] = 0;
                        for (int w = 0; w < 3; w++) {
                            v[j] += (Mx[j][w] / t + My[j][w]) * Vv[n[w]];
                            u[j] += (Mx[j][w] / t + t * My[j][w]) * Vv[n[w]];
                        }
                    }
                    K = -100. * c * c * c * dv / (a);
                    for (int j = 0; j < 3; j++)
                        for (int w = 0; w < 3; w++) Mn[j][w] = K * (v[j] * u[w] + v[w] * u[j]);
                }
            }

            for (int j = 0; j < 3; j++)
                for (int k = 0; k < 3; k++) {
                    Me[j][k] += (Mx[j][k] / mu2[i] + My[j][k] / mu1[i] + Mxy[j][k] * v12[i] + Mn[j][k]);
                    be[j] += Mn[j][k] * Vv[n[k]];
                }
            for (int j = 0; j < 3; j++) {
                for (int k = j; k < 3; k++) ops->addto(L, -Me[j][k], n[j], n[k]);
                b[n[j]] -= be[j];
            }
        }

        /* point currents (static2d.cpp:818-825) */
        for (int i = 0; i < NN; i++)
            if (pr->marker[i] >= 0) b[i] += (0.01 * pr->points[pr->marker[i]].J_re);
        /* fixed A at points (static2d.cpp:827-838) */
        for (int i = 0; i < NN; i++)
            if (pr->marker[i] >= 0) {
                const ora_point *pp = &pr->points[pr->marker[i]];
                if ((pp->J_re == 0) && (pp->J_im == 0)) ops->setvalue(L, i, pp->A_re / c);
            }
        /* fixed A along segments (static2d.cpp:840-926) */
        for (int i = 0; i < NE; i++)
            for (int j = 0; j < 3; j++) {
                int k = j + 1;
                if (k == 3) k = 0;
                int s = pr->e[3 * i + j];
                if (s >= 0 && pr->lines[s].BdryFormat == 0) {
                    const ora_line *ln = &pr->lines[s];
                    int nodes2[2] = {pr->p[3 * i + j], pr->p[3 * i + k]};
                    for (int m = 0; m < 2; m++) {
                        double x = pr->x[nodes2[m]], y = pr->y[nodes2[m]], a;
                        if (pr->coords == 0) {
                            x /= units[pr->length_units];
                            y /= units[pr->length_units];
                            a = ln->A0 + x * ln->A1 + y * ln->A2;
                        } else {
                            double r = sqrt(x * x + y * y), t;
                            if ((x == 0) && (y == 0)) t = 0;
                            else t = atan2(y, x) / ORA_DEG;
                            r /= units[pr->length_units];
                            a = ln->A0 + r * ln->A1 + t * ln->A2;
                        }
                        a *= cos(ln->phi * ORA_DEG);
                        ops->setvalue(L, nodes2[m], a / c);
                    }
                }
            }
        /* (anti)periodic boundary conditions (static2d.cpp:929-940) */
        for (int k = 0; k < pr->n_pbc; k++) {
            if (pr->pbc[3 * k + 2] == 0) ops->periodicity(L, pr->pbc[3 * k], pr->pbc[3 * k + 1]);
            if (pr->pbc[3 * k + 2] == 1) ops->antiperiodicity(L, pr->pbc[3 * k], pr->pbc[3 * k + 1]);
        }

    *LinearFlag_io = LinearFlag;
}

/* one Newton iteration of FSolver::StaticAxisymmetric (staticaxi.cpp:146-697):
 * x is r, y is z (cm) */
static void ora_assemble_axi(ora_problem *pr, const ora_linprob_ops *ops, void *L, int Iter,
                             double *mu1, double *mu2, double *v12, int *LinearFlag_io)
{
    const double c = ORA_PI * 4.e-05;
    const double units[] = {2.54, 0.1, 1., 100., 0.00254, 1.e-04};
    const int NN = pr->n_nodes, NE = pr->n_elems;
    const double extRo = pr->ext_ro * units[pr->length_units];   /* staticaxi.cpp:70-72 */
    const double extRi = pr->ext_ri * units[pr->length_units];
    const double extZo = pr->ext_zo * units[pr->length_units];
    int LinearFlag = *LinearFlag_io;
    double *b = ops->b(L);
    double *Vv = ops->V(L);
    const double *X = pr->x, *Y = pr->y;

    for (int i = 0; i < NE; i++) {
        double Me[3][3], be[3], Mx[3][3], My[3][3], Mxy[3][3], Mn[3][3];
        double l[3], p[3], q[3], g[3], v[3], u[3], rn[3];
        int n[3];
        double a, K, t = 0., r, B, mu, dv, R, a_hat, vol, R_hat = 0.;
        for (int j = 0; j < 3; j++) {
            for (int k = 0; k < 3; k++) {
                Me[j][k] = 0.; Mx[j][k] = 0.; My[j][k] = 0.; Mxy[j][k] = 0.; Mn[j][k] = 0.;
            }
            be[j] = 0.;
        }
        for (int k = 0; k < 3; k++) {
            n[k] = pr->p[3 * i + k];
            rn[k] = X[n[k]];
        }
        p[0] = Y[n[1]] - Y[n[2]];
        p[1] = Y[n[2]] - Y[n[0]];
        p[2] = Y[n[0]] - Y[n[1]];
        q[0] = X[n[2]] - X[n[1]];
        q[1] = X[n[0]] - X[n[2]];
        q[2] = X[n[1]] - X[n[0]];
        g[0] = (X[n[2]] + X[n[1]]) / 2.;
        g[1] = (X[n[0]] + X[n[2]]) / 2.;
        g[2] = (X[n[1]] + X[n[0]]) / 2.;
        for (int j = 0, k = 1; j < 3; k++, j++) {
            if (k == 3) k = 0;
            l[j] = sqrt(pow(X[n[k]] - X[n[j]], 2.) + pow(Y[n[k]] - Y[n[j]], 2.));
        }
        a = (p[0] * q[1] - p[1] * q[0]) / 2.;
        R = (X[n[0]] + X[n[1]] + X[n[2]]) / 3.;
        a_hat = 0;
        for (int j = 0; j < 3; j++) a_hat += (rn[j] * rn[j] * p[j] / (4. * R));
        vol = 2. * R * a_hat;

        /* R_hat: the element's 1/r-weighted mean radius (staticaxi.cpp:208-254) */
        int flag = 0;
        for (int j = 0; j < 3; j++)
            if (rn[j] < 1.e-06) flag++;
        if (flag == 2) {
            R_hat = R;
        } else if (flag == 1) {
            if (rn[0] < 1.e-06) {
                if (fabs(rn[1] - rn[2]) < 1.e-06) R_hat = rn[2] / 2.;
                else R_hat = (rn[1] - rn[2]) / (2. * log(rn[1]) - 2. * log(rn[2]));
            }
            if (rn[1] < 1.e-06) {
                if (fabs(rn[2] - rn[0]) < 1.e-06) R_hat = rn[0] / 2.;
                else R_hat = (rn[2] - rn[0]) / (2. * log(rn[2]) - 2. * log(rn[0]));
            }
            if (rn[2] < 1.e-06) {
                if (fabs(rn[0] - rn[1]) < 1.e-06) R_hat = rn[1] / 2.;
                else R_hat = (rn[0] - rn[1]) / (2. * log(rn[0]) - 2. * log(rn[1]));
            }
        } else {
            if (fabs(q[0]) < 1.e-06)
                R_hat = (q[1] * q[1]) / (2. * (-q[1] + rn[0] * log(rn[0] / rn[2])));
            else if (fabs(q[1]) < 1.e-06)
                R_hat = (q[2] * q[2]) / (2. * (-q[2] + rn[1] * log(rn[1] / rn[0])));
            else if (fabs(q[2]) < 1.e-06)
                R_hat = (q[0] * q[0]) / (2. * (-q[0] + rn[2] * log(rn[2] / rn[1])));
            else
                R_hat = -(q[0] * q[1] * q[2]) /
                        (2. * (q[0] * rn[0] * log(rn[0]) + q[1] * rn[1] * log(rn[1]) + q[2] * rn[2] * log(rn[2])));
        }

        /* Mr, Mz, Mrz (staticaxi.cpp:256-296) */
        K = (-1. / (2. * a_hat * R));
        for (int j = 0; j < 3; j++)
            for (int k = j; k < 3; k++) Mx[j][k] += K * p[j] * rn[j] * p[k] * rn[k];
        for (int j = 0; j < 3; j++)
            if (rn[j] < 1.e-06) Mx[j][j] += Mx[0][0] + Mx[1][1] + Mx[2][2];
        K = (-1. / (2. * a_hat * R_hat));
        for (int j = 0; j < 3; j++)
            for (int k = j; k < 3; k++) My[j][k] += K * (q[j] * rn[j]) * (q[k] * rn[k]) * (g[j] / R) * (g[k] / R);
        for (int j = 0; j < 3; j++)
            for (int k = j; k < 3; k++)
                Mxy[j][k] += K * ((q[j] * rn[j]) * (g[j] / R)) * (p[k] * rn[k]) +
                             K * ((q[k] * rn[k]) * (g[k] / R)) * (p[j] * rn[j]);
        Mx[1][0] = Mx[0][1]; Mx[2][0] = Mx[0][2]; Mx[2][1] = Mx[1][2];
        My[1][0] = My[0][1]; My[2][0] = My[0][2]; My[2][1] = My[1][2];
        Mxy[1][0] = Mxy[0][1]; Mxy[2][0] = Mxy[0][2]; Mxy[2][1] = Mxy[1][2];

        /* mixed boundary conditions, r-weighted (staticaxi.cpp:298-320) */
        for (int j = 0; j < 3; j++) {
            int ej = pr->e[3 * i + j];
            if (ej >= 0 && pr->lines[ej].BdryFormat == 2) {
                int k = j + 1;
                if (k == 3) k = 0;
                r = (X[n[j]] + X[n[k]]) / 2.;
                K = -0.0001 * c * 2. * r * pr->lines[ej].c0 * l[j] / 6.;
                Me[j][j] += K * 2.;
                Me[k][k] += K * 2.;
                Me[j][k] += K;
                Me[k][j] += K;
                K = (pr->lines[ej].c1 * l[j] / 2.) * 0.0001 * 2 * r;
                be[j] += K;
                be[k] += K;
            }
        }

        const ora_label *lab = &pr->labels[pr->lbl[i]];
        const ora_block *bp = &pr->blocks[pr->blk[i]];
        /* source current density (staticaxi.cpp:322-337) */
        for (int j = 0; j < 3; j++) {
            if (lab->InCircuit >= 0) {
                const ora_circ *cp = &pr->circs[lab->InCircuit];
                if (cp->Case == 1) t = cp->J;
                if (cp->Case == 0) t = -100. * cp->dV * bp->Cduct / R;
            } else {
                t = 0;
            }
            K = -2. * R * (bp->J_re + t) * a / 3.;
            be[j] += K;
        }
        /* magnetization, r-weighted (staticaxi.cpp:339-407) */
        t = pr->elem_magdir ? pr->elem_magdir[i] : lab->MagDir;
        for (int j = 0; j < 3; j++) {
            int k = j + 1;
            if (k == 3) k = 0;
            r = (X[n[j]] + X[n[k]]) / 2.;
            K = -0.0001 * r * bp->H_c *
                (cos(t * ORA_PI / 180.) * (X[n[k]] - X[n[j]]) + sin(t * ORA_PI / 180.) * (Y[n[k]] - Y[n[j]]));
            be[j] += K;
            be[k] += K;
        }

        /* permeability (staticaxi.cpp:409-623; no incremental problems) */
        if (Iter == 0) {
            if (bp->LamType == 0) {
                mu = bp->LamFill;
                mu1[i] = bp->mu_x * mu;
                mu2[i] = bp->mu_y * mu;
            }
            if (bp->LamType == 1) {
                mu = bp->LamFill;
                K = bp->mu_x;
                mu1[i] = K * mu + (1. - mu);
                mu2[i] = K / (mu + K * (1. - mu));
            }
            if (bp->LamType == 2) {
                mu = bp->LamFill;
                K = bp->mu_y;
                mu1[i] = K * mu + (1. - mu);
                mu2[i] = K / (mu + K * (1. - mu));
            }
            if (bp->LamType > 2) { mu1[i] = 1; mu2[i] = 1; }
            if (bp->BHpoints != 0) LinearFlag = 0;
        } else {
            if ((bp->LamType == 0) && (mu1[i] == mu2[i]) && (bp->BHpoints > 0)) {
                /* B directly from the energy */
                v[0] = 0; v[1] = 0; v[2] = 0;
                for (int j = 0; j < 3; j++)
                    for (int w = 0; w < 3; w++) v[j] += (Mx[j][w] + My[j][w]) * Vv[n[w]];
                dv = 0;
                for (int j = 0; j < 3; j++) dv += Vv[n[j]] * v[j];
                dv *= (10000. * c * c / vol);
                B = sqrt(fabs(dv));
                ora_get_bh_props(bp, B, &mu, &dv);
                mu = 1. / (ORA_MUO * mu);
                mu1[i] = mu;
                mu2[i] = mu;
                for (int j = 0; j < 3; j++) {
                    v[j] = 0;
                    for (int w = 0; w < 3; w++) v[j] += (Mx[j][w] + My[j][w]) * Vv[n[w]];
                }
                K = -200. * c * c * c * dv / vol;
                for (int j = 0; j < 3; j++)
                    for (int w = 0; w < 3; w++) Mn[j][w] = K * v[j] * v[w];
            }
            if ((bp->LamType == 1) && (bp->BHpoints > 0)) {
                t = bp->LamFill;
                v[0] = 0; v[1] = 0; v[2] = 0;
                for (int j = 0; j < 3; j++)
                    for (int w = 0; w < 3; w++) v[j] += (Mx[j][w] + My[j][w] / (t * t)) * Vv[n[w]];
                dv = 0;
                for (int j = 0; j < 3; j++) dv += Vv[n[j]] * v[j];
                dv *= (10000. * c * c / vol);
                B = sqrt(fabs(dv));
                ora_get_bh_props(bp, B, &mu, &dv);
                mu = 1. / (ORA_MUO * mu);
                mu1[i] = mu * t;
                mu2[i] = mu / (t + mu * (1. - t));
                for (int j = 0; j < 3; j++) {
                    v[j] = 0; u[j] = 0;
                    for (int w = 0; w < 3; w++) {
                        v[j] += (My[j][w] / t + Mx[j][w]) * Vv[n[w]];
                        u[j] += (My[j][w] / t + t * Mx[j][w]) * Vv[n[w]];
                    }
                }
                K = -100. * c * c * c * dv / (vol);
                for (int j = 0; j < 3; j++)
                    for (int w = 0; w < 3; w++) Mn[j][w] = K * (v[j] * u[w] + v[w] * u[j]);
            }
            if ((bp->LamType == 2) && (bp->BHpoints > 0)) {
                t = bp->LamFill;
                v[0] = 0; v[1] = 0; v[2] = 0;
                for (int j = 0; j < 3; j++)
                    for (int w = 0; w < 3; w++) v[j] += (Mx[j][w] / (t * t) + My[j][w]) * Vv[n[w]];
                dv = 0;
                for (int j = 0; j < 3; j++) dv += Vv[n[j]] * v[j];
                dv *= (10000. * c * c / vol);
                B = sqrt(fabs(dv));
                ora_get_bh_props(bp, B, &mu, &dv);
                mu = 1. / (ORA_MUO * mu);
                mu2[i] = mu * t;
                mu1[i] = mu / (t + mu * (1. - t));
                for (int j = 0; j < 3; j++) {
                    v[j] = 0; u[j] = 0;
                    for (int w = 0; w < 3; w++) {
                        v[j] += (Mx[j][w] / t + My[j][w]) * Vv[n[w]];
                        u[j] += (Mx[j][w] / t + t * My[j][w]) * Vv[n[w]];
                    }
                }
                K = -100. * c * c * c * dv / (vol);
                for (int j = 0; j < 3; j++)
                    for (int w = 0; w < 3; w++) Mn[j][w] = K * (v[j] * u[w] + v[w] * u[j]);
            }
        }

        /* the conformally mapped exterior region (staticaxi.cpp:625-632) */
        if (lab->IsExternal && (Iter == 0)) {
            double Z = (Y[n[0]] + Y[n[1]] + Y[n[2]]) / 3. - extZo;
            double kludge = (R * R + Z * Z) * extRi / (extRo * extRo * extRo);
            mu1[i] /= kludge;
            mu2[i] /= kludge;
        }

        for (int j = 0; j < 3; j++)
            for (int k = 0; k < 3; k++) {
                Me[j][k] += (Mx[j][k] / mu2[i] + My[j][k] / mu1[i] + Mxy[j][k] * v12[i] + Mn[j][k]);
                be[j] += Mn[j][k] * Vv[n[k]];
            }
        for (int j = 0; j < 3; j++) {
            for (int k = j; k < 3; k++) ops->addto(L, -Me[j][k], n[j], n[k]);
            b[n[j]] -= be[j];
        }
    }

    /* point currents (staticaxi.cpp:644-650) */
    for (int i = 0; i < NN; i++)
        if (pr->marker[i] >= 0) b[i] += (0.01 * pr->points[pr->marker[i]].J_re * 2. * X[i]);
    /* A = 0 on the axis, fixed A at points (staticaxi.cpp:652-659) */
    for (int i = 0; i < NN; i++) {
        if (fabs(X[i]) < (units[pr->length_units] * 1.e-06)) {
            ops->setvalue(L, i, 0.);
        } else if (pr->marker[i] >= 0) {
            const ora_point *pp = &pr->points[pr->marker[i]];
            if ((pp->J_re == 0) && (pp->J_im == 0)) ops->setvalue(L, i, pp->A_re / c);
        }
    }
    /* fixed A along segments, skipped on the axis (staticaxi.cpp:661-728) */
    for (int i = 0; i < NE; i++)
        for (int j = 0; j < 3; j++) {
            int k = j + 1;
            if (k == 3) k = 0;
            int s = pr->e[3 * i + j];
            if (s >= 0 && pr->lines[s].BdryFormat == 0) {
                const ora_line *ln = &pr->lines[s];
                int nodes2[2] = {pr->p[3 * i + j], pr->p[3 * i + k]};
                for (int m = 0; m < 2; m++) {
                    double x = X[nodes2[m]], y = Y[nodes2[m]], av;
                    if (pr->coords == 0) {
                        x /= units[pr->length_units];
                        y /= units[pr->length_units];
                        av = ln->A0 + x * ln->A1 + y * ln->A2;
                    } else {
                        double rr = sqrt(x * x + y * y), tt;
                        if ((x == 0) && (y == 0)) tt = 0;
                        else tt = atan2(y, x) / ORA_DEG;
                        rr /= units[pr->length_units];
                        av = ln->A0 + rr * ln->A1 + tt * ln->A2;
                    }
                    av *= cos(ln->phi * ORA_DEG);
                    if (x != 0) ops->setvalue(L, nodes2[m], av / c);
                }
            }
        }
    for (int k = 0; k < pr->n_pbc; k++) {
        if (pr->pbc[3 * k + 2] == 0) ops->periodicity(L, pr->pbc[3 * k], pr->pbc[3 * k + 1]);
        if (pr->pbc[3 * k + 2] == 1) ops->antiperiodicity(L, pr->pbc[3 * k], pr->pbc[3 * k + 1]);
    }
    *LinearFlag_io = LinearFlag;
}

int ora_static2d(ora_problem *pr, const ora_linprob_ops *ops, double *A_out, ora_stats *stats)
{
    if (!ops) ops = &k_builtin;
    const double c = ORA_PI * 4.e-05;
    const int NN = pr->n_nodes, NE = pr->n_elems;
    double res = 0, lastres = 0, Relax = pr->relax;
    int Iter = 0, LinearFlag = 1;
    long long cg_total = 0;

    void *L = ops->create(NN, pr->bandwidth, pr->precision);
    double *V_old = (double *)calloc(NN, sizeof(double));
    double *mu1 = (double *)malloc(sizeof(double) * NE);
    double *mu2 = (double *)malloc(sizeof(double) * NE);
    double *v12 = (double *)calloc(NE, sizeof(double));
    for (int i = 0; i < NE; i++) { mu1[i] = -1.; mu2[i] = -1.; }

    ora_circuits(pr);

    do {
        if (Iter > 0) ops->wipe(L);
        if (pr->axisymmetric) ora_assemble_axi(pr, ops, L, Iter, mu1, mu2, v12, &LinearFlag);
        else ora_assemble(pr, ops, L, Iter, mu1, mu2, v12, &LinearFlag);
        double *Vv;
        Vv = ops->V(L);
        for (int j = 0; j < NN; j++) V_old[j] = Vv[j];
        long long it = 0;
        if (!ops->pcgsolve(L, Iter, &it)) {
            ops->destroy(L);
            free(V_old); free(mu1); free(mu2); free(v12);
            return 0;
        }
        if (it < 0 || cg_total < 0) cg_total = -1; else cg_total += it;
        Vv = ops->V(L);

        if (LinearFlag == 0) {
            double x = 0, y = 0;
            for (int j = 0; j < NN; j++) {
                x += (Vv[j] - V_old[j]) * (Vv[j] - V_old[j]);
                y += (Vv[j] * Vv[j]);
            }
            if (y == 0) LinearFlag = 1;
            else { lastres = res; res = sqrt(x / y); }
            if (Iter > 5) {
                if ((res > lastres) && (Relax > 0.125)) Relax /= 2.;
                else Relax += 0.1 * (1. - Relax);
                for (int j = 0; j < NN; j++) Vv[j] = Relax * Vv[j] + (1.0 - Relax) * V_old[j];
            }
        }
        if ((res < 100. * pr->precision) && (Iter > 0)) LinearFlag = 1;
        Iter++;
    } while (LinearFlag == 0);

    double *Vv = ops->V(L);
    for (int i = 0; i < NN; i++) A_out[i] = Vv[i] * c;
    if (pr->axisymmetric)   /* Webers: 2 pi r A (staticaxi.cpp:774-779) */
        for (int i = 0; i < NN; i++) A_out[i] *= (pr->x[i] * 0.01 * 2 * ORA_PI);
    if (stats) {
        stats->newton_iters = Iter;
        stats->cg_iters = cg_total;
        stats->last_res = res;
    }
    ops->destroy(L);
    free(V_old); free(mu1); free(mu2); free(v12);
    return 1;
}

int ora_static2d_system(ora_problem *pr, int *rows, int *cols, double *vals, long long cap,
                        double *b_out, long long *nnz_out)
{
    const int NN = pr->n_nodes, NE = pr->n_elems;
    int LinearFlag = 1;
    void *L = ora_lp_create(NN, pr->bandwidth, pr->precision);
    double *mu1 = (double *)malloc(sizeof(double) * NE);
    double *mu2 = (double *)malloc(sizeof(double) * NE);
    double *v12 = (double *)calloc(NE, sizeof(double));
    /* circuits are computed by ora_static2d; do the same prologue here */
    ora_circuits(pr);
    if (pr->axisymmetric) ora_assemble_axi(pr, &k_builtin, L, 0, mu1, mu2, v12, &LinearFlag);
    else ora_assemble(pr, &k_builtin, L, 0, mu1, mu2, v12, &LinearFlag);
    *nnz_out = ora_lp_export_upper(L, rows, cols, vals, cap);
    for (int i = 0; i < NN; i++) b_out[i] = ((ora_lp *)L)->b[i];
    ora_lp_destroy(L);
    free(mu1); free(mu2); free(v12);
    return 1;
}
