/* CPU oracle for the fsolver harmonic-2D path -- TEST INFRASTRUCTURE ONLY.
 * See harmonic2d_oracle.h for scope and the reference lines each part follows.
 *
 * Every complex operation restates femmcomplex.cpp's formula (products as
 * (ac - bd, ad + bc), quotients through the scaled reciprocal) and every loop
 * keeps the reference's order, so that the restated CBigComplexLinProb gives
 * results bit-identical with the reference's cspars.cpp.
 */
#include "harmonic2d_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ORA_PI 3.141592653589793238462643383
#define ORA_DEG 0.01745329251994329576923690768

/* ------------------------------------------------------------------------ */
/* CComplex restatement (femmcomplex.cpp)                                   */
/* ------------------------------------------------------------------------ */

typedef struct {
    double re, im;
} cx;

static cx C(double re, double im) { cx z = {re, im}; return z; }
static cx cadd(cx x, cx y) { return C(x.re + y.re, x.im + y.im); }
static cx csub(cx x, cx y) { return C(x.re - y.re, x.im - y.im); }
static cx cneg(cx y) { return C(-y.re, -y.im); }
static cx cmul(cx x, cx y) { return C(x.re * y.re - x.im * y.im, x.re * y.im + x.im * y.re); }   /* :355 */
static cx cmuld(cx x, double z) { return C(x.re * z, x.im * z); }                                /* :323 */
static cx dmulc(double x, cx y) { return C(x * y.re, x * y.im); }                                /* :350 */
static cx cdivd(cx x, double z) { return C(x.re / z, x.im / z); }                                /* :388 */
static cx cconj(cx x) { return C(x.re, -x.im); }
static cx crecip(cx z)
{   /* the scaled reciprocal of every CComplex quotient (:362-380) */
    double c;
    cx y;
    if (fabs(z.re) > fabs(z.im)) {
        c = z.im / z.re;
        y.re = 1. / (z.re * (1. + c * c));
        y.im = (-c) * y.re;
    } else {
        c = z.re / z.im;
        y.im = (-1.) / (z.im * (1. + c * c));
        y.re = (-c) * y.im;
    }
    return y;
}
static cx cdiv(cx x, cx z) { return cmul(x, crecip(z)); }                                        /* :456 */
static cx ddivc(double x, cx z) { cx y = crecip(z); y.re *= x; y.im *= x; return y; }            /* :433 */
static cx dplusc(double x, cx y) { return C(x + y.re, y.im); }                                 /* :244 */
static cx cplusd(cx x, double z) { return C(x.re + z, x.im); }                                 /* :218 */
static int cnz(cx z) { return (z.re != 0) || (z.im != 0); }
static cx cx_exp(cx x)
{   /* :622-634 */
    const double e = exp(x.re);
    return C(cos(x.im) * e, sin(x.im) * e);
}
static cx cx_tanh(cx x)
{   /* :675-687 */
    if (x.re > 0) {
        cx e = cx_exp(dmulc(-2.0, x));
        return cdiv(C(1 - e.re, -e.im), C(1 + e.re, e.im));
    }
    cx e = cx_exp(dmulc(2.0, x));
    return cdiv(C(e.re - 1, e.im), C(e.re + 1, e.im));
}

static const cx I = {0.0, 1.0};

/* ------------------------------------------------------------------------ */
/* CBigComplexLinProb restatement (cspars.cpp)                              */
/* ------------------------------------------------------------------------ */

typedef struct {
    int len, cap;
    int *c;
    cx *x;
} crow;

typedef struct {
    int n, bdw, nodes;
    double precision, lambda;
    crow *M;
    cx *b, *V, *P, *R, *U, *Z;
    /* Newton AC solver (cspars.cpp:58, 160-184): auxiliary matrices, allocated
       by the first Put with k > 0 */
    int bnewton;
    crow *Mh, *Ms, *Ma;
    cx *uu, *vv;
} clp;

static void crow_reserve(crow *r, int cap)
{
    if (cap <= r->cap) return;
    int nc = r->cap ? r->cap * 2 : 8;
    while (nc < cap) nc *= 2;
    r->c = (int *)realloc(r->c, sizeof(int) * nc);
    r->x = (cx *)realloc(r->x, sizeof(cx) * nc);
    r->cap = nc;
}

static void *clp_create(int n, int bw, int nodes, double precision)
{   /* cspars.cpp:40-45, 119-145 */
    clp *L = (clp *)calloc(1, sizeof(clp));
    L->n = n;
    L->bdw = bw;
    L->nodes = nodes;
    L->precision = precision;
    L->lambda = 1.5;
    L->M = (crow *)calloc(n, sizeof(crow));
    L->b = (cx *)calloc(n, sizeof(cx));
    L->V = (cx *)calloc(n, sizeof(cx));
    L->P = (cx *)calloc(n, sizeof(cx));
    L->R = (cx *)calloc(n, sizeof(cx));
    L->U = (cx *)calloc(n, sizeof(cx));
    L->Z = (cx *)calloc(n, sizeof(cx));
    for (int i = 0; i < n; i++) {
        crow_reserve(&L->M[i], 8);
        L->M[i].len = 1;
        L->M[i].c[0] = i;
        L->M[i].x[0] = C(0, 0);
    }
    return L;
}

static crow *crows_new(int n)
{
    crow *M = (crow *)calloc(n, sizeof(crow));
    for (int i = 0; i < n; i++) {
        crow_reserve(&M[i], 8);
        M[i].len = 1;
        M[i].c[0] = i;
        M[i].x[0] = C(0, 0);
    }
    return M;
}

static void crows_free(crow *M, int n)
{
    if (!M) return;
    for (int i = 0; i < n; i++) {
        free(M[i].c);
        free(M[i].x);
    }
    free(M);
}

static void crows_zero(crow *M, int n)
{
    for (int i = 0; i < n; i++)
        for (int k = 0; k < M[i].len; k++) M[i].x[k] = C(0, 0);
}

static void clp_wipe(void *lp)
{   /* cspars.cpp:539-590 */
    clp *L = (clp *)lp;
    for (int i = 0; i < L->n; i++) {
        L->b[i] = C(0, 0);
        for (int k = 0; k < L->M[i].len; k++) L->M[i].x[k] = C(0, 0);
    }
    if (!L->bnewton) return;
    crows_zero(L->Mh, L->n);
    crows_zero(L->Ma, L->n);
    crows_zero(L->Ms, L->n);
}

static void clp_destroy(void *lp)
{
    clp *L = (clp *)lp;
    if (!L) return;
    for (int i = 0; i < L->n; i++) {
        free(L->M[i].c);
        free(L->M[i].x);
    }
    free(L->M);
    crows_free(L->Mh, L->n);
    crows_free(L->Ms, L->n);
    crows_free(L->Ma, L->n);
    free(L->b); free(L->V); free(L->P); free(L->R); free(L->U); free(L->Z);
    free(L->uu); free(L->vv);
    free(L);
}

static crow *lp_mat(clp *L, int k)
{
    return k == 1 ? L->Mh : (k == 2 ? L->Ms : (k == 3 ? L->Ma : L->M));
}

static void lp_putk(clp *L, cx v, int p, int q, int k)
{   /* cspars.cpp:147-233 */
    if (q < p) {
        int t = p; p = q; q = t;
        if (k == 1) v = cconj(v);           /* hermitian matrix */
        if (k == 3) v = cneg(cconj(v));     /* antihermitian matrix */
    }
    if (k > 0 && !L->bnewton) {             /* allocate the auxiliary matrices on first use */
        L->bnewton = 1;
        L->Mh = crows_new(L->n);
        L->Ma = crows_new(L->n);
        L->Ms = crows_new(L->n);
        L->uu = (cx *)calloc(L->n, sizeof(cx));
        L->vv = (cx *)calloc(L->n, sizeof(cx));
    }
    crow *r = &lp_mat(L, k)[p];
    int t = 0;
    while (t < r->len && r->c[t] < q) t++;
    if (t < r->len && r->c[t] == q) { r->x[t] = v; return; }
    crow_reserve(r, r->len + 1);
    memmove(r->c + t + 1, r->c + t, sizeof(int) * (r->len - t));
    memmove(r->x + t + 1, r->x + t, sizeof(cx) * (r->len - t));
    r->c[t] = q;
    r->x[t] = v;
    r->len++;
}

static cx lp_getk(clp *L, int p, int q, int k)
{   /* cspars.cpp:235-283 */
    int flip = 0;
    if (q < p) { int t = p; p = q; q = t; flip = 1; }
    if (k > 0 && !L->bnewton) return C(0, 0);
    const crow *r = &lp_mat(L, k)[p];
    for (int t = 0; t < r->len; t++) {
        if (r->c[t] == q) {
            if (flip && k == 1) return cconj(r->x[t]);
            if (flip && k == 3) return cneg(cconj(r->x[t]));
            return r->x[t];
        }
        if (r->c[t] > q) break;
    }
    return C(0, 0);
}

static void lp_put(clp *L, cx v, int p, int q)
{   /* cspars.cpp:147-233 (k = 0) */
    if (q < p) { int t = p; p = q; q = t; }
    crow *r = &L->M[p];
    int k = 0;
    while (k < r->len && r->c[k] < q) k++;
    if (k < r->len && r->c[k] == q) { r->x[k] = v; return; }
    crow_reserve(r, r->len + 1);
    memmove(r->c + k + 1, r->c + k, sizeof(int) * (r->len - k));
    memmove(r->x + k + 1, r->x + k, sizeof(cx) * (r->len - k));
    r->c[k] = q;
    r->x[k] = v;
    r->len++;
}

static cx lp_get(clp *L, int p, int q)
{   /* cspars.cpp:235-283 (k = 0) */
    if (q < p) { int t = p; p = q; q = t; }
    const crow *r = &L->M[p];
    for (int k = 0; k < r->len; k++) {
        if (r->c[k] == q) return r->x[k];
        if (r->c[k] > q) break;
    }
    return C(0, 0);
}

static void clp_addto(void *lp, double vr, double vi, int p, int q)
{   /* cspars.cpp:285-288 */
    clp *L = (clp *)lp;
    lp_put(L, cadd(lp_get(L, p, q), C(vr, vi)), p, q);
}

static void clp_get(void *lp, int p, int q, double *vr, double *vi)
{
    cx z = lp_get((clp *)lp, p, q);
    *vr = z.re;
    *vi = z.im;
}

static void clp_put(void *lp, double vr, double vi, int p, int q) { lp_put((clp *)lp, C(vr, vi), p, q); }
static double *clp_b(void *lp) { return (double *)((clp *)lp)->b; }
static double *clp_V(void *lp) { return (double *)((clp *)lp)->V; }

static void clp_setvalue(void *lp, int i, double xr, double xi)
{   /* cspars.cpp:482-537 (bNewton false) */
    clp *L = (clp *)lp;
    cx x = C(xr, xi);
    int fst, lst;
    if (L->bdw == 0) {
        fst = 0;
        lst = L->n;
    } else {
        fst = i - L->bdw;
        if (fst < 0) fst = 0;
        lst = i + L->bdw;
        if (lst > L->nodes) lst = L->nodes;
    }
    for (int k = fst; k < L->n; k++) {
        if (k == lst) k = L->nodes;
        if (k >= L->n) break;
        cx z = lp_get(L, k, i);
        if (cnz(z)) {
            L->b[k] = csub(L->b[k], cmul(z, x));
            if (i != k) lp_put(L, C(0, 0), k, i);
        }
        if (L->bnewton) {   /* cspars.cpp:511-534 (Ma, like Ms, acts on conj(x) here) */
            z = lp_getk(L, k, i, 1);
            if (cnz(z)) {
                if (i != k) L->b[k] = csub(L->b[k], cmul(z, x));
                lp_putk(L, C(0, 0), k, i, 1);
            }
            z = lp_getk(L, k, i, 2);
            if (cnz(z)) {
                if (i != k) L->b[k] = csub(L->b[k], cmul(z, cconj(x)));
                lp_putk(L, C(0, 0), k, i, 2);
            }
            z = lp_getk(L, k, i, 3);
            if (cnz(z)) {
                if (i != k) L->b[k] = csub(L->b[k], cmul(z, cconj(x)));
                lp_putk(L, C(0, 0), k, i, 3);
            }
        }
    }
    L->b[i] = cmul(lp_get(L, i, i), x);
}

static void clp_pair(clp *L, int i, int j, int anti)
{   /* cspars.cpp:592-675 (AntiPeriodicity), 677-758 (Periodicity), bNewton false */
    int fst, lst;
    if (j < i) { int t = j; j = i; i = t; }
    if (L->bdw == 0) {
        fst = 0;
        lst = L->n;
    } else {
        fst = i - L->bdw;
        if (fst < 0) fst = 0;
        lst = j + L->bdw;
        if (lst > L->nodes - 1) lst = L->nodes - 1;
    }
    for (int k = fst; k < L->n; k++) {
        if ((k != i) && (k != j)) {
            cx v1 = lp_get(L, k, i), v2 = lp_get(L, k, j);
            if (cnz(v1) || cnz(v2)) {
                if (anti) {
                    cx c = cdivd(csub(v1, v2), 2.);
                    lp_put(L, c, k, i);
                    lp_put(L, cneg(c), k, j);
                } else {
                    cx c = cdivd(cadd(v1, v2), 2.);
                    lp_put(L, c, k, i);
                    lp_put(L, c, k, j);
                }
            }
        }
        if ((k == i + L->bdw) && (k < j - L->bdw) && (L->bdw != 0)) k = j - L->bdw;
        else if (k == lst) k = L->nodes;
    }
    cx c = anti ? dmulc(0.5, cadd(lp_get(L, i, i), lp_get(L, j, j)))
                : cdivd(cadd(lp_get(L, i, i), lp_get(L, j, j)), 2.);
    lp_put(L, c, i, i);
    lp_put(L, c, j, j);
    if (anti) {
        c = dmulc(0.5, csub(L->b[i], L->b[j]));
        L->b[i] = c;
        L->b[j] = cneg(c);
    } else {
        c = dmulc(0.5, cadd(L->b[i], L->b[j]));
        L->b[i] = c;
        L->b[j] = c;
    }
    if (!L->bnewton) return;
    for (int h = 1; h <= 3; h++) {   /* cspars.cpp:648-671 / 732-755 */
        for (int k = fst; k < L->n; k++) {
            if ((k != i) && (k != j)) {
                cx v1 = lp_getk(L, k, i, h), v2 = lp_getk(L, k, j, h);
                if (cnz(v1) || cnz(v2)) {
                    if (anti) {
                        cx cc = cdivd(csub(v1, v2), 2.);
                        lp_putk(L, cc, k, i, h);
                        lp_putk(L, cneg(cc), k, j, h);
                    } else {
                        cx cc = cdivd(cadd(v1, v2), 2.);
                        lp_putk(L, cc, k, i, h);
                        lp_putk(L, cc, k, j, h);
                    }
                }
            }
            if ((k == i + L->bdw) && (k < j - L->bdw) && (L->bdw != 0)) k = j - L->bdw;
            else if (k == lst) k = L->nodes;
        }
        if (anti) {
            cx cc = cdivd(cadd(csub(csub(lp_getk(L, i, i, h), lp_getk(L, i, j, h)), lp_getk(L, j, i, h)),
                               lp_getk(L, j, j, h)), 4.);
            lp_putk(L, cc, i, i, h);
            lp_putk(L, cneg(cc), i, j, h);
            lp_putk(L, cc, j, j, h);
        } else {
            cx cc = cdivd(cadd(cadd(cadd(lp_getk(L, i, i, h), lp_getk(L, i, j, h)), lp_getk(L, j, i, h)),
                               lp_getk(L, j, j, h)), 4.);
            lp_putk(L, cc, i, i, h);
            lp_putk(L, cc, i, j, h);
            lp_putk(L, cc, j, j, h);
        }
    }
}

static void clp_periodicity(void *lp, int i, int j) { clp_pair((clp *)lp, i, j, 0); }
static void clp_antiperiodicity(void *lp, int i, int j) { clp_pair((clp *)lp, i, j, 1); }

static void lp_multA(clp *L, const cx *X, cx *Y)
{   /* cspars.cpp:290-360 (k = 0: complex symmetric) */
    for (int i = 0; i < L->n; i++) Y[i] = C(0, 0);
    for (int i = 0; i < L->n; i++) {
        const crow *r = &L->M[i];
        Y[i] = cadd(Y[i], cmul(r->x[0], X[i]));
        for (int k = 1; k < r->len; k++) {
            int c = r->c[k];
            Y[i] = cadd(Y[i], cmul(r->x[k], X[c]));
            Y[c] = cadd(Y[c], cmul(r->x[k], X[i]));
        }
    }
}

static cx lp_dot(const cx *x, const cx *y, int n)
{   /* cspars.cpp:417-426 */
    cx z = C(0, 0);
    for (int i = 0; i < n; i++) z = cadd(z, cmul(x[i], y[i]));
    return z;
}

static cx lp_conjdot(const cx *x, const cx *y, int n)
{   /* cspars.cpp:428-437 */
    cx z = C(0, 0);
    for (int i = 0; i < n; i++) z = cadd(z, cmul(cconj(x[i]), y[i]));
    return z;
}

static double lp_nrm(const cx *x, int n) { return sqrt(lp_conjdot(x, x, n).re); }   /* cspars.cpp:30 */

static void lp_multpc(clp *L, const cx *X, cx *Y)
{   /* cspars.cpp:439-480: SSOR */
    int n = L->n;
    double lam = L->lambda;
    cx c = C(lam * (2. - lam), 0);
    for (int i = 0; i < n; i++) Y[i] = cmul(X[i], c);
    for (int i = 0; i < n; i++) {
        const crow *r = &L->M[i];
        Y[i] = cdiv(Y[i], r->x[0]);
        for (int k = 1; k < r->len; k++)
            Y[r->c[k]] = csub(Y[r->c[k]], cmuld(cmul(r->x[k], Y[i]), lam));
    }
    for (int i = 0; i < n; i++) Y[i] = cmul(Y[i], L->M[i].x[0]);
    for (int i = n - 1; i >= 0; i--) {
        const crow *r = &L->M[i];
        for (int k = 1; k < r->len; k++) Y[i] = csub(Y[i], cmuld(cmul(r->x[k], Y[r->c[k]]), lam));
        Y[i] = cdiv(Y[i], r->x[0]);
    }
}

static void lp_multappa(clp *L, const cx *X, cx *Y)
{   /* cspars.cpp:406-415 */
    lp_multA(L, X, L->Z);
    lp_multpc(L, L->Z, Y);
    for (int i = 0; i < L->n; i++) Y[i].im = -Y[i].im;
    lp_multpc(L, Y, L->Z);
    lp_multA(L, L->Z, Y);
    for (int i = 0; i < L->n; i++) Y[i].im = -Y[i].im;
}

static int lp_pcgsqstart(clp *L)
{   /* cspars.cpp:764-820 */
    int n = L->n;
    for (int i = 0; i < n; i++)
        if ((L->M[i].x[0].re == 0) && (L->M[i].x[0].im == 0)) {
            fprintf(stderr, "singular flag tripped.");
            return 0;
        }
    lp_multpc(L, L->b, L->Z);
    for (int i = 0; i < n; i++) L->Z[i].im = -L->Z[i].im;
    lp_multpc(L, L->Z, L->P);
    lp_multA(L, L->P, L->Z);
    for (int i = 0; i < n; i++) L->P[i] = cconj(L->Z[i]);
    for (int i = 0; i < n; i++) L->V[i] = C(0, 0);
    lp_multappa(L, L->V, L->R);
    for (int i = 0; i < n; i++) L->R[i] = csub(L->P[i], L->R[i]);
    for (int i = 0; i < n; i++) L->P[i] = L->R[i];
    cx res = lp_conjdot(L->R, L->R, n);
    for (int k = 0; k < 3; k++) {
        lp_multappa(L, L->P, L->U);
        cx pAp = lp_conjdot(L->P, L->U, n);
        cx del = cdiv(res, pAp);
        for (int i = 0; i < n; i++) L->V[i] = cadd(L->V[i], cmul(del, L->P[i]));
        for (int i = 0; i < n; i++) L->R[i] = csub(L->R[i], cmul(del, L->U[i]));
        cx res_new = lp_conjdot(L->R, L->R, n);
        cx rho = cdiv(res_new, res);
        res = res_new;
        for (int i = 0; i < n; i++) L->P[i] = cadd(L->R[i], cmul(rho, L->P[i]));
    }
    return 1;
}

static long long g_iters;

static int lp_pbcgsolve(clp *L, int flag)
{   /* cspars.cpp:822-895 */
    int n = L->n;
    if (flag == 0)
        for (int i = 0; i < n; i++) L->V[i] = C(0, 0);
    lp_multA(L, L->V, L->R);
    for (int i = 0; i < n; i++) L->R[i] = csub(L->b[i], L->R[i]);
    double normb = lp_nrm(L->b, n);
    double er;
    lp_multpc(L, L->R, L->Z);
    for (int i = 0; i < n; i++) L->P[i] = L->Z[i];
    cx res = lp_dot(L->Z, L->R, n);
    g_iters = 0;
    do {
        lp_multA(L, L->P, L->U);
        cx pAp = lp_dot(L->P, L->U, n);
        cx del = cdiv(res, pAp);
        for (int i = 0; i < n; i++) L->V[i] = cadd(L->V[i], cmul(del, L->P[i]));
        for (int i = 0; i < n; i++) L->R[i] = csub(L->R[i], cmul(del, L->U[i]));
        lp_multpc(L, L->R, L->Z);
        cx res_new = lp_dot(L->Z, L->R, n);
        cx rho = cdiv(res_new, res);
        res = res_new;
        for (int i = 0; i < n; i++) L->P[i] = cadd(L->Z[i], cmul(rho, L->P[i]));
        er = lp_nrm(L->R, n) / normb;
        g_iters++;
    } while (er > L->precision);
    return 1;
}

/* Y = M_k X for k = 1 (hermitian), 2 (complex symmetric), 3 (antihermitian)
   stored as their upper triangles (cspars.cpp:290-360) */
static void lp_multA_k(clp *L, const cx *X, cx *Y, int k)
{
    const crow *M = lp_mat(L, k);
    for (int i = 0; i < L->n; i++) Y[i] = C(0, 0);
    for (int i = 0; i < L->n; i++) {
        const crow *r = &M[i];
        Y[i] = cadd(Y[i], cmul(r->x[0], X[i]));
        for (int t = 1; t < r->len; t++) {
            const int c = r->c[t];
            Y[i] = cadd(Y[i], cmul(r->x[t], X[c]));
            if (k == 1) Y[c] = cadd(Y[c], cmul(cconj(r->x[t]), X[i]));
            else if (k == 3) Y[c] = cadd(Y[c], cmul(cneg(cconj(r->x[t])), X[i]));
            else Y[c] = cadd(Y[c], cmul(r->x[t], X[i]));
        }
    }
}

/* Y = conj(M_2) X (cspars.cpp:362-404, k = 2: the complex-symmetric branch) */
static void lp_multconjA_2(clp *L, const cx *X, cx *Y)
{
    const crow *M = L->Ms;
    for (int i = 0; i < L->n; i++) Y[i] = C(0, 0);
    for (int i = 0; i < L->n; i++) {
        const crow *r = &M[i];
        Y[i] = cadd(Y[i], cmul(cconj(r->x[0]), X[i]));
        for (int t = 1; t < r->len; t++) {
            const int c = r->c[t];
            Y[i] = cadd(Y[i], cmul(cconj(r->x[t]), X[c]));
            Y[c] = cadd(Y[c], cmul(cconj(r->x[t]), X[i]));
        }
    }
}

/* the full Newton operator, MultA(X, Y, -1) (cspars.cpp:303-312):
   Y = M X + Mh X + Ms conj(X) + Ma X */
static void lp_multA_full(clp *L, const cx *X, cx *Y)
{
    lp_multA(L, X, Y);
    lp_multA_k(L, X, L->uu, 1);
    for (int i = 0; i < L->n; i++) Y[i] = cadd(Y[i], L->uu[i]);
    lp_multconjA_2(L, X, L->uu);
    lp_multA_k(L, X, L->vv, 3);
    for (int i = 0; i < L->n; i++) Y[i] = cadd(cadd(Y[i], cconj(L->uu[i])), L->vv[i]);
}

/* CBigComplexLinProb::KludgeSolve (cspars.cpp:983-1059): outer iterations on
   the non-complex-linear Newton system, each a complex-symmetric PBCGSolve of
   the main matrix against the RHS moved by the auxiliary matrices at the
   current V, then a least-squares step length along the update */
static int lp_kludgesolve(clp *L, int flag)
{
    const int n = L->n;
    cx *borig = (cx *)calloc(n, sizeof(cx)), *v = (cx *)calloc(n, sizeof(cx)), *r = (cx *)calloc(n, sizeof(cx));
    if (flag == 0)
        for (int i = 0; i < n; i++) L->V[i] = C(0, 0);
    const double normb = lp_nrm(L->b, n);
    for (int i = 0; i < n; i++) {
        borig[i] = L->b[i];
        v[i] = L->V[i];
    }
    lp_multA_full(L, L->V, r);
    for (int i = 0; i < n; i++) r[i] = csub(L->b[i], r[i]);
    double er = lp_nrm(r, n) / normb;
    long long its = 0;
    if (!(er < L->precision)) {
        for (int k = 0; k < 10; k++) {
            lp_multA_k(L, L->V, L->P, 1);
            lp_multconjA_2(L, L->V, L->U);
            lp_multA_k(L, L->V, L->R, 3);
            for (int i = 0; i < n; i++)
                L->b[i] = csub(csub(csub(borig[i], L->P[i]), cconj(L->U[i])), L->R[i]);
            lp_pbcgsolve(L, 1);
            its += g_iters;
            for (int i = 0; i < n; i++) L->P[i] = csub(L->V[i], v[i]);
            lp_multA_full(L, L->P, L->U);
            const double cstep = lp_conjdot(r, L->U, n).re / lp_conjdot(L->U, L->U, n).re;
            for (int i = 0; i < n; i++) {
                L->V[i] = cadd(v[i], dmulc(cstep, L->P[i]));
                r[i] = csub(r[i], dmulc(cstep, L->U[i]));
                v[i] = L->V[i];
            }
            er = lp_nrm(r, n) / normb;
            if (getenv("ORACLE_TRACE_NONLINEAR"))
                fprintf(stderr, "  kludge %d: c %.6e er %.6e (cocg %lld)\n", k, cstep, er, (long long)g_iters);
            if (er < L->precision * 10.) break;
        }
    }
    g_iters = its;
    free(borig);
    free(v);
    free(r);
    return 1;
}

static int clp_solve(void *lp, int flag)
{   /* cspars.cpp:1062-1081 */
    clp *L = (clp *)lp;
    if (L->bnewton) return lp_kludgesolve(L, flag);
    if (flag == 0)
        if (lp_pcgsqstart(L) == 0) return 0;
    return lp_pbcgsolve(L, 2);
}

static void clp_put_k(void *lp, double vr, double vi, int p, int q, int k) { lp_putk((clp *)lp, C(vr, vi), p, q, k); }
static void clp_get_k(void *lp, int p, int q, int k, double *vr, double *vi)
{
    cx z = lp_getk((clp *)lp, p, q, k);
    *vr = z.re;
    *vi = z.im;
}
static int clp_newton(void *lp) { return ((clp *)lp)->bnewton; }
static void clp_set_precision(void *lp, double p) { ((clp *)lp)->precision = p; }

static const orh_linprob_ops g_builtin = {clp_create, clp_destroy, clp_addto, clp_get, clp_put,
                                          clp_b, clp_V, clp_setvalue, clp_periodicity,
                                          clp_antiperiodicity, clp_solve, clp_wipe,
                                          clp_put_k, clp_get_k, clp_newton, clp_set_precision};

const orh_linprob_ops *orh_builtin_linprob(void) { return &g_builtin; }

/* ------------------------------------------------------------------------ */
/* FSolver::Harmonic2D (harmonic2d.cpp), linear problems                    */
/* ------------------------------------------------------------------------ */

typedef struct {
    cx mu0, mu1;
} effmu;

#define ORH_MUO 1.2566370614359173e-6

/* abs(CComplex) (femmcomplex.cpp:749-757) */
static double cx_abs(cx x)
{
    if ((x.re == 0) && (x.im == 0)) return 0.;
    if (fabs(x.re) > fabs(x.im)) return fabs(x.re) * sqrt(1. + (x.im / x.re) * (x.im / x.re));
    return fabs(x.im) * sqrt(1. + (x.re / x.im) * (x.re / x.im));
}

/* ---- the complex curve of a nonlinear block ---- */
static cx bh_H(const orh_block *b, int i) { return C(b->H_re[i], b->H_im[i]); }
static cx bh_S(const orh_block *b, int i) { return C(b->S_re[i], b->S_im[i]); }

/* CMMaterialProp::GetH(CComplex) (CMaterialProp.cpp:493-518) for x = B >= 0 */
static cx bh_geth(const orh_block *m, double B)
{
    const int n = m->BHpoints;
    const double b = B;                 /* abs(CComplex(B)) */
    if (b == 0) return C(0, 0);
    const cx pp = cdivd(C(B, 0), b);    /* p = x / b */
    if (b > m->B[n - 1]) return cmul(pp, cadd(bh_H(m, n - 1), cmuld(bh_S(m, n - 1), b - m->B[n - 1])));
    for (int i = 0; i < n - 1; i++)
        if ((b >= m->B[i]) && (b <= m->B[i + 1])) {
            double l = m->B[i + 1] - m->B[i], z = (b - m->B[i]) / l, z2 = z * z;
            cx h = dmulc(1. - 3. * z2 + 2. * z2 * z, bh_H(m, i));
            h = cadd(h, dmulc(z * (1. - 2. * z + z2) * l, bh_S(m, i)));
            h = cadd(h, dmulc(z2 * (3. - 2. * z), bh_H(m, i + 1)));
            h = cadd(h, dmulc(z2 * (z - 1.) * l, bh_S(m, i + 1)));
            return cmul(pp, h);
        }
    return C(0, 0);
}

/* Get_v(B) (CMaterialProp.cpp:899-903): the base-class GetH(double) is the
 * real part of GetH(CComplex) (:488-491) */
static cx bh_getv(const orh_block *m, double B)
{
    if (B == 0) return bh_S(m, 0);
    return C(bh_geth(m, B).re / B, 0);
}

/* GetdHdB(B) (CMaterialProp.cpp:461-486) */
static cx bh_dhdb(const orh_block *m, double B)
{
    const int n = m->BHpoints;
    const double b = fabs(B);
    if (b > m->B[n - 1]) return bh_S(m, n - 1);
    for (int i = 0; i < n - 1; i++)
        if ((b >= m->B[i]) && (b <= m->B[i + 1])) {
            double l = m->B[i + 1] - m->B[i], z = (b - m->B[i]) / l;
            cx h = cdivd(dmulc(6. * z * (z - 1.), bh_H(m, i)), l);
            h = cadd(h, dmulc(1. - 4. * z + 3. * z * z, bh_S(m, i)));
            h = cadd(h, cdivd(dmulc(6. * z * (1. - z), bh_H(m, i + 1)), l));
            h = cadd(h, dmulc(z * (3. * z - 2.), bh_S(m, i + 1)));
            return h;
        }
    return C(0, 0);
}

/* CMSolverMaterialProp::GetBHProps(double, CComplex&, CComplex&) (CMaterialProp.cpp:1008-1057) */
static void bh_getbhprops(const orh_block *m, double B, cx *v, cx *dv)
{
    const double b = fabs(B);
    const int n = m->BHpoints;
    if (b == 0) {
        *v = bh_S(m, 0);
        *dv = C(0, 0);
        return;
    }
    if (b > m->B[n - 1]) {
        const cx h = cadd(bh_H(m, n - 1), cmuld(bh_S(m, n - 1), b - m->B[n - 1]));
        const cx dh = bh_S(m, n - 1);
        *v = cdivd(h, b);
        *dv = dmulc(0.5, csub(cdivd(dh, b * b), cdivd(h, b * b * b)));
        return;
    }
    for (int i = 0; i < n - 1; i++)
        if ((b >= m->B[i]) && (b <= m->B[i + 1])) {
            const double l = m->B[i + 1] - m->B[i], z = (b - m->B[i]) / l, z2 = z * z;
            cx h = dmulc(1. - 3. * z2 + 2. * z2 * z, bh_H(m, i));
            h = cadd(h, dmulc(z * (1. - 2. * z + z2) * l, bh_S(m, i)));
            h = cadd(h, dmulc(z2 * (3. - 2. * z), bh_H(m, i + 1)));
            h = cadd(h, dmulc(z2 * (z - 1.) * l, bh_S(m, i + 1)));
            cx dh = cdivd(dmulc(6. * z * (z - 1.), bh_H(m, i)), l);
            dh = cadd(dh, dmulc(1. - 4. * z + 3. * z * z, bh_S(m, i)));
            dh = cadd(dh, cdivd(dmulc(6. * z * (1. - z), bh_H(m, i + 1)), l));
            dh = cadd(dh, dmulc(z * (3. * z - 2.), bh_S(m, i + 1)));
            *v = cdivd(h, b);
            *dv = dmulc(0.5, csub(cdivd(dh, b * b), cdivd(h, b * b * b)));
            return;
        }
}

/* Newton terms of one nonlinear element (harmonic2d.cpp:610-639,
   harmonicaxi.cpp:519-545): mu from GetBHProps, v = (Mx + My) V, K =
   -200 c^3 dv / a (a: area, or the r-weighted volume of the axisymmetric
   element), Mn = K Re(v v^H), Mnh / Mna the Hermitian / anti-Hermitian
   remainders of 0.5 Re(K) v v^H / 0.5 I Im(K) v v^H, Mns = 0.5 K v v^T */
static void newton_terms(const orh_block *blk, double B, double c, double a, const cx (*Mx)[3], const cx (*My)[3],
                         const cx *Vn, cx *mu_out, cx (*Mn)[3], cx (*Mnh)[3], cx (*Mna)[3], cx (*Mns)[3])
{
    cx mu, dv, v[3];
    bh_getbhprops(blk, B, &mu, &dv);
    mu = ddivc(1., cmuld(mu, ORH_MUO));   /* 1./(muo*mu): double * CComplex */
    *mu_out = mu;
    for (int j = 0; j < 3; j++) {
        v[j] = C(0, 0);
        for (int w = 0; w < 3; w++) v[j] = cadd(v[j], cmul(cadd(Mx[j][w], My[j][w]), Vn[w]));
    }
    const cx K = cdivd(dmulc(-200. * c * c * c, dv), a);
    const cx half_im = cmuld(cmuld(I, 0.5), K.im);   /* I*0.5*Im(K) */
    for (int j = 0; j < 3; j++)
        for (int w = 0; w < 3; w++) {
            const cx vv = cmul(v[j], cconj(v[w]));
            Mn[j][w] = cmuld(K, vv.re);
            Mnh[j][w] = C(cmul(dmulc(0.5 * K.re, v[j]), cconj(v[w])).re - Mn[j][w].re,
                          cmul(dmulc(0.5 * K.re, v[j]), cconj(v[w])).im);
            Mna[j][w] = csub(cmul(cmul(half_im, v[j]), cconj(v[w])), cmuld(I, Mn[j][w].im));
            Mns[j][w] = cmul(cmul(dmulc(0.5, K), v[j]), v[w]);
        }
}

void orh_acprops(const orh_block *b, const double *Bq, int nq, double *v, double *dhdb)
{
    for (int i = 0; i < nq; i++) {
        cx a = bh_getv(b, Bq[i]), d = bh_dhdb(b, Bq[i]);
        v[2 * i] = a.re;
        v[2 * i + 1] = a.im;
        dhdb[2 * i] = d.re;
        dhdb[2 * i + 1] = d.im;
    }
}

/* effective permeability of each block (harmonic2d.cpp:190-235) */
/* -I Theta DEG (harmonic2d.cpp) or -I Theta PI / 180 (harmonicaxi.cpp:133-151), halved for the half-lag */
static cx lagarg(double th, int axi, int half)
{
    if (axi) return cdivd(cmuld(cmuld(cneg(I), th), ORA_PI), half ? 360. : 180.);
    return half ? cdivd(cmuld(cmuld(cneg(I), th), ORA_DEG), 2.) : cmuld(cmuld(cneg(I), th), ORA_DEG);
}

static void effective_mu(const orh_problem *pr, double w, effmu *Mu)
{
    const cx deg45 = C(1, 1);
    const int axi = pr->problem_type == 1;
    for (int k = 0; k < pr->n_blocks; k++) {
        const orh_block *b = &pr->blocks[k];
        if (b->LamType == 0) {
            Mu[k].mu0 = dmulc(b->mu_x, cx_exp(lagarg(b->Theta_hx, axi, 0)));
            Mu[k].mu1 = dmulc(b->mu_y, cx_exp(lagarg(b->Theta_hy, axi, 0)));
            if (b->Lam_d != 0) {
                if (b->Cduct != 0) {
                    cx halflag = cx_exp(lagarg(b->Theta_hx, axi, 1));
                    double ds = sqrt(2. / (0.4 * ORA_PI * w * b->Cduct * b->mu_x));
                    cx K = cdivd(cmuld(cmuld(cmul(halflag, deg45), b->Lam_d), 0.001), 2. * ds);
                    Mu[k].mu0 = cplusd(cmuld(cdiv(cmul(Mu[k].mu0, cx_tanh(K)), K), b->LamFill), 1. - b->LamFill);
                    halflag = cx_exp(lagarg(b->Theta_hy, axi, 1));
                    ds = sqrt(2. / (0.4 * ORA_PI * w * b->Cduct * b->mu_y));
                    K = cdivd(cmuld(cmuld(cmul(halflag, deg45), b->Lam_d), 0.001), 2. * ds);
                    Mu[k].mu1 = cplusd(cmuld(cdiv(cmul(Mu[k].mu1, cx_tanh(K)), K), b->LamFill), 1. - b->LamFill);
                } else {
                    Mu[k].mu0 = cplusd(cmuld(Mu[k].mu0, b->LamFill), 1. - b->LamFill);
                    Mu[k].mu1 = cplusd(cmuld(Mu[k].mu1, b->LamFill), 1. - b->LamFill);
                }
            }
        } else {
            Mu[k].mu0 = C(1, 0);
            Mu[k].mu1 = C(1, 0);
        }
    }
}

/* circuit cases (harmonic2d.cpp:86-170) */
static void circuits(orh_problem *pr)
{
    int nc = pr->n_circs;
    if (nc <= 0) return;
    cx *I1 = (cx *)calloc(nc, sizeof(cx)), *I2 = (cx *)calloc(nc, sizeof(cx)), *I3 = (cx *)calloc(nc, sizeof(cx));
    for (int i = 0; i < pr->n_elems; i++) {
        if (pr->lbl[i] < 0) continue;
        const orh_label *lb = &pr->labels[pr->lbl[i]];
        if (lb->InCircuit == -1) continue;
        const int *n = pr->p + 3 * i;
        double p0 = pr->y[n[1]] - pr->y[n[2]], p1 = pr->y[n[2]] - pr->y[n[0]];
        double q0 = pr->x[n[2]] - pr->x[n[1]], q1 = pr->x[n[0]] - pr->x[n[2]];
        double a = (p0 * q1 - p1 * q0) / 2.;
        const orh_block *b = &pr->blocks[pr->blk[i]];
        double Cduct = b->Cduct;
        if (lb->bIsWound) Cduct = 0;
        int k = lb->InCircuit;
        I1[k] = cplusd(I1[k], a);
        if (pr->problem_type == 1) {   /* conductivity / R (harmonicaxi.cpp:86-87) */
            double r = (pr->x[n[0]] + pr->x[n[1]] + pr->x[n[2]]) / 3.;
            I2[k] = cplusd(I2[k], a * Cduct / (0.01 * r));
        } else {
            I2[k] = cplusd(I2[k], a * Cduct);
        }
        I3[k] = cadd(I3[k], cmuld(cmuld(dplusc(b->J_re, cmuld(I, b->J_im)), a), 100.));
    }
    for (int k = 0; k < nc; k++) {
        orh_circ *c = &pr->circs[k];
        c->J_re = c->J_im = c->dV_re = c->dV_im = 0;
        if (c->CircType == 0) {
            if (!cnz(I2[k])) {
                c->Case = 1;
                if (!cnz(I1[k])) {
                    c->J_re = c->J_im = 0;
                } else {
                    cx amps = dplusc(c->Amps_re, cmuld(I, c->Amps_im));
                    cx J = cdiv(dmulc(0.01, csub(amps, I3[k])), I1[k]);
                    c->J_re = J.re;
                    c->J_im = J.im;
                }
            } else {
                c->Case = 2;
            }
        } else {
            c->Case = 0;
            cx dV = dplusc(c->dVolts_re, cmuld(I, c->dVolts_im));
            c->dV_re = dV.re;
            c->dV_im = dV.im;
        }
    }
    free(I1); free(I2); free(I3);
}

/* one element of HarmonicAxisymmetric (harmonicaxi.cpp:215-605) */
/* Element matrices into the system (harmonic2d.cpp:671-705, harmonicaxi.cpp:588-623).
   ACSolver 0: Me += Mx/mu2 + My/mu1 (+ Mxy v12 planar), be += Mn V.
   ACSolver 1 (every element, Newton terms zero unless it is nonlinear): Me +=
   Mx/mu2 + My/mu1 + Mn, be += (Mnh + Mna + Mn) V + Mns conj(V), and the nonzero
   upper-triangle Newton terms accumulate into the auxiliary matrices 1, 2, 3
   (Put(Get(k) + m, k)). */
static void element_to_system(const orh_problem *pr, const orh_linprob_ops *ops, void *L, const int *n, cx (*Me)[3],
                              cx *be, cx (*Mx)[3], cx (*My)[3], cx (*Mxy)[3], cx v12, cx (*Mn)[3], cx (*Mnh)[3],
                              cx (*Mna)[3], cx (*Mns)[3], cx mu1, cx mu2, const cx *VL, cx *bL, int planar)
{
    static const cx Z3[3][3];
    const int ac1 = pr->ac_solver == 1;
    if (ac1 && !Mnh) {   /* linear element of a Newton problem: the zeroed Mnh / Mna / Mns (:399-404) */
        Mnh = (cx(*)[3])Z3;
        Mna = (cx(*)[3])Z3;
        Mns = (cx(*)[3])Z3;
    }
    for (int j = 0; j < 3; j++)
        for (int k = 0; k < 3; k++) {
            if (ac1) {
                Me[j][k] = cadd(Me[j][k], cadd(cadd(cdiv(Mx[j][k], mu2), cdiv(My[j][k], mu1)), Mn[j][k]));
                be[j] = cadd(be[j], cmul(cadd(cadd(Mnh[j][k], Mna[j][k]), Mn[j][k]), VL[n[k]]));
                be[j] = cadd(be[j], cmul(Mns[j][k], cconj(VL[n[k]])));
            } else if (planar) {
                Me[j][k] = cadd(Me[j][k], cadd(cadd(cdiv(Mx[j][k], mu2), cdiv(My[j][k], mu1)), cmul(Mxy[j][k], v12)));
                be[j] = cadd(be[j], cmul(Mn[j][k], VL[n[k]]));
            } else {
                Me[j][k] = cadd(Me[j][k], cadd(cdiv(Mx[j][k], mu2), cdiv(My[j][k], mu1)));
                be[j] = cadd(be[j], cmul(Mn[j][k], VL[n[k]]));
            }
        }
    for (int j = 0; j < 3; j++) {
        for (int k = j; k < 3; k++) {
            ops->addto(L, Me[j][k].re, Me[j][k].im, n[j], n[k]);
            if (ac1) {
                const cx *aux[3] = {&Mnh[j][k], &Mns[j][k], &Mna[j][k]};
                for (int m = 0; m < 3; m++) {
                    if (aux[m]->re == 0 && aux[m]->im == 0) continue;
                    double gr, gi;
                    ops->get_k(L, n[j], n[k], m + 1, &gr, &gi);
                    const cx s = cadd(C(gr, gi), *aux[m]);
                    ops->put_k(L, s.re, s.im, n[j], n[k], m + 1);
                }
            }
        }
        bL[n[j]] = cadd(bL[n[j]], be[j]);
    }
}

static void axi_element(orh_problem *pr, const orh_linprob_ops *ops, void *L, const effmu *Mu, double w, int Iter,
                        int i, cx *VL, cx *bL)
{
    const double c = ORA_PI * 4.e-05;
    const double units[] = {2.54, 0.1, 1., 100., 0.00254, 1.e-04};
    const cx deg45 = C(1, 1);
    const int NN = pr->n_nodes;
    cx Me[3][3], be[3], Mx[3][3], My[3][3], Mn[3][3], K;
    double p[3], q[3], g[3], rn[3], l[3];
    int n[3];
    for (int j = 0; j < 3; j++) {
        for (int k = 0; k < 3; k++) Me[j][k] = Mx[j][k] = My[j][k] = Mn[j][k] = C(0, 0);
        be[j] = C(0, 0);
    }
    for (int k = 0; k < 3; k++) {
        n[k] = pr->p[3 * i + k];
        rn[k] = pr->x[n[k]];
    }
    p[0] = pr->y[n[1]] - pr->y[n[2]];
    p[1] = pr->y[n[2]] - pr->y[n[0]];
    p[2] = pr->y[n[0]] - pr->y[n[1]];
    q[0] = pr->x[n[2]] - pr->x[n[1]];
    q[1] = pr->x[n[0]] - pr->x[n[2]];
    q[2] = pr->x[n[1]] - pr->x[n[0]];
    g[0] = (pr->x[n[2]] + pr->x[n[1]]) / 2.;
    g[1] = (pr->x[n[0]] + pr->x[n[2]]) / 2.;
    g[2] = (pr->x[n[1]] + pr->x[n[0]]) / 2.;
    for (int j = 0, k = 1; j < 3; k++, j++) {
        if (k == 3) k = 0;
        l[j] = sqrt(pow(pr->x[n[k]] - pr->x[n[j]], 2.) + pow(pr->y[n[k]] - pr->y[n[j]], 2.));
    }
    const double a = (p[0] * q[1] - p[1] * q[0]) / 2.;
    const double R = (pr->x[n[0]] + pr->x[n[1]] + pr->x[n[2]]) / 3.;
    double a_hat = 0, R_hat = 0;
    for (int j = 0; j < 3; j++) a_hat += (rn[j] * rn[j] * p[j] / (4. * R));
    const double vol = 2. * R * a_hat;
    int flag = 0;
    for (int j = 0; j < 3; j++)
        if (rn[j] < 1.e-06) flag++;
    if (flag == 2) {
        R_hat = R;
    } else if (flag == 1) {
        if (rn[0] < 1.e-06)
            R_hat = (fabs(rn[1] - rn[2]) < 1.e-06) ? rn[2] / 2. : (rn[1] - rn[2]) / (2. * log(rn[1]) - 2. * log(rn[2]));
        if (rn[1] < 1.e-06)
            R_hat = (fabs(rn[2] - rn[0]) < 1.e-06) ? rn[0] / 2. : (rn[2] - rn[0]) / (2. * log(rn[2]) - 2. * log(rn[0]));
        if (rn[2] < 1.e-06)
            R_hat = (fabs(rn[0] - rn[1]) < 1.e-06) ? rn[1] / 2. : (rn[0] - rn[1]) / (2. * log(rn[0]) - 2. * log(rn[1]));
    } else {
        if (fabs(q[0]) < 1.e-06) R_hat = (q[1] * q[1]) / (2. * (-q[1] + rn[0] * log(rn[0] / rn[2])));
        else if (fabs(q[1]) < 1.e-06) R_hat = (q[2] * q[2]) / (2. * (-q[2] + rn[1] * log(rn[1] / rn[0])));
        else if (fabs(q[2]) < 1.e-06) R_hat = (q[0] * q[0]) / (2. * (-q[0] + rn[2] * log(rn[2] / rn[1])));
        else
            R_hat = -(q[0] * q[1] * q[2]) /
                    (2. * (q[0] * rn[0] * log(rn[0]) + q[1] * rn[1] * log(rn[1]) + q[2] * rn[2] * log(rn[2])));
    }
    /* Mr, Mz (:293-321) */
    K = C(-1. / (2. * a_hat * R), 0);
    for (int j = 0; j < 3; j++)
        for (int k = j; k < 3; k++) Mx[j][k] = cadd(Mx[j][k], cmuld(cmuld(cmuld(cmuld(K, p[j]), rn[j]), p[k]), rn[k]));
    for (int j = 0; j < 3; j++)
        if (rn[j] < 1.e-06) Mx[j][j] = cadd(Mx[j][j], cadd(cadd(Mx[0][0], Mx[1][1]), Mx[2][2]));
    K = C(-1. / (2. * a_hat * R_hat), 0);
    for (int j = 0; j < 3; j++)
        for (int k = j; k < 3; k++)
            My[j][k] = cadd(My[j][k], cmuld(cmuld(cmuld(cmuld(K, q[j] * rn[j]), q[k] * rn[k]), g[j] / R), g[k] / R));
    Mx[1][0] = Mx[0][1]; Mx[2][0] = Mx[0][2]; Mx[2][1] = Mx[1][2];
    My[1][0] = My[0][1]; My[2][0] = My[0][2]; My[2][1] = My[1][2];
    const orh_block *blk = &pr->blocks[pr->blk[i]];
    const orh_label *lab = &pr->labels[pr->lbl[i]];
    /* eddy currents (:333-347) */
    K = cdivd(cmuld(cmuld(cmuld(cmuld(cmuld(cneg(I), R), a), w), blk->Cduct), c), 6.);
    if ((blk->LamType == 0) && (blk->Lam_d > 0)) K = C(0, 0);
    if (lab->bIsWound) K = C(0, 0);
    for (int j = 0; j < 3; j++)
        for (int k = 0; k < 3; k++) Me[j][k] = cadd(Me[j][k], cdivd(cmuld(K, 4.), 3.));
    /* derivative boundary conditions (:349-383) */
    for (int j = 0; j < 3; j++) {
        int k = j + 1;
        if (k == 3) k = 0;
        double r = (pr->x[n[j]] + pr->x[n[k]]) / 2.;
        int ej = pr->e ? pr->e[3 * i + j] : -1;
        if (ej < 0) continue;
        const orh_line *ln = &pr->lines[ej];
        if (ln->BdryFormat == 2) {
            K = cdivd(cmuld(dmulc(-0.0001 * c * 2. * r, C(ln->c0_re, ln->c0_im)), l[j]), 6.);
            Me[j][j] = cadd(Me[j][j], dmulc(2.0, K));
            Me[k][k] = cadd(Me[k][k], dmulc(2.0, K));
            Me[j][k] = cadd(Me[j][k], K);
            Me[k][j] = cadd(Me[k][j], K);
            K = cmuld(cmuld(cmuld(cdivd(cmuld(C(ln->c1_re, ln->c1_im), l[j]), 2.), 2.), r), 0.0001);
            be[j] = cadd(be[j], K);
            be[k] = cadd(be[k], K);
        }
        if (ln->BdryFormat == 1) {
            double ds = sqrt(2. / (0.4 * ORA_PI * w * ln->Sig * ln->Mu));
            K = cdivd(deg45, -ds * ln->Mu * 100.);
            K = cmuld(K, 2. * r * l[j] / 6.);
            Me[j][j] = cadd(Me[j][j], dmulc(2.0, K));
            Me[k][k] = cadd(Me[k][k], dmulc(2.0, K));
            Me[j][k] = cadd(Me[j][k], K);
            Me[k][j] = cadd(Me[k][j], K);
        }
    }
    /* sources (:385-405) */
    for (int j = 0; j < 3; j++) {
        cx Jv = C(0, 0);
        if (lab->InCircuit >= 0) {
            const orh_circ *cc = &pr->circs[lab->InCircuit];
            if (cc->Case == 1) Jv = C(cc->J_re, cc->J_im);
            if (cc->Case == 0) Jv = cdivd(cmuld(dmulc(-100., C(cc->dV_re, cc->dV_im)), blk->Cduct), R);
        }
        K = cdivd(cmuld(dmulc(-2. * R, cadd(dplusc(blk->J_re, cmuld(I, blk->J_im)), Jv)), a), 3.);
        be[j] = cadd(be[j], K);
        if (lab->InCircuit >= 0 && pr->circs[lab->InCircuit].Case == 2) {
            int row = NN + lab->InCircuit;
            bL[row] = cadd(bL[row], cdivd(K, R));
        }
    }
    /* Case 2 circuit couplings (:407-417) */
    if (lab->InCircuit >= 0 && pr->circs[lab->InCircuit].Case == 2) {
        int cr = NN + lab->InCircuit;
        cx Kc = cmuld(cmuld(cmuld(cmuld(dmulc(-2., I), a), w), blk->Cduct), c);
        for (int j = 0; j < 3; j++) {
            double gr, gi;
            ops->get(L, n[j], cr, &gr, &gi);
            cx v = cadd(C(gr, gi), cdivd(Kc, 3.));
            ops->put(L, v.re, v.im, n[j], cr);
        }
        double gr, gi;
        ops->get(L, cr, cr, &gr, &gi);
        cx v = cadd(C(gr, gi), cdivd(Kc, R));
        ops->put(L, v.re, v.im, cr, cr);
    }
    /* permeability: the block's / successive approximation with B from the
     * element energy (:425-560) / the exterior warp (:567-574) */
    cx mu1 = Mu[pr->blk[i]].mu0, mu2 = Mu[pr->blk[i]].mu1;
    if (blk->LamType > 2) mu1 = mu2 = C(lab->ProxMu_re, lab->ProxMu_im);   /* prox. effects (:571-575) */
    cx Mnh[3][3], Mna[3][3], Mns[3][3];
    int updated = 0, newton = 0;
    if (Iter > 0 && blk->LamType == 0 && blk->BHpoints > 0 && mu1.re == mu2.re && mu1.im == mu2.im) {
        cx v[3], dv = C(0, 0);
        for (int j = 0; j < 3; j++) {
            v[j] = C(0, 0);
            for (int ww = 0; ww < 3; ww++) v[j] = cadd(v[j], cmul(cadd(Mx[j][ww], My[j][ww]), VL[n[ww]]));
        }
        for (int j = 0; j < 3; j++) dv = cadd(dv, cmul(cconj(VL[n[j]]), v[j]));
        dv = cmuld(dv, (10000. * c * c / vol));
        double B = sqrt(cx_abs(dv));
        if (pr->ac_solver == 1) {   /* Newton (harmonicaxi.cpp:520-547): K over vol */
            const cx Vn[3] = {VL[n[0]], VL[n[1]], VL[n[2]]};
            newton_terms(blk, B, c, vol, (const cx(*)[3])Mx, (const cx(*)[3])My, Vn, &mu1, Mn, Mnh, Mna, Mns);
            mu2 = mu1;
            newton = 1;
            updated = 1;
        } else {
        cx murel = ddivc(1., cmuld(bh_getv(blk, B), ORH_MUO));
        cx muinc = ddivc(1., cmuld(bh_dhdb(blk, B), ORH_MUO));
        K = cdiv(cmul(dmulc(2., murel), muinc), cadd(murel, muinc));
        mu1 = K;
        mu2 = K;
        K = cneg(csub(ddivc(1., murel), ddivc(1., K)));
        for (int j = 0; j < 3; j++)
            for (int k = 0; k < 3; k++) Mn[j][k] = cmul(K, cadd(Mx[j][k], My[j][k]));
        updated = 1;
        }
    }
    if (lab->IsExternal && !updated) {   /* set at Iter 0 and kept by linear elements */
        double u = units[pr->length_units];
        double Z = (pr->y[n[0]] + pr->y[n[1]] + pr->y[n[2]]) / 3. - pr->extZo * u;
        double kludge = (R * R + Z * Z) * (pr->extRi * u) / ((pr->extRo * u) * (pr->extRo * u) * (pr->extRo * u));
        mu1 = cdivd(mu1, kludge);
        mu2 = cdivd(mu2, kludge);
    }
    element_to_system(pr, ops, L, n, Me, be, Mx, My, NULL, C(0, 0), Mn, newton ? Mnh : NULL, Mna, Mns, mu1, mu2, VL,
                      bL, 0);
}

static void hage_emit(void *ctx, double v, int p, int q)
{
    struct hage_ctx { const orh_linprob_ops *ops; void *L; } *a = ctx;
    a->ops->addto(a->L, -v, 0.0, p, q);   /* opposite sign to Static2D (harmonic2d.cpp:382) */
}

static int assemble_and_bc(orh_problem *pr, const orh_linprob_ops *ops, void *L, const effmu *Mu, double w,
                           int Iter)
{
    const double c = ORA_PI * 4.e-05;
    const double units[] = {2.54, 0.1, 1., 100., 0.00254, 1.e-04};
    const cx deg45 = C(1, 1);
    const int NN = pr->n_nodes;
    cx *bL = (cx *)ops->b(L);
    cx *VL = (cx *)ops->V(L);
    const int axi = pr->problem_type == 1;
    if (!axi) {   /* air-gap elements first (harmonic2d.cpp:227-380), real entries */
        struct hage_ctx { const orh_linprob_ops *ops; void *L; } actx = {ops, L};
        ora_age_assemble(pr->n_ages, pr->ages, 1, hage_emit, &actx);
    }
    for (int i = 0; i < pr->n_elems; i++) {
        if (axi) {
            axi_element(pr, ops, L, Mu, w, Iter, i, VL, bL);
            continue;
        }
        cx Me[3][3], be[3], Mx[3][3], My[3][3], Mxy[3][3], Mn[3][3];
        double p[3], q[3], l[3];
        int n[3];
        for (int j = 0; j < 3; j++) {
            for (int k = 0; k < 3; k++) Me[j][k] = Mx[j][k] = My[j][k] = Mxy[j][k] = Mn[j][k] = C(0, 0);
            be[j] = C(0, 0);
        }
        for (int k = 0; k < 3; k++) n[k] = pr->p[3 * i + k];
        p[0] = pr->y[n[1]] - pr->y[n[2]];
        p[1] = pr->y[n[2]] - pr->y[n[0]];
        p[2] = pr->y[n[0]] - pr->y[n[1]];
        q[0] = pr->x[n[2]] - pr->x[n[1]];
        q[1] = pr->x[n[0]] - pr->x[n[2]];
        q[2] = pr->x[n[1]] - pr->x[n[0]];
        for (int j = 0, k = 1; j < 3; k++, j++) {
            if (k == 3) k = 0;
            l[j] = sqrt(pow(pr->x[n[k]] - pr->x[n[j]], 2.) + pow(pr->y[n[k]] - pr->y[n[j]], 2.));
        }
        double a = (p[0] * q[1] - p[1] * q[0]) / 2.;
        const orh_block *blk = &pr->blocks[pr->blk[i]];
        const orh_label *lab = &pr->labels[pr->lbl[i]];
        cx K = C(-1. / (4. * a), 0);
        for (int j = 0; j < 3; j++)
            for (int k = j; k < 3; k++) {
                cx t = cmuld(cmuld(K, p[j]), p[k]);
                Mx[j][k] = cadd(Mx[j][k], t);
                if (j != k) Mx[k][j] = cadd(Mx[k][j], t);
            }
        for (int j = 0; j < 3; j++)
            for (int k = j; k < 3; k++) {
                cx t = cmuld(cmuld(K, q[j]), q[k]);
                My[j][k] = cadd(My[j][k], t);
                if (j != k) My[k][j] = cadd(My[k][j], t);
            }
        for (int j = 0; j < 3; j++)
            for (int k = j; k < 3; k++) {
                cx t = cmuld(K, p[j] * q[k] + p[k] * q[j]);
                Mxy[j][k] = cadd(Mxy[j][k], t);
                if (j != k) Mxy[k][j] = cadd(Mxy[k][j], t);
            }
        /* eddy currents (:387-402) */
        K = cmuld(cmuld(cmuld(cmuld(cneg(I), a), w), blk->Cduct), c);
        K = cdivd(K, 12.);
        if ((blk->LamType == 0) && (blk->Lam_d > 0)) K = C(0, 0);
        if (lab->bIsWound) K = C(0, 0);
        for (int j = 0; j < 3; j++)
            for (int k = j; k < 3; k++) {
                Me[j][k] = cadd(Me[j][k], K);
                Me[k][j] = cadd(Me[k][j], K);
            }
        /* derivative boundary conditions (:404-438) */
        for (int j = 0; j < 3; j++) {
            int ej = pr->e ? pr->e[3 * i + j] : -1;
            if (ej < 0) continue;
            const orh_line *ln = &pr->lines[ej];
            int k = j + 1;
            if (k == 3) k = 0;
            if (ln->BdryFormat == 2) {
                K = cdivd(cmuld(dmulc(-0.0001 * c, C(ln->c0_re, ln->c0_im)), l[j]), 6.);
                Me[j][j] = cadd(Me[j][j], dmulc(2.0, K));
                Me[k][k] = cadd(Me[k][k], dmulc(2.0, K));
                Me[j][k] = cadd(Me[j][k], K);
                Me[k][j] = cadd(Me[k][j], K);
                K = cmuld(cdivd(cmuld(C(ln->c1_re, ln->c1_im), l[j]), 2.), 0.0001);
                be[j] = cadd(be[j], K);
                be[k] = cadd(be[k], K);
            }
            if (ln->BdryFormat == 1) {
                double ds = sqrt(2. / (0.4 * ORA_PI * w * ln->Sig * ln->Mu));
                K = cdivd(deg45, -ds * ln->Mu * 100.);
                K = cmuld(K, l[j] / 6.);
                Me[j][j] = cadd(Me[j][j], dmulc(2.0, K));
                Me[k][k] = cadd(Me[k][k], dmulc(2.0, K));
                Me[j][k] = cadd(Me[j][k], K);
                Me[k][j] = cadd(Me[k][j], K);
            }
        }
        /* sources (:441-460) */
        for (int j = 0; j < 3; j++) {
            cx Jv = C(0, 0);
            if (lab->InCircuit >= 0) {
                const orh_circ *cc = &pr->circs[lab->InCircuit];
                if (cc->Case == 1) Jv = C(cc->J_re, cc->J_im);
                if (cc->Case == 0) Jv = cmuld(cneg(C(cc->dV_re, cc->dV_im)), blk->Cduct);
            }
            K = cdivd(cmuld(cneg(cadd(dplusc(blk->J_re, cmuld(I, blk->J_im)), Jv)), a), 3.);
            be[j] = cadd(be[j], K);
            if (lab->InCircuit >= 0 && pr->circs[lab->InCircuit].Case == 2) {
                int row = NN + lab->InCircuit;
                bL[row] = cadd(bL[row], K);
            }
        }
        /* Case 2 circuit couplings (:463-472) */
        if (lab->InCircuit >= 0 && pr->circs[lab->InCircuit].Case == 2) {
            int cr = NN + lab->InCircuit;
            cx Kc = cmuld(cmuld(cmuld(cmuld(cneg(I), a), w), blk->Cduct), c);
            for (int j = 0; j < 3; j++) {
                double gr, gi;
                ops->get(L, n[j], cr, &gr, &gi);
                cx v = cadd(C(gr, gi), cdivd(Kc, 3.));
                ops->put(L, v.re, v.im, n[j], cr);
            }
            double gr, gi;
            ops->get(L, cr, cr, &gr, &gi);
            cx v = cadd(C(gr, gi), Kc);
            ops->put(L, v.re, v.im, cr, cr);
        }
        /* element permeability: Iter 0 / linear blocks the block's (:557-563);
         * later passes, nonlinear LamType-0 blocks: successive approximation
         * (:588-660, ACSolver 0) */
        cx mu1 = Mu[pr->blk[i]].mu0, mu2 = Mu[pr->blk[i]].mu1, v12 = C(0, 0);
        if (blk->LamType > 2) mu1 = mu2 = C(lab->ProxMu_re, lab->ProxMu_im);   /* prox. effects (:664-668) */
        cx Mnh[3][3], Mna[3][3], Mns[3][3];
        int newton = 0;
        if (Iter > 0 && blk->LamType == 0 && blk->BHpoints > 0 && mu1.re == mu2.re && mu1.im == mu2.im) {
            cx B1 = C(0, 0), B2 = C(0, 0);
            for (int j = 0; j < 3; j++) {
                B1 = cadd(B1, cmuld(VL[n[j]], q[j]));
                B2 = cadd(B2, cmuld(VL[n[j]], p[j]));
            }
            cx s1 = cmul(B1, cconj(B1)), s2 = cmul(B2, cconj(B2));
            double B = c * sqrt(cx_abs(s1) + cx_abs(s2)) / (0.02 * a);
            if (pr->ac_solver == 1) {   /* Newton (:611-639) */
                const cx Vn[3] = {VL[n[0]], VL[n[1]], VL[n[2]]};
                newton_terms(blk, B, c, a, (const cx(*)[3])Mx, (const cx(*)[3])My, Vn, &mu1, Mn, Mnh, Mna, Mns);
                mu2 = mu1;
                newton = 1;
            } else {
            cx murel = ddivc(1., cmuld(bh_getv(blk, B), ORH_MUO));   /* muo * Get_v: CComplex * double */
            cx muinc = ddivc(1., cmuld(bh_dhdb(blk, B), ORH_MUO));
            cx K = cdiv(cmul(dmulc(2., murel), muinc), cadd(murel, muinc));
            mu1 = K;
            mu2 = K;
            K = cneg(csub(ddivc(1., murel), ddivc(1., K)));
            for (int j = 0; j < 3; j++)
                for (int k = 0; k < 3; k++) Mn[j][k] = cmul(K, cadd(Mx[j][k], My[j][k]));
            }
        }
        element_to_system(pr, ops, L, n, Me, be, Mx, My, Mxy, v12, Mn, newton ? Mnh : NULL, Mna, Mns, mu1, mu2, VL,
                          bL, 1);
    }
    /* point currents (:634-641) */
    for (int i = 0; i < NN; i++) {
        int m = pr->marker ? pr->marker[i] : -1;
        if (m >= 0) {   /* axisymmetric: (2 r 0.01) J (harmonicaxi.cpp:610-617) */
            cx K = dmulc(axi ? (2. * pr->x[i] * 0.01) : 0.01, dplusc(pr->points[m].J_re, cmuld(I, pr->points[m].J_im)));
            bL[i] = axi ? csub(bL[i], K) : cadd(bL[i], cneg(K));
        }
    }
    /* Case 2 total current constraints (:644-650) */
    for (int i = 0; i < pr->n_circs; i++)
        if (pr->circs[i].Case == 2)
            bL[NN + i] = cadd(bL[NN + i], dmulc(axi ? 2. * 0.01 : 0.01,
                                                dplusc(pr->circs[i].Amps_re, cmuld(I, pr->circs[i].Amps_im))));
    /* fixed points (:653-661) */
    for (int i = 0; i < NN; i++) {
        int m = pr->marker ? pr->marker[i] : -1;
        if (axi && pr->x[i] < (units[pr->length_units] * 1.e-06)) {   /* A = 0 on the axis (:626-631) */
            ops->setvalue(L, i, 0., 0.);
            continue;
        }
        if (m >= 0 && pr->points[m].J_re == 0 && pr->points[m].J_im == 0) {
            cx K = cdivd(dplusc(pr->points[m].A_re, cmuld(I, pr->points[m].A_im)), c);
            ops->setvalue(L, i, K.re, K.im);
        }
    }
    /* fixed segments (:664-730) */
    for (int i = 0; i < pr->n_elems; i++)
        for (int j = 0; j < 3; j++) {
            int k = j + 1;
            if (k == 3) k = 0;
            int s = pr->e ? pr->e[3 * i + j] : -1;
            if (s < 0 || pr->lines[s].BdryFormat != 0) continue;
            const orh_line *ln = &pr->lines[s];
            int nodes2[2] = {pr->p[3 * i + j], pr->p[3 * i + k]};
            for (int m = 0; m < 2; m++) {
                double x = pr->x[nodes2[m]], y = pr->y[nodes2[m]], av;
                if (pr->coords == 0) {
                    x /= units[pr->length_units];
                    y /= units[pr->length_units];
                    av = ln->A0 + x * ln->A1 + y * ln->A2;
                } else {
                    double r = sqrt(x * x + y * y), t;
                    if ((x == 0) && (y == 0)) t = 0;
                    else t = atan2(y, x) / ORA_DEG;
                    r /= units[pr->length_units];
                    av = ln->A0 + r * ln->A1 + t * ln->A2;
                }
                cx K = dmulc(av / c, cx_exp(cmuld(cmuld(I, ln->phi), ORA_DEG)));
                ops->setvalue(L, nodes2[m], K.re, K.im);
            }
        }
    /* circuits with a priori current / voltage: keep their rows regular (:734-736) */
    for (int j = 0; j < pr->n_circs; j++)
        if (pr->circs[j].Case < 2) {
            double gr, gi;
            ops->get(L, 0, 0, &gr, &gi);
            ops->put(L, gr, gi, NN + j, NN + j);
        }
    for (int k = 0; k < pr->n_pbc; k++) {
        if (pr->pbc[3 * k + 2] == 0) ops->periodicity(L, pr->pbc[3 * k], pr->pbc[3 * k + 1]);
        if (pr->pbc[3 * k + 2] == 1) ops->antiperiodicity(L, pr->pbc[3 * k], pr->pbc[3 * k + 1]);
    }
    return 1;
}

static int check_linear(const orh_problem *pr)
{
    for (int k = 0; k < pr->n_blocks; k++) {
        if (pr->blocks[k].BHpoints != 0 && !(pr->blocks[k].B && pr->blocks[k].H_re && pr->blocks[k].H_im &&
                                             pr->blocks[k].S_re && pr->blocks[k].S_im))
            return 0;
        if (pr->blocks[k].LamType == 1 || pr->blocks[k].LamType == 2) return 0;
    }
    return 1;
}

int orh_harmonic2d(orh_problem *pr, const orh_linprob_ops *ops, double *A_out, ora_stats *stats)
{
    if (!ops) ops = orh_builtin_linprob();
    if (!check_linear(pr)) return 0;
    const double c = ORA_PI * 4.e-05;
    const double w = pr->frequency * 2. * ORA_PI;
    const int NN = pr->n_nodes, n = NN + pr->n_circs;
    effmu *Mu = (effmu *)calloc(pr->n_blocks > 0 ? pr->n_blocks : 1, sizeof(effmu));
    circuits(pr);
    effective_mu(pr, w, Mu);
    void *L = ops->create(n, pr->bandwidth, NN, pr->precision);
    /* LinearFlag = false when any element lies in a B-H block (:559-569) */
    int linear = 1;
    for (int i = 0; i < pr->n_elems && linear; i++) linear = pr->blocks[pr->blk[i]].BHpoints == 0;
    cx *Vold = (cx *)calloc(n, sizeof(cx));
    double res = 0, lastres = 0, Relax = 1.;   /* FSolver::Relax (fsolver.cpp:210) */
    int Iter = 0, ok = 0;
    long long iters_total = 0;
    do {   /* :219-873 */
        if (Iter > 0) ops->wipe(L);
        assemble_and_bc(pr, ops, L, Mu, w, Iter);
        cx *VL = (cx *)ops->V(L);
        for (int j = 0; j < n; j++) Vold[j] = VL[j];
        if (ops->newton(L)) {   /* :821-825 */
            double lp = 1.e-4 < 0.001 * res ? 1.e-4 : 0.001 * res;
            if (lp < pr->precision) lp = pr->precision;
            ops->set_precision(L, lp);
        }
        g_iters = -1;
        ok = ops->solve(L, Iter);
        if (!ok) break;
        if (g_iters > 0) iters_total += g_iters;
        VL = (cx *)ops->V(L);
        if (!linear) {
            double x = 0, y = 0;
            for (int j = 0; j < NN; j++) {
                x += cmul(csub(VL[j], Vold[j]), cconj(csub(VL[j], Vold[j]))).re;
                y += cmul(VL[j], cconj(VL[j])).re;
            }
            if (y == 0) linear = 1;
            else {
                lastres = res;
                res = sqrt(x / y);
            }
            if (getenv("ORACLE_TRACE_NONLINEAR")) fprintf(stderr, "pass %d: res %.6e relax %.4f\n", Iter, res, Relax);
            if (Iter > 5) {
                if ((res > lastres) && (Relax > 0.1)) Relax /= 2.;
                else Relax += 0.1 * (1. - Relax);
                for (int j = 0; j < n; j++) VL[j] = cadd(dmulc(Relax, VL[j]), dmulc(1.0 - Relax, Vold[j]));
            }
        }
        if ((res < 100. * pr->precision) && Iter > 0) linear = 1;
        Iter++;
        if (Iter > 1000) {
            ok = 0;
            break;
        }
    } while (!linear);
    free(Vold);
    if (ok) {
        const cx *V = (const cx *)ops->V(L);
        for (int i = 0; i < NN; i++) {
            if (pr->problem_type == 1) {   /* the flux (harmonicaxi.cpp:790) */
                cx f = cmuld(cmuld(cmuld(cmuld(cmuld(V[i], c), 2.), ORA_PI), pr->x[i]), 0.01);
                A_out[2 * i] = f.re;
                A_out[2 * i + 1] = f.im;
            } else {
                A_out[2 * i] = V[i].re * c;
                A_out[2 * i + 1] = V[i].im * c;
            }
        }
        for (int i = 0; i < pr->n_circs; i++)
            if (pr->circs[i].Case == 2) {   /* L.b[NumNodes+i] = I*c*w*V (:784) and .ans writes it as dV */
                cx dv = pr->problem_type == 1 ? cmul(cmuld(cmuld(cmuld(I, w), c), 0.01), V[NN + i])   /* :791 */
                                              : cmul(cmuld(cmuld(I, c), w), V[NN + i]);
                pr->circs[i].dV_re = dv.re;
                pr->circs[i].dV_im = dv.im;
            }
    }
    if (stats) {
        stats->newton_iters = Iter;
        stats->cg_iters = (ops == orh_builtin_linprob()) ? iters_total : -1;
        stats->last_res = res;
    }
    ops->destroy(L);
    free(Mu);
    return ok;
}

int orh_harmonic2d_system(orh_problem *pr, int *rows, int *cols, double *vals, long long cap, double *b_out,
                          long long *nnz_out)
{
    if (!check_linear(pr)) return 0;
    const double w = pr->frequency * 2. * ORA_PI;
    const int NN = pr->n_nodes, n = NN + pr->n_circs;
    effmu *Mu = (effmu *)calloc(pr->n_blocks > 0 ? pr->n_blocks : 1, sizeof(effmu));
    circuits(pr);
    effective_mu(pr, w, Mu);
    clp *L = (clp *)clp_create(n, pr->bandwidth, NN, pr->precision);
    assemble_and_bc(pr, orh_builtin_linprob(), L, Mu, w, 0);
    long long k = 0;
    for (int i = 0; i < NN; i++) {
        const crow *r = &L->M[i];
        for (int t = 0; t < r->len; t++) {
            if (r->c[t] >= NN) continue;
            if (k < cap) {
                rows[k] = i;
                cols[k] = r->c[t];
                vals[2 * k] = r->x[t].re;
                vals[2 * k + 1] = r->x[t].im;
            }
            k++;
        }
        b_out[2 * i] = L->b[i].re;
        b_out[2 * i + 1] = L->b[i].im;
    }
    *nnz_out = k;
    clp_destroy(L);
    free(Mu);
    return 1;
}
