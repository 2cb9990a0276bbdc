// Time-harmonic planar problems on MI355X (gfx950): FSolver::Harmonic2D
// (cfemm/fsolver/harmonic2d.cpp:36-790) with the complex-symmetric solve of
// CBigComplexLinProb (cfemm/libfemm/cspars.cpp).
//
// Shares the static path's symbolic phase (CSR pattern, element colouring,
// CSR slots, Dirichlet row/column lists, the composed periodic averaging map)
// and stores the complex matrix as two value arrays over that pattern
// (val = real parts, val_im), so the real-weighted periodic map applies to
// each part unchanged.  Complex arithmetic follows femmcomplex.cpp's formulas
// (products (ac - bd, ad + bc), quotients through the scaled reciprocal).
//
// Solver: the reference's PBCGSolve is COCG -- preconditioned CG with the
// UNCONJUGATED bilinear form x.y, for complex-symmetric A -- stopping at
// |r| / |b| <= Precision (cspars.cpp:822-895).  Here it runs in the
// Chronopoulos-Gear arrangement of xfk_pcg.hip (two launches per iteration,
// every inner product from one reduction phase) preconditioned by the
// smoothed-aggregation V-cycle of a real SPD surrogate (or complex Jacobi) in
// place of the sequential SSOR sweep; the three CGNE
// start-up iterations of PCGSQStart (cspars.cpp:764-820) are not needed by it
// and are omitted (the answer is the solution to the same tolerance).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <complex>

#include "xfk_age.h"
#include "xfk_amg.h"
#include "xfk_axi.h"
#include "xfk_comm.h"
#include "xfk_kernels.h"
#include "xfk_spmv.h"

namespace xfk {

namespace {

// ---- complex helpers (femmcomplex.cpp) ----
__host__ __device__ __forceinline__ double2 cx(double re, double im) { return make_double2(re, im); }
__host__ __device__ __forceinline__ double2 cadd(double2 a, double2 b) { return cx(a.x + b.x, a.y + b.y); }
__host__ __device__ __forceinline__ double2 csub(double2 a, double2 b) { return cx(a.x - b.x, a.y - b.y); }
__host__ __device__ __forceinline__ double2 cmul(double2 a, double2 b)
{
    return cx(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__host__ __device__ __forceinline__ double2 cscale(double2 a, double s) { return cx(a.x * s, a.y * s); }
__host__ __device__ __forceinline__ double2 crecip(double2 z)
{
    double c;
    double2 y;
    if (fabs(z.x) > fabs(z.y)) {
        c = z.y / z.x;
        y.x = 1. / (z.x * (1. + c * c));
        y.y = (-c) * y.x;
    } else {
        c = z.x / z.y;
        y.y = (-1.) / (z.y * (1. + c * c));
        y.x = (-c) * y.y;
    }
    return y;
}
__host__ __device__ __forceinline__ double2 cdiv(double2 a, double2 b) { return cmul(a, crecip(b)); }
__host__ __device__ __forceinline__ double2 cexp_(double2 x)
{
    const double e = exp(x.x);
    return cx(cos(x.y) * e, sin(x.y) * e);
}
__host__ __device__ __forceinline__ double2 ctanh_(double2 x)
{
    if (x.x > 0) {
        double2 e = cexp_(cscale(x, -2.0));
        return cdiv(cx(1 - e.x, -e.y), cx(1 + e.x, e.y));
    }
    double2 e = cexp_(cscale(x, 2.0));
    return cdiv(cx(e.x - 1, e.y), cx(e.x + 1, e.y));
}

struct HarmArgs {
    const int4 *erec;
    const int *ebits;
    const int *slot;
    const double *x, *y;
    const DevLabel *labels;
    const DevBlockAC *blocks;
    const DevLineAC *lines;
    const DevCircAC *circs;
    double *val, *val_im, *b, *b_im;
    double w;
    // HarmonicAxisymmetric (x is r, y is z; exterior-region warp in cm)
    int axi;
    double ext_ro, ext_ri, ext_zo;
    // successive approximation (nonlinear blocks, iter > 0)
    int iter;
    const double2 *V;                  // the current iterate
    const double *bhB;                 // complex B-H curves (DevBlockAC::bh_off / bh_n)
    const double2 *bhH, *bhS;
    // Newton AC solver (ACSolver 1, iter > 0): Newton terms of the nonlinear
    // elements, the auxiliary matrices Mh, Ms, Ma (6 arrays of nnz: re, im each)
    int newton;
    double *aux;
    long long nnz;
};

// Get_v(B) of the harmonic solver's curve (CMaterialProp.cpp:899-903): the
// base-class GetH(double), i.e. the REAL part of the Hermite interpolant
// (CMaterialProp.cpp:488-518), over B; slope[0] at B = 0
__device__ double2 hbh_v(double Bq, int n, const double *__restrict__ B, const double2 *__restrict__ H,
                         const double2 *__restrict__ S)
{
    if (Bq == 0) return S[0];
    const double b = fabs(Bq);
    double h = 0.0;
    if (b > B[n - 1]) {
        h = H[n - 1].x + S[n - 1].x * (b - B[n - 1]);
    } else {
        for (int i = 0; i < n - 1; i++)
            if ((b >= B[i]) && (b <= B[i + 1])) {
                const double l = B[i + 1] - B[i], z = (b - B[i]) / l, z2 = z * z;
                h = (1. - 3. * z2 + 2. * z2 * z) * H[i].x + z * (1. - 2. * z + z2) * l * S[i].x +
                    z2 * (3. - 2. * z) * H[i + 1].x + z2 * (z - 1.) * l * S[i + 1].x;
                break;
            }
    }
    return cx(h / Bq, 0.0);
}

// GetdHdB(B) on the complex curve (CMaterialProp.cpp:461-486)
__device__ double2 hbh_dhdb(double Bq, int n, const double *__restrict__ B, const double2 *__restrict__ H,
                            const double2 *__restrict__ S)
{
    const double b = fabs(Bq);
    if (b > B[n - 1]) return S[n - 1];
    for (int i = 0; i < n - 1; i++)
        if ((b >= B[i]) && (b <= B[i + 1])) {
            const double l = B[i + 1] - B[i], z = (b - B[i]) / l;
            const double c0 = 6. * z * (z - 1.), c1 = 1. - 4. * z + 3. * z * z, c2 = 6. * z * (1. - z),
                         c3 = z * (3. * z - 2.);
            double2 h = cx(c0 * H[i].x / l, c0 * H[i].y / l);
            h = cadd(h, cscale(S[i], c1));
            h = cadd(h, cx(c2 * H[i + 1].x / l, c2 * H[i + 1].y / l));
            return cadd(h, cscale(S[i + 1], c3));
        }
    return cx(0, 0);
}

// GetBHProps(B, v, dv) of the complex curve (CMaterialProp.cpp:1008-1057):
// v = h / b and dv = d(h / b) / d(b^2) = (dh / b^2 - h / b^3) / 2
__device__ void hbh_props(double Bq, int n, const double *__restrict__ B, const double2 *__restrict__ H,
                          const double2 *__restrict__ S, double2 &v, double2 &dv)
{
    const double b = fabs(Bq);
    v = S[0];
    dv = cx(0, 0);
    if (b == 0) return;
    double2 h, dh;
    if (b > B[n - 1]) {
        h = cadd(H[n - 1], cscale(S[n - 1], b - B[n - 1]));
        dh = S[n - 1];
    } else {
        int i = 0;
        while (i < n - 2 && !((b >= B[i]) && (b <= B[i + 1]))) ++i;
        const double l = B[i + 1] - B[i], z = (b - B[i]) / l, z2 = z * z;
        h = cscale(H[i], 1. - 3. * z2 + 2. * z2 * z);
        h = cadd(h, cscale(S[i], z * (1. - 2. * z + z2) * l));
        h = cadd(h, cscale(H[i + 1], z2 * (3. - 2. * z)));
        h = cadd(h, cscale(S[i + 1], z2 * (z - 1.) * l));
        const double c0 = 6. * z * (z - 1.), c2 = 6. * z * (1. - z);
        dh = cx(c0 * H[i].x / l, c0 * H[i].y / l);
        dh = cadd(dh, cscale(S[i], 1. - 4. * z + 3. * z * z));
        dh = cadd(dh, cx(c2 * H[i + 1].x / l, c2 * H[i + 1].y / l));
        dh = cadd(dh, cscale(S[i + 1], z * (3. * z - 2.)));
    }
    v = cx(h.x / b, h.y / b);
    const double2 t = csub(cx(dh.x / (b * b), dh.y / (b * b)), cx(h.x / (b * b * b), h.y / (b * b * b)));
    dv = cscale(t, 0.5);
}

// Newton terms of entry (j, k) of a nonlinear element (harmonic2d.cpp:626-638):
// Mn = K Re(v_j conj v_k); Mnh, Mna the Hermitian / anti-Hermitian remainders
// of 0.5 Re(K) v_j conj v_k and 0.5 I Im(K) v_j conj v_k; Mns = 0.5 K v_j v_k
__device__ __forceinline__ void newton_entry(double2 vj, double2 vk, double2 K, double2 &Mn, double2 &Mnh,
                                             double2 &Mna, double2 &Mns)
{
    const double2 ck = cx(vk.x, -vk.y);
    Mn = cscale(K, cmul(vj, ck).x);
    const double2 t = cmul(cscale(vj, 0.5 * K.x), ck);
    Mnh = cx(t.x - Mn.x, t.y);
    const double2 a = cmul(cmul(cx(0.0, 0.5 * K.y), vj), ck);
    Mna = cx(a.x, a.y - Mn.y);
    Mns = cmul(cmul(cscale(K, 0.5), vj), vk);
}

// the element's Newton contribution to row j: Mn into Me (added by the
// caller), (Mnh + Mna + Mn) V + Mns conj(V) into be (harmonic2d.cpp:676-681)
__device__ __forceinline__ double2 newton_be(const double2 (&vn)[3], double2 K, int j, const double2 (&Vn)[3])
{
    double2 be = cx(0, 0);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        double2 Mn, Mnh, Mna, Mns;
        newton_entry(vn[j], vn[k], K, Mn, Mnh, Mna, Mns);
        be = cadd(be, cmul(cadd(cadd(Mnh, Mna), Mn), Vn[k]));
        be = cadd(be, cmul(Mns, cx(Vn[k].x, -Vn[k].y)));
    }
    return be;
}

// scatter of the auxiliary entries of local row j: the upper entries (k >= j)
// as computed, the lower ones through Put's flip (cspars.cpp:147-160):
// Hermitian conj, complex-symmetric as is, anti-Hermitian -conj
__device__ __forceinline__ void newton_scatter(const HarmArgs &A, const int *sl, int j, const double2 (&vn)[3],
                                               double2 K)
{
    double *Mh = A.aux, *Ms = A.aux + 2 * A.nnz, *Ma = A.aux + 4 * A.nnz;
    const long long nz = A.nnz;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        double2 Mn, Mnh, Mna, Mns;
        if (k >= j) {
            newton_entry(vn[j], vn[k], K, Mn, Mnh, Mna, Mns);
        } else {
            newton_entry(vn[k], vn[j], K, Mn, Mnh, Mna, Mns);
            Mnh = cx(Mnh.x, -Mnh.y);
            Mna = cx(-Mna.x, Mna.y);
        }
        const int q = sl[3 * j + k];
        Mh[q] += Mnh.x;
        Mh[nz + q] += Mnh.y;
        Ms[q] += Mns.x;
        Ms[nz + q] += Mns.y;
        Ma[q] += Mna.x;
        Ma[nz + q] += Mna.y;
    }
}

// the averaged permeability of successive approximation at flux density B
// (harmonic2d.cpp:648-656, harmonicaxi.cpp:543-553): mu = K, correction Kn
__device__ __forceinline__ void hbh_update(double B, const DevBlockAC &bp, const HarmArgs &A, double2 &mu,
                                           double2 &Kn)
{
    const double *cb = A.bhB + bp.bh_off;
    const double2 *ch = A.bhH + bp.bh_off, *cs = A.bhS + bp.bh_off;
    const double2 gv = hbh_v(B, bp.bh_n, cb, ch, cs), gd = hbh_dhdb(B, bp.bh_n, cb, ch, cs);
    const double2 murel = crecip(cscale(gv, kMUO)), muinc = crecip(cscale(gd, kMUO));
    mu = cdiv(cmul(cscale(murel, 2.), muinc), cadd(murel, muinc));
    const double2 d = csub(crecip(murel), crecip(mu));
    Kn = cx(-d.x, -d.y);
}

// femmcomplex abs (femmcomplex.cpp:749-757)
__device__ __forceinline__ double cabs_(double2 x)
{
    if ((x.x == 0) && (x.y == 0)) return 0.;
    if (fabs(x.x) > fabs(x.y)) return fabs(x.x) * sqrt(1. + (x.y / x.x) * (x.y / x.x));
    return fabs(x.y) * sqrt(1. + (x.x / x.y) * (x.x / x.y));
}

// HarmonicAxisymmetric element (harmonicaxi.cpp:215-605): the r-weighted flux
// formulation of xfk_axi.h, eddy currents lumped to the element mean, r-weighted
// boundary terms and sources, B from the element energy, the exterior warp
__device__ void hax_element(int i, const HarmArgs &A, const int (&n)[3], const double (&X)[3],
                            const double (&Y)[3], const DevLabel &lab, const DevBlockAC &bp, double2 (&Me)[3][3],
                            double2 (&be)[3], bool &nt, double2 (&vn)[3], double2 &Kt)
{
    nt = false;
    AxiGeom Gm;
    axi_geometry(X, Y, Gm);
    const double R = Gm.R, a = Gm.a;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
#pragma unroll
        for (int k = 0; k < 3; ++k) Me[j][k] = cx(0, 0);
        be[j] = cx(0, 0);
    }
    // eddy currents, induced current constant over the element (:333-347)
    if (bp.eddy && !lab.is_wound) {
        double2 Ke = cx(-0.0 * R, -R);
        Ke = cx(Ke.x * a, Ke.y * a);
        Ke = cx(Ke.x * A.w, Ke.y * A.w);
        Ke = cx(Ke.x * bp.Cduct, Ke.y * bp.Cduct);
        Ke = cx(Ke.x * kC / 6., Ke.y * kC / 6.);
        Ke = cx(Ke.x * 4. / 3., Ke.y * 4. / 3.);
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int k = 0; k < 3; ++k) Me[j][k] = cadd(Me[j][k], Ke);
    }
    // derivative boundary conditions (:349-383)
    const int eb = A.ebits[i];
    if (eb) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int ej = ((eb >> (10 * j)) & 1023) - 1;
            if (ej < 0) continue;
            const DevLineAC ln = A.lines[ej];
            if (ln.format != 1 && ln.format != 2) continue;
            const int k = (j + 1) % 3;
            const double r = (X[j] + X[k]) / 2.;
            const double lj = sqrt(pow(X[k] - X[j], 2.) + pow(Y[k] - Y[j], 2.));
            double2 Kb;
            if (ln.format == 2) {
                const double s = -0.0001 * kC * 2. * r;
                Kb = cscale(ln.c0, s);
                Kb = cx(Kb.x * lj / 6., Kb.y * lj / 6.);
                const double2 Kc = cx(ln.c1.x * lj / 2. * 2. * r * 0.0001, ln.c1.y * lj / 2. * 2. * r * 0.0001);
                be[j] = cadd(be[j], Kc);
                be[k] = cadd(be[k], Kc);
            } else {
                Kb = cscale(ln.zs, (2. * r * lj / 6.));
            }
            Me[j][j] = cadd(Me[j][j], cscale(Kb, 2.));
            Me[k][k] = cadd(Me[k][k], cscale(Kb, 2.));
            Me[j][k] = cadd(Me[j][k], Kb);
            Me[k][j] = cadd(Me[k][j], Kb);
        }
    }
    // source current density (:385-405)
    double2 Jv = cx(0, 0);
    if (lab.in_circuit >= 0) {
        const DevCircAC C = A.circs[lab.in_circuit];
        if (C.ccase == 1) Jv = C.J;
        if (C.ccase == 0) Jv = cx(-100. * C.dV.x * bp.Cduct / R, -100. * C.dV.y * bp.Cduct / R);
    }
    {
        const double2 Jt = cadd(bp.J, Jv);
        const double s = -2. * R;
        const double2 Ks = cx(s * Jt.x * a / 3., s * Jt.y * a / 3.);
        be[0] = cadd(be[0], Ks);
        be[1] = cadd(be[1], Ks);
        be[2] = cadd(be[2], Ks);
    }
    // permeability: the block's (+ the exterior warp), or successive
    // approximation with B derived from the element energy (:468-560)
    double2 mu1 = bp.mu1, mu2 = bp.mu2, Kn = cx(0, 0);
    if (bp.prox) mu1 = mu2 = lab.prox_mu;   // wound region (harmonicaxi.cpp:571-575), then the warp below
    const bool nl = bp.bh_n > 0 && A.iter > 0;
    if (nl) {
        double2 v[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            v[j] = cx(0, 0);
#pragma unroll
            for (int w = 0; w < 3; ++w) v[j] = cadd(v[j], cscale(A.V[n[w]], Gm.Mx[j][w] + Gm.My[j][w]));
        }
        double2 dv = cx(0, 0);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const double2 vn = A.V[n[j]];
            dv = cadd(dv, cmul(cx(vn.x, -vn.y), v[j]));
        }
        const double s = (10000. * kC * kC / Gm.vol);
        dv = cx(dv.x * s, dv.y * s);
        if (A.newton) {   // Newton (harmonicaxi.cpp:520-547): K over the r-weighted volume
            double2 gv, gd;
            hbh_props(sqrt(cabs_(dv)), bp.bh_n, A.bhB + bp.bh_off, A.bhH + bp.bh_off, A.bhS + bp.bh_off, gv, gd);
            mu1 = crecip(cscale(gv, kMUO));
            Kt = cscale(gd, -200. * kC * kC * kC);
            Kt = cx(Kt.x / Gm.vol, Kt.y / Gm.vol);
#pragma unroll
            for (int j = 0; j < 3; ++j) vn[j] = v[j];
            nt = true;
        } else {
            hbh_update(sqrt(cabs_(dv)), bp, A, mu1, Kn);
        }
        mu2 = mu1;
    } else if (lab.external) {
        const double Z = (Y[0] + Y[1] + Y[2]) / 3. - A.ext_zo;
        const double kludge = (R * R + Z * Z) * A.ext_ri / (A.ext_ro * A.ext_ro * A.ext_ro);
        mu1 = cx(mu1.x / kludge, mu1.y / kludge);
        mu2 = cx(mu2.x / kludge, mu2.y / kludge);
    }
    const double2 r1 = crecip(mu1), r2 = crecip(mu2);
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double mx = Gm.Mx[j][k], my = Gm.My[j][k];
            if (nt) {
                double2 Mn, Mnh, Mna, Mns;
                newton_entry(vn[j], vn[k], Kt, Mn, Mnh, Mna, Mns);
                Me[j][k] = cadd(Me[j][k], cadd(cadd(cscale(r2, mx), cscale(r1, my)), Mn));
            } else {
                Me[j][k] = cadd(Me[j][k], cadd(cscale(r2, mx), cscale(r1, my)));
                if (nl) be[j] = cadd(be[j], cmul(cscale(Kn, mx + my), A.V[n[k]]));
            }
        }
    if (nt) {
        const double2 Vn[3] = {A.V[n[0]], A.V[n[1]], A.V[n[2]]};
#pragma unroll
        for (int j = 0; j < 3; ++j) be[j] = cadd(be[j], newton_be(vn, Kt, j, Vn));
    }
}

// One colour of the element loop (harmonic2d.cpp:352-700; v12 == 0):
// element matrices, eddy-current and boundary terms, sources, for nonlinear
// blocks after the first pass the averaged permeability of the element's
// flux density and the residual correction Mn V (successive approximation,
// harmonic2d.cpp:616-660), colour-exclusive scatter into the complex CSR.
__global__ void __launch_bounds__(kBlock) k_hassemble_color(int begin, int end, HarmArgs A)
{
    __shared__ int s_slot[kBlock * 9 + kBlock / 8];
    const int tile0 = begin + blockIdx.x * kBlock;
    const int ntile = min(kBlock, end - tile0);
    if (ntile <= 0) return;
    for (int k = threadIdx.x; k < ntile * 9; k += kBlock) {
        int e = k / 9;
        s_slot[k + (e >> 3)] = A.slot[(size_t)tile0 * 9 + k];
    }
    __syncthreads();
    const int li = threadIdx.x;
    if (li >= ntile) return;
    const int i = tile0 + li;
    const int4 r = A.erec[i];
    const int n[3] = {r.x, r.y, r.z};
    const DevLabel lab = A.labels[r.w];
    const DevBlockAC bp = A.blocks[lab.blk];
    const double X[3] = {A.x[n[0]], A.x[n[1]], A.x[n[2]]};
    const double Y[3] = {A.y[n[0]], A.y[n[1]], A.y[n[2]]};
    if (A.axi) {
        double2 Me[3][3], be[3], vn[3], Kt = cx(0, 0);
        bool nt;
        hax_element(i, A, n, X, Y, lab, bp, Me, be, nt, vn, Kt);
        const int *sl = &s_slot[li * 9 + (li >> 3)];
        for (int j = 0; j < 3; ++j) {
            if (sl[3 * j] < 0) continue;
            for (int k = 0; k < 3; ++k) {
                const double2 m = (k >= j) ? Me[j][k] : Me[k][j];
                A.val[sl[3 * j + k]] += m.x;
                A.val_im[sl[3 * j + k]] += m.y;
            }
            if (nt) newton_scatter(A, sl, j, vn, Kt);
            A.b[n[j]] += be[j].x;
            A.b_im[n[j]] += be[j].y;
        }
        return;
    }
    double p[3], q[3];
    p[0] = Y[1] - Y[2]; p[1] = Y[2] - Y[0]; p[2] = Y[0] - Y[1];
    q[0] = X[2] - X[1]; q[1] = X[0] - X[2]; q[2] = X[1] - X[0];
    const double a = (p[0] * q[1] - p[1] * q[0]) / 2.;
    const double K = (-1. / (4. * a));
    double2 Me[3][3], be[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
#pragma unroll
        for (int k = 0; k < 3; ++k) Me[j][k] = cx(0, 0);
        be[j] = cx(0, 0);
    }
    // eddy currents (harmonic2d.cpp:387-410)
    if (bp.eddy && !lab.is_wound && bp.Cduct != 0.0) {
        const double2 Ke = cx(-0.0 * a * A.w * bp.Cduct * kC / 12., -a * A.w * bp.Cduct * kC / 12.);
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int k = j; k < 3; ++k) {
                Me[j][k] = cadd(Me[j][k], Ke);
                Me[k][j] = cadd(Me[k][j], Ke);
            }
    }
    // derivative boundary conditions (harmonic2d.cpp:412-438)
    const int eb = A.ebits[i];
    if (eb) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            int ej = ((eb >> (10 * j)) & 1023) - 1;
            if (ej < 0) continue;
            const DevLineAC ln = A.lines[ej];
            if (ln.format != 1 && ln.format != 2) continue;
            int k = (j + 1) % 3;
            double lj = sqrt(pow(X[k] - X[j], 2.) + pow(Y[k] - Y[j], 2.));
            double2 Kb;
            if (ln.format == 2) {
                Kb = cscale(cscale(ln.c0, -0.0001 * kC), lj);
                Kb = cx(Kb.x / 6., Kb.y / 6.);
                const double2 Kc = cx(ln.c1.x * lj / 2. * 0.0001, ln.c1.y * lj / 2. * 0.0001);
                be[j] = cadd(be[j], Kc);
                be[k] = cadd(be[k], Kc);
            } else {
                Kb = cscale(ln.zs, lj / 6.);
            }
            Me[j][j] = cadd(Me[j][j], cscale(Kb, 2.));
            Me[k][k] = cadd(Me[k][k], cscale(Kb, 2.));
            Me[j][k] = cadd(Me[j][k], Kb);
            Me[k][j] = cadd(Me[k][j], Kb);
        }
    }
    // source current density (harmonic2d.cpp:441-460)
    double2 Jv = cx(0, 0);
    if (lab.in_circuit >= 0) {
        const DevCircAC C = A.circs[lab.in_circuit];
        if (C.ccase == 1) Jv = C.J;
        if (C.ccase == 0) Jv = cscale(C.dV, -bp.Cduct);
    }
    const double2 Jt = cadd(bp.J, Jv);
    const double2 Ks = cx((-Jt.x * a) / 3., (-Jt.y * a) / 3.);
    be[0] = cadd(be[0], Ks);
    be[1] = cadd(be[1], Ks);
    be[2] = cadd(be[2], Ks);
    double2 mu1 = bp.mu1, mu2 = bp.mu2;
    if (bp.prox) mu1 = mu2 = lab.prox_mu;   // wound region (harmonic2d.cpp:664-668)
    double2 Kn = cx(0, 0), Kt = cx(0, 0), vn[3];
    const bool nl = bp.bh_n > 0 && A.iter > 0;
    const bool nt = nl && A.newton;
    if (nl) {
        // flux density of the element from the current iterate
        double2 B1 = cx(0, 0), B2 = cx(0, 0);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const double2 v = A.V[n[j]];
            B1 = cadd(B1, cscale(v, q[j]));
            B2 = cadd(B2, cscale(v, p[j]));
        }
        const double s1 = B1.x * B1.x - B1.y * (-B1.y), s2 = B2.x * B2.x - B2.y * (-B2.y);
        const double B = kC * sqrt(fabs(s1) + fabs(s2)) / (0.02 * a);
        if (nt) {   // Newton (harmonic2d.cpp:611-639)
            double2 gv, gd;
            hbh_props(B, bp.bh_n, A.bhB + bp.bh_off, A.bhH + bp.bh_off, A.bhS + bp.bh_off, gv, gd);
            mu1 = crecip(cscale(gv, kMUO));
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                vn[j] = cx(0, 0);
#pragma unroll
                for (int w = 0; w < 3; ++w) vn[j] = cadd(vn[j], cscale(A.V[n[w]], K * p[j] * p[w] + K * q[j] * q[w]));
            }
            Kt = cscale(gd, -200. * kC * kC * kC);
            Kt = cx(Kt.x / a, Kt.y / a);
        } else {
            hbh_update(B, bp, A, mu1, Kn);   // averaged secant / incremental permeability
        }
        mu2 = mu1;
    }
    // Mx / mu2 + My / mu1 (+ Mn, the correction moved to the right-hand side)
    const double2 r1 = crecip(mu1), r2 = crecip(mu2);
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double mx = K * p[j] * p[k], my = K * q[j] * q[k];
            if (nt) {
                double2 Mn, Mnh, Mna, Mns;
                newton_entry(vn[j], vn[k], Kt, Mn, Mnh, Mna, Mns);
                Me[j][k] = cadd(Me[j][k], cadd(cadd(cscale(r2, mx), cscale(r1, my)), Mn));
            } else {
                Me[j][k] = cadd(Me[j][k], cadd(cscale(r2, mx), cscale(r1, my)));
                if (nl) be[j] = cadd(be[j], cmul(cscale(Kn, mx + my), A.V[n[k]]));
            }
        }
    if (nt) {
        const double2 Vn[3] = {A.V[n[0]], A.V[n[1]], A.V[n[2]]};
#pragma unroll
        for (int j = 0; j < 3; ++j) be[j] = cadd(be[j], newton_be(vn, Kt, j, Vn));
    }
    const int *sl = &s_slot[li * 9 + (li >> 3)];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        if (sl[3 * j] < 0) continue;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double2 m = (k >= j) ? Me[j][k] : Me[k][j];
            A.val[sl[3 * j + k]] += m.x;
            A.val_im[sl[3 * j + k]] += m.y;
        }
        if (nt) newton_scatter(A, sl, j, vn, Kt);
        A.b[n[j]] += be[j].x;
        A.b_im[n[j]] += be[j].y;
    }
}

__global__ void k_hpoint(int n, const int *__restrict__ nodes, const double *__restrict__ J, double *__restrict__ b,
                         double *__restrict__ b_im)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    b[nodes[i]] += J[2 * i];
    b_im[nodes[i]] += J[2 * i + 1];
}

// CBigComplexLinProb::SetValue (cspars.cpp:482-537), column half: b[k] -= A(k,i) x_i
// (first value set), A(k,i) = 0
// With the Newton AC solver's auxiliary matrices (aux != nullptr, cspars.cpp:511-533):
// b[k] -= Mh(k,i) x, Ms(k,i) conj(x) and -- as the reference does -- Ma(k,i) conj(x)
__global__ void k_hdir_cols(int n, const int *__restrict__ rows, const int *__restrict__ rowptr,
                            const int *__restrict__ col, const unsigned char *__restrict__ fixed,
                            const double *__restrict__ first, double *__restrict__ val, double *__restrict__ val_im,
                            double *__restrict__ b, double *__restrict__ b_im, double *__restrict__ aux,
                            long long nnz)
{
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    int r = rows[t];
    double2 br = cx(b[r], b_im[r]);
    for (int k = rowptr[r]; k < rowptr[r + 1]; ++k) {
        int c = col[k];
        if (!fixed[c]) continue;
        const double2 x = cx(first[2 * c], first[2 * c + 1]);
        const double2 z = cx(val[k], val_im[k]);
        if (z.x != 0 || z.y != 0) {
            br = csub(br, cmul(z, x));
            val[k] = 0.0;
            val_im[k] = 0.0;
        }
        if (aux) {
            for (int h = 0; h < 3; ++h) {
                double *re = aux + 2 * h * nnz, *im = re + nnz;
                const double2 za = cx(re[k], im[k]);
                if (za.x != 0 || za.y != 0) {
                    br = csub(br, cmul(za, h == 0 ? x : cx(x.x, -x.y)));
                    re[k] = 0.0;
                    im[k] = 0.0;
                }
            }
        }
    }
    b[r] = br.x;
    b_im[r] = br.y;
}

// row half: the fixed row keeps its diagonal, b = A_ii x_i (last value set)
// (the auxiliary matrices lose the whole row, diagonal included)
__global__ void k_hdir_rows(int n, const int *__restrict__ rows, const int *__restrict__ rowptr,
                            const int *__restrict__ diag, double *__restrict__ val, double *__restrict__ val_im,
                            double *__restrict__ b, double *__restrict__ b_im, const double *__restrict__ last,
                            double *__restrict__ aux, long long nnz)
{
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    int r = rows[t];
    int d = diag[r];
    for (int k = rowptr[r]; k < rowptr[r + 1]; ++k) {
        if (k != d) {
            val[k] = 0.0;
            val_im[k] = 0.0;
        }
        if (aux)
            for (int h = 0; h < 6; ++h) aux[h * nnz + k] = 0.0;
    }
    const double2 v = cmul(cx(val[d], val_im[d]), cx(last[2 * r], last[2 * r + 1]));
    b[r] = v.x;
    b_im[r] = v.y;
}

// complex Jacobi preconditioner + the reference's singularity check (cspars.cpp:772-777)
__global__ void k_hdiag_inv(int N, const int *__restrict__ diag, const double *__restrict__ val,
                            const double *__restrict__ val_im, double2 *__restrict__ dinv, CcgState *S)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const double2 d = cx(val[diag[i]], val_im[diag[i]]);
    if (d.x == 0.0 && d.y == 0.0) {
        S->singular = 1;
        dinv[i] = cx(0, 0);
    } else {
        dinv[i] = crecip(d);
    }
}

// ---- COCG kernels ----
constexpr int kHcCap = 4 * kCgBlock;   // complex products staged per LDS pass (64 KiB)
constexpr int kHcAxBlock = 256;
constexpr int kHcAxGrid = 1024;
constexpr int kHcParts = 9;            // gam0 re/im, gam1 re/im, del re/im, rr0, rr1, bb

// w = A u over the rows of one tile (CSR-stream through LDS, complex)
__device__ __forceinline__ double2 hc_tile_spmv(int r0, int N, const int *__restrict__ rowptr,
                                                const int *__restrict__ col, const double *__restrict__ val,
                                                const double *__restrict__ val_im, const double2 *__restrict__ X,
                                                double2 *lds)
{
    const int r = r0 + threadIdx.x;
    const int rend = min(r0 + kCgBlock, N);
    const int s = rowptr[r0], e = rowptr[rend];
    const int my_s = (r < N) ? rowptr[r] : 0, my_e = (r < N) ? rowptr[r + 1] : 0;
    double2 acc = cx(0, 0);
    for (int c0 = s; c0 < e; c0 += kHcCap) {
        const int c1 = min(e, c0 + kHcCap);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int k = c0 + threadIdx.x + m * kCgBlock;
            if (k < c1) lds[k - c0] = cmul(cx(val[k], val_im[k]), X[col[k]]);
        }
        __syncthreads();
        const int a = max(my_s, c0), z = min(my_e, c1);
        for (int k = a; k < z; ++k) acc = cadd(acc, lds[k - c0]);
        __syncthreads();
    }
    return acc;
}

// the same with X given as split real / imaginary arrays
__device__ __forceinline__ double2 hc_tile_spmv_split(int r0, int N, const int *__restrict__ rowptr,
                                                      const int *__restrict__ col, const double *__restrict__ val,
                                                      const double *__restrict__ val_im,
                                                      const double *__restrict__ Xr, const double *__restrict__ Xi,
                                                      double2 *lds)
{
    const int r = r0 + threadIdx.x;
    const int rend = min(r0 + kCgBlock, N);
    const int s = rowptr[r0], e = rowptr[rend];
    const int my_s = (r < N) ? rowptr[r] : 0, my_e = (r < N) ? rowptr[r + 1] : 0;
    double2 acc = cx(0, 0);
    for (int c0 = s; c0 < e; c0 += kHcCap) {
        const int c1 = min(e, c0 + kHcCap);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int k = c0 + threadIdx.x + m * kCgBlock;
            if (k < c1) {
                const int j = col[k];
                lds[k - c0] = cmul(cx(val[k], val_im[k]), cx(Xr[j], Xi[j]));
            }
        }
        __syncthreads();
        const int a = max(my_s, c0), z = min(my_e, c1);
        for (int k = a; k < z; ++k) acc = cadd(acc, lds[k - c0]);
        __syncthreads();
    }
    return acc;
}

// sums of NV values over the workgroup, broadcast
template <int NV>
__device__ __forceinline__ void hc_block_sum(double (&v)[NV], double *red)
{
#pragma unroll
    for (int q = 0; q < NV; ++q) v[q] = cg_wave_sum(v[q]);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0)
#pragma unroll
        for (int q = 0; q < NV; ++q) red[NV * wid + q] = v[q];
    __syncthreads();
    const int nw = blockDim.x >> 6;
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        double t = 0.0;
        for (int w = 0; w < nw; ++w) t += red[NV * w + q];
        v[q] = t;
    }
}

struct HcArgs {
    int N;
    const int *rowptr, *col;
    const double *val, *val_im;
    double2 *x, *r, *u, *w, *z, *p;
    const double2 *dinv;
    double *part;     // kHcParts arrays of G (written)
    const double *part_rd;   // what the update reads: part, or its sum over the ranks (sharded)
    int G;
    int Gred;         // partial entries the update reduces (0: the local grids)
    CcgState *S;
    // AMG mode: the real V-cycle preconditions real and imaginary parts; r is
    // also written split (r_re, r_im), u comes back split (u_re, u_im)
    int amg;
    double *r_re, *r_im;
    const double *u_re, *u_im;
};

// r = b - A x0, u = M^-1 r, z = p = 0; partials gamma_0, |r0|^2, |b|^2.
// WARM: x0 is the current iterate (later passes of the nonlinear loop:
// PBCGSolveMod(Iter > 0) keeps V), else x0 = 0
template <bool WARM>
__global__ void __launch_bounds__(kCgBlock) k_hc_init(HcArgs A, const double *__restrict__ b,
                                                      const double *__restrict__ b_im)
{
    __shared__ double red[4 * (kCgBlock / 64) + 4];
    __shared__ double2 lds[WARM ? kHcCap : 1];
    const int i = blockIdx.x * kCgBlock + threadIdx.x;
    double2 ax = cx(0, 0);
    if (WARM) ax = hc_tile_spmv(blockIdx.x * kCgBlock, A.N, A.rowptr, A.col, A.val, A.val_im, A.x, lds);
    double v[4] = {0, 0, 0, 0};
    double bb = 0;
    if (i < A.N) {
        const double2 bi = cx(b[i], b_im[i]);
        const double2 rr = WARM ? csub(bi, ax) : bi;
        bb = bi.x * bi.x + bi.y * bi.y;
        if (!WARM) A.x[i] = cx(0, 0);
        A.r[i] = rr;
        A.z[i] = cx(0, 0);
        A.p[i] = cx(0, 0);
        if (A.amg) {   // u and gamma_0 come from the V-cycle and the SpMV
            A.r_re[i] = rr.x;
            A.r_im[i] = rr.y;
        } else {
            const double2 u = cmul(A.dinv[i], rr);
            A.u[i] = u;
            const double2 g = cmul(rr, u);
            v[0] = g.x;
            v[1] = g.y;
        }
        v[2] = rr.x * rr.x + rr.y * rr.y;
    }
    double s4[4] = {v[0], v[1], v[2], bb};
    hc_block_sum<4>(s4, red);
    if (threadIdx.x == 0) {
        if (!A.amg) {
            A.part[0 * A.G + blockIdx.x] = s4[0];
            A.part[1 * A.G + blockIdx.x] = s4[1];
        }
        A.part[6 * A.G + blockIdx.x] = s4[2];
        A.part[8 * A.G + blockIdx.x] = s4[3];
    }
}

// nonlinear loop: sum |V - V_old|^2 and |V|^2 over the nodes (harmonic2d.cpp:831-845)
__global__ void __launch_bounds__(256) k_hres(int N, const double2 *__restrict__ V, const double2 *__restrict__ Vo,
                                              double *__restrict__ part)
{
    __shared__ double red[2 * 4 + 2];
    double s2[2] = {0, 0};
    for (int i = blockIdx.x * 256 + threadIdx.x; i < N; i += gridDim.x * 256) {
        const double2 d = csub(V[i], Vo[i]), v = V[i];
        s2[0] += d.x * d.x - d.y * (-d.y);
        s2[1] += v.x * v.x - v.y * (-v.y);
    }
    hc_block_sum<2>(s2, red);
    if (threadIdx.x == 0) {
        part[blockIdx.x] = s2[0];
        part[gridDim.x + blockIdx.x] = s2[1];
    }
}
// Case-2 border: per-block partials of C . y (unconjugated, C split re / im)
__global__ void __launch_bounds__(256) k_hc_cdot(int N, const double *__restrict__ cr, const double *__restrict__ ci,
                                                 const double2 *__restrict__ y, double *__restrict__ part)
{
    __shared__ double red[2 * 4 + 2];
    double s2[2] = {0, 0};
    for (int i = blockIdx.x * 256 + threadIdx.x; i < N; i += gridDim.x * 256) {
        const double2 t = cmul(cx(cr[i], ci[i]), y[i]);
        s2[0] += t.x;
        s2[1] += t.y;
    }
    hc_block_sum<2>(s2, red);
    if (threadIdx.x == 0) {
        part[blockIdx.x] = s2[0];
        part[gridDim.x + blockIdx.x] = s2[1];
    }
}
// x = y0 - sum_q Y_q u_q (Y_q at stride ld: node vectors with the halo's room)
__global__ void k_hc_border_combine(int N, int nc2, const double2 *__restrict__ y0, const double2 *__restrict__ Y,
                                    int ld, const double2 *__restrict__ u, double2 *__restrict__ x)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    double2 v = y0[i];
    for (int q = 0; q < nc2; ++q) v = csub(v, cmul(Y[(size_t)q * ld + i], u[q]));
    x[i] = v;
}

// y += sign sum_q C_q u_q (the border columns applied to the circuit unknowns)
__global__ void k_hc_add_cu(int N, int nc2, const double *__restrict__ Cb, const double2 *__restrict__ u,
                            double sign, double2 *__restrict__ y)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    double2 a = y[i];
    for (int q = 0; q < nc2; ++q) {
        const double2 t = cmul(cx(Cb[2 * (size_t)q * N + i], Cb[2 * (size_t)q * N + N + i]), u[q]);
        a = cx(a.x + sign * t.x, a.y + sign * t.y);
    }
    y[i] = a;
}

// V = Relax V + (1 - Relax) V_old (harmonic2d.cpp:851)
__global__ void k_hrelax(int N, double relax, double2 *__restrict__ V, const double2 *__restrict__ Vo)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const double2 v = V[i], o = Vo[i];
    V[i] = cx(relax * v.x + (1.0 - relax) * o.x, relax * v.y + (1.0 - relax) * o.y);
}

// w = A u; partials delta = u.w (unconjugated).  AMG mode: u is gathered from
// the V-cycle's split output (and stored interleaved for the update kernel),
// and gamma = r.u goes to the partial arrays of parity gpar
__global__ void __launch_bounds__(kCgBlock) k_hc_spmv(HcArgs A, int gpar)
{
    if (A.S->done) return;
    __shared__ __attribute__((aligned(16))) double2 lds[kHcCap];
    __shared__ double red[4 * (kCgBlock / 64)];
    const int r0 = blockIdx.x * kCgBlock;
    const int i = r0 + threadIdx.x;
    double2 w;
    if (A.amg) {
        const double *ur = A.u_re, *ui = A.u_im;
        w = hc_tile_spmv_split(r0, A.N, A.rowptr, A.col, A.val, A.val_im, ur, ui, lds);
    } else {
        w = hc_tile_spmv(r0, A.N, A.rowptr, A.col, A.val, A.val_im, A.u, lds);
    }
    double s4[4] = {0, 0, 0, 0};
    if (i < A.N) {
        A.w[i] = w;
        const double2 u = A.amg ? cx(A.u_re[i], A.u_im[i]) : A.u[i];
        if (A.amg) A.u[i] = u;
        const double2 d = cmul(u, w);
        s4[0] = d.x;
        s4[1] = d.y;
        if (A.amg) {
            const double2 g = cmul(A.r[i], u);
            s4[2] = g.x;
            s4[3] = g.y;
        }
    }
    hc_block_sum<4>(s4, red);
    if (threadIdx.x == 0) {
        A.part[4 * A.G + blockIdx.x] = s4[0];
        A.part[5 * A.G + blockIdx.x] = s4[1];
        if (A.amg) {
            A.part[(2 * gpar) * A.G + blockIdx.x] = s4[2];
            A.part[(2 * gpar + 1) * A.G + blockIdx.x] = s4[3];
        }
    }
}

// iteration `it`: reduce gamma_it, delta_it, |r_it|^2 (and |b|^2) -> alpha,
// beta, the reference's stop test |r| / |b| <= Precision; then
// z = w + beta z, p = u + beta p, x += alpha p, r -= alpha z, u = M^-1 r,
// partials gamma_it+1, |r_it+1|^2
__global__ void __launch_bounds__(kHcAxBlock) k_hc_axpy(HcArgs A, long long it, int Ggam, int Grr)
{
    __shared__ double red[5 * (kHcAxBlock / 64)];
    CcgState *S = A.S;
    if (S->done) return;
    const int par = (int)(it & 1);
    double s5[5] = {0, 0, 0, 0, 0};
    const int Gcg = A.Gred ? A.Gred : (A.N + kCgBlock - 1) / kCgBlock;
    const double *pr = A.part_rd;
    for (int k = threadIdx.x; k < Ggam; k += blockDim.x) {
        s5[0] += pr[(2 * par) * A.G + k];
        s5[1] += pr[(2 * par + 1) * A.G + k];
    }
    for (int k = threadIdx.x; k < Grr; k += blockDim.x) s5[2] += pr[(6 + par) * A.G + k];
    for (int k = threadIdx.x; k < Gcg; k += blockDim.x) {
        s5[3] += pr[4 * A.G + k];
        s5[4] += pr[5 * A.G + k];
    }
    hc_block_sum<5>(s5, red);
    const double2 gam = cx(s5[0], s5[1]), del = cx(s5[3], s5[4]);
    const double rr = s5[2];
    double bb;
    if (it == 0) {
        double sb[1] = {0};
        for (int k = threadIdx.x; k < Gcg; k += blockDim.x) sb[0] += pr[8 * A.G + k];
        hc_block_sum<1>(sb, red);
        bb = sb[0];
    } else {
        bb = S->bb;
    }
    double2 beta = cx(0, 0), alpha;
    if (it == 0) {
        alpha = cdiv(gam, del);
    } else {
        const double2 gp = cx(S->gam[(it - 1) & 1][0], S->gam[(it - 1) & 1][1]);
        const double2 ap = cx(S->alp[(it - 1) & 1][0], S->alp[(it - 1) & 1][1]);
        beta = cdiv(gam, gp);
        alpha = cdiv(gam, csub(del, cdiv(cmul(beta, gam), ap)));
    }
    const double er = (bb == 0.0) ? 0.0 : sqrt(rr / bb);
    const bool stop = (bb == 0.0) || (it >= 1 && er <= S->tol);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (it == 0) S->bb = bb;
        S->er = er;
        S->iters = it;
        if (stop) S->done = 1;
        S->gam[it & 1][0] = gam.x;
        S->gam[it & 1][1] = gam.y;
        S->alp[it & 1][0] = alpha.x;
        S->alp[it & 1][1] = alpha.y;
    }
    if (stop) return;
    double g[3] = {0, 0, 0};
    if (A.amg) {   // u = M^-1 r by the V-cycle after this launch: r also split
        for (int i = blockIdx.x * kHcAxBlock + threadIdx.x; i < A.N; i += gridDim.x * kHcAxBlock) {
            const double2 z = cadd(A.w[i], cmul(beta, A.z[i]));
            const double2 pp = cadd(A.u[i], cmul(beta, A.p[i]));
            const double2 rn = csub(A.r[i], cmul(alpha, z));
            A.x[i] = cadd(A.x[i], cmul(alpha, pp));
            A.z[i] = z;
            A.p[i] = pp;
            A.r[i] = rn;
            A.r_re[i] = rn.x;
            A.r_im[i] = rn.y;
            g[2] += rn.x * rn.x + rn.y * rn.y;
        }
        hc_block_sum<3>(g, red);
        if (threadIdx.x == 0) A.part[(6 + (int)((it + 1) & 1)) * A.G + blockIdx.x] = g[2];
        return;
    }
    for (int i = blockIdx.x * kHcAxBlock + threadIdx.x; i < A.N; i += gridDim.x * kHcAxBlock) {
        const double2 z = cadd(A.w[i], cmul(beta, A.z[i]));
        const double2 pp = cadd(A.u[i], cmul(beta, A.p[i]));
        const double2 rn = csub(A.r[i], cmul(alpha, z));
        const double2 u = cmul(A.dinv[i], rn);
        A.x[i] = cadd(A.x[i], cmul(alpha, pp));
        A.z[i] = z;
        A.p[i] = pp;
        A.r[i] = rn;
        A.u[i] = u;
        const double2 gg = cmul(rn, u);
        g[0] += gg.x;
        g[1] += gg.y;
        g[2] += rn.x * rn.x + rn.y * rn.y;
    }
    hc_block_sum<3>(g, red);
    if (threadIdx.x == 0) {
        const int np = (int)((it + 1) & 1);
        A.part[(2 * np) * A.G + blockIdx.x] = g[0];
        A.part[(2 * np + 1) * A.G + blockIdx.x] = g[1];
        A.part[(6 + np) * A.G + blockIdx.x] = g[2];
    }
}

// the real SPD surrogate the AMG hierarchy is built on: Re A + sgn Im A with
// the sign that makes the imaginary part (eddy-current mass, loss terms)
// positive semi-definite, so that the surrogate is spectrally equivalent to A
__global__ void k_hc_surrogate(int N, double sgn, const int *__restrict__ rowptr, const int *__restrict__ col,
                               const double *__restrict__ val, const double *__restrict__ val_im,
                               double *__restrict__ out)
{
    // positive off-diagonal parts of sgn Im A (the consistent eddy-current
    // mass) are lumped onto the diagonal: B stays definite (negative definite
    // in FEMM's sign convention: Re A has a negative diagonal and positive
    // couplings), within a factor of two of the unlumped surrogate, and keeps
    // the sign pattern the aggregation's strength test (relative to the
    // diagonal's sign) and the Jacobi smoother expect
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    double lump = 0;
    int kd = -1;
    for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) {
        const double m = sgn * val_im[k];
        if (col[k] == i) {
            kd = k;
            out[k] = val[k] + m;
        } else if (m > 0) {
            lump += m;
            out[k] = val[k];
        } else {
            out[k] = val[k] + m;
        }
    }
    if (kd >= 0) out[kd] += lump;
}
// per-block sums of the imaginary diagonal (its sign picks sgn above)
__global__ void __launch_bounds__(256) k_hc_diag_im(int N, const int *__restrict__ diag,
                                                    const double *__restrict__ val_im, double *__restrict__ part)
{
    __shared__ double red[4];
    const int i = blockIdx.x * 256 + threadIdx.x;
    double v = (i < N) ? val_im[diag[i]] : 0.0;
    v = cg_wave_sum(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ---- Newton AC solver: KludgeSolve (cspars.cpp:1000-1060) kernels ----
// mode 0: Y = F(X) = M X + Mh X + Ms conj(X) + Ma X   (MultA(X, Y, -1))
// mode 1: (ore, oim) = b0 - (Mh X + Ms conj(X) + Ma X) (the right-hand side of the inner solve)
// mode 2: Y = b0 - F(X)                               (the true residual)
__global__ void __launch_bounds__(256) k_hk_apply(int N, const int *__restrict__ rowptr, const int *__restrict__ col,
                                                  const double *__restrict__ val, const double *__restrict__ val_im,
                                                  const double *__restrict__ aux, long long nnz,
                                                  const double2 *__restrict__ X, const double2 *__restrict__ b0,
                                                  int mode, double2 *__restrict__ Y, double *__restrict__ ore,
                                                  double *__restrict__ oim)
{
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= N) return;
    const double *hr = aux, *hi = aux + nnz, *sr = aux + 2 * nnz, *si = aux + 3 * nnz, *ar = aux + 4 * nnz,
                 *ai = aux + 5 * nnz;
    double2 m = cx(0, 0), q = cx(0, 0);
    for (int k = rowptr[r]; k < rowptr[r + 1]; ++k) {
        const double2 x = X[col[k]];
        if (mode != 1) m = cadd(m, cmul(cx(val[k], val_im[k]), x));
        q = cadd(q, cmul(cx(hr[k] + ar[k], hi[k] + ai[k]), x));
        q = cadd(q, cmul(cx(sr[k], si[k]), cx(x.x, -x.y)));
    }
    if (mode == 0) {
        Y[r] = cadd(m, q);
    } else if (mode == 1) {
        const double2 t = csub(b0[r], q);
        ore[r] = t.x;
        oim[r] = t.y;
    } else {
        Y[r] = csub(b0[r], cadd(m, q));
    }
}
// partials of Re(conj(a) . b), |b|^2, |a|^2 (ConjDot, the norms)
__global__ void __launch_bounds__(256) k_hk_dots(int N, const double2 *__restrict__ a, const double2 *__restrict__ b,
                                                 double *__restrict__ part)
{
    __shared__ double red[3 * 4 + 3];
    double s3[3] = {0, 0, 0};
    for (int i = blockIdx.x * 256 + threadIdx.x; i < N; i += gridDim.x * 256) {
        const double2 x = a[i], y = b[i];
        s3[0] += x.x * y.x + x.y * y.y;
        s3[1] += y.x * y.x + y.y * y.y;
        s3[2] += x.x * x.x + x.y * x.y;
    }
    hc_block_sum<3>(s3, red);
    if (threadIdx.x == 0) {
        part[blockIdx.x] = s3[0];
        part[gridDim.x + blockIdx.x] = s3[1];
        part[2 * gridDim.x + blockIdx.x] = s3[2];
    }
}
// P = V - v (the step of the inner solve)
__global__ void k_hk_diff(int N, const double2 *__restrict__ V, const double2 *__restrict__ v, double2 *__restrict__ P)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) P[i] = csub(V[i], v[i]);
}
// line search step: V = v + c P, r -= c U, v = V
__global__ void k_hk_update(int N, double c, double2 *__restrict__ V, double2 *__restrict__ v,
                            const double2 *__restrict__ P, double2 *__restrict__ r, const double2 *__restrict__ U)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const double2 x = cadd(v[i], cscale(P[i], c));
    V[i] = x;
    v[i] = x;
    r[i] = csub(r[i], cscale(U[i], c));
}
// b (split) -> interleaved
__global__ void k_hk_join(int N, const double *__restrict__ re, const double *__restrict__ im, double2 *__restrict__ o)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) o[i] = cx(re[i], im[i]);
}

inline int nb256(long long n) { return (int)((n + kBlock - 1) / kBlock); }
int hc_axpy_grid(int N)
{
    int g = (N + kHcAxBlock - 1) / kHcAxBlock;
    return g < 1 ? 1 : (g < kHcAxGrid ? g : kHcAxGrid);
}

// ---- host: effective permeability and boundary constants (harmonic2d.cpp) ----
using hcx = std::complex<double>;
inline double2 h2(hcx z) { return cx(z.real(), z.imag()); }
inline hcx hc(double2 z) { return hcx(z.x, z.y); }

// the lag angle argument -I Theta DEG (harmonic2d.cpp) or -I Theta PI / 180
// (harmonicaxi.cpp:133-151), halved for the lamination half-lag
double2 lag_arg(double theta, bool axi, bool half)
{
    if (axi) return half ? cx(-0.0 * theta * kPI / 360., -theta * kPI / 360.) : cx(-0.0 * theta * kPI / 180., -theta * kPI / 180.);
    return half ? cx(-0.0 * theta * kDEG / 2., -theta * kDEG / 2.) : cx(-0.0 * theta * kDEG, -theta * kDEG);
}

DevBlockAC effective_block(const xfk_block_desc &b, const xfk_block_ac_desc &ac, double w, bool axi)
{
    // harmonic2d.cpp:190-235 / harmonicaxi.cpp:128-170 with femmcomplex.cpp's
    // exp / tanh / quotient formulas
    DevBlockAC o{};
    const double2 deg45 = cx(1, 1);
    double2 m0, m1;
    if (b.LamType == 0) {
        m0 = cscale(cexp_(lag_arg(ac.Theta_hx, axi, false)), b.mu_x);
        m1 = cscale(cexp_(lag_arg(ac.Theta_hy, axi, false)), b.mu_y);
        if (ac.Lam_d != 0) {
            if (b.Cduct != 0) {
                double2 halflag = cexp_(lag_arg(ac.Theta_hx, axi, true));
                double ds = sqrt(2. / (0.4 * kPI * w * b.Cduct * b.mu_x));
                double2 K = cscale(cscale(cmul(halflag, deg45), ac.Lam_d), 0.001);
                K = cx(K.x / (2. * ds), K.y / (2. * ds));
                m0 = cscale(cdiv(cmul(m0, ctanh_(K)), K), b.LamFill);
                m0.x += (1. - b.LamFill);
                halflag = cexp_(lag_arg(ac.Theta_hy, axi, true));
                ds = sqrt(2. / (0.4 * kPI * w * b.Cduct * b.mu_y));
                K = cscale(cscale(cmul(halflag, deg45), ac.Lam_d), 0.001);
                K = cx(K.x / (2. * ds), K.y / (2. * ds));
                m1 = cscale(cdiv(cmul(m1, ctanh_(K)), K), b.LamFill);
                m1.x += (1. - b.LamFill);
            } else {
                m0 = cscale(m0, b.LamFill);
                m0.x += (1. - b.LamFill);
                m1 = cscale(m1, b.LamFill);
                m1.x += (1. - b.LamFill);
            }
        }
    } else {
        m0 = cx(1, 0);
        m1 = cx(1, 0);
    }
    o.mu1 = m0;
    o.mu2 = m1;
    o.J = cx(b.J_re, ac.J_im);
    o.Cduct = b.Cduct;
    o.eddy = !((b.LamType == 0) && (ac.Lam_d > 0));
    o.prox = b.LamType > 2;
    return o;
}

}  // namespace

}  // namespace xfk

using namespace xfk;

namespace {

int harmonic_validate(const xfk_problem_desc *d, const xfk_harmonic_desc *ac)
{
    XFK_REQUIRE(ac && ac->frequency > 0, XFK_ERR_ARG, "harmonic problems need a frequency > 0");
    XFK_REQUIRE(ac->ac_solver == 0 || ac->ac_solver == 1, XFK_ERR_ARG, "ac_solver must be 0 or 1");
    XFK_REQUIRE(d->n_blocks == 0 || ac->blocks, XFK_ERR_ARG, "missing AC block table");
    XFK_REQUIRE(d->n_lines == 0 || ac->lines, XFK_ERR_ARG, "missing AC boundary table");
    XFK_REQUIRE(d->n_circs == 0 || ac->circs, XFK_ERR_ARG, "missing AC circuit table");
    for (int k = 0; k < d->n_blocks; ++k) {
        if (d->blocks[k].BHpoints > 0) {
            XFK_REQUIRE(ac->blocks[k].H_im && ac->blocks[k].slope_im && d->blocks[k].B && d->blocks[k].H &&
                            d->blocks[k].slope && d->blocks[k].BHpoints >= 2,
                        XFK_ERR_ARG, "nonlinear harmonic block needs its complex B-H curve (GetSlopes(omega))");
        }
        XFK_REQUIRE(d->blocks[k].LamType != 1 && d->blocks[k].LamType != 2, XFK_ERR_UNSUPPORTED,
                    "On-edge lamination not supported in AC analyses");   // harmonic2d.cpp:76-85
    }
    return XFK_OK;
}

}  // namespace

namespace {

// the harmonic problem of one device (comm == nullptr) or of comm's rank
int create_harmonic(const xfk_problem_desc *d, const xfk_harmonic_desc *ac, int device, xfk_comm *comm,
                    xfk_problem **out)
{
    XFK_REQUIRE(d && out, XFK_ERR_ARG, "null argument");
    *out = nullptr;
    int rc = validate_desc(d);
    if (rc == XFK_OK) rc = harmonic_validate(d, ac);
    if (rc == XFK_OK) rc = check_device(device);
    if (rc != XFK_OK) return rc;
    const int N = d->n_nodes, NE = d->n_elems;
    const double c = kC, w = ac->frequency * 2. * kPI;
    const double units[] = {2.54, 0.1, 1., 100., 0.00254, 1.e-04};
    GlobalPrep G;
    prepare_global(d, G);
    G.pbc_aux = ac->ac_solver == 1;   // (the Newton AC solver's auxiliary matrices go through the periodic map)
    rc = age_entries(d, -1.0, G.age_key, G.age_val);   // air-gap elements, negated (harmonic2d.cpp:227-382)
    if (rc != XFK_OK) return rc;
    const bool axi = G.axi;   // HarmonicAxisymmetric (harmonicaxi.cpp)

    // blocks, lines
    std::vector<DevBlockAC> blk(std::max(1, d->n_blocks));
    std::vector<double> bhB;
    std::vector<double2> bhH, bhS;
    for (int k = 0; k < d->n_blocks; ++k) {
        blk[k] = effective_block(d->blocks[k], ac->blocks[k], w, axi);
        const xfk_block_desc &b = d->blocks[k];
        // only LamType 0 blocks follow their curve (harmonic2d.cpp:598-600)
        if (b.BHpoints > 0 && b.LamType == 0) {   // the complex curve of GetSlopes(omega)
            blk[k].bh_n = b.BHpoints;
            blk[k].bh_off = (int)bhB.size();
            for (int i = 0; i < b.BHpoints; ++i) {
                bhB.push_back(b.B[i]);
                bhH.push_back(cx(b.H[i], ac->blocks[k].H_im[i]));
                bhS.push_back(cx(b.slope[i], ac->blocks[k].slope_im[i]));
            }
        }
    }
    // the reference starts its successive approximation when any element
    // lies in a block with a B-H curve (harmonic2d.cpp:559-569)
    bool nonlin = false;
    for (int i = 0; i < NE && !nonlin; ++i) nonlin = d->blocks[G.lab[d->lbl[i]].blk].BHpoints > 0;
    // proximity-effect permeabilities of wound LamType > 2 regions
    for (size_t k = 0; k < G.lab.size(); ++k)
        G.lab[k].prox_mu = ac->label_prox_mu ? cx(ac->label_prox_mu[2 * k], ac->label_prox_mu[2 * k + 1]) : cx(1, 0);
    if (bhB.empty()) {
        bhB.push_back(0.0);
        bhH.push_back(cx(0, 0));
        bhS.push_back(cx(0, 0));
    }
    std::vector<DevLineAC> lin(std::max<size_t>(1, G.lin_used.size()));   // compact, as the edge fields
    for (size_t m = 0; m < G.lin_used.size(); ++m) {
        const int k = G.lin_used[m];
        DevLineAC &o = lin[m];
        const xfk_line_desc &l = d->lines[k];
        o.format = l.format;
        o.c0 = cx(l.c0, ac->lines[k].c0_im);
        o.c1 = cx(l.c1, ac->lines[k].c1_im);
        o.zs = cx(0, 0);
        if (l.format == 1) {   // harmonic2d.cpp:424-437
            const double Mu = ac->lines[k].Mu, Sig = ac->lines[k].Sig;
            XFK_REQUIRE(Mu > 0 && Sig > 0, XFK_ERR_ARG, "small-skin-depth boundary needs Mu > 0 and Sig > 0");
            const double ds = sqrt(2. / (0.4 * kPI * w * Sig * Mu));
            const double den = -ds * Mu * 100.;
            o.zs = cx(1. / den, 1. / den);
        }
    }
    // circuits (harmonic2d.cpp:86-170)
    std::vector<DevCircAC> circ(std::max(1, d->n_circs));
    if (d->n_circs > 0) {
        std::vector<hcx> I1(d->n_circs), I2(d->n_circs), I3(d->n_circs);
        for (int i = 0; i < NE; ++i) {
            const DevLabel &L = G.lab[d->lbl[i]];
            if (L.in_circuit == -1) continue;
            const int *n = d->p + 3LL * i;
            double p0 = d->y[n[1]] - d->y[n[2]], p1 = d->y[n[2]] - d->y[n[0]];
            double q0 = d->x[n[2]] - d->x[n[1]], q1 = d->x[n[0]] - d->x[n[2]];
            double a = (p0 * q1 - p1 * q0) / 2.;
            double Cduct = d->blocks[L.blk].Cduct;
            if (L.is_wound) Cduct = 0;
            I1[L.in_circuit] += a;
            if (axi) {   // conductivity / R (harmonicaxi.cpp:86-87)
                const double r = (d->x[n[0]] + d->x[n[1]] + d->x[n[2]]) / 3.;
                I2[L.in_circuit] += a * Cduct / (0.01 * r);
            } else {
                I2[L.in_circuit] += a * Cduct;
            }
            I3[L.in_circuit] += hc(blk[L.blk].J) * a * 100.;
        }
        for (int k = 0; k < d->n_circs; ++k) {
            DevCircAC &C = circ[k];
            C.J = cx(0, 0);
            C.dV = cx(0, 0);
            if (d->circs[k].type == 0) {
                if (I2[k] != 0.0) {   // Case 2: the voltage gradient is an extra unknown
                    C.ccase = 2;
                    continue;
                }
                C.ccase = 1;
                if (I1[k] != 0.0) {
                    const hcx amps(d->circs[k].amps_re, ac->circs[k].amps_im);
                    C.J = cdiv(h2(0.01 * (amps - I3[k])), h2(I1[k]));
                }
            } else {
                C.ccase = 0;
                C.dV = cx(d->circs[k].dvolts_re, ac->circs[k].dvolts_im);
            }
        }
    }
    // point currents and complex Dirichlet values, in SetValue order
    std::vector<int> pt_nodes;
    std::vector<double> pt_J;
    std::vector<unsigned char> fixed(N, 0);
    std::vector<double> first(2 * (size_t)N, 0.0), last(2 * (size_t)N, 0.0);
    auto set_value = [&](int i, hcx x) {
        if (!fixed[i]) {
            first[2 * i] = x.real();
            first[2 * i + 1] = x.imag();
        }
        fixed[i] = 1;
        last[2 * i] = x.real();
        last[2 * i + 1] = x.imag();
    };
    auto marker = [&](int i) { return d->marker ? d->marker[i] : -1; };
    for (int i = 0; i < N; ++i) {
        int m = marker(i);
        if (m >= 0 && (d->points[m].J_re != 0 || d->points[m].J_im != 0)) {   // harmonic2d.cpp:634-641
            pt_nodes.push_back(i);
            const double s = axi ? (2. * d->x[i] * 0.01) : 0.01;   // harmonicaxi.cpp:610-617
            pt_J.push_back(-(s * d->points[m].J_re));
            pt_J.push_back(-(s * d->points[m].J_im));
        }
    }
    for (int i = 0; i < N; ++i) {
        int m = marker(i);
        if (axi && d->x[i] < (units[d->length_units] * 1.e-06)) {   // A = 0 on the axis (harmonicaxi.cpp:626-631)
            set_value(i, hcx(0, 0));
            continue;
        }
        if (m >= 0 && d->points[m].J_re == 0 && d->points[m].J_im == 0)
            set_value(i, hcx(d->points[m].A_re, d->points[m].A_im) / c);
    }
    auto edge = [&](long long k) { return d->e ? d->e[k] : -1; };
    for (int i = 0; i < NE; ++i)
        for (int j = 0; j < 3; ++j) {
            int k = (j + 1) % 3;
            int sgi = edge(3LL * i + j);
            if (sgi < 0 || d->lines[sgi].format != 0) continue;
            const xfk_line_desc &ln = d->lines[sgi];
            int nodes2[2] = {d->p[3LL * i + j], d->p[3LL * i + k]};
            for (int m = 0; m < 2; ++m) {
                double x = d->x[nodes2[m]], y = d->y[nodes2[m]], a;
                if (d->coords == 0) {
                    x /= units[d->length_units];
                    y /= units[d->length_units];
                    a = ln.A0 + x * ln.A1 + y * ln.A2;
                } else {
                    double r = sqrt(x * x + y * y), t;
                    if ((x == 0) && (y == 0)) t = 0;
                    else t = atan2(y, x) / kDEG;
                    r /= units[d->length_units];
                    a = ln.A0 + r * ln.A1 + t * ln.A2;
                }
                const double2 e = cexp_(cx(0.0 * ln.phi * kDEG, ln.phi * kDEG));
                set_value(nodes2[m], hcx((a / c) * e.x, (a / c) * e.y));   // harmonic2d.cpp:664-730
            }
        }
    for (int i = 0; i < N; ++i)
        XFK_REQUIRE((fixed[i] != 0) == (G.fixed[i] != 0), XFK_ERR_ARG, "internal: Dirichlet node sets differ");

    // Case-2 circuits: the border of the system (harmonic2d.cpp:441-472, 644-650;
    // harmonicaxi.cpp:385-417, 619-623) -- column C_k over the nodes of the
    // circuit's region, diagonal D_k, right-hand side f_k -- depends only on the
    // geometry, so it is built here once; SetValue moves the fixed nodes'
    // column entries (first value) to f_k
    std::vector<int> c2;   // circuit index of each bordered unknown
    for (int k = 0; k < d->n_circs; ++k)
        if (circ[k].ccase == 2) c2.push_back(k);
    const int nc2 = (int)c2.size();
    std::vector<double> Cb(2 * (size_t)nc2 * N, 0.0);   // per unknown: N re, then N im
    std::vector<double2> Db(nc2, cx(0, 0)), fb(nc2, cx(0, 0));
    if (nc2 > 0) {
        std::vector<int> slot(std::max(1, d->n_circs), -1);
        for (int q = 0; q < nc2; ++q) slot[c2[q]] = q;
        for (int i = 0; i < NE; ++i) {
            const DevLabel &L = G.lab[d->lbl[i]];
            if (L.in_circuit < 0 || circ[L.in_circuit].ccase != 2) continue;
            const int q = slot[L.in_circuit];
            const int *n = d->p + 3LL * i;
            const double p0 = d->y[n[1]] - d->y[n[2]], p1 = d->y[n[2]] - d->y[n[0]];
            const double q0 = d->x[n[2]] - d->x[n[1]], q1 = d->x[n[0]] - d->x[n[2]];
            const double a = (p0 * q1 - p1 * q0) / 2.;
            const double R = (d->x[n[0]] + d->x[n[1]] + d->x[n[2]]) / 3.;
            const double Cd = d->blocks[L.blk].Cduct;
            const double2 Jb = blk[L.blk].J;
            // source of the element, added once per node to the circuit row
            double2 Ks;
            if (axi) {
                const double s = -2. * R;
                Ks = cx(s * Jb.x * a / 3., s * Jb.y * a / 3.);
                Ks = cx(Ks.x / R, Ks.y / R);
            } else {
                Ks = cx((-Jb.x * a) / 3., (-Jb.y * a) / 3.);
            }
            for (int j = 0; j < 3; ++j) fb[q] = cadd(fb[q], Ks);
            // coupling -I a w sigma c (axi: -2 I a w sigma c)
            double2 Kc = axi ? cx(-2. * 0.0, -2. * 1.0) : cx(-0.0, -1.0);
            Kc = cx(Kc.x * a * w * Cd * c, Kc.y * a * w * Cd * c);
            for (int j = 0; j < 3; ++j) {
                double *cr = &Cb[2 * (size_t)q * N], *ci = cr + N;
                cr[n[j]] += Kc.x / 3.;
                ci[n[j]] += Kc.y / 3.;
            }
            Db[q] = cadd(Db[q], axi ? cx(Kc.x / R, Kc.y / R) : Kc);
        }
        for (int q = 0; q < nc2; ++q) {
            const int k = c2[q];
            const double s = axi ? 2. * 0.01 : 0.01;
            fb[q] = cadd(fb[q], cx(s * d->circs[k].amps_re, s * ac->circs[k].amps_im));
            double *cr = &Cb[2 * (size_t)q * N], *ci = cr + N;
            for (int i = 0; i < N; ++i)
                if (fixed[i] && (cr[i] != 0 || ci[i] != 0)) {
                    fb[q] = csub(fb[q], cmul(cx(cr[i], ci[i]), cx(first[2 * i], first[2 * i + 1])));
                    cr[i] = 0;
                    ci[i] = 0;
                }
            // then the periodic / antiperiodic pairs, in pbclist order: their
            // loops over the rows of the whole bordered matrix reach the
            // circuit's row too (cspars.cpp:677-716 Periodicity, 592-640
            // AntiPeriodicity: rows k >= NumNodes after the band), averaging
            // the border column at the pair's two nodes; D_k and f_k stay
            for (int k2 = 0; k2 < d->n_pbc; ++k2) {
                int i = d->pbc[3 * k2], j = d->pbc[3 * k2 + 1];
                const int t = d->pbc[3 * k2 + 2];
                if (t != 0 && t != 1) continue;
                if (j < i) std::swap(i, j);
                const double2 v1 = cx(cr[i], ci[i]), v2 = cx(cr[j], ci[j]);
                if (v1.x == 0 && v1.y == 0 && v2.x == 0 && v2.y == 0) continue;
                if (t == 0) {
                    const double2 h = cx((v1.x + v2.x) / 2., (v1.y + v2.y) / 2.);
                    cr[i] = cr[j] = h.x;
                    ci[i] = ci[j] = h.y;
                } else {
                    const double2 h = cx((v1.x - v2.x) / 2., (v1.y - v2.y) / 2.);
                    cr[i] = h.x;
                    ci[i] = h.y;
                    cr[j] = -h.x;
                    ci[j] = -h.y;
                }
            }
        }
    }

    // sharded: the row-block plan, then the per-node tables in local numbering
    PartPlan plan;
    if (comm) {
        if ((rc = plan_rank(d, G, comm, plan)) != XFK_OK) return rc;
        const int NL = plan.n_own + plan.n_halo, NR = plan.n_own + plan.n_extra;
        if (nc2 > 0) {   // Case-2 border columns (made on the global numbering above): the owned rows
            const int no = plan.n_own;
            std::vector<double> Cl(2 * (size_t)nc2 * no);
            for (int q = 0; q < nc2; ++q)
                for (int l = 0; l < no; ++l) {
                    const size_t g = (size_t)plan.l2g[l];
                    Cl[2 * (size_t)q * no + l] = Cb[2 * (size_t)q * N + g];
                    Cl[2 * (size_t)q * no + no + l] = Cb[2 * (size_t)q * N + N + g];
                }
            Cb.swap(Cl);
        }
        std::vector<double> f2(2 * (size_t)NL), l2(2 * (size_t)NL);
        for (int l = 0; l < NL; ++l)
            for (int q = 0; q < 2; ++q) {
                f2[2 * (size_t)l + q] = first[2 * (size_t)plan.l2g[l] + q];
                l2[2 * (size_t)l + q] = last[2 * (size_t)plan.l2g[l] + q];
            }
        first.swap(f2);
        last.swap(l2);
        std::vector<int> g2l_row(N, -1);   // assembled rows (owned, then the coupled extra rows)
        for (int l = 0; l < NR; ++l) g2l_row[plan.l2g[l]] = l;
        std::vector<int> pn;
        std::vector<double> pj;
        for (size_t k = 0; k < pt_nodes.size(); ++k) {
            const int l = g2l_row[pt_nodes[k]];
            if (l < 0) continue;
            pn.push_back(l);
            pj.push_back(pt_J[2 * k]);
            pj.push_back(pt_J[2 * k + 1]);
        }
        pt_nodes.swap(pn);
        pt_J.swap(pj);
    }
    xfk_problem *P = nullptr;
    rc = build_local(d, G, comm ? &plan : nullptr, device, comm, &P);
    if (rc != XFK_OK) return rc;
    P->harmonic = true;
    P->omega = w;
    P->hc2_circ = c2;
    P->hc2_D = Db;
    P->hc2_f = fb;
    P->hc2_u.assign(nc2, cx(0, 0));
    P->any_nonlinear = nonlin;
    P->ac_solver = ac->ac_solver;
    P->axi = axi;
    if (axi) P->axi_x.assign(d->x, d->x + N);
    P->ext_ro = G.ext_ro;
    P->ext_ri = G.ext_ri;
    P->ext_zo = G.ext_zo;
    P->hcircs = circ;
    P->nhpt = (int)pt_nodes.size();
    hipStream_t s = P->stream;
    hipError_t e = hipSuccess;
#define UP(buf, ptr, n) if (e == hipSuccess) e = upload(buf, ptr, n, s)
    UP(P->blocks_ac, blk.data(), blk.size());
    UP(P->lines_ac, lin.data(), lin.size());
    UP(P->circs_ac, circ.data(), circ.size());
    UP(P->hpt_nodes, pt_nodes.data(), pt_nodes.size());
    UP(P->hpt_J, pt_J.data(), pt_J.size());
    UP(P->hfix_first, first.data(), first.size());
    UP(P->hfix_last, last.data(), last.size());
    UP(P->hbh_B, bhB.data(), bhB.size());
    if (nc2 > 0) UP(P->hc2_C, Cb.data(), Cb.size());
    UP(P->hbh_H, bhH.data(), bhH.size());
    UP(P->hbh_S, bhS.data(), bhS.size());
#undef UP
    if (e == hipSuccess) e = pinned_malloc((void **)&P->hc_host, sizeof(CcgState));
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        set_error(std::string("upload failed: ") + hipGetErrorString(e));
        xfk_problem_destroy(P);
        return XFK_ERR_HIP;
    }
    *out = P;
    return XFK_OK;
}

}  // namespace

namespace xfk {
static int harmonic2d_run(xfk_problem *P, int flags, xfk_result *res);
void problem_recycle(xfk_problem *P);
}

extern "C" {

int xfk_problem_create_harmonic(const xfk_problem_desc *d, const xfk_harmonic_desc *ac, int device,
                                xfk_problem **out)
{
    return create_harmonic(d, ac, device, nullptr, out);
}

int xfk_problem_create_harmonic_dist(const xfk_problem_desc *d, const xfk_harmonic_desc *ac, int device,
                                     xfk_comm *comm, xfk_problem **out)
{
    XFK_REQUIRE(comm, XFK_ERR_ARG, "null communicator");
    return create_harmonic(d, ac, device, comm, out);
}

int xfk_harmonic2d(xfk_problem *P, int flags, xfk_result *res)
{
    ArenaScope arena_scope(P ? &P->arena : nullptr);
    const int rc = harmonic2d_run(P, flags, res);
    problem_recycle(P);
    return rc;
}

}  // extern "C"

namespace xfk {
static int harmonic2d_run(xfk_problem *P, int flags, xfk_result *res)
{
    ArenaScope arena_scope(P ? &P->arena : nullptr);
    XFK_REQUIRE(P && P->harmonic, XFK_ERR_ARG, "not a harmonic problem (xfk_problem_create_harmonic)");
    XFK_CHECK(hipSetDevice(P->device));
    hipStream_t s = P->stream;
    ScopedEvents<3> ev;
    XFK_CHECK(ev.create());
    hipEvent_t e0 = ev[0], e1 = ev[1], e2 = ev[2];
    xfk_result R{};
    float ms = 0;
    XFK_CHECK(hipEventRecord(e0, s));
    if (!P->symbolic_ready || (flags & XFK_REBUILD_SYMBOLIC)) {
        P->symbolic_ready = false;
        int rc = build_symbolic(P);
        if (rc != XFK_OK) return rc;
    }
    XFK_CHECK(hipEventRecord(e1, s));
    XFK_CHECK(hipEventSynchronize(e1));
    XFK_CHECK(hipEventElapsedTime(&ms, e0, e1));
    R.ms_symbolic = ms;

    const int N = P->N, NL = P->NL;   // owned rows; local nodes (owned, then the halo)
    const long long nnz = P->nnz;
    // sharded (xfk_problem_create_harmonic_dist): row blocks as the static
    // path -- the halo of x / u exchanged before each SpMV (x: interleaved
    // complex; u: the V-cycle's split real / imaginary outputs), the
    // per-block partials all-reduced after each SpMV, the setup-time
    // decisions and the nonlinear residual summed over the ranks
    xfk_comm *comm = P->comm;
    XFK_CHECK(P->val.alloc((size_t)nnz));
    XFK_CHECK(P->val_im.alloc((size_t)nnz));
    const int NR = P->NR;   // assembled rows: owned, then (sharded, periodic) the coupled rows folded in
    XFK_CHECK(P->b.alloc((size_t)NR));
    XFK_CHECK(P->b_im.alloc((size_t)NR));
    const int Gcg = (N + kCgBlock - 1) / kCgBlock, Gax = hc_axpy_grid(N);
    int G = std::max(Gcg, Gax);
    if (comm)   // one partial layout for every rank: the largest block's grids
        for (int q = 0; q < P->nranks; ++q) {
            const int nq = (int)(row_begin(P->N_global, q + 1, P->nranks) - row_begin(P->N_global, q, P->nranks));
            G = std::max(G, std::max((nq + kCgBlock - 1) / kCgBlock, hc_axpy_grid(nq)));
        }
    if (comm && P->halo2.send.empty() && P->halo2.recv.empty()) {
        for (const HaloRange &h : P->halo.send) P->halo2.send.push_back(HaloRange{h.peer, 2 * h.off, 2 * h.len, h.g0});
        for (const HaloRange &h : P->halo.recv) P->halo2.recv.push_back(HaloRange{h.peer, 2 * h.off, 2 * h.len, h.g0});
    }
    XFK_CHECK(P->hc_vec.alloc(7 * (size_t)NL));
    XFK_CHECK(P->hc_part.alloc((comm ? 2 : 1) * (size_t)kHcParts * G));
    XFK_CHECK(P->hc_state.alloc(1));
    XFK_CHECK(P->hc_split.alloc(4 * (size_t)NL));
    double2 *v = P->hc_vec.p;
    auto exch_c = [&](double2 *vec) -> int {   // halo of an interleaved complex node vector
        return comm ? comm->exchange(P->halo2, reinterpret_cast<double *>(vec), s) : XFK_OK;
    };
    auto exch_r = [&](double *vec) -> int { return comm ? comm->exchange(P->halo, vec, s) : XFK_OK; };
    auto reduce_parts = [&]() -> int {
        return comm ? comm->allreduce_sum(P->hc_part.p, P->hc_part.p + (size_t)kHcParts * G, (size_t)kHcParts * G, s)
                    : XFK_OK;
    };
    const bool nonlin = P->any_nonlinear;
    constexpr int kResGrid = 256;
    // Newton AC solver: auxiliary matrices from the second pass on (the
    // reference's bNewton, set by the first auxiliary Put)
    const bool ac1 = nonlin && P->ac_solver == 1;
    const bool trace = std::getenv("XFK_TRACE_NONLINEAR") != nullptr;
    if (nonlin) {
        XFK_CHECK(P->hV_old.alloc((size_t)N));
        XFK_CHECK(P->hres_part.alloc(3 * kResGrid));
    }
    if (ac1) {
        XFK_CHECK(P->haux.alloc(6 * (size_t)nnz));
        XFK_CHECK(P->hk_vec.alloc(5 * (size_t)NL));   // (node vectors with the halo's room: Pd is exchanged)
        XFK_CHECK(P->hk_b.alloc(2 * (size_t)N));
    }
    HarmArgs A;
    A.erec = P->erec.p;
    A.ebits = P->ebits.p;
    A.slot = P->slot.p;
    A.x = P->x.p;
    A.y = P->y.p;
    A.labels = P->labels.p;
    A.blocks = P->blocks_ac.p;
    A.lines = P->lines_ac.p;
    A.circs = P->circs_ac.p;
    A.val = P->val.p;
    A.val_im = P->val_im.p;
    A.b = P->b.p;
    A.b_im = P->b_im.p;
    A.w = P->omega;
    A.axi = P->axi ? 1 : 0;
    A.ext_ro = P->ext_ro;
    A.ext_ri = P->ext_ri;
    A.ext_zo = P->ext_zo;
    A.V = v;
    A.bhB = P->hbh_B.p;
    A.bhH = P->hbh_H.p;
    A.bhS = P->hbh_S.p;
    A.newton = 0;
    A.aux = ac1 ? P->haux.p : nullptr;
    A.nnz = nnz;
    HcArgs H;
    H.N = N;
    H.rowptr = P->rowptr.p;
    H.col = P->col.p;
    H.val = P->val.p;
    H.val_im = P->val_im.p;
    H.x = v;
    H.r = v + NL;
    H.u = v + 2 * (size_t)NL;
    H.w = v + 3 * (size_t)NL;
    H.z = v + 4 * (size_t)NL;
    H.p = v + 5 * (size_t)NL;
    double2 *dinv = v + 6 * (size_t)NL;
    H.dinv = dinv;
    H.part = P->hc_part.p;
    H.part_rd = comm ? P->hc_part.p + (size_t)kHcParts * G : P->hc_part.p;
    H.G = G;
    H.Gred = comm ? G : 0;
    H.S = P->hc_state.p;
    H.r_re = P->hc_split.p;
    H.r_im = P->hc_split.p + NL;
    double *u_re = P->hc_split.p + 2 * (size_t)NL, *u_im = P->hc_split.p + 3 * (size_t)NL;
    H.u_re = u_re;
    H.u_im = u_im;
    const int *done = &P->hc_state.p->done;

    // successive approximation (harmonic2d.cpp:219-873; a single pass for
    // linear problems): assemble from the current iterate, solve warm-started,
    // relax, stop at |dV| / |V| < 100 Precision
    double Relax = P->relax, resn = 0, lastres = 0;
    long long cg_total = 0;
    float ms_asm = 0, ms_sol = 0, ms_setup = 0;
    bool amg = false, reusable = false, fresh = false;
    long long fresh_iters = 0, last_iters = 0;
    int iter = 0;
    for (;; ++iter) {
        XFK_CHECK(hipEventRecord(e0, s));
        if (nonlin && iter > 0) {   // the elements' B reads V at their halo nodes
            const int xrc = exch_c(v);
            if (xrc != XFK_OK) return xrc;
        }
        XFK_CHECK(hipMemsetAsync(P->val.p, 0, sizeof(double) * nnz, s));
        XFK_CHECK(hipMemsetAsync(P->val_im.p, 0, sizeof(double) * nnz, s));
        XFK_CHECK(hipMemsetAsync(P->b.p, 0, sizeof(double) * NR, s));
        XFK_CHECK(hipMemsetAsync(P->b_im.p, 0, sizeof(double) * NR, s));
        A.iter = iter;
        A.newton = (ac1 && iter > 0) ? 1 : 0;
        double *aux = A.newton ? P->haux.p : nullptr;
        if (aux) XFK_CHECK(hipMemsetAsync(aux, 0, sizeof(double) * 6 * nnz, s));
        for (int cl = 0; cl < P->ncolors; ++cl) {
            const int n = P->color_off[cl + 1] - P->color_off[cl];
            if (n > 0) k_hassemble_color<<<nb256(n), kBlock, 0, s>>>(P->color_off[cl], P->color_off[cl + 1], A);
        }
        launch_add_at_slots(s, P->age_n, P->age_slot.p, P->age_v.p, P->val.p);   // air-gap elements (real)
        if (P->nhpt > 0)
            k_hpoint<<<nb256(P->nhpt), kBlock, 0, s>>>(P->nhpt, P->hpt_nodes.p, P->hpt_J.p, P->b.p, P->b_im.p);
        if (P->nfix_cols > 0) {
            // rows that are not fixed but couple to a fixed node: k_hdir_cols walks those rows
            k_hdir_cols<<<nb256(P->nfix_cols), kBlock, 0, s>>>(P->nfix_cols, P->fix_cols_row.p, P->rowptr.p,
                                                               P->col.p, P->fixed.p, P->hfix_first.p, P->val.p,
                                                               P->val_im.p, P->b.p, P->b_im.p, aux, nnz);
        }
        if (P->nfix_rows > 0)
            k_hdir_rows<<<nb256(P->nfix_rows), kBlock, 0, s>>>(P->nfix_rows, P->fix_rows.p, P->rowptr.p,
                                                               P->diag.p, P->val.p, P->val_im.p, P->b.p,
                                                               P->b_im.p, P->hfix_last.p, aux, nnz);
        launch_map(s, P->pm_n, P->pm_dst.p, P->pm_ptr.p, P->pm_src.p, P->pm_w.p, P->val.p, P->pm_tmp.p);
        launch_map(s, P->pm_n, P->pm_dst.p, P->pm_ptr.p, P->pm_src.p, P->pm_w.p, P->val_im.p, P->pm_tmp.p);
        launch_map(s, P->pb_n, P->pb_dst.p, P->pb_ptr.p, P->pb_src.p, P->pb_w.p, P->b.p, P->pb_tmp.p);
        launch_map(s, P->pb_n, P->pb_dst.p, P->pb_ptr.p, P->pb_src.p, P->pb_w.p, P->b_im.p, P->pb_tmp.p);
        if (aux)
            for (int h = 0; h < 6; ++h)
                launch_map(s, P->pa_n, P->pa_dst.p, P->pa_ptr.p, P->pa_src.p, P->pa_w.p, aux + h * nnz,
                           P->pa_tmp.p);
        if (nonlin) XFK_CHECK(hipMemcpyAsync(P->hV_old.p, v, sizeof(double2) * N, hipMemcpyDeviceToDevice, s));
        XFK_CHECK(hipGetLastError());
        XFK_CHECK(hipEventRecord(e1, s));

        // COCG, Chronopoulos-Gear arrangement; preconditioner: the AMG V-cycle of
        // the real surrogate B = Re A + sgn Im A applied to real and imaginary
        // parts (a real symmetric M keeps COCG's complex-symmetric structure; with
        // K_r, K_i both positive semi-definite, the eigenvalues of B^-1 (K_r + i K_i)
        // lie in the box [0,1] x [0,1] away from 0, so the iteration count is the
        // V-cycle's, not the mesh's), or complex Jacobi
        amg = false;
        if (P->precond == XFK_PRECOND_AMG) {
            const int nbd = nb256(N);
            XFK_CHECK(P->hc_bval.alloc((size_t)std::max<long long>(P->nnz, nbd)));
            k_hc_diag_im<<<nbd, 256, 0, s>>>(N, P->diag.p, P->val_im.p, P->hc_bval.p);
            std::vector<double> hp(nbd);
            XFK_CHECK(d2h(hp.data(), P->hc_bval.p, sizeof(double) * nbd, s));
            double sdi = 0;
            for (double q : hp) sdi += q;
            if (comm) {   // the same sign on every rank
                const int arc0 = allreduce_host(P, sdi);
                if (arc0 != XFK_OK) return arc0;
            }
            k_hc_surrogate<<<nb256(N), kBlock, 0, s>>>(N, sdi >= 0 ? 1.0 : -1.0, P->rowptr.p, P->col.p, P->val.p,
                                                       P->val_im.p, P->hc_bval.p);
            if (!P->amg) P->amg = new Amg();
            P->amg->theta = P->amg_theta;
            P->amg->sweeps = P->amg_sweeps;
            P->amg->omega = P->amg_omega;
            P->amg->rep_rows = P->amg_replicate;
            ScopedEvents<2> aev;
            XFK_CHECK(aev.create());
            hipEvent_t a0 = aev[0], a1 = aev[1];
            XFK_CHECK(hipEventRecord(a0, s));
            // later passes of the nonlinear loop keep the hierarchy (fine-level
            // smoother refreshed) while COCG stays within 1.25x + 1 the
            // iterations of the last fresh build (tighter than the static
            // loop's 2x: a COCG iteration costs two V-cycles); the reference
            // count is taken on a warm-started pass (pass 1 is built fresh),
            // the cold first pass needing several times more
            const bool reuse = P->amg_reuse && reusable && iter > 1 &&
                               4 * last_iters <= 5 * fresh_iters + 4;
            fresh = !reuse;
            const bool sharded = comm && comm->size > 1;   // (one rank: the single-device hierarchy)
            const int arc = reuse     ? P->amg->refresh(s)
                            : sharded ? P->amg->setup_dist(s, comm, P->halo, N, NL - N, P->rowptr.p, P->col.p,
                                                           P->hc_bval.p, P->nnz_own)
                                      : P->amg->setup(s, N, N, P->rowptr.p, P->col.p, P->hc_bval.p, P->nnz_own);
            XFK_CHECK(hipEventRecord(a1, s));
            XFK_CHECK(hipEventSynchronize(a1));
            float mss = 0;
            XFK_CHECK(hipEventElapsedTime(&mss, a0, a1));
            ms_setup += mss;
            if (arc != XFK_OK && arc != XFK_ERR_UNSUPPORTED) return arc;
            double okv = arc == XFK_OK ? 0.0 : 1.0;   // every rank takes the same preconditioner
            if (comm) {
                const int arc1 = allreduce_host(P, okv);
                if (arc1 != XFK_OK) return arc1;
            }
            amg = okv == 0.0;
            reusable = amg;
        }
        H.amg = amg ? 1 : 0;
        auto precondition = [&]() -> int {
            int rc = P->amg->vcycle(s, H.r_re, u_re, done);
            if (rc == XFK_OK) rc = P->amg->vcycle(s, H.r_im, u_im, done);
            if (rc == XFK_OK) rc = exch_r(u_re);   // (the SpMV gathers u at the halo columns)
            if (rc == XFK_OK) rc = exch_r(u_im);
            return rc;
        };
        // the SpMV of the current u, then the partials of every rank summed
        auto spmv = [&](int gpar) -> int {
            int rc = amg ? XFK_OK : exch_c(H.u);
            if (rc != XFK_OK) return rc;
            k_hc_spmv<<<Gcg, kCgBlock, 0, s>>>(H, gpar);
            return reduce_parts();
        };
        // one COCG solve A x = b (warm: from the current x)
        // the linear solver's precision: adaptive once the auxiliary matrices
        // exist (harmonic2d.cpp:821-825, harmonicaxi.cpp:745-749)
        double lprec = P->precision;
        if (A.newton) {
            lprec = std::min(1.e-4, 0.001 * resn);
            if (lprec < P->precision) lprec = P->precision;
        }
        auto solve_one = [&](double2 *xv, const double *bre, const double *bim, bool warm) -> int {
            H.x = xv;
            XFK_CHECK(hipMemsetAsync(P->hc_part.p, 0, sizeof(double) * kHcParts * G, s));   // (the written half)
            CcgState init{};
            init.tol = lprec;
            XFK_CHECK(hipMemcpyAsync(P->hc_state.p, &init, sizeof(CcgState), hipMemcpyHostToDevice, s));
            k_hdiag_inv<<<nb256(N), kBlock, 0, s>>>(N, P->diag.p, P->val.p, P->val_im.p, dinv, P->hc_state.p);
            XFK_CHECK(hipMemcpyAsync(P->hc_host, P->hc_state.p, sizeof(CcgState), hipMemcpyDeviceToHost, s));
            XFK_CHECK(hipStreamSynchronize(s));
            if (comm) {   // every rank must agree before the collective iterations
                double sg = P->hc_host->singular ? 1.0 : 0.0;
                const int grc = allreduce_host(P, sg);
                if (grc != XFK_OK) return grc;
                P->hc_host->singular = sg != 0.0;
            }
            if (P->hc_host->singular) {
                set_error("singular flag tripped: zero diagonal entry in the assembled matrix");
                return XFK_ERR_SINGULAR;
            }
            int prc;
            if (warm && (prc = exch_c(xv)) != XFK_OK) return prc;   // (r = b - A x0 reads x0's halo)
            if (warm) k_hc_init<true><<<Gcg, kCgBlock, 0, s>>>(H, bre, bim);
            else k_hc_init<false><<<Gcg, kCgBlock, 0, s>>>(H, bre, bim);
            if (amg && (prc = precondition()) != XFK_OK) return prc;
            if ((prc = spmv(0)) != XFK_OK) return prc;
            long long it = 0;
            int batch = amg ? 8 : 32;
            const long long cap = std::max<long long>(100000, 20LL * N);
            // batches end with an update (its convergence test is what the
            // poll reads); that iteration's preconditioner + SpMV open the
            // next batch, so a converged solve launches no exiting tail
            bool tail = false;
            for (;;) {
                for (int k = 0; k < batch; ++k, ++it) {
                    if (tail) {
                        if (amg && (prc = precondition()) != XFK_OK) return prc;
                        if ((prc = spmv((int)(it & 1))) != XFK_OK) return prc;   // iteration it - 1's
                    }
                    if (comm) {
                        // every partial array is read over all G entries (zero
                        // beyond a rank's grids); the init's gamma / |r|^2 arrays
                        // (k_hc_init grid) are next written by the update (its own
                        // grid): cleared once the first update has read them
                        k_hc_axpy<<<Gax, kHcAxBlock, 0, s>>>(H, it, G, G);
                        if (it == 0) {
                            XFK_CHECK(hipMemsetAsync(P->hc_part.p, 0, sizeof(double) * 2 * G, s));
                            XFK_CHECK(hipMemsetAsync(P->hc_part.p + 6 * (size_t)G, 0, sizeof(double) * G, s));
                        }
                    } else if (amg) k_hc_axpy<<<Gax, kHcAxBlock, 0, s>>>(H, it, Gcg, it == 0 ? Gcg : Gax);
                    else k_hc_axpy<<<Gax, kHcAxBlock, 0, s>>>(H, it, it == 0 ? Gcg : Gax, it == 0 ? Gcg : Gax);
                    tail = true;
                }
                XFK_CHECK(hipGetLastError());
                XFK_CHECK(hipMemcpyAsync(P->hc_host, P->hc_state.p, sizeof(CcgState), hipMemcpyDeviceToHost, s));
                XFK_CHECK(hipStreamSynchronize(s));
                const CcgState &S = *P->hc_host;
                if (S.done) break;
                if (it >= cap) {
                    set_error("COCG did not converge within the iteration cap");
                    return XFK_ERR_NOCONV;
                }
                double rate = (S.iters > 0 && S.er > 0 && S.er < 1) ? std::log(S.er) / (double)S.iters : 0.0;
                long long rem = rate < 0 ? (long long)std::ceil(std::log(S.tol / S.er) / rate) : 2 * batch;
                batch = (int)std::max<long long>(8, std::min<long long>(rem + 2, 512));
            }
            cg_total += P->hc_host->iters;
            return XFK_OK;
        };
        // KludgeSolve (cspars.cpp:1000-1060): M V + Mh V + Ms conj(V) + Ma V = b
        // by at most 10 COCG solves on M with the auxiliary terms of the
        // current iterate on the right-hand side, each step scaled by the
        // line search c = Re(r^H U) / |U|^2 on the true residual
        auto dots = [&](const double2 *a, const double2 *bb, double (&out)[3]) -> int {
            k_hk_dots<<<kResGrid, 256, 0, s>>>(N, a, bb, P->hres_part.p);
            std::vector<double> hp(3 * kResGrid);
            XFK_CHECK(d2h(hp.data(), P->hres_part.p, sizeof(double) * hp.size(), s));
            for (int q = 0; q < 3; ++q) {
                out[q] = 0;
                for (int k = 0; k < kResGrid; ++k) out[q] += hp[q * kResGrid + k];
            }
            return allreduce_host_n(P, out, 3);   // (sharded: over every rank's owned rows)
        };
        auto kludge = [&]() -> int {
            double2 *bo = P->hk_vec.p, *vs = bo + NL, *rr = bo + 2 * (size_t)NL, *Pd = bo + 3 * (size_t)NL,
                    *U = bo + 4 * (size_t)NL;
            double *bre = P->hk_b.p, *bim = P->hk_b.p + N;
            const int nbn = nb256(N);
            k_hk_join<<<nbn, kBlock, 0, s>>>(N, P->b.p, P->b_im.p, bo);
            XFK_CHECK(hipMemcpyAsync(vs, v, sizeof(double2) * N, hipMemcpyDeviceToDevice, s));
            if (int xrc = exch_c(v)) return xrc;   // (the products read V at the halo columns)
            k_hk_apply<<<nbn, 256, 0, s>>>(N, P->rowptr.p, P->col.p, P->val.p, P->val_im.p, aux, nnz, v, bo, 2, rr,
                                           nullptr, nullptr);
            double d3[3];
            int rc = dots(rr, bo, d3);
            if (rc != XFK_OK) return rc;
            const double normb = std::sqrt(d3[1]);
            if (normb == 0.0) return XFK_OK;
            double er = std::sqrt(d3[2]) / normb;
            if (!(er < lprec)) {
                for (int k = 0; k < 10; ++k) {
                    if ((rc = exch_c(v)) != XFK_OK) return rc;
                    k_hk_apply<<<nbn, 256, 0, s>>>(N, P->rowptr.p, P->col.p, P->val.p, P->val_im.p, aux, nnz, v, bo,
                                                   1, nullptr, bre, bim);
                    if ((rc = solve_one(v, bre, bim, true)) != XFK_OK) return rc;
                    k_hk_diff<<<nbn, kBlock, 0, s>>>(N, v, vs, Pd);
                    if ((rc = exch_c(Pd)) != XFK_OK) return rc;
                    k_hk_apply<<<nbn, 256, 0, s>>>(N, P->rowptr.p, P->col.p, P->val.p, P->val_im.p, aux, nnz, Pd,
                                                   nullptr, 0, U, nullptr, nullptr);
                    if ((rc = dots(rr, U, d3)) != XFK_OK) return rc;
                    const double cstep = d3[0] / d3[1];
                    k_hk_update<<<nbn, kBlock, 0, s>>>(N, cstep, v, vs, Pd, rr, U);
                    if ((rc = dots(rr, rr, d3)) != XFK_OK) return rc;
                    er = std::sqrt(d3[2]) / normb;
                    if (trace) std::fprintf(stderr, "  kludge %d: c %.6e er %.6e (cocg %lld)\n", k, cstep, er,
                                            (long long)P->hc_host->iters);
                    if (er < lprec * 10.) break;
                }
            } else if (trace) {
                std::fprintf(stderr, "  kludge: er %.6e < %.3e at start\n", er, lprec);
            }
            return XFK_OK;
        };
        const int nc2 = (int)P->hc2_circ.size();
        const double *Cb = P->hc2_C.p;
        // C_q . y (unconjugated) of the Case-2 border column q
        auto cdot = [&](int q, const double2 *y, hcx &out) -> int {
            k_hc_cdot<<<kResGrid, 256, 0, s>>>(N, Cb + 2 * (size_t)q * N, Cb + 2 * (size_t)q * N + N, y,
                                               P->hres_part.p);
            std::vector<double> hp(2 * kResGrid);
            XFK_CHECK(d2h(hp.data(), P->hres_part.p, sizeof(double) * hp.size(), s));
            double re = 0, im = 0;
            for (int k = 0; k < kResGrid; ++k) {
                re += hp[k];
                im += hp[kResGrid + k];
            }
            double ri[2] = {re, im};
            const int arc = allreduce_host_n(P, ri, 2);   // (sharded: over every rank's owned rows)
            out = hcx(ri[0], ri[1]);
            return arc;
        };
        // Schur complement D - C^T Y of this pass's matrix (Y = M^-1 C)
        auto schur = [&](std::vector<hcx> &Sm) -> int {
            Sm.assign((size_t)nc2 * nc2, hcx(0, 0));
            for (int q = 0; q < nc2; ++q)
                for (int r = 0; r < nc2; ++r) {
                    hcx t;
                    int rc = cdot(q, P->hc2_Y.p + (size_t)r * NL, t);
                    if (rc != XFK_OK) return rc;
                    Sm[(size_t)q * nc2 + r] = (q == r ? hc(P->hc2_D[q]) : hcx(0, 0)) - t;
                }
            return XFK_OK;
        };
        // small dense complex solve S u = g, partial pivoting (S, g by value)
        auto dense_solve = [&](std::vector<hcx> S, std::vector<hcx> g, std::vector<double2> &u) -> int {
            for (int k = 0; k < nc2; ++k) {
                int pv = k;
                for (int r = k + 1; r < nc2; ++r)
                    if (std::abs(S[(size_t)r * nc2 + k]) > std::abs(S[(size_t)pv * nc2 + k])) pv = r;
                if (std::abs(S[(size_t)pv * nc2 + k]) == 0.0) {
                    set_error("singular circuit system (Case-2 circuits)");
                    return XFK_ERR_SINGULAR;
                }
                if (pv != k) {
                    for (int c2 = 0; c2 < nc2; ++c2) std::swap(S[(size_t)k * nc2 + c2], S[(size_t)pv * nc2 + c2]);
                    std::swap(g[k], g[pv]);
                }
                for (int r = k + 1; r < nc2; ++r) {
                    const hcx f = S[(size_t)r * nc2 + k] / S[(size_t)k * nc2 + k];
                    for (int c2 = k; c2 < nc2; ++c2) S[(size_t)r * nc2 + c2] -= f * S[(size_t)k * nc2 + c2];
                    g[r] -= f * g[k];
                }
            }
            u.assign(nc2, cx(0, 0));
            for (int k = nc2 - 1; k >= 0; --k) {
                hcx t = g[k];
                for (int c2 = k + 1; c2 < nc2; ++c2) t -= S[(size_t)k * nc2 + c2] * hc(u[c2]);
                u[k] = h2(t / S[(size_t)k * nc2 + k]);
            }
            return XFK_OK;
        };
        // KludgeSolve on the bordered system (cspars.cpp:1000-1060 over the
        // full unknown vector [V; u], harmonic2d.cpp:800-826): the residual,
        // the step and the line search run over nodes and circuit unknowns
        // alike (the auxiliary matrices are zero on the border rows); each
        // inner solve is the bordered [M C; C^T D] solve through the Schur
        // complement with this pass's Y = M^-1 C
        auto kludge2 = [&]() -> int {
            double2 *bo = P->hk_vec.p, *vs = bo + NL, *rr = bo + 2 * (size_t)NL, *Pd = bo + 3 * (size_t)NL,
                    *U = bo + 4 * (size_t)NL;
            double *bre = P->hk_b.p, *bim = P->hk_b.p + N;
            const int nbn = nb256(N);
            int rc;
            for (int q = 0; q < nc2; ++q)
                if ((rc = solve_one(P->hc2_Y.p + (size_t)q * NL, Cb + 2 * (size_t)q * N, Cb + 2 * (size_t)q * N + N,
                                    true)) != XFK_OK)
                    return rc;
            std::vector<hcx> Sm;
            if ((rc = schur(Sm)) != XFK_OK) return rc;
            DBuf<double2> ud;
            XFK_CHECK(ud.alloc((size_t)nc2));
            auto put = [&](const std::vector<double2> &w) -> int {
                XFK_CHECK(hipMemcpyAsync(ud.p, w.data(), sizeof(double2) * nc2, hipMemcpyHostToDevice, s));
                XFK_CHECK(hipStreamSynchronize(s));
                return XFK_OK;
            };
            std::vector<double2> u = P->hc2_u, un, Pb(nc2);
            std::vector<hcx> rb(nc2), Ub(nc2), g(nc2);
            k_hk_join<<<nbn, kBlock, 0, s>>>(N, P->b.p, P->b_im.p, bo);
            XFK_CHECK(hipMemcpyAsync(vs, v, sizeof(double2) * N, hipMemcpyDeviceToDevice, s));
            if (int xrc = exch_c(v)) return xrc;   // (the products read V at the halo columns)
            k_hk_apply<<<nbn, 256, 0, s>>>(N, P->rowptr.p, P->col.p, P->val.p, P->val_im.p, aux, nnz, v, bo, 2, rr,
                                           nullptr, nullptr);
            if ((rc = put(u)) != XFK_OK) return rc;
            k_hc_add_cu<<<nbn, kBlock, 0, s>>>(N, nc2, Cb, ud.p, -1.0, rr);
            double fb2 = 0, rb2 = 0;
            for (int q = 0; q < nc2; ++q) {
                hcx t;
                if ((rc = cdot(q, v, t)) != XFK_OK) return rc;
                rb[q] = hc(P->hc2_f[q]) - t - hc(P->hc2_D[q]) * hc(u[q]);
                fb2 += std::norm(hc(P->hc2_f[q]));
                rb2 += std::norm(rb[q]);
            }
            double d3[3];
            if ((rc = dots(rr, bo, d3)) != XFK_OK) return rc;
            const double normb = std::sqrt(d3[1] + fb2);
            if (normb == 0.0) return XFK_OK;
            double er = std::sqrt(d3[2] + rb2) / normb;
            if (!(er < lprec)) {
                for (int k = 0; k < 10; ++k) {
                    if ((rc = exch_c(v)) != XFK_OK) return rc;
                    k_hk_apply<<<nbn, 256, 0, s>>>(N, P->rowptr.p, P->col.p, P->val.p, P->val_im.p, aux, nnz, v, bo,
                                                   1, nullptr, bre, bim);
                    if ((rc = solve_one(P->hc2_y0.p, bre, bim, true)) != XFK_OK) return rc;
                    for (int q = 0; q < nc2; ++q) {
                        hcx t;
                        if ((rc = cdot(q, P->hc2_y0.p, t)) != XFK_OK) return rc;
                        g[q] = hc(P->hc2_f[q]) - t;
                    }
                    if ((rc = dense_solve(Sm, g, un)) != XFK_OK) return rc;
                    if ((rc = put(un)) != XFK_OK) return rc;
                    k_hc_border_combine<<<nbn, kBlock, 0, s>>>(N, nc2, P->hc2_y0.p, P->hc2_Y.p, NL, ud.p, v);
                    k_hk_diff<<<nbn, kBlock, 0, s>>>(N, v, vs, Pd);
                    for (int q = 0; q < nc2; ++q) Pb[q] = cx(un[q].x - u[q].x, un[q].y - u[q].y);
                    if ((rc = exch_c(Pd)) != XFK_OK) return rc;
                    k_hk_apply<<<nbn, 256, 0, s>>>(N, P->rowptr.p, P->col.p, P->val.p, P->val_im.p, aux, nnz, Pd,
                                                   nullptr, 0, U, nullptr, nullptr);
                    if ((rc = put(Pb)) != XFK_OK) return rc;
                    k_hc_add_cu<<<nbn, kBlock, 0, s>>>(N, nc2, Cb, ud.p, 1.0, U);
                    double bn = 0, bd = 0;
                    for (int q = 0; q < nc2; ++q) {
                        hcx t;
                        if ((rc = cdot(q, Pd, t)) != XFK_OK) return rc;
                        Ub[q] = t + hc(P->hc2_D[q]) * hc(Pb[q]);
                        bn += (std::conj(rb[q]) * Ub[q]).real();
                        bd += std::norm(Ub[q]);
                    }
                    if ((rc = dots(rr, U, d3)) != XFK_OK) return rc;
                    const double cstep = (d3[0] + bn) / (d3[1] + bd);
                    k_hk_update<<<nbn, kBlock, 0, s>>>(N, cstep, v, vs, Pd, rr, U);
                    rb2 = 0;
                    for (int q = 0; q < nc2; ++q) {
                        u[q] = cx(u[q].x + cstep * Pb[q].x, u[q].y + cstep * Pb[q].y);
                        rb[q] -= cstep * Ub[q];
                        rb2 += std::norm(rb[q]);
                    }
                    if ((rc = dots(rr, rr, d3)) != XFK_OK) return rc;
                    er = std::sqrt(d3[2] + rb2) / normb;
                    if (trace) std::fprintf(stderr, "  kludge2 %d: c %.6e er %.6e (cocg %lld)\n", k, cstep, er,
                                            (long long)P->hc_host->iters);
                    if (er < lprec * 10.) break;
                }
            } else if (trace) {
                std::fprintf(stderr, "  kludge2: er %.6e < %.3e at start\n", er, lprec);
            }
            P->hc2_u_old = P->hc2_u;
            P->hc2_u = u;
            return XFK_OK;
        };
        int src;
        if (nc2 == 0) {
            if (A.newton) {
                if ((src = kludge()) != XFK_OK) return src;
            } else if ((src = solve_one(v, P->b.p, P->b_im.p, iter > 0)) != XFK_OK) {
                return src;
            }
        } else if (A.newton) {
            if ((src = kludge2()) != XFK_OK) return src;
        } else {
            // bordered system [A C; C^T D][V; u] = [b; f] through the Schur
            // complement: Y = A^-1 C, y0 = A^-1 b, (D - C^T Y) u = f - C^T y0,
            // V = y0 - Y u (one COCG solve per Case-2 circuit and one for b)
            if (iter == 0) {
                XFK_CHECK(P->hc2_Y.alloc((size_t)nc2 * NL));   // (solve_one's x: room for the halo)
                XFK_CHECK(P->hc2_y0.alloc((size_t)NL));
                XFK_CHECK(P->hres_part.alloc(2 * kResGrid));
            }
            for (int q = 0; q < nc2; ++q)
                if ((src = solve_one(P->hc2_Y.p + (size_t)q * NL, Cb + 2 * (size_t)q * N,
                                     Cb + 2 * (size_t)q * N + N, iter > 0)) != XFK_OK)
                    return src;
            if ((src = solve_one(P->hc2_y0.p, P->b.p, P->b_im.p, iter > 0)) != XFK_OK) return src;
            std::vector<hcx> S, g(nc2);
            if ((src = schur(S)) != XFK_OK) return src;
            for (int q = 0; q < nc2; ++q) {
                hcx t;
                if ((src = cdot(q, P->hc2_y0.p, t)) != XFK_OK) return src;
                g[q] = hc(P->hc2_f[q]) - t;
            }
            std::vector<double2> u;
            if ((src = dense_solve(S, g, u)) != XFK_OK) return src;
            P->hc2_u_old = P->hc2_u;
            P->hc2_u = u;
            DBuf<double2> ud;
            XFK_CHECK(ud.alloc((size_t)nc2));
            XFK_CHECK(hipMemcpyAsync(ud.p, u.data(), sizeof(double2) * nc2, hipMemcpyHostToDevice, s));
            k_hc_border_combine<<<nb256(N), kBlock, 0, s>>>(N, nc2, P->hc2_y0.p, P->hc2_Y.p, NL, ud.p, v);
            XFK_CHECK(hipStreamSynchronize(s));
        }
        last_iters = P->hc_host->iters;
        if (fresh) fresh_iters = last_iters;
        XFK_CHECK(hipEventRecord(e2, s));
        XFK_CHECK(hipEventSynchronize(e2));
        float ms = 0;
        XFK_CHECK(hipEventElapsedTime(&ms, e0, e1));
        ms_asm += ms;
        XFK_CHECK(hipEventElapsedTime(&ms, e1, e2));
        ms_sol += ms;
        if (!nonlin) break;
        // the change of this pass (harmonic2d.cpp:829-852)
        k_hres<<<kResGrid, 256, 0, s>>>(N, v, P->hV_old.p, P->hres_part.p);
        std::vector<double> hp(2 * kResGrid);
        XFK_CHECK(d2h(hp.data(), P->hres_part.p, sizeof(double) * hp.size(), s));
        double sx = 0, sy = 0;
        for (int k = 0; k < kResGrid; ++k) {
            sx += hp[k];
            sy += hp[kResGrid + k];
        }
        if (comm) {   // over every rank's owned rows
            int rrc = allreduce_host(P, sx);
            if (rrc == XFK_OK) rrc = allreduce_host(P, sy);
            if (rrc != XFK_OK) return rrc;
        }
        if (sy == 0) break;
        lastres = resn;
        resn = std::sqrt(sx / sy);
        if (trace) std::fprintf(stderr, "pass %d: res %.6e relax %.4f lprec %.3e\n", iter, resn, Relax, lprec);
        if (iter > 5) {
            if ((resn > lastres) && (Relax > 0.1)) Relax /= 2.;
            else Relax += 0.1 * (1. - Relax);
            k_hrelax<<<nb256(N), kBlock, 0, s>>>(N, Relax, v, P->hV_old.p);
            for (size_t q = 0; q < P->hc2_u.size(); ++q) {   // the circuit unknowns relax alike
                const double2 a2 = P->hc2_u[q], o = P->hc2_u_old[q];
                P->hc2_u[q] = cx(Relax * a2.x + (1.0 - Relax) * o.x, Relax * a2.y + (1.0 - Relax) * o.y);
            }
        }
        if ((resn < 100. * P->precision) && iter > 0) break;
        if (iter >= 10000) {
            set_error("harmonic successive approximation did not converge within the iteration cap");
            return XFK_ERR_NOCONV;
        }
    }
    // Case-2 circuits: the voltage gradient from the bordered unknown
    // (harmonic2d.cpp:784-785: I c w V[N+k]; harmonicaxi.cpp:791: I w c 0.01 V[N+k])
    for (size_t q = 0; q < P->hc2_circ.size(); ++q) {
        const double2 f = P->axi ? cx(0.0 * P->omega * kC * 0.01, P->omega * kC * 0.01)
                                 : cx(0.0 * kC * P->omega, kC * P->omega);
        P->hcircs[P->hc2_circ[q]].dV = cmul(f, P->hc2_u[q]);
    }
    R.ms_assemble = ms_asm;
    R.ms_solve = ms_sol;
    R.newton_iters = iter + 1;
    R.cg_iters = cg_total;
    R.final_er = P->hc_host->er;
    R.nnz = P->nnz_own;
    R.ncolors = P->ncolors;
    R.color_rounds = P->color_rounds;
    R.precond = amg ? XFK_PRECOND_AMG : XFK_PRECOND_JACOBI;
    if (amg) {
        R.amg_levels = P->amg->stats.levels;
        R.amg_op_complexity = P->amg->stats.op_complexity;
        R.ms_amg_setup = ms_setup;
    }
    P->last = R;
    if (res) *res = R;
    return XFK_OK;
}

}  // namespace xfk

extern "C" {

int xfk_get_solution_complex(xfk_problem *P, double *A)
{
    XFK_REQUIRE(P && A && P->harmonic, XFK_ERR_ARG, "null argument or not a harmonic problem");
    XFK_REQUIRE(P->symbolic_ready && P->hc_vec.p, XFK_ERR_ARG, "no solution yet");
    XFK_CHECK(hipSetDevice(P->device));
    hipStream_t s = P->stream;
    const int Ng = P->N_global;
    if (!P->comm) {
        XFK_CHECK(d2h(A, P->hc_vec.p, sizeof(double2) * P->N, s));
    } else {   // sharded: all-gather the owned rows (padded to the largest block), collective
        const int R = P->nranks;
        size_t maxn = 0;
        for (int q = 0; q < R; ++q) maxn = std::max<size_t>(maxn, row_begin(Ng, q + 1, R) - row_begin(Ng, q, R));
        XFK_CHECK(P->gather_buf.alloc(2 * maxn * (1 + R)));
        double *send = P->gather_buf.p, *recv = P->gather_buf.p + 2 * maxn;
        XFK_CHECK(hipMemsetAsync(send, 0, sizeof(double) * 2 * maxn, s));
        XFK_CHECK(hipMemcpyAsync(send, P->hc_vec.p, sizeof(double2) * P->N, hipMemcpyDeviceToDevice, s));
        const int rc = P->comm->allgather(send, recv, 2 * maxn, s);
        if (rc != XFK_OK) return rc;
        std::vector<double> h(2 * maxn * R);
        XFK_CHECK(d2h(h.data(), recv, sizeof(double) * h.size(), s));
        for (int q = 0; q < R; ++q) {
            const long long r0 = row_begin(Ng, q, R), r1 = row_begin(Ng, q + 1, R);
            for (long long i = r0; i < r1; ++i)
                for (int c = 0; c < 2; ++c) A[2 * i + c] = h[2 * ((size_t)q * maxn + (i - r0)) + c];
        }
    }
    if (P->axi) {   // the flux 2 pi r A (harmonicaxi.cpp:790)
        for (int i = 0; i < Ng; ++i)
            for (int q = 0; q < 2; ++q) A[2 * i + q] = A[2 * i + q] * kC * 2. * kPI * P->axi_x[i] * 0.01;
    } else {
        for (long long i = 0; i < 2LL * Ng; ++i) A[i] *= kC;   // harmonic2d.cpp:783
    }
    return XFK_OK;
}

int xfk_get_circuits_complex(xfk_problem *P, int *ccase, double *J, double *dV)
{
    XFK_REQUIRE(P && P->harmonic, XFK_ERR_ARG, "not a harmonic problem");
    for (int k = 0; k < P->ncircs; ++k) {
        const DevCircAC &C = P->hcircs[k];
        if (ccase) ccase[k] = C.ccase;
        if (J) { J[2 * k] = C.J.x; J[2 * k + 1] = C.J.y; }
        if (dV) { dV[2 * k] = C.dV.x; dV[2 * k + 1] = C.dV.y; }
    }
    return XFK_OK;
}

int xfk_get_csr_complex(xfk_problem *P, int *rowptr, int *col, double *val, double *b)
{
    XFK_REQUIRE(P && P->harmonic && P->symbolic_ready && P->val_im.p, XFK_ERR_ARG, "no assembled harmonic system");
    XFK_CHECK(hipSetDevice(P->device));
    hipStream_t s = P->stream;
    XFK_CHECK(hipStreamSynchronize(s));
    if (rowptr) XFK_CHECK(d2h(rowptr, P->rowptr.p, sizeof(int) * (P->N + 1), s));
    if (col) XFK_CHECK(d2h(col, P->col.p, sizeof(int) * P->nnz_own, s));
    if (val) {
        std::vector<double> re(P->nnz_own), im(P->nnz_own);
        XFK_CHECK(d2h(re.data(), P->val.p, sizeof(double) * P->nnz_own, s));
        XFK_CHECK(d2h(im.data(), P->val_im.p, sizeof(double) * P->nnz_own, s));
        for (long long k = 0; k < P->nnz_own; ++k) {
            val[2 * k] = re[k];
            val[2 * k + 1] = im[k];
        }
    }
    if (b) {
        std::vector<double> re(P->N), im(P->N);
        XFK_CHECK(d2h(re.data(), P->b.p, sizeof(double) * P->N, s));
        XFK_CHECK(d2h(im.data(), P->b_im.p, sizeof(double) * P->N, s));
        for (int i = 0; i < P->N; ++i) {
            b[2 * i] = re[i];
            b[2 * i + 1] = im[i];
        }
    }
    return XFK_OK;
}

}  // extern "C"

// xfk_device_init: loads this translation unit's code object onto the device
// (the first use of any of its kernels would otherwise do it inside a solve)
hipError_t xfk::warm_module_harmonic()
{
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&k_hassemble_color));
}
