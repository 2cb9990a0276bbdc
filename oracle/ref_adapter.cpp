// C adapter over the REFERENCE's own solver sources, compiled from
// /root/reference by oracle/Makefile into oracle/_ref/libxfemm_ref.so.
//
// TEST INFRASTRUCTURE ONLY (oracle pinning and the bench's cpu_baseline leg).
// Nothing of the reference is copied: this file only calls
//   CBigLinProb            cfemm/libfemm/spars.h:38-83   (spars.cpp)
//   CMSolverMaterialProp   cfemm/libfemm/CMaterialProp.h:193 (CMaterialProp.cpp)
//   CBigComplexLinProb     cfemm/libfemm/cspars.h (cspars.cpp)
// through extern "C" surfaces matching ora_linprob_ops (static2d_oracle.h) and
// orh_linprob_ops (harmonic2d_oracle.h).
#include <sstream>
#include <string>
#include <vector>

#include "CMaterialProp.h"
#include "femmcomplex.h"
#include "cspars.h"
#include "spars.h"

extern "C" {

void *ref_lp_create(int n, int bw, double precision)
{
    CBigLinProb *L = new CBigLinProb();
    L->Precision = precision;
    L->Create(n, bw);
    return L;
}

void ref_lp_destroy(void *L) { delete static_cast<CBigLinProb *>(L); }
void ref_lp_addto(void *L, double v, int p, int q) { static_cast<CBigLinProb *>(L)->AddTo(v, p, q); }
double *ref_lp_b(void *L) { return static_cast<CBigLinProb *>(L)->b; }
double *ref_lp_V(void *L) { return static_cast<CBigLinProb *>(L)->V; }
void ref_lp_setvalue(void *L, int i, double x) { static_cast<CBigLinProb *>(L)->SetValue(i, x); }
void ref_lp_periodicity(void *L, int i, int j) { static_cast<CBigLinProb *>(L)->Periodicity(i, j); }
void ref_lp_antiperiodicity(void *L, int i, int j) { static_cast<CBigLinProb *>(L)->AntiPeriodicity(i, j); }
void ref_lp_wipe(void *L) { static_cast<CBigLinProb *>(L)->Wipe(); }
double ref_lp_get(void *L, int p, int q) { return static_cast<CBigLinProb *>(L)->Get(p, q); }
void ref_lp_multA(void *L, double *X, double *Y) { static_cast<CBigLinProb *>(L)->MultA(X, Y); }

int ref_lp_pcgsolve(void *L, int flag, long long *iters)
{
    if (iters) *iters = -1;  // the reference does not report its iteration count
    return static_cast<CBigLinProb *>(L)->PCGSolve(flag) ? 1 : 0;
}

// Parse one <BeginBlock> ... <EndBlock> text with the reference parser, run
// GetSlopes(omega=0) and return the processed curve (B, H.re, slope.re) and mu_x.
// Returns BHpoints, or -1 on a parse problem.  Arrays must hold `cap` values.
int ref_block_slopes(const char *block_text, double *B, double *H, double *slope,
                     int cap, double *mu_x)
{
    std::istringstream in(block_text);
    std::ostringstream err;
    femm::CMSolverMaterialProp prop = femm::CMSolverMaterialProp::fromStream(in, err);
    if (prop.BHpoints > 0) prop.GetSlopes(0.0);
    int n = prop.BHpoints;
    if (n > cap) return -1;
    for (int i = 0; i < n; i++) {
        B[i] = prop.Bdata[i];
        H[i] = prop.Hdata[i].re;
        slope[i] = prop.slope[i].re;
    }
    *mu_x = prop.mu_x;
    return n;
}

// GetSlopes(omega) (omega > 0: the harmonic solver's complex curve); returns
// BHpoints (or -1), the complex H and slopes split into re / im arrays.
int ref_block_slopes_ac(const char *block_text, double omega, double *B, double *Hr, double *Hi, double *Sr,
                        double *Si, int cap, double *mu_x, double *mu_max)
{
    std::istringstream in(block_text);
    std::ostringstream err;
    femm::CMSolverMaterialProp prop = femm::CMSolverMaterialProp::fromStream(in, err);
    if (prop.BHpoints > 0) prop.GetSlopes(omega);
    int n = prop.BHpoints;
    if (n > cap) return -1;
    for (int i = 0; i < n; i++) {
        B[i] = prop.Bdata[i];
        Hr[i] = prop.Hdata[i].re;
        Hi[i] = prop.Hdata[i].im;
        Sr[i] = prop.slope[i].re;
        Si[i] = prop.slope[i].im;
    }
    *mu_x = prop.mu_x;
    *mu_max = prop.MuMax;
    return n;
}

// Get_v(B) and GetdHdB(B) of the AC-processed block (what the harmonic
// nonlinear update evaluates, harmonic2d.cpp:648-650), for a batch of B.
int ref_block_acprops(const char *block_text, double omega, const double *Bq, int nq, double *vr, double *vi,
                      double *dr, double *di)
{
    std::istringstream in(block_text);
    std::ostringstream err;
    femm::CMSolverMaterialProp prop = femm::CMSolverMaterialProp::fromStream(in, err);
    if (prop.BHpoints > 0) prop.GetSlopes(omega);
    for (int i = 0; i < nq; i++) {
        CComplex v = prop.Get_v(Bq[i]), d = prop.GetdHdB(Bq[i]);
        vr[i] = v.re;
        vi[i] = v.im;
        dr[i] = d.re;
        di[i] = d.im;
    }
    return prop.BHpoints;
}

// GetBHProps(B) of the processed block, for a batch of flux densities.
int ref_block_bhprops(const char *block_text, const double *Bq, int nq, double *v, double *dv)
{
    std::istringstream in(block_text);
    std::ostringstream err;
    femm::CMSolverMaterialProp prop = femm::CMSolverMaterialProp::fromStream(in, err);
    if (prop.BHpoints > 0) prop.GetSlopes(0.0);
    for (int i = 0; i < nq; i++) {
        double vv = 0, dd = 0;
        prop.GetBHProps(Bq[i], vv, dd);
        v[i] = vv;
        dv[i] = dd;
    }
    return prop.BHpoints;
}

// ---- CBigComplexLinProb (harmonic path) ----
static CBigComplexLinProb *CL(void *L) { return static_cast<CBigComplexLinProb *>(L); }

void *ref_clp_create(int n, int bw, int nodes, double precision)
{
    CBigComplexLinProb *L = new CBigComplexLinProb();
    L->Precision = precision;
    L->Create(n, bw, nodes);
    return L;
}

void ref_clp_destroy(void *L) { delete CL(L); }
void ref_clp_addto(void *L, double vr, double vi, int p, int q) { CL(L)->AddTo(CComplex(vr, vi), p, q); }
void ref_clp_get(void *L, int p, int q, double *vr, double *vi)
{
    CComplex z = CL(L)->Get(p, q);
    *vr = z.re;
    *vi = z.im;
}
void ref_clp_put(void *L, double vr, double vi, int p, int q) { CL(L)->Put(CComplex(vr, vi), p, q); }
double *ref_clp_b(void *L) { return reinterpret_cast<double *>(CL(L)->b); }
double *ref_clp_V(void *L) { return reinterpret_cast<double *>(CL(L)->V); }
void ref_clp_setvalue(void *L, int i, double xr, double xi) { CL(L)->SetValue(i, CComplex(xr, xi)); }
void ref_clp_periodicity(void *L, int i, int j) { CL(L)->Periodicity(i, j); }
void ref_clp_antiperiodicity(void *L, int i, int j) { CL(L)->AntiPeriodicity(i, j); }
int ref_clp_solve(void *L, int flag) { return CL(L)->PBCGSolveMod(flag, false) ? 1 : 0; }
void ref_clp_wipe(void *L) { CL(L)->Wipe(); }
void ref_clp_put_k(void *L, double vr, double vi, int p, int q, int k) { CL(L)->Put(CComplex(vr, vi), p, q, k); }
void ref_clp_get_k(void *L, int p, int q, int k, double *vr, double *vi)
{
    CComplex v = CL(L)->Get(p, q, k);
    *vr = v.re;
    *vi = v.im;
}
int ref_clp_newton(void *L) { return CL(L)->bNewton ? 1 : 0; }
void ref_clp_set_precision(void *L, double precision) { CL(L)->Precision = precision; }

}  // extern "C"
