/* CPU oracle for the fsolver harmonic-2D (time-harmonic planar) path.
 *
 * TEST INFRASTRUCTURE ONLY: the checker, never the thing measured or shipped.
 * Only tests/ and __graft_entry__.smoke() may load it.
 *
 * Restates, in plain C:
 *   CComplex arithmetic               cfemm/libfemm/liblua/femmcomplex.cpp:300-760
 *   CBigComplexLinProb                cfemm/libfemm/cspars.cpp:40-1081
 *     (upper-triangular linked rows, complex-symmetric MultA, SSOR MultPC,
 *      SetValue, (Anti)Periodicity, PCGSQStart + PBCGSolve = PBCGSolveMod)
 *   FSolver::Harmonic2D               cfemm/fsolver/harmonic2d.cpp:36-873
 *   FSolver::HarmonicAxisymmetric     cfemm/fsolver/harmonicaxi.cpp:1-800
 *     (r-weighted flux formulation, eddy current lumped to the element mean,
 *      r-weighted boundary terms / sources / point currents / circuits, A = 0
 *      on the axis, B from the element energy, exterior-region warp; answers
 *      are the flux 2 pi r A)
 *     (effective permeabilities with hysteresis lag and laminations, eddy
 *      currents, mixed and small-skin-depth boundaries, complex sources,
 *      circuits of Case 0 / 1 / 2, point currents, Dirichlet, periodicity;
 *      nonlinear blocks: the successive approximation of ACSolver 0 --
 *      averaged permeability from Get_v / GetdHdB, the Mn V correction,
 *      relaxation -- on the complex curve GetSlopes(omega) produced, which is
 *      an INPUT here: the host restatement of that preprocessing is pinned
 *      separately against the reference's CMaterialProp.cpp,
 *      tests/test_oracle_acslopes.py)
 *
 * As for the static oracle, the linear algebra is reached through
 * orh_linprob_ops so the restated element loop can drive either the restated
 * CBigComplexLinProb or the reference's own cspars.cpp compiled from
 * /root/reference into oracle/_ref (ref_adapter.cpp); identical results pin
 * the restatement.
 */
#ifndef XFEMM_HARMONIC2D_ORACLE_H
#define XFEMM_HARMONIC2D_ORACLE_H

#include "static2d_oracle.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    double mu_x, mu_y;          /* relative permeabilities */
    double Theta_hx, Theta_hy;  /* hysteresis lag, degrees */
    double Lam_d, LamFill;      /* lamination thickness (mm), fill factor */
    double J_re, J_im;          /* MA/m^2 */
    double Cduct;               /* MS/m */
    int LamType;
    int BHpoints;               /* 0 = linear */
    /* BHpoints > 0: the curve processed by GetSlopes(omega) (B, complex H, complex slope) */
    const double *B, *H_re, *H_im, *S_re, *S_im;
} orh_block;

typedef struct {
    int InCircuit;
    int bIsWound;
    int IsExternal;             /* exterior region (axisymmetric) */
    double ProxMu_re, ProxMu_im;   /* ProximityMu (GetFillFactor): LamType > 2 wound regions */
} orh_label;

typedef struct {
    int BdryFormat;             /* 0 prescribed A, 1 small skin depth, 2 mixed, 4/5 (anti)periodic */
    double A0, A1, A2, phi;
    double c0_re, c0_im, c1_re, c1_im;
    double Mu, Sig;             /* small-skin-depth parameters */
} orh_line;

typedef struct {
    int CircType;               /* 0 specified current, 1 specified voltage gradient */
    double Amps_re, Amps_im, dVolts_re, dVolts_im;
    int Case;                   /* out */
    double J_re, J_im;          /* out (Case 1) */
    double dV_re, dV_im;        /* out (Case 0 / 2) */
} orh_circ;

typedef struct {
    int n_nodes;
    const double *x, *y;        /* cm */
    const int *marker;          /* point-prop index or -1 */
    int n_elems;
    const int *p, *e, *lbl, *blk;
    int n_blocks;  const orh_block *blocks;
    int n_labels;  const orh_label *labels;
    int n_lines;   const orh_line *lines;
    int n_points;  const ora_point *points;
    int n_circs;   orh_circ *circs;
    int n_pbc;     const int *pbc;
    double precision;
    double frequency;           /* Hz */
    int length_units;
    int coords;
    int bandwidth;              /* CBigComplexLinProb bdw (0 = full scan) */
    int problem_type;           /* 0 planar (Harmonic2D), 1 axisymmetric (HarmonicAxisymmetric) */
    double extZo, extRo, extRi; /* exterior region (axisymmetric), length units of the file */
    int n_ages;  const ora_age *ages;   /* air-gap elements (planar only) */
    int ac_solver;              /* [ACSolver]: 0 successive approximation, 1 Newton (KludgeSolve) */
} orh_problem;

typedef struct {
    void *(*create)(int n, int bw, int nodes, double precision);
    void (*destroy)(void *L);
    void (*addto)(void *L, double vr, double vi, int p, int q);
    void (*get)(void *L, int p, int q, double *vr, double *vi);
    void (*put)(void *L, double vr, double vi, int p, int q);
    double *(*b)(void *L);      /* interleaved re, im */
    double *(*V)(void *L);
    void (*setvalue)(void *L, int i, double xr, double xi);
    void (*periodicity)(void *L, int i, int j);
    void (*antiperiodicity)(void *L, int i, int j);
    int (*solve)(void *L, int flag);   /* PBCGSolveMod(flag, false) */
    void (*wipe)(void *L);             /* Wipe(): matrix and b to zero, V kept */
    /* Newton AC solver: the auxiliary matrices k = 1 (Hermitian Mh), 2 (symmetric
     * Ms, applied to conj(x)), 3 (anti-Hermitian Ma) of Put / Get (cspars.cpp:147-283) */
    void (*put_k)(void *L, double vr, double vi, int p, int q, int k);
    void (*get_k)(void *L, int p, int q, int k, double *vr, double *vi);
    int (*newton)(void *L);            /* bNewton */
    void (*set_precision)(void *L, double precision);
} orh_linprob_ops;

const orh_linprob_ops *orh_builtin_linprob(void);

/* FSolver::Harmonic2D; A = V * c (the values written to .ans), interleaved
 * re/im per node; circuit results in pr->circs. */
int orh_harmonic2d(orh_problem *pr, const orh_linprob_ops *ops, double *A_out, ora_stats *stats);

/* Get_v(B) and GetdHdB(B) of a nonlinear block's complex curve
 * (CMaterialProp.cpp:461-486, 899-903), interleaved re/im, for nq values. */
void orh_acprops(const orh_block *b, const double *Bq, int nq, double *v, double *dhdb);

/* The assembled system after all boundary conditions (node rows only), as
 * upper-triangular COO (interleaved complex values) plus b. */
int orh_harmonic2d_system(orh_problem *pr, int *rows, int *cols, double *vals, long long cap, double *b_out,
                          long long *nnz_out);

#ifdef __cplusplus
}
#endif
#endif
