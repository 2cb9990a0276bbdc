/* CPU oracle for the fsolver static-2D hot path.
 *
 * TEST INFRASTRUCTURE ONLY: the checker, never the thing measured or shipped.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it.
 *
 * Restates, in plain C:
 *   CBigLinProb (linked-list symmetric sparse matrix + SSOR-PCG)
 *       cfemm/libfemm/spars.cpp:35-495, spars.h:38-83
 *   FSolver::Static2D (element assembly, BCs, nonlinear B-H Newton loop)
 *       cfemm/fsolver/static2d.cpp:53-1033
 *   FSolver::StaticAxisymmetric (r-weighted element matrices with the
 *       logarithmic R_hat, r-weighted sources, A = 0 on the axis, output
 *       converted to flux 2 pi r A)  cfemm/fsolver/staticaxi.cpp:45-794
 *   CMSolverMaterialProp::GetBHProps (cubic Hermite B-H interpolation)
 *       cfemm/libfemm/CMaterialProp.cpp:997-1057
 *
 * The linear-algebra layer is reached through ora_linprob_ops so the same
 * Static2D restatement can drive either this file's CBigLinProb restatement
 * or the reference's own spars.cpp compiled from /root/reference
 * (oracle/ref_adapter.cpp -> oracle/_ref/libxfemm_ref.so); identical results
 * of the two pin the restatement bit for bit.
 */
#ifndef XFEMM_STATIC2D_ORACLE_H
#define XFEMM_STATIC2D_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    double mu_x, mu_y;      /* relative permeabilities (GetSlopes overwrites for B-H) */
    double H_c;             /* coercivity, A/m */
    double J_re;            /* source current density, MA/m^2 */
    double Cduct;           /* conductivity, MS/m */
    double LamFill;
    int LamType;
    int BHpoints;
    const double *Bdata;    /* BHpoints entries, after GetSlopes */
    const double *Hdata;    /* real parts */
    const double *slope;    /* real parts */
} ora_block;

typedef struct {
    int InCircuit;          /* -1 if none */
    double MagDir;          /* degrees */
    int bIsWound;
    int IsExternal;         /* axisymmetric: conformally mapped exterior region */
} ora_label;

typedef struct {
    int BdryFormat;
    double A0, A1, A2, phi;
    double c0, c1;          /* real parts */
} ora_line;

typedef struct {
    double A_re, A_im, J_re, J_im;
} ora_point;

typedef struct {
    int CircType;
    double Amps_re;
    double dVolts_re;
    int Case;               /* out */
    double J;               /* out */
    double dV;              /* out */
} ora_circ;

/* CAirGapElement after FSolver::LoadMesh (fsolver.cpp:425-515). */
typedef struct {
    int BdryFormat;             /* 0 periodic, 1 antiperiodic copies */
    double ri, ro, totalArcLength, InnerShift, OuterShift;
    int totalArcElements;
    const int *qn;              /* quadNode[k].n0..n3 at 4k+0..3, k = 0..totalArcElements */
    const double *qw;           /* quadNode[k].w0..w3 */
} ora_age;

typedef void (*ora_age_emit)(void *ctx, double v, int p, int q);
/* MG of one arc element (row-major 10x10), static2d.cpp:209-263. */
void ora_age_matrix(double ci, double co, double K, double Ki, double *MG);
/* Every air-gap contribution as AddTo(v, p, q) calls in the reference's order
 * (static2d.cpp:191-344). */
void ora_age_assemble(int n_ages, const ora_age *ages, int harmonic, ora_age_emit emit, void *ctx);

typedef struct {
    int n_nodes;
    const double *x, *y;        /* cm */
    const int *marker;          /* point-prop index or -1 */
    int n_elems;
    const int *p;               /* 3 per element */
    const int *e;               /* 3 per element: boundary-prop index or -1 */
    const int *lbl;
    const int *blk;
    int n_blocks;  const ora_block *blocks;
    int n_labels;  const ora_label *labels;
    int n_lines;   const ora_line *lines;
    int n_points;  const ora_point *points;
    int n_circs;   ora_circ *circs;
    int n_pbc;     const int *pbc;      /* 3 per pair: x, y, t (0 periodic, 1 anti) */
    double precision;
    int length_units;
    int coords;                 /* 0 cartesian, 1 polar */
    int bandwidth;              /* CBigLinProb bdw (0 = full scan) */
    double relax;               /* FSolver::Relax (1.0 after LoadProblemFile) */
    int axisymmetric;           /* ProblemType: 0 planar (Static2D), 1 axisymmetric */
    double ext_ro, ext_ri, ext_zo;   /* exterior-region parameters (user units) */
    int n_ages;  const ora_age *ages;   /* air-gap elements (planar only, as the reference) */
    const double *elem_magdir;  /* per element: the direction a label's MagDirFctn gives (degrees,
                                   from the reference's own Lua, oracle/ref_lua.cpp); NULL = the
                                   labels' constant MagDir */
} ora_problem;

typedef struct {
    int newton_iters;           /* number of linear solves */
    long long cg_iters;         /* total PCG iterations (-1 if unknown) */
    double last_res;            /* last nonlinear residual */
} ora_stats;

typedef struct {
    void *(*create)(int n, int bw, double precision);
    void (*destroy)(void *L);
    void (*addto)(void *L, double v, int p, int q);
    double *(*b)(void *L);
    double *(*V)(void *L);
    void (*setvalue)(void *L, int i, double x);
    void (*periodicity)(void *L, int i, int j);
    void (*antiperiodicity)(void *L, int i, int j);
    void (*wipe)(void *L);
    int (*pcgsolve)(void *L, int flag, long long *iters);
} ora_linprob_ops;

/* The built-in CBigLinProb restatement. */
const ora_linprob_ops *ora_builtin_linprob(void);

/* FSolver::Static2D / StaticAxisymmetric (pr->axisymmetric); A_out[i] is
 * the value written to .ans: V[i] * c, times 2 pi r (m) when axisymmetric. */
int ora_static2d(ora_problem *pr, const ora_linprob_ops *ops, double *A_out,
                 ora_stats *stats);

/* Iter-0 system after assembly and all boundary conditions, exported as the
 * upper-triangular COO of the restated CBigLinProb plus b. */
int ora_static2d_system(ora_problem *pr, int *rows, int *cols, double *vals, long long cap,
                        double *b_out, long long *nnz_out);

/* CMSolverMaterialProp::GetBHProps(B, v, dv) on the real axis. */
void ora_get_bh_props(const ora_block *m, double B, double *v, double *dv);

/* Stand-alone access to the restated CBigLinProb for tests. */
void *ora_lp_create(int n, int bw, double precision);
void ora_lp_destroy(void *L);
void ora_lp_addto(void *L, double v, int p, int q);
double ora_lp_get(void *L, int p, int q);
double *ora_lp_b(void *L);
double *ora_lp_V(void *L);
void ora_lp_setvalue(void *L, int i, double x);
void ora_lp_periodicity(void *L, int i, int j);
void ora_lp_antiperiodicity(void *L, int i, int j);
int ora_lp_pcgsolve(void *L, int flag, long long *iters);
void ora_lp_multA(void *L, const double *X, double *Y);
/* Export the (symmetric) matrix as upper-triangular COO; returns nnz stored. */
long long ora_lp_export_upper(void *L, int *rows, int *cols, double *vals, long long cap);

#ifdef __cplusplus
}
#endif
#endif
