/* xfemm_kernels.h -- C-ABI of the MI355X (gfx950) fsolver hot path.
 *
 * Thin boundary between the C++ host side (FSolver, include/xfemm_fsolver.h)
 * and the hand-written HIP kernels: plain pointers and sizes, no C++ or torch
 * types.  One xfk_problem holds one static-2D magnetostatic problem resident
 * in HBM; xfk_static2d() runs the whole reference Static2D on the GPU:
 * element assembly into CSR, point/segment/(anti)periodic boundary conditions,
 * the preconditioned conjugate-gradient solve and the nonlinear B-H Newton loop.
 *
 * Reference interfaces replaced (temudschin/xfemm @ 2025-02-04):
 *   xfk_static2d          FSolver::Static2D(CBigLinProb&)   cfemm/fsolver/static2d.cpp:53
 *                         (called from FSolver::runSolver   cfemm/fsolver/fsolver.cpp:1266)
 *   xfk_pcg_solve         CBigLinProb::PCGSolve(int flag)   cfemm/libfemm/spars.cpp:238
 *   xfk_csr_*             CBigLinProb::MultA / Dot          cfemm/libfemm/spars.cpp:167,187
 *   xfk_problem_create    the state FSolver::LoadMesh + LoadProblemFile leave behind
 *                         (meshnode, meshele, the prop lists)      cfemm/fsolver/fsolver.cpp:202,350
 *
 * All functions return XFK_OK (0) or a negative error code; xfk_last_error()
 * gives the message of the last failure on the calling thread.  There is no
 * CPU fallback: without a usable gfx950 device every call fails.
 */
#ifndef XFEMM_KERNELS_H
#define XFEMM_KERNELS_H

#ifdef __cplusplus
extern "C" {
#endif

enum {
    XFK_OK = 0,
    XFK_ERR_ARG = -1,
    XFK_ERR_HIP = -2,
    XFK_ERR_SINGULAR = -3,      /* zero diagonal: "singular flag tripped" (spars.cpp:245) */
    XFK_ERR_NOCONV = -4,        /* iteration cap reached */
    XFK_ERR_UNSUPPORTED = -5
};

/* CMSolverMaterialProp after GetSlopes(0) (CMaterialProp.h:193). */
typedef struct {
    double mu_x, mu_y;          /* relative permeability */
    double H_c;                 /* coercivity, A/m */
    double J_re;                /* applied current density, MA/m^2 */
    double Cduct;               /* conductivity, MS/m */
    double LamFill;
    int LamType;
    int BHpoints;               /* 0 = linear */
    const double *B;            /* BHpoints: processed B-H curve (T) */
    const double *H;            /* BHpoints: A/m (real parts) */
    const double *slope;        /* BHpoints: dH/dB at the knots */
} xfk_block_desc;

/* CMBlockLabel (CBlockLabel.h:153) after FSolver::GetFillFactor. */
typedef struct {
    int block;                  /* index into blocks */
    int in_circuit;             /* -1 = none */
    double mag_dir;             /* magnetisation direction, degrees */
    int is_wound;
    int is_external;            /* axisymmetric: conformally mapped exterior region ([IsExternal]) */
    const char *mag_dir_fctn;   /* MagDirFctn: Lua expression of the element centroid (x y r z theta R)
                                   giving the direction per element (static2d.cpp:511-581,
                                   staticaxi.cpp:354-404); NULL or "" = the constant mag_dir.
                                   Static problems only, as in the reference. */
} xfk_label_desc;

/* CMBoundaryProp (CBoundaryProp.h). */
typedef struct {
    int format;                 /* BdryFormat: 0 prescribed A, 2 mixed, 4 periodic, 5 antiperiodic */
    double A0, A1, A2, phi;
    double c0, c1;
} xfk_line_desc;

/* CMPointProp (CPointProp.h). */
typedef struct {
    double A_re, A_im, J_re, J_im;
} xfk_point_desc;

/* CMCircuit (CCircuit.h) after FSolver::LoadProblemFile's serial expansion. */
typedef struct {
    int type;                   /* 0 parallel/voltage, 1 not expected here */
    double amps_re;
    double dvolts_re;
} xfk_circuit_desc;

/* CAirGapElement (cfemm/libfemm/CAirGapElement.h) as FSolver::LoadMesh reads it
 * from the .pbc file (fsolver.cpp:425-515): an unmeshed annulus between two
 * rings of equally spaced boundary nodes, coupled by totalArcElements
 * "air-gap elements" (static2d.cpp:191-344, harmonic2d.cpp:227-380). */
typedef struct {
    int format;                 /* BdryFormat: 0 periodic, 1 antiperiodic copies */
    double ri, ro;              /* inner / outer radius */
    double total_arc_length;    /* degrees spanned by the AGE */
    double inner_shift, outer_shift;   /* InnerShift / OuterShift, in arc elements */
    int n_arc;                  /* totalArcElements */
    const int *qn;              /* 4 * (n_arc + 1): quadNode[k].n0 n1 n2 n3 */
    const double *qw;           /* 4 * (n_arc + 1): quadNode[k].w0 w1 w2 w3 */
} xfk_age_desc;

typedef struct {
    int n_nodes;
    const double *x, *y;        /* node coordinates, cm */
    const int *marker;          /* point-prop index or -1 (may be NULL) */
    int n_elems;
    const int *p;               /* 3 per element */
    const int *e;               /* 3 per element: boundary-prop index or -1 (may be NULL) */
    const int *lbl;             /* block label of each element */
    int n_blocks;  const xfk_block_desc *blocks;
    int n_labels;  const xfk_label_desc *labels;
    int n_lines;   const xfk_line_desc *lines;
    int n_points;  const xfk_point_desc *points;
    int n_circs;   const xfk_circuit_desc *circs;
    int n_pbc;     const int *pbc;      /* 3 per pair: node, node, type (0 periodic, 1 anti) */
    double precision;           /* [Precision] */
    int length_units;           /* femm::LengthUnit */
    int coords;                 /* 0 cartesian, 1 polar */
    double relax;               /* FSolver::Relax, 1.0 */
    int problem_type;           /* [ProblemType]: XFK_PLANAR (Static2D) or XFK_AXISYMMETRIC
                                   (FSolver::StaticAxisymmetric, staticaxi.cpp:45-794: x is r, y is z) */
    double ext_zo, ext_ro, ext_ri;   /* [extZo] [extRo] [extRi]: axisymmetric exterior region, user units */
    int n_ages;  const xfk_age_desc *ages;   /* air-gap elements (planar; ignored when axisymmetric,
                                                as StaticAxisymmetric / HarmonicAxisymmetric do) */
} xfk_problem_desc;

enum { XFK_PLANAR = 0, XFK_AXISYMMETRIC = 1 };

typedef struct {
    int newton_iters;           /* linear solves performed */
    long long cg_iters;         /* total PCG iterations */
    double last_res;            /* last nonlinear residual */
    double final_er;            /* last PCG preconditioned residual ratio */
    long long nnz;              /* CSR nonzeros (full symmetric storage) */
    int ncolors;                /* element colours of the assembly scatter */
    double ms_symbolic;         /* device time, ms */
    double ms_assemble;
    double ms_solve;
    double spmv_ms_avg;         /* XFK_TIME_SPMV: mean HIP-event time of one SpMV launch */
    int spmv_samples;           /* launches sampled (every 16th PCG iteration) */
    int color_rounds;           /* Jones-Plassmann rounds of the element colouring */
    int precond;                /* preconditioner of the last solve (XFK_PRECOND_*) */
    int amg_levels;             /* AMG: levels of the last hierarchy */
    double amg_op_complexity;   /* AMG: sum of level nonzeros / fine nonzeros */
    double ms_amg_setup;        /* AMG: device time of the hierarchy setups, ms (inside ms_solve) */
    /* sharded solves with XFK_TIME_TAIL: device time of the replicated coarse
     * levels (every rank builds and applies them): the V-cycles' all-gather of
     * the coarse right-hand side + the replicated cycle, summed over the solve,
     * and the setup's build of the replicated levels */
    double ms_rep_cycle;
    int rep_cycles;             /* V-cycles timed */
    double ms_rep_setup;
    int prec_fallback;          /* 1: a stagnating PCG switched the AMG's f32 parts (level-0 transfers,
                                   coarsest inverse) to f64 and restarted; kept for the problem's life */
} xfk_result;

typedef struct xfk_problem xfk_problem;

const char *xfk_last_error(void);
int xfk_device_count(void);
/* Bring up the HIP runtime on `device` ahead of the first solve: the runtime
 * and the device context (~0.4 s in a fresh process), every code object of
 * this library, and a few streams for the process's stream pool.  Idempotent
 * and thread-safe; the FSolver runs it on a thread of its own beside
 * LoadMesh / Cuthill, so a fresh `fsolver` process does not wait for it in
 * series.  XFK_OK, or XFK_ERR_HIP when there is no such device. */
int xfk_device_init(int device);

/* Upload a problem; nothing is computed yet.  Host arrays may be freed after. */
int xfk_problem_create(const xfk_problem_desc *desc, int device, xfk_problem **out);
void xfk_problem_destroy(xfk_problem *prob);

enum { XFK_REBUILD_SYMBOLIC = 1, XFK_TIME_SPMV = 2, XFK_TIME_TAIL = 4 };

/* Solver options.  The reference preconditions its PCG with a sequential
 * SSOR sweep (spars.cpp:186-236, CBigLinProb::MultPC); the device offers
 *   XFK_PRECOND_AMG    smoothed-aggregation AMG V-cycle (default; rebuilt for
 *                      every matrix the Newton loop assembles; sharded solves
 *                      use it as a rank-local block preconditioner)
 *   XFK_PRECOND_JACOBI diag(A)
 * Both keep the reference's stopping test sqrt(z.r / z0.b) <= Precision.
 * A hierarchy whose SpGEMM rows overflow the LDS tables falls back to Jacobi
 * for that solve (xfk_result.precond tells which one ran). */
enum { XFK_PRECOND_JACOBI = 0, XFK_PRECOND_AMG = 1 };
enum {
    XFK_OPT_PRECOND = 1,        /* XFK_PRECOND_* */
    XFK_OPT_AMG_SWEEPS = 2,     /* Jacobi sweeps before and after the coarse correction (1..8, default 1) */
    XFK_OPT_AMG_THETA = 3,      /* strength threshold (0..1, default 0.08) */
    XFK_OPT_AMG_OMEGA = 4,      /* Jacobi weight factor: weight = omega / rho(D^-1 A) (0..2, default 1.75) */
    XFK_OPT_AMG_REPLICATE = 5,  /* sharded solve: coarse levels of at most this many global rows are
                                   replicated on every rank, larger ones stay sharded (default 250000) */
    XFK_OPT_AMG_REUSE = 6,      /* 1 (default): later Newton iterations of one solve keep the hierarchy
                                   and refresh only the fine-level smoother, rebuilt when the PCG needs
                                   2x the iterations of the last fresh build; 0: rebuild every time */
    XFK_OPT_AMG_DENSE = 7,      /* coarsening stops at a level of at most this many rows, which is
                                   solved by its dense inverse (16..2048, default 2048) */
    XFK_OPT_AMG_FOLD = 8,       /* 1 (default, or XFK_AMG_FOLD from the environment): V(1,1) levels
                                   run folded (one pass over P~ = (I - w D^-1 A) P for prolongation +
                                   post-sweep, coarse pre-steps with R~ = P~^T); 0: the plain cycle */
    XFK_OPT_AMG_COL16 = 9,      /* 1 (default, unless XFK_NO_COL16 is set): single-device level-0
                                   operators (the PCG SpMV, the sweeps, P~, R) read 16-bit column
                                   offsets per row tile (tiles spanning > 65535 columns read the int
                                   columns); 0: int columns.  The same column indices: the same bits. */
    XFK_OPT_AMG_WLEVEL = 10,    /* the folded coarse level that runs a W-cycle (two coarse
                                   corrections); -2 (default): the level above the last V-cycle
                                   level (XFK_AMG_W overrides), -1: a plain V-cycle */
    XFK_OPT_AMG_F32 = 11,       /* 1 (default, unless XFK_AMG_F32=0 is set; needs 16-bit columns):
                                   the V-cycle's level-0 transfers (R, P~) store f32 values,
                                   products and sums in f64; 0: f64 values.  The sweeps and the
                                   PCG's own SpMV keep A in f64. */
    XFK_OPT_NEWTON_INEXACT = 12 /* 1 (default, unless XFK_NEWTON_INEXACT=0 is set): the nonlinear
                                   loop's passes before the last solve their linear system to a
                                   forcing tolerance (Eisenstat-Walker: eta times the last Newton
                                   change |dV| / |V|, clamped to [Precision, 1e-3]); a pass that
                                   meets the loop's stop test (|dV| / |V| < 100 Precision) at a
                                   tolerance looser than Precision is followed by one more pass
                                   solved to Precision, so the answer is always that of a pass
                                   solved to the reference's tolerance.  0: every pass to
                                   Precision, as the reference (static2d.cpp:997-1008). */
};
int xfk_set_option(xfk_problem *prob, int option, double value);

/* FSolver::Static2D on the device.  flags: XFK_REBUILD_SYMBOLIC rebuilds the
 * CSR pattern, colouring and boundary maps (they are cached otherwise);
 * XFK_TIME_SPMV brackets every 16th SpMV launch with HIP events on the
 * solver stream and reports the mean launch duration; XFK_TIME_TAIL (sharded
 * solves) brackets the replicated coarse levels of every V-cycle and of the
 * setup (ms_rep_cycle, ms_rep_setup). */
int xfk_static2d(xfk_problem *prob, int flags, xfk_result *res);

/* A at every node (V * c, the value fsolver writes to .ans), host copy. */
int xfk_get_solution(xfk_problem *prob, double *A_host);

/* Circuit results after xfk_static2d: case (0/1), J, dV per circuit. */
int xfk_get_circuits(xfk_problem *prob, int *ccase, double *J, double *dV);

/* ---------------------------------------------------------------------------
 * Sharded solve (one large mesh across ranks, configs[4]).
 *
 * Rows (nodes, in the caller's -- normally Cuthill-McKee -- numbering) are
 * split into contiguous blocks, one per rank; each rank assembles the
 * elements touching its rows (ghost elements replicated, no communication),
 * exchanges the halo of the PCG vector before every SpMV, and all-reduces the
 * PCG's per-block dot-product partials once per iteration.  Boundary
 * conditions and circuits are evaluated on the GLOBAL mesh, so every rank
 * passes the same global description.  Periodic / antiperiodic pairs and
 * air-gap nodes ("coupled nodes") are assembled on every rank that needs them
 * (the averaging map of its owned rows then finds every entry locally).
 *
 * xfk_static2d and xfk_get_solution are collective over the communicator
 * (every rank calls them); xfk_get_solution returns the global solution on
 * every rank.
 * ------------------------------------------------------------------------- */
typedef struct xfk_comm xfk_comm;

/* RCCL, one process per GPU: rank 0 creates the 128-byte unique id, the caller
 * distributes it (e.g. torch.distributed broadcast), every rank then calls
 * xfk_comm_create_rccl (collective). */
int xfk_comm_unique_id(void *out, int bytes);
int xfk_comm_create_rccl(const void *unique_id, int bytes, int rank, int nranks, int device, xfk_comm **out);
/* In-process group of nranks communicators (one host thread per rank, any
 * devices, including several ranks on one device): the test transport. */
int xfk_comm_create_local(int nranks, xfk_comm **out_array);
void xfk_comm_destroy(xfk_comm *comm);
int xfk_comm_rank(const xfk_comm *comm);
int xfk_comm_size(const xfk_comm *comm);

/* Issue order and recording.  Every collective of a communicator runs after
 * the previous one in device order: when a collective is enqueued on another
 * stream than the previous collective, the communicator first makes that
 * stream wait for the event recorded after the previous one (RCCL matches
 * collectives by issue order; the sharded path issues halo exchanges on a side
 * stream and all-reduces / all-gathers on the main stream).
 *
 * xfk_comm_record(comm, mode) starts an empty recording (mode 1: the sequence
 * of collectives; mode 2: the sequence and every byte the rank receives, kept
 * in device memory, for xfk_comm_create_replay), or stops it (mode 0; the log
 * is kept).  xfk_comm_log copies the log: one ALLREDUCE / ALLGATHER / EXCHANGE
 * record per collective call, each EXCHANGE followed by one SEND / RECV
 * record per halo range.  Every rank of a correct program produces the same
 * sequence of calls (op, stream, bytes), and the send of rank a to rank b in
 * exchange k matches the receive of b from a in the same exchange. */
enum { XFK_COMM_ALLREDUCE = 1, XFK_COMM_EXCHANGE = 2, XFK_COMM_SEND = 3, XFK_COMM_RECV = 4, XFK_COMM_ALLGATHER = 5 };
typedef struct {
    long long seq;              /* collective number since the recording started */
    int op;                     /* XFK_COMM_* */
    int stream;                 /* stream index in first-use order (0: the first stream this communicator saw) */
    int waited;                 /* 1: another stream than the previous collective's; the communicator
                                   made it wait for that collective's completion event */
    int peer;                   /* SEND / RECV: the peer rank; -1 otherwise */
    long long bytes;            /* payload: ALLREDUCE the reduced bytes, ALLGATHER the bytes per rank,
                                   SEND / RECV the range; EXCHANGE 0 */
    long long g0;               /* SEND / RECV: the range's first global row; EXCHANGE: its range count */
} xfk_comm_op;
int xfk_comm_record(xfk_comm *comm, int mode);
int xfk_comm_log(const xfk_comm *comm, xfk_comm_op *out, int cap, int *count);
/* A communicator that replays the recording (mode 2) of `recorded`: same rank
 * and size, no peers; every collective checks that it is the next one of the
 * recording (op and sizes, else XFK_ERR_ARG) and copies the recorded received
 * bytes into place.  The recording is cut into one segment per solve
 * (xfk_static2d); replayed solve k is served segment k, the last segment
 * repeating, and must issue exactly that segment's collectives (a first and a
 * repeated solve differ: the PCG's batching uses the last solve's iteration
 * count).  It runs one rank of a sharded solve alone on its GPU with the
 * exact inputs of the recorded run: the per-rank compute time without the
 * transport. */
int xfk_comm_create_replay(const xfk_comm *recorded, xfk_comm **out);
/* Time inside collectives (the N > 1 bench line's diagnosis).  With timing on
 * (xfk_comm_time(comm, 1)) every collective is bracketed by two HIP events on
 * the stream it is issued on: the interval covers the transfer and any wait
 * for the peers' matching call (an RCCL kernel starts only when its peers'
 * have).  xfk_comm_timing waits for those events and returns, per op
 * (index 0 all-reduce, 1 halo exchange, 2 all-gather), the number of calls
 * and the summed and longest microseconds since the last read, then clears
 * them.  Timing off (the default): no events. */
int xfk_comm_time(xfk_comm *comm, int on);
int xfk_comm_timing(xfk_comm *comm, long long calls[3], double us_total[3], double us_max[3]);

typedef struct {
    int rank, nranks;
    int n_global;               /* global nodes */
    int row0, n_own;            /* owned rows [row0, row0 + n_own) */
    int n_halo;                 /* halo nodes (local ids n_own .. n_own + n_halo - 1) */
    int n_elems;                /* local (owned + ghost) elements */
    int n_send, n_recv;         /* halo ranges */
    int n_extra;                /* coupled nodes owned elsewhere, assembled here (local ids n_own ..) */
} xfk_dist_info;

/* Host-only partition plan (no device needed).  Call once with null arrays to
 * get the sizes in *info, then with l2g[n_own + n_halo], elems[n_elems],
 * recv[4 * n_recv] and send[4 * n_send] ({peer, local offset, length, first
 * global row} per range). */
int xfk_partition_plan(int n_nodes, int n_elems, const int *p, int rank, int nranks, xfk_dist_info *info,
                       int *l2g, int *elems, int *recv, int *send);
/* The same with coupled nodes (periodic pairs, air-gap quad nodes): every
 * element touching one is local on every rank, the coupled nodes owned
 * elsewhere are the first n_extra halo nodes (assembled rows), and a peer may
 * send several ranges (coupled nodes first).  xfk_problem_create_dist plans
 * this way for problems with periodic boundaries or air gaps. */
int xfk_partition_plan_coupled(int n_nodes, int n_elems, const int *p, int rank, int nranks, int n_coupled,
                               const int *coupled, xfk_dist_info *info, int *l2g, int *elems, int *recv, int *send);

/* This rank's part of the global problem `desc` on `device`. */
int xfk_problem_create_dist(const xfk_problem_desc *desc, int device, xfk_comm *comm, xfk_problem **out);
int xfk_dist_get_info(const xfk_problem *prob, xfk_dist_info *info);

/* ---------------------------------------------------------------------------
 * Time-harmonic planar problems: FSolver::Harmonic2D
 * (cfemm/fsolver/harmonic2d.cpp:36-790) with CBigComplexLinProb::PBCGSolveMod
 * (cspars.cpp:822-895, 1062-1081) as the solver.
 *
 * The base descriptor carries the real parts; these arrays (same lengths as
 * desc->blocks / lines / circs) carry what the AC formulation adds.  Blocks
 * with a B-H curve run the reference's successive-approximation loop
 * (ACSolver 0: averaged secant / incremental permeability per element,
 * residual correction on the right-hand side, relaxation after 5 iterations,
 * stop at |dV| / |V| < 100 Precision).  Case-2 circuits -- a specified
 * current in a conducting region, whose voltage gradient is an extra
 * unknown -- are solved through the Schur complement of the bordered system
 * (one extra COCG solve per such circuit; not with periodic boundaries).
 * ac_solver = 1 selects the reference's Newton AC solver instead
 * (harmonic2d.cpp:611-639, harmonicaxi.cpp:520-547): after the first pass the
 * nonlinear elements add their Newton terms -- Mn to the matrix, the
 * Hermitian / conj-symmetric / anti-Hermitian remainders to three auxiliary
 * matrices -- and every pass solves M V + Mh V + Ms conj(V) + Ma V = b by the
 * reference's KludgeSolve (cspars.cpp:1000-1060: at most 10 COCG solves on M
 * with the auxiliary terms moved to the right-hand side, each followed by a
 * line search on the true residual) at the adaptive precision
 * min(1e-4, 0.001 res) >= Precision (harmonic2d.cpp:821-825).
 * The reference itself rejects LamType 1/2 in AC analyses; wound regions
 * with proximity effects (LamType > 2) return XFK_ERR_UNSUPPORTED.  Single
 * device.
 * ------------------------------------------------------------------------- */
typedef struct {
    double J_im;                /* imaginary part of the source current density, MA/m^2 */
    double Theta_hx, Theta_hy;  /* hysteresis lag, degrees */
    double Lam_d;               /* lamination thickness, mm */
    /* nonlinear blocks (desc->blocks[k].BHpoints > 0, LamType 0): the curve
     * processed by GetSlopes(omega) (xfemm_bh_get_slopes_ac) -- B and the real
     * parts of H and slope in desc->blocks[k], the imaginary parts here; mu_x /
     * mu_y there are the curve's initial permeability, Theta_hx / Theta_hy
     * its Theta_hn.  NULL for linear blocks. */
    const double *H_im;
    const double *slope_im;
} xfk_block_ac_desc;

typedef struct {
    double c0_im, c1_im;        /* mixed BC, imaginary parts */
    double Mu, Sig;             /* small-skin-depth BC (BdryFormat 1): relative mu, MS/m */
} xfk_line_ac_desc;

typedef struct {
    double amps_im, dvolts_im;
} xfk_circuit_ac_desc;

typedef struct {
    double frequency;           /* Hz, > 0 */
    const xfk_block_ac_desc *blocks;
    const xfk_line_ac_desc *lines;      /* may be NULL when n_lines == 0 */
    const xfk_circuit_ac_desc *circs;   /* may be NULL when n_circs == 0 */
    int ac_solver;              /* [ACSolver]: 0 successive approximation, 1 Newton */
    const double *label_prox_mu;   /* 2 per label (re, im): CMBlockLabel::ProximityMu after
                                      FSolver::GetFillFactor (fsolver.cpp:1083-1193), the relative
                                      permeability of a wound region of a LamType > 2 block
                                      (harmonic2d.cpp:664-668); read for those labels only;
                                      NULL: 1 for every label */
} xfk_harmonic_desc;

int xfk_problem_create_harmonic(const xfk_problem_desc *desc, const xfk_harmonic_desc *ac, int device,
                                xfk_problem **out);
/* The same problem sharded over comm's ranks (row blocks, as
 * xfk_problem_create_dist): every rank passes the GLOBAL descriptors;
 * xfk_harmonic2d and xfk_get_solution_complex are collective.  COCG exchanges
 * the halo of its vectors before every SpMV and all-reduces its per-block
 * partials once per iteration; the AMG preconditioner is the sharded hierarchy
 * of the real surrogate (Amg::setup_dist).  Linear problems and the
 * successive-approximation nonlinear loop (ACSolver 0), the Newton AC solver
 * (ACSolver 1: the auxiliary matrices assembled per rank, the KludgeSolve
 * products exchange V / the step at the halo, its dot products all-reduced)
 * and Case-2 circuits (each rank holds the border columns of its rows; C . y
 * all-reduced, the small circuit system solved on every rank alike). */
int xfk_problem_create_harmonic_dist(const xfk_problem_desc *desc, const xfk_harmonic_desc *ac, int device,
                                     xfk_comm *comm, xfk_problem **out);
/* FSolver::Harmonic2D, or HarmonicAxisymmetric (harmonicaxi.cpp:1-800) when
 * desc->problem_type is XFK_AXISYMMETRIC, on the device (complex-symmetric
 * COCG, the reference's stopping test |r| / |b| <= Precision).  flags as for
 * xfk_static2d. */
int xfk_harmonic2d(xfk_problem *prob, int flags, xfk_result *res);
/* A = V * c at every node, interleaved (re, im); axisymmetric problems: the
 * flux V * c * 2 pi r * 0.01 (harmonicaxi.cpp:790). */
int xfk_get_solution_complex(xfk_problem *prob, double *A_host);
/* Circuit results: case, J and dV interleaved (re, im) per circuit. */
int xfk_get_circuits_complex(xfk_problem *prob, int *ccase, double *J, double *dV);
/* Assembled complex system after all boundary conditions (val, b interleaved). */
int xfk_get_csr_complex(xfk_problem *prob, int *rowptr, int *col, double *val, double *b);

/* Device views for the bench / tests (stream-ordered on the problem's stream). */
int xfk_get_csr(xfk_problem *prob, int *rowptr, int *col, double *val, double *b);
long long xfk_get_nnz(xfk_problem *prob);
/* Column-index bytes per nonzero the last solve's PCG SpMV read: 2 with the
   AMG's 16-bit tile offsets (plus 2 for every nonzero of a tile whose columns
   span more than 65535), 4 without them; -1 for a null problem. */
double xfk_spmv_col_bytes(xfk_problem *prob);
int xfk_get_stream(xfk_problem *prob, void **hip_stream);

/* Stand-alone PCG on a host-supplied full symmetric CSR (testing the solver
 * alone, CBigLinProb::PCGSolve semantics with the device preconditioner).
 * V is the initial guess (used when flag != 0) and receives the solution. */
int xfk_pcg_solve_csr(int n, const int *rowptr, const int *col, const double *val,
                      const double *b, double *V, int flag, double precision,
                      int device, long long *iters, double *er);
/* The same with a chosen preconditioner (XFK_PRECOND_*). */
int xfk_pcg_solve_csr_pc(int n, const int *rowptr, const int *col, const double *val,
                         const double *b, double *V, int flag, double precision,
                         int device, int precond, long long *iters, double *er);

/* Air-gap element matrix of one arc element (host math, no device needed):
 * MG (10 x 10, row-major) for the reduced ring shifts ci, co and
 * K = dr / (R dtheta), Ki = 1 / K.  Replaces the closed form of
 * cfemm/fsolver/static2d.cpp:209-263 (harmonic2d.cpp:245-300). */
int xfk_age_element_matrix(double ci, double co, double K, double Ki, double *MG);

/* Timing probe of the CG kernels (profiles / roofline): run `iters` PCG
 * iterations on the assembled system without a convergence stop; returns the
 * mean device time (ms) of the SpMV kernel and of one whole iteration. */
int xfk_pcg_time(xfk_problem *prob, int iters, double *ms_spmv, double *ms_iter);

/* Per-phase profile of a solved static problem (single device, AMG
 * preconditioner): with XFK_PROFILE_SETUP the AMG hierarchy is rebuilt for the
 * assembled matrix, then `iters` PCG iterations run without a convergence stop;
 * every phase -- setup steps per level, each V-cycle launch per level, the
 * PCG SpMV and update -- is bracketed by HIP events on the problem's stream.
 * Phases come back in first-seen order, aggregated by name: launches, total
 * device time, algorithmic bytes per launch (0 where the phase is not a
 * streaming kernel).  *count = phases written (<= cap). */
typedef struct {
    char name[64];
    int calls;
    double ms_total;
    double bytes_per_call;
} xfk_phase;
enum { XFK_PROFILE_SETUP = 1 };
int xfk_phase_profile(xfk_problem *prob, int iters, int flags, xfk_phase *out, int cap, int *count);

/* Diagnostics: device allocations of the library since the last reset, process
 * wide -- out[0] hipMalloc calls, out[1] their host ms, out[2] hipFree calls,
 * out[3] their host ms (a hipFree waits for the device).  Blocks served from
 * the process cache (what destroyed problems returned: xfk_problem_destroy
 * keeps their device blocks for the next problem of the process) are not
 * counted.  reset != 0 zeroes the counters after reading. */
int xfk_alloc_stats(double *out4, int reset);

/* Device memory of one problem (diagnostics): out4[0] bytes of the arena
 * chunks it holds, out4[1] their count, out4[2] bytes carved and live,
 * out4[3] bytes freed by its solves and kept for reuse by the next ones.  A
 * problem solved repeatedly stays at the footprint of its largest solve. */
int xfk_problem_memory(const xfk_problem *prob, long long *out4);
/* The process-wide caches a destroyed problem leaves for the next one: device
 * blocks (at most XFK_POOL_CAP_MB, default 64 GiB), pinned host buffers (at
 * most XFK_PIN_CAP_MB, default 1 GiB) and idle streams.  xfk_cache_stats:
 * out3[0] cached device bytes, out3[1] cached pinned bytes, out3[2] idle
 * streams.  xfk_release_cache gives all of them back to HIP (live problems
 * keep theirs). */
int xfk_cache_stats(long long *out3);
int xfk_release_cache(void);

/* AMG hints across problems (no reference counterpart: the reference rebuilds
 * nothing on the device).  The last single-device AMG setup of the process
 * leaves its SpGEMM slot capacities, MIS-2 round counts and coarsest
 * nested-dissection plan behind, keyed by the fine level's rows and nonzeros;
 * the next fresh problem of that size takes them as speculation checked on
 * the device (a capacity must be the class a measurement would pick, the plan
 * must match the coarsest pattern -- else that part is measured and redone),
 * so answers are bit-identical with or without them.  xfk_amg_forget_hints
 * drops them (XFK_AMG_NO_FOREIGN=1 never keeps any). */
int xfk_amg_forget_hints(void);

/* FEASolver::SortElements (cfemm/libfemm/cuthill.cpp:39-86; called from
 * FSolver::Cuthill) on the device: the reference's comb sort -- gap * 10 / 13
 * (9, 10 -> 11), swap on a strictly greater score, stop after the first pass
 * without a swap or after the first gap-1 pass (`while ((gap > 1) && (i > 0))`,
 * so the result need not be fully sorted) -- of the elements by
 * score[i] = p0 + p1 + p2 of element i, every pass simulated: the reference's
 * order, equal scores included.  perm[k] = the element at position k after
 * the sort. */
int xfk_sort_elements(int n_elems, const unsigned *score, int device, int *perm);

/* Magnetisation-direction function of a block label, evaluated for elements
 * as the reference's element loop does (FSolver::Static2D,
 * cfemm/fsolver/static2d.cpp:509-583; StaticAxisymmetric staticaxi.cpp:350-406):
 * the centroid of element i (nodes p[3i..3i+2], coordinates x, y in cm)
 * in drawing units gives x y r z theta R, and t[i] is the real part of the
 * last value `fctn` returns, in degrees (mag_dir when it returns nothing).
 * The chunk runs on a native restatement of the reference's Lua 4
 * interpreter (complex numbers; the base, string and math libraries; tables,
 * closures, LuaInstance's Complex and pi; xfk_lua.h lists what is refused),
 * one interpreter for all n_elems elements in order, globals persisting from
 * one to the next; errors carry the reference's messages ("Lua error occurred
 * when evaluating: ...", "... does not evaluate to a numerical value").
 * Host only: no device is needed. */
int xfk_magdir_eval(const char *fctn, int n_elems, const int *p, const double *x, const double *y,
                    int length_units, double mag_dir, double *t);

/* A whole problem's element loop (what xfk_problem_create runs): element i
 * runs its label lbl[i]'s function fctns[lbl[i]] (NULL or "": the label's
 * mag_dirs[lbl[i]], nothing run) on ONE interpreter, in element order, as the
 * reference's one Lua state per FSolver does; `axisymmetric` selects
 * staticaxi.cpp's chunk (r and z set first).  `repeats` != 0: the problem is
 * nonlinear, whose Newton loop re-runs the element loop every pass
 * (static2d.cpp:997-1008) -- refused (XFK_ERR_ARG, "not supported") when a
 * chunk changed state a later pass would see or left values on the stack. */
/* A whole Lua chunk on a fresh interpreter of the kind MagDirFctn runs on (a
 * femmcli-style script: the reference's LuaInstance, LuaInstance.cpp:185-208,
 * through lua_dostring): what print / write send to the standard output is
 * returned in out (NUL-terminated, at most cap - 1 bytes; *out_len the full
 * length).  0; -2 when the chunk raised a Lua error (syntax or run-time), -1
 * for a construct the interpreter refuses.  Host only. */
int xfk_lua_run(const char *chunk, char *out, long long cap, long long *out_len);

int xfk_magdir_eval_labels(int n_labels, const char *const *fctns, const double *mag_dirs, int n_elems,
                           const int *p, const int *lbl, const double *x, const double *y, int length_units,
                           int axisymmetric, int repeats, double *t);

#ifdef __cplusplus
}
#endif
#endif
