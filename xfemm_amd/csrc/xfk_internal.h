// Internal definitions of the MI355X (gfx950) fsolver hot path.
//
// Device-resident layout of one static-2D magnetostatic problem
// (FSolver::Static2D, reference cfemm/fsolver/static2d.cpp:53-1033):
//
//   nodes     x[N], y[N]            f64 SoA, cm (FSolver::LoadMesh converts to cm)
//   elements  erec[NE] int4         {p0, p1, p2, label} in COLOUR order
//             ebits[NE] int32       3 x 10-bit (boundary-prop index + 1) per edge
//             slot[NE][9] int32     CSR positions of the 3x3 element matrix
//             mu1[NE], mu2[NE] f64  element permeabilities (Newton state)
//   matrix    rowptr[N+1], col[nnz] int32, val[nnz] f64 -- full symmetric CSR
//             (the reference keeps the upper triangle in linked lists,
//             spars.h:38-83; full storage makes SpMV a pure gather)
//   vectors   b, V, R, P, U, dinv   f64[N]
//
// Everything here is plain C++/HIP for gfx950; no CUDA shims.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <map>
#include <string>
#include <unordered_map>
#include <thread>
#include <vector>

#include "../../include/xfemm_kernels.h"
#include "xfk_partition.h"

struct xfk_comm;

namespace xfk {

struct Amg;

constexpr int kBlock = 256;          // 4 waves of 64
constexpr int kRedGrid = 1024;       // fixed grid of the reduction kernels (4 WG/CU)
constexpr double kPI = 3.141592653589793238462643383;
constexpr double kDEG = 0.01745329251994329576923690768;
constexpr double kMUO = 1.2566370614359173e-6;
constexpr double kC = kPI * 4.e-05;  // static2d.cpp:66

#define XFK_CHECK(call)                                                          \
    do {                                                                         \
        hipError_t _e = (call);                                                  \
        if (_e != hipSuccess) {                                                  \
            ::xfk::set_error(std::string(#call) + ": " + hipGetErrorString(_e)); \
            return XFK_ERR_HIP;                                                  \
        }                                                                        \
    } while (0)

// hipEvents owned by one function: destroyed on every return path
template <int N>
struct ScopedEvents {
    hipEvent_t e[N] = {};
    hipError_t create()
    {
        for (auto &x : e)
            if (hipError_t r = hipEventCreate(&x); r != hipSuccess) return r;
        return hipSuccess;
    }
    hipEvent_t operator[](int i) const { return e[i]; }
    ~ScopedEvents()
    {
        for (auto &x : e)
            if (x) (void)hipEventDestroy(x);
    }
};

#define XFK_REQUIRE(cond, code, msg)  \
    do {                              \
        if (!(cond)) {                \
            ::xfk::set_error(msg);    \
            return code;              \
        }                             \
    } while (0)

void set_error(const std::string &msg);

// Per-block material parameters, as read by Static2D (CMSolverMaterialProp).
struct DevBlock {
    double mu_x, mu_y, H_c, J_re, Cduct, LamFill;
    int LamType, BHpoints, bh_off;
    int bh_sorted;   // B knots non-decreasing: the interval lookup may bisect
};

// Per-label parameters; the magnetisation direction is pre-evaluated on the
// host exactly as static2d.cpp:593-595 does (cos/sin of MagDir*PI/180).
struct DevLabel {
    double cos_m, sin_m;
    int blk, in_circuit, is_wound, external;
    double2 prox_mu;    // harmonic: ProximityMu of a LamType > 2 label
};

struct DevLine {
    double c0, c1;     // mixed BC coefficients (real parts)
    int format, pad;
};

struct DevCirc {
    double amps_re, dvolts_re;  // inputs
    double J, dV;               // outputs
    int type, ccase;
};

// Scalars of one PCG solve, device resident (written by the last-arriving
// block of each reduction kernel, read by the next launch).
struct PcgScalars {
    double res;       // z.r of the current iterate
    double res_o;     // (M^-1 b).b
    double del;       // res / pAp
    double rho;       // res_new / res
    double er;        // sqrt(res / res_o)
    double tol;
    int done;         // 1 once er <= tol (or res_o == 0)
    int singular;
    long long iters;
};

// State of the fused PCG (xfk_pcg.hip), device resident.  gam/alp are
// rings indexed by iteration parity: launch i writes slot i&1 and reads
// slot (i-1)&1, which the previous launch wrote.
struct CgState {
    double res_o;     // (M^-1 b).b
    double gam[2];    // gamma_i = r_i . M^-1 r_i
    double alp[2];    // alpha_i
    double er;        // sqrt(gamma_i / res_o)
    double tol;
    double tol_rel;   // inexact Newton passes: stop also at er <= tol_rel er0 (0: off)
    double er0;       // er of iteration 0
    int done;
    int singular;
    long long iters;
};

// Time-harmonic tables (xfk_harmonic.hip): complex values as double2 {re, im}.
struct DevBlockAC {
    double2 mu1, mu2;   // effective permeabilities Mu[k][0], Mu[k][1] (harmonic2d.cpp:190-235)
    double2 J;          // source current density
    double Cduct;
    int eddy;           // 0: laminated (Lam_d > 0) blocks carry no bulk eddy current (harmonic2d.cpp:392-394)
    int bh_n;           // nonlinear: knots of the complex B-H curve (0: linear)
    int bh_off;         // first knot in the problem's curve tables
    int prox;           // LamType > 2: wound region, the label's ProximityMu (harmonic2d.cpp:664-668)
};

struct DevLineAC {
    double2 c0, c1;     // mixed BC
    double2 zs;         // small-skin-depth BC: (1+I) / (-ds Mu 100) (harmonic2d.cpp:424-437), times l/6 per edge
    int format, pad;
};

struct DevCircAC {
    double2 J;          // Case 1: applied current density
    double2 dV;         // Case 0: voltage gradient
    int ccase, pad;
};

// State of the complex-symmetric Chronopoulos-Gear COCG (xfk_harmonic.hip)
struct CcgState {
    double bb;            // |b|^2
    double gam[2][2];     // gamma_i = r.u (unconjugated), parity rings, {re, im}
    double alp[2][2];
    double er, tol;
    int done, singular;
    long long iters;
};

struct NewtonScalars {
    double dx2;       // sum (V - Vold)^2
    double v2;        // sum V^2
};

// Small device buffer helper.
// device allocations of the library (counted for xfk_alloc_stats)
hipError_t dev_malloc(void **p, size_t bytes);
void dev_free(void *p);
// pinned host buffers through a process-wide cache: pinned_free returns the
// buffer to it inside a PoolRelease scope (a problem being destroyed, its
// device work synchronised), else hipHostFree
hipError_t pinned_malloc(void **p, size_t bytes);
void pinned_free(void *p);

// A problem's device arena: while an ArenaScope of the problem is active on
// the calling thread, dev_malloc carves buffers out of chunks (32 MiB, then
// doubling up to 256 MiB: a few hipMalloc per problem instead of one per
// buffer -- ~130 in a first solve, ~1 ms).  dev_free of a carved buffer (a
// function's scratch, the old block of a growing DBuf) keeps it `pending`:
// queued work may still read it.  At the end of every solve, with every
// stream of the problem idle, recycle() makes the pending blocks reusable,
// and later carvings take a reusable block of a fitting size before cutting
// new space, so a problem solved again and again (a rotor-angle loop) stays
// at the footprint of its largest solve.  The chunks go back to the process
// cache when the problem is destroyed.
struct DevArena {
    std::vector<std::pair<char *, size_t>> chunks;
    size_t off = 0;                                   // used bytes of the last chunk
    size_t next_chunk = 32ull << 20;                  // size of the next chunk (doubling to 256 MiB)
    std::unordered_map<void *, size_t> carved;        // live carved blocks -> block bytes
    std::multimap<size_t, char *> reuse;              // freed blocks no device work can read any more
    std::vector<std::pair<char *, size_t>> pending;   // freed during the current solve
    size_t chunk_bytes() const;
    // room for `bytes` more in the last chunk (a new chunk of that size
    // otherwise): a problem's creation reserves its first solve's footprint,
    // so the solve carves without a hipMalloc
    hipError_t reserve(size_t bytes);
    void release();   // (the problem's device work finished)
    void recycle();   // (every stream of the problem idle) pending -> reuse
    bool retire(void *p);   // p carved here: pending until the next recycle()
};
// p carved from the arena active on this thread: retire it there (true)
bool arena_retire(void *p);
struct ArenaScope {
    DevArena *prev;
    explicit ArenaScope(DevArena *a);
    ~ArenaScope();
};

template <class T>
struct DBuf {
    T *p = nullptr;
    size_t n = 0;
    DBuf() = default;
    DBuf(const DBuf &) = delete;
    DBuf &operator=(const DBuf &) = delete;
    ~DBuf() { free(); }
    // growing keeps the old block until the buffer itself is freed (or, for a
    // block carved from the problem's arena, until the solve's end): work
    // still queued may read it, and a hipFree here would wait for the device
    // in the middle of a solve (the grows of a problem's first setup)
    hipError_t alloc(size_t count) {
        if (count <= n && p) return hipSuccess;
        if (p && !arena_retire(p)) retired.push_back(p);
        p = nullptr;
        n = 0;
        if (count == 0) return hipSuccess;
        hipError_t e = dev_malloc(reinterpret_cast<void **>(&p), count * sizeof(T));
        if (e == hipSuccess) n = count;
        return e;
    }
    void free() {
        if (p) dev_free(p);
        for (T *q : retired) dev_free(q);
        retired.clear();
        p = nullptr;
        n = 0;
    }
    std::vector<T *> retired;
};

// Halo exchange overlapped with computation on a sharded operator.  Tiles of
// B rows (the tile kernels' workgroups) are split once per operator into the
// interior tiles -- every column owned (< n) -- and the boundary tiles that
// read a halo column.  The exchange runs on a side stream while the interior
// tiles run on the main stream; the boundary tiles follow the exchange.
// Every tile computes exactly what the unsplit launch computes (same tile
// ids, same partial-sum slots), so the split changes no bit of the result.
struct TileSplit {
    DBuf<int> tiles;                  // interior tile ids, then boundary tile ids (ascending)
    int B = 0, n_in = 0, n_bd = 0;
    bool ready() const { return B > 0; }
};
// host-synchronising (once per operator)
int build_tile_split(hipStream_t s, int n, int B, const int *rowptr, const int *col, TileSplit &ts);
// f(begin, end) over [0, n) in contiguous chunks on up to 16 host threads
// (one chunk below 2 min_per_thread items); the problem-creation loops over
// the mesh (validation, boundary preparation) are independent per item
template <class F>
void host_par_for(long long n, long long min_per_thread, F f)
{
    const long long hw = std::max(1u, std::thread::hardware_concurrency());
    const int T = (int)std::max(1LL, std::min({std::min(hw, 16LL), n / std::max(1LL, min_per_thread)}));
    if (T <= 1) {
        f(0LL, n);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back([&, t] { f(n * t / T, n * (t + 1) / T); });
    f(0LL, n / T);
    for (auto &x : th) x.join();
}
// Process-wide pool of non-blocking streams on the current device: creating a
// HIP stream costs ~4 ms on MI355X (a hardware queue), so a problem returns its
// streams here when it is destroyed and the next problem takes them back.
hipError_t stream_acquire(hipStream_t *s);
// one kernel of each translation unit queried, so its code object is loaded
// (xfk_device_init)
hipError_t warm_module_amg();
hipError_t warm_module_comm();
hipError_t warm_module_device();
hipError_t warm_module_harmonic();
hipError_t warm_module_pcg();
hipError_t warm_module_sort();
void stream_release(hipStream_t s);   // idle streams only (the caller synchronised it)
void stream_pool_drain();
// xfk_sort.hip: the reference's comb sort of the element scores on the device
// (perm_dev may alias score_dev: the scores are read first)
int sort_elements_device(hipStream_t s, int n, const unsigned *score_dev, int *perm_dev, unsigned long long *key,
                         unsigned long long *tmp, unsigned long long *red, unsigned long long *cin, int *flag,
                         int *passes);             // destroy the idle pooled streams (xfk_release_cache)
long long stream_pool_idle();
struct SideStream {
    hipStream_t cs = nullptr;
    hipEvent_t a = nullptr, b = nullptr, c = nullptr;
    int init();
    ~SideStream();
};
// off unless XFK_OVERLAP=1 (otherwise: exchange, then one launch over every tile)
bool overlap_enabled();
// exch(side stream) once the main stream's work so far is done; interior()
// meanwhile on s; boundary() on s after the exchange
template <class Ex, class In, class Bd>
int exchange_overlapped(hipStream_t s, SideStream &ss, Ex &&exch, In &&interior, Bd &&boundary)
{
    XFK_CHECK(hipEventRecord(ss.a, s));
    XFK_CHECK(hipStreamWaitEvent(ss.cs, ss.a, 0));
    const int rc = exch(ss.cs);
    if (rc != XFK_OK) return rc;
    XFK_CHECK(hipEventRecord(ss.b, ss.cs));
    interior();
    XFK_CHECK(hipStreamWaitEvent(s, ss.b, 0));
    boundary();
    return XFK_OK;
}

}  // namespace xfk

// The opaque problem handle of the C-ABI.
struct xfk_problem {
    xfk::DevArena arena;             // (declared first: destroyed after every buffer carved from it)
    int device = 0;
    hipStream_t stream = nullptr;

    // sizes: N owned rows (= all nodes unless sharded), NL local nodes
    // (owned rows first, then the halo), NE local elements
    int N = 0, NL = 0, NE = 0;
    // rows assembled: the owned rows, then (sharded periodic / air-gap
    // problems) the extra rows of coupled nodes owned elsewhere (xfk_partition.h)
    int NR = 0;
    long long nnz = 0;       // entries of the assembled rows (NR)
    long long nnz_own = 0;   // entries of the owned rows (N): the solved matrix
    int row_max = 0;         // longest assembled row (0: not measured; read with the lengths)
    int ncolors = 0;
    std::vector<int> color_off;      // ncolors + 1 (host)

    // sharded solve (xfk_problem_create_dist); comm == nullptr otherwise
    xfk_comm *comm = nullptr;
    int rank = 0, nranks = 1;
    int N_global = 0, row0 = 0;
    std::vector<int> l2g;            // local node -> global node
    xfk::HaloPlan halo;              // slices of the node vectors exchanged with peers
    xfk::HaloPlan halo2;             // the same for interleaved complex (double2) node vectors
    int Gpart = 0;                   // length of each per-block partial array (agreed by all ranks)
    xfk::TileSplit ts;               // sharded PCG SpMV: interior / boundary tiles (exchange overlap)
    int *hpin = nullptr;             // pinned scratch for small device -> host reads
    hipEvent_t nnz_ev = nullptr;     // the pattern's lengths landed in hpin[0..1] (deferred read)
    bool nnz_pending = false;        // nnz / nnz_own not read back yet (xfk_resolve_nnz)
    int pcg_hint0 = 0;               // PCG iterations of the last solve's first pass (first batch)
    double pcg_rate = 0;             // log(er) per iteration in the last converged solve (< 0; 0: none yet)
    std::vector<hipEvent_t> setup_ev;   // AMG setup event pairs, read after the solve
    int setup_used = 0;
    double setup_ms_pending = 0;        // pairs read out early when the pool filled
    xfk::SideStream side;

    // host copies kept for host-side setup (periodic maps)
    std::vector<int> hp, hpbc;
    int length_units = 0, coords = 0;
    bool axi = false;                // StaticAxisymmetric (x is r)
    std::vector<double> axi_x;       // global node radii (cm): the answer is 2 pi r A
    double ext_ro = 0, ext_ri = 0, ext_zo = 0;   // exterior region, cm
    double precision = 1e-8, relax = 1.0;
    bool any_nonlinear = false;

    // raw mesh (original element order)
    xfk::DBuf<double> x, y;
    xfk::DBuf<int> p_raw;            // 3*NE
    xfk::DBuf<int> lbl_raw;          // NE
    xfk::DBuf<int> ebits_raw;        // NE

    // tables
    xfk::DBuf<xfk::DevBlock> blocks;
    xfk::DBuf<xfk::DevLabel> labels;
    xfk::DBuf<xfk::DevLine> lines;
    xfk::DBuf<xfk::DevCirc> circs;
    xfk::DBuf<double> bhB, bhH, bhS;
    int nblocks = 0, nlabels = 0, nlines = 0, ncircs = 0;

    // symbolic
    bool symbolic_ready = false;
    xfk::DBuf<int> n2e_ptr, n2e;     // node -> incident elements (sorted)
    xfk::DBuf<int> rowptr, col, diag;
    xfk::DBuf<int> color;            // per raw element
    int color_rounds = 0;            // Jones-Plassmann rounds of the last symbolic build
    xfk::DBuf<char> cub_tmp;         // hipcub temporary storage
    xfk::DBuf<char> sym_tmp;         // symbolic-phase temporaries (SymTmp in xfk_api.hip)
    xfk::DBuf<int> fill_ptr, fill_col;   // periodic fill-in entries by row
    xfk::DBuf<int> perm;             // colour order -> raw element
    xfk::DBuf<int4> erec;            // colour order
    xfk::DBuf<int> ebits;            // colour order
    xfk::DBuf<int> slot;             // colour order, 9 per element
    xfk::DBuf<double> mu1, mu2;      // element permeability state (colour order: harmonic; raw order: static)
    xfk::DBuf<double> mu1b, mu2b;    // static row-gather assembly: the state written by the current assembly
    xfk::DBuf<double> dv_el;         // planar Newton passes: the element's dv (k_planar_state)
    xfk::DBuf<unsigned char> on_el;  // ... and whether its Newton terms apply
    xfk::DBuf<int> asm_miss;         // static assembly: 1 when an element entry found no slot in its row
    bool miss_checked = false;       // asm_miss read since the last symbolic build

    // boundary conditions
    xfk::DBuf<int> pt_nodes;         // nodes with a point current / fixed point value
    xfk::DBuf<double> pt_J;          // 0.01*J_re per pt node
    int npt = 0;
    xfk::DBuf<unsigned char> fixed;  // N
    xfk::DBuf<double> fix_first, fix_last;
    xfk::DBuf<int> fix_rows;         // fixed nodes
    int nfix_rows = 0;
    xfk::DBuf<int> fix_cols;         // slots (k, c) with c fixed, k not fixed
    xfk::DBuf<int> fix_cols_node;    // the fixed column c of each such slot
    xfk::DBuf<int> fix_cols_row;     // row k of each such slot
    int nfix_cols = 0;                // -1: the count is on the device (nfix_dev)
    xfk::DBuf<int> nfix_dev;
    // periodic map: dst <- sum_s w_s * src_s (values), and the same for b
    xfk::DBuf<int> pm_dst, pm_ptr, pm_src;
    xfk::DBuf<double> pm_w, pm_tmp;
    int pm_n = 0;
    xfk::DBuf<int> pb_dst, pb_ptr, pb_src;
    xfk::DBuf<double> pb_w, pb_tmp;
    int pb_n = 0;
    // fill-in entries requested by the periodic map (row, col) -> pattern
    std::vector<long long> pbc_fill;   // packed (row<<32)|col: periodic fill-in and air-gap couplings
    std::vector<long long> age_key;    // air-gap element entries (r <= c), xfk_age.h
    std::vector<double> age_val;
    xfk::DBuf<int> age_slot;           // CSR slot of every full-storage air-gap entry
    xfk::DBuf<double> age_v;
    int age_n = 0;
    // host form, entry m's terms at [pbc_entry_ptr[m], pbc_entry_ptr[m + 1]) of pbc_entry_terms
    std::vector<std::pair<long long, double>> pbc_entry_terms;
    std::vector<int> pbc_entry_ptr;
    std::vector<long long> pbc_entry_key;
    std::vector<std::pair<int, double>> pbc_b_terms;   // (the same layout, pbc_b_ptr)
    std::vector<int> pbc_b_ptr;
    std::vector<int> pbc_b_key;
    // the same composition for the Newton AC solver's auxiliary matrices
    // (cspars.cpp:648-670, 732-754): ordered (row, col) entries -- they are
    // Hermitian / anti-Hermitian, not symmetric -- whose (i, j) block of each
    // pair is the mean of its four entries; the entries (i, j) it creates
    std::vector<std::pair<long long, double>> pbca_entry_terms;   // (pbca_entry_ptr)
    std::vector<int> pbca_entry_ptr;
    std::vector<long long> pbca_entry_key;
    std::vector<long long> pbca_fill;
    xfk::DBuf<int> pa_dst, pa_ptr, pa_src;
    xfk::DBuf<double> pa_w, pa_tmp;
    int pa_n = 0;

    // numeric: V (the PCG iterate x) and U (= M^-1 r) span the NL local
    // nodes, their halo slices filled by exchanges; the rest span N rows
    xfk::DBuf<double> val, b, V, Vold, P, dinv;
    xfk::DBuf<double> R2, W2, Z2;     // r; w = A u; z (N) followed by u (NL)
    // per-block partials of the PCG inner products, 4 arrays of Gpart:
    // gamma (2 parities), delta, (M^-1 b).b.  part_loc is written by the
    // kernels; part_glob is what they read: the sum over ranks when sharded
    // (all-reduce), the same memory as part_loc otherwise
    xfk::DBuf<double> part_loc, part_glob_buf;
    double *part_glob = nullptr;
    xfk::DBuf<double> nws_glob;       // all-reduced Newton sums (sharded)
    xfk::DBuf<double> gather_buf;     // solution all-gather (sharded)
    xfk::DBuf<double> partials;       // kRedGrid * 2 (Newton residual)
    xfk::DBuf<unsigned> counters;     // ticket counters
    xfk::DBuf<xfk::CgState> pcg;
    xfk::DBuf<xfk::NewtonScalars> nws;
    xfk::CgState *pcg_host = nullptr;  // pinned mirror
    xfk::NewtonScalars *nws_host = nullptr;
    // single device, nonlinear static pass: the Newton residual is enqueued
    // at every PCG poll and read with it; nws_ready once the final (done)
    // poll's copy holds this pass's |dV|^2, |V|^2 -- the Newton loop then
    // needs no host round trip of its own
    bool nws_at_poll = false;
    bool nws_ready = false;

    // preconditioner (xfk_set_option): XFK_PRECOND_AMG (default) or XFK_PRECOND_JACOBI
    int precond = XFK_PRECOND_AMG;
    int amg_sweeps = 1;
    double amg_theta = 0.08;
    double amg_omega = 1.75;
    int amg_replicate = 250000;
    int amg_dense = 2048;
    int amg_fold = -1;                // XFK_OPT_AMG_FOLD (-1: the XFK_AMG_FOLD environment default)
    int amg_col16 = -1;               // XFK_OPT_AMG_COL16 (-1: on unless XFK_NO_COL16)
    int amg_wlevel = -2;              // XFK_OPT_AMG_WLEVEL (-2: the default level)
    int amg_f32 = -1;                 // XFK_OPT_AMG_F32 (-1: on unless XFK_AMG_F32=0)
    int newton_inexact = -1;          // XFK_OPT_NEWTON_INEXACT (-1: on unless XFK_NEWTON_INEXACT=0)
    double pcg_tol = 0;               // PCG stopping tolerance of the running pass (0: precision)
    double pcg_tol_rel = 0;           // ... and its relative stop (er <= tol_rel er0; 0: none)
    bool f64_fallback = false;        // a stagnating PCG switched the f32 parts of the AMG to f64 (sticky)
    long long pcg_discarded = 0;     // PCG iterations of this solve spent before a restart (stale hierarchy / f64)
    int amg_reuse = 1;
    bool amg_reusable = false;        // the hierarchy belongs to this solve's matrix pattern
    bool amg_fresh = false;           // built from scratch for the running PCG solve
    long long amg_fresh_iters = 0, amg_last_iters = 0;
    xfk::Amg *amg = nullptr;         // hierarchy of the current matrix (xfk_amg.hip)
    int pc_used = XFK_PRECOND_JACOBI;  // preconditioner of the running solve

    // time-harmonic problem (xfk_problem_create_harmonic, xfk_harmonic.hip)
    bool harmonic = false;
    double omega = 0;                  // 2 pi f
    xfk::DBuf<xfk::DevBlockAC> blocks_ac;
    xfk::DBuf<xfk::DevLineAC> lines_ac;
    xfk::DBuf<xfk::DevCircAC> circs_ac;
    std::vector<xfk::DevCircAC> hcircs;          // host copy (circuit results)
    xfk::DBuf<double> val_im, b_im;              // imaginary parts of val, b
    xfk::DBuf<double> hfix_first, hfix_last;     // 2 per node {re, im}
    xfk::DBuf<int> hpt_nodes;
    xfk::DBuf<double> hpt_J;                     // 2 per point node: -0.01 J
    int nhpt = 0;
    xfk::DBuf<double2> hc_vec;                   // COCG vectors: x, r, u, w, z, p, dinv (N each)
    xfk::DBuf<double> hc_split;                  // AMG: r and u split into real / imaginary parts
    xfk::DBuf<double> hc_bval;                   // AMG: values of the real surrogate Re A +- Im A
    // nonlinear harmonic (successive approximation, harmonic2d.cpp:616-660, 826-873)
    xfk::DBuf<double> hbh_B;                     // complex B-H curves of all nonlinear blocks
    xfk::DBuf<double2> hbh_H, hbh_S;
    xfk::DBuf<double2> hV_old;                   // the iterate before the solve
    xfk::DBuf<double> hres_part;                 // residual partial sums
    // Case-2 circuits: bordered unknowns solved through their Schur complement
    std::vector<int> hc2_circ;                   // circuit of each bordered unknown
    std::vector<double2> hc2_D, hc2_f, hc2_u;    // diagonal, right-hand side, solution (u: V[N + k])
    std::vector<double2> hc2_u_old;
    xfk::DBuf<double> hc2_C;                     // border columns, per unknown N re then N im
    xfk::DBuf<double2> hc2_Y, hc2_y0;            // A^-1 C_k and A^-1 b
    // Newton AC solver (ac_solver == 1): Mh, Ms, Ma over the CSR pattern as
    // six arrays of nnz (re, im of each), the KludgeSolve vectors
    int ac_solver = 0;
    xfk::DBuf<double> haux;
    xfk::DBuf<double2> hk_vec;                   // borig, v, r, P(dir), U (N each)
    xfk::DBuf<double> hk_b;                      // b' split: re, im (N each)
    xfk::DBuf<double> hc_part;                   // per-block partials, 9 arrays
    xfk::DBuf<xfk::CcgState> hc_state;
    xfk::CcgState *hc_host = nullptr;            // pinned mirror

    // live SpMV launch timing (XFK_TIME_SPMV)
    bool time_spmv = false;
    std::vector<hipEvent_t> spmv_ev;   // pairs
    std::vector<hipEvent_t> pass_ev;   // static Newton loop: (start, assembled, solved) per pass, read at the end
    int spmv_used = 0;

    // last-solve statistics
    xfk_result last{};
};

// Host-side helpers shared by the static (xfk_api.hip) and harmonic
// (xfk_harmonic.hip) drivers.
namespace xfk {

// Per-phase timing for xfk_phase_profile: while g_prof is set, the PCG and
// V-cycle launch sites bracket each launch with a pair of HIP events on the
// launch stream, tagged with the phase name and its algorithmic bytes.
struct PhaseProf {
    hipStream_t s = nullptr;
    struct Rec {
        std::string name;
        double bytes;
        int ev0, ev1;   // begin / end events (ev1 < 0: never closed, ignored)
    };
    std::vector<hipEvent_t> ev;
    int used = 0;
    std::vector<Rec> recs;
    hipError_t record()
    {
        if (used == (int)ev.size()) {
            hipEvent_t e;
            hipError_t r = hipEventCreate(&e);
            if (r != hipSuccess) return r;
            ev.push_back(e);
        }
        return hipEventRecord(ev[used++], s);
    }
    void begin(const std::string &name, double bytes)
    {
        if (!recs.empty() && recs.back().ev1 < 0) recs.back().ev0 = -1;   // an unclosed phase: dropped
        recs.push_back({name, bytes, used, -1});
        (void)record();
    }
    void end()
    {
        if (recs.empty() || recs.back().ev1 >= 0 || recs.back().ev0 < 0) return;
        recs.back().ev1 = used;
        (void)record();
    }
    ~PhaseProf()
    {
        for (auto &e : ev) (void)hipEventDestroy(e);
    }
};
extern thread_local PhaseProf *g_prof;
#define XFK_PHASE(name, bytes, ...)                       \
    do {                                                  \
        if (::xfk::g_prof) ::xfk::g_prof->begin(name, bytes); \
        __VA_ARGS__;                                      \
        if (::xfk::g_prof) ::xfk::g_prof->end();          \
    } while (0)

// Everything Static2D derives from the GLOBAL problem before the mesh is split
// (so a sharded solve sees the same boundary values, point currents and
// circuit currents as the single-device one).
struct GlobalPrep {
    std::vector<DevBlock> blk;
    std::vector<double> hB, hH, hS;
    std::vector<DevLabel> lab;           // labels, then one per element of a MagDirFctn label
    std::vector<int> elab;               // per element: index into lab (empty: the mesh's lbl)
    std::vector<DevLine> lin;            // boundary properties used on edges, compacted
    std::vector<int> lmap, lin_used;     // property -> compact index (-1: unused); compact -> property
    std::vector<DevCirc> circ;
    std::vector<int> ebits;              // per element: 3 x 10-bit boundary-prop index + 1
    std::vector<int> pt_nodes;           // nodes with a point current, ascending
    std::vector<double> pt_J;            // 0.01 * J of each
    std::vector<unsigned char> fixed;    // per node: Dirichlet value set
    std::vector<double> first, last;     // first / last value set (CBigLinProb::SetValue order)
    bool any_nonlinear = false;
    bool axi = false;                    // FSolver::StaticAxisymmetric
    double ext_ro = 0, ext_ri = 0, ext_zo = 0;   // exterior region, cm
    std::vector<long long> age_key;      // air-gap element entries, (r << 32) | c with r <= c
    std::vector<double> age_val;
    bool pbc_aux = false;                // compose the periodic map of the Newton AC auxiliary matrices too
};

int validate_desc(const xfk_problem_desc *d);
int check_device(int device);
void prepare_global(const xfk_problem_desc *d, GlobalPrep &G);
// static problems: per-element magnetisation directions of MagDirFctn labels
int prepare_magdir(const xfk_problem_desc *d, GlobalPrep &G);
// the device problem of one rank (plan == nullptr: the whole mesh)
int build_local(const xfk_problem_desc *d, const GlobalPrep &G, const PartPlan *plan, int device, xfk_comm *comm,
                xfk_problem **out);
int build_symbolic(xfk_problem *P);
// sum of a host scalar over the ranks of P's communicator (no-op on one device)
int allreduce_host(xfk_problem *P, double &v);
int allreduce_host_n(xfk_problem *P, double *v, int n);   // n doubles summed over the ranks (host in, host out)
// the row-block plan of comm's rank (coupled nodes assembled on every rank)
int plan_rank(const xfk_problem_desc *d, const GlobalPrep &G, xfk_comm *comm, PartPlan &plan);
hipError_t d2h(void *dst, const void *src, size_t bytes, hipStream_t s);
// host -> device copy into a (re)allocated buffer, ordered on `s`
template <class T>
inline hipError_t upload(DBuf<T> &d, const T *h, size_t n, hipStream_t s)
{
    hipError_t e = d.alloc(n ? n : 1);
    if (e != hipSuccess || n == 0) return e;
    return hipMemcpyAsync(d.p, h, n * sizeof(T), hipMemcpyHostToDevice, s);
}

}  // namespace xfk
