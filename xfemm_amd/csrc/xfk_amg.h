// Smoothed-aggregation algebraic multigrid preconditioner of the PCG
// (xfk_amg.hip), device resident on one GPU.
//
// The reference preconditions CBigLinProb::PCGSolve with a sequential SSOR
// sweep (cfemm/libfemm/spars.cpp:186-236, MultPC); a triangular sweep has no
// parallelism to offer a GPU, and Jacobi -- the first device preconditioner --
// needs O(sqrt(DoF)) iterations (3537 at 1M DoF).  This is the replacement:
// a symmetric V-cycle whose iteration count is nearly mesh independent.
//
// Setup, per level l (all on the device, deterministic):
//   strength    |a_ij| > theta sqrt(|a_ii a_jj|)             (1 flag byte per nonzero)
//   MIS-2       parallel maximal distance-2 independent set of the strength
//               graph, keys (state, hash(i), i), two max-propagation sweeps per round
//   aggregates  roots, then distance-1 and distance-2 joins (max-key neighbour)
//   P           (I - W D_F^-1 A_F) P_tent, A_F = strong part + weak entries lumped
//               onto the diagonal, W_ii = 4 / (3 max(rho_i, 2)), rho_i the row's
//               Gershgorin bound of D_F^-1 A_F
//   R = P^T     counting transpose, rows sorted, values looked up in P
//   A_{l+1}     R (A P), two wave-per-row SpGEMMs with LDS hash tables and an
//               ordered per-product accumulation (bit-reproducible)
// until the level has <= kAmgDenseMax rows, whose dense inverse is formed by
// blocked Gauss-Jordan (64-wide block columns, tile GEMM updates).
//
// V-cycle: nu damped-Jacobi sweeps (weight omega / rho_A, rho_A the Gershgorin
// bound of D^-1 A, default nu = 1, omega = 1.75) before and after the coarse
// correction; the first sweep starts from x = 0 implicitly.
// With equal pre/post sweeps and R = P^T the cycle is a symmetric positive
// definite operator, as CG requires.
#pragma once

#include <hip/hip_runtime.h>

#include <map>
#include <memory>
#include <vector>

#include "xfk_internal.h"
#include "xfk_partition.h"

struct xfk_comm;

namespace xfk {

constexpr int kAmgDenseMax = 2048;    // coarsest level solved by its dense inverse (blocked Gauss-Jordan)
constexpr int kAmgMaxLevels = 16;
constexpr int kAmgDeferSlots = 64;    // deferred SpGEMM (overflow flag, length) pairs per setup
constexpr int kAmgDeferTotal = kAmgDeferSlots + kAmgDeferSlots / 2;   // + a class-check flag per pair

struct AmgLevel {
    int n = 0;                        // rows
    long long nnz = 0;
    int ncol_lim = 0;                 // columns >= ncol_lim are ignored by the coarsening (sharded level 0: halo)
    int ncol_smooth = 0;              // columns the smoother and residual read (sharded level 0: owned + halo)
    const int *rowptr = nullptr, *col = nullptr;
    const double *val = nullptr;
    DBuf<int> rowptr_o, col_o;        // storage of levels >= 1
    DBuf<double> val_o;
    DBuf<double> dinv;
    // transfer to the next level (absent on the coarsest)
    int nc = 0;
    long long pnnz = 0;
    DBuf<int> prow, pcol, rrow, rcol;
    DBuf<double> pval, rval;
    // folded level (xfk_amg.hip: k_fold_pre): P~ = (I - w D^-1 A) P and R~ = P~^T
    bool fold = false;
    bool fold_formed = false;         // the setup formed P~ (a refresh may fold or not)
    long long fnnz = 0;
    DBuf<int> ftrow, ftcol, frrow, frcol;
    DBuf<double> ftval, frval;
    // V-cycle vectors: b (right-hand side, levels >= 1), two iterate buffers, residual
    DBuf<double> b, xa, xb, r;
    // sharded level: rows owned by this rank, halo columns n .. ncol_smooth-1
    // filled by exchanges over `plan` (level 0: the problem's node plan;
    // coarser: spans of the peers' aggregate ids)
    bool dist = false;
    HaloPlan plan;
    TileSplit ts;                     // sharded level run by the tile kernels: exchange overlap
    // 16-bit column offsets per tile (single-device level 0, xfk_spmv.h
    // k_tile_col16): A and P~ in the 512-row tiles of the SpMV / sweeps /
    // folded post-step, R in the restriction's 256-row tiles
    bool has16 = false;
    DBuf<unsigned short> a16, f16, r16, p16;
    DBuf<int> a16b, f16b, r16b, p16b;
    // level 0 (with has16): the V-cycle's transfers R and P~ with f32 values
    // (products and sums in f64; A keeps f64 -- a32 only with XFK_AMG_F32_SWEEP=1);
    // a sharded level 0 (unfolded) keeps R and P in f32, P with 16-bit
    // columns in 256-row tiles (p16)
    bool has32 = false;
    DBuf<float> a32, r32, f32v, p32;
    // stored bytes per nonzero of the level's V-cycle transfers (column + value)
    double nz_bytes() const { return (has16 ? 2.0 : 4.0) + (has32 ? 4.0 : 8.0); }
};

struct AmgStats {
    int levels = 0;
    int n[kAmgMaxLevels] = {};
    long long nnz[kAmgMaxLevels] = {};
    int mis_rounds[kAmgMaxLevels] = {};
    double op_complexity = 0;         // sum nnz / nnz(level 0)
};

struct Amg {
    // parameters
    double theta = 0.08;              // strength threshold
    double theta_coarse = -1.0;       // levels >= 1 (< 0: theta; XFK_AMG_THETA_COARSE overrides)
    double theta_at(int l) const;
    int sweeps = 1;                   // Jacobi sweeps before and after the coarse correction
    int wlevel = -2;                  // W-cycle (two coarse corrections) at this folded level (-1: none; -2: XFK_AMG_W)
    int wcycle_level() const;
    bool w_at(int l) const;
    double omega = 1.75;              // Jacobi weight = omega / rho_A (rho_A: Gershgorin bound of D^-1 A);
                                      // omega < 2 keeps the cycle SPD since rho_A >= rho(D^-1 A)

    std::vector<std::unique_ptr<AmgLevel>> L;
    int nlev = 0;
    bool dense_coarse = false;
    DBuf<double> cinv;                // dense inverse of the coarsest level (row major, padded)
    int cinv_ld = 0;
    DBuf<float> cinv_o;               // the inverse the V-cycle applies: unpermuted, symmetrised, scaled M (f32)
    DBuf<double> cinv_o64;            // the same in f64 (prec32 == 0)
    DBuf<double> cinv_sc;             // the scale S (original order): A_c^-1 = S M S
    bool cinv_f64 = false;
    // the hierarchy applies f32 values somewhere (level-0 transfers or the coarsest inverse)
    bool f32_active() const { return (dense_coarse && !cinv_f64) || (!L.empty() && L[0]->has32); }
    const float *cinv_apply = nullptr;
    DBuf<int> cinv_perm, cinv_iperm, nd_tiles;
    DBuf<unsigned char> nd_mask;
    struct NdPhase {                  // one tree level of the nested-dissection order
        int nch = 0, steps = 0;       // pivot chains (<= 8) and their block steps
        int base[8] = {}, next_slot[8] = {};
        int tiles_off = 0, ntiles = 0;
    };
    std::vector<NdPhase> nd_phases;
    std::vector<int> nd_key;          // coarsest pattern (rowptr, col) the cached plan was made for
    DBuf<int> nd_key_dev;             // its device copy (compared on the device by the next setup)
    int nd_key_n = -1;
    long long nd_key_nnz = 0;
    std::vector<NdPhase> nd_phases_key;
    int nd_ld = 0;
    char *nd_stage = nullptr;         // pinned upload staging of the plan
    size_t nd_stage_n = 0;
    DBuf<double> bgj_tmp;             // blocked Gauss-Jordan panels
    DBuf<unsigned long long> rho;     // per level {rho_A, rho_F} as ordered bit patterns
    AmgStats stats;

    // setup scratch (reused across setups)
    DBuf<double> absd, dfinv, wF, rho_part;
    DBuf<unsigned char> sflag;
    DBuf<unsigned> key, t1;           // MIS-2 keys (state:2 | priority:30)
    DBuf<unsigned char> act;          // MIS-2: the row's strong neighbourhood still holds an undecided row
    DBuf<int> cnt, agg1, agg, flag, cursor;
    DBuf<int> ap_row, ap_col;
    DBuf<int> pad_col;                // single-pass SpGEMM: padded rows
    DBuf<double> pad_val;
    DBuf<double> ap_val;
    DBuf<int> dev_int;                // small device scalars (undecided flag, overflow flags)
    std::map<int, int> cap_hint;      // SpGEMM slot capacity of each call site in the last setup
    std::map<int, int> mis_hint;      // MIS-2 rounds each level needed in the last setup
    int row_max0 = 0;                 // longest row of the fine matrix (the caller's symbolic phase; 0: unknown)
    // a fresh hierarchy (no setup yet): capacities and MIS rounds from the
    // longest fine row instead of host-checked measurements
    void seed_hints();
    DBuf<int> def_dev;                // deferred SpGEMM results: (overflow flag, length) pairs
    int *def_host = nullptr;          // pinned mirror
    int def_n = 0;
    long long *def_target[kAmgDeferSlots / 2] = {};
    int def_verify[kAmgDeferSlots / 2] = {};   // capacity whose class the device checks (0: none)
    bool foreign = false;
    std::vector<char> nd_plan;        // host copy of the plan's device arrays (for the hint store)
    size_t nd_tl_n = 0, nd_mask_n = 0;             // the capacity hints came from another problem (load_hints)
    int load_hints(hipStream_t s, int n0, long long nnz0);
    void save_hints(int n0, long long nnz0);
    int *host_int = nullptr;          // pinned mirror (16 ints; 8..10: the aggregation's packed check)
    hipEvent_t ev_host = nullptr;     // host waits for a check while later setup work runs
    DBuf<int> mis_out;                // packed aggregation check
    DBuf<char> cub_tmp;

    // sharded hierarchy (setup_dist): levels 0 .. lrep-1 are sharded (each rank
    // aggregates its own rows; the Galerkin product uses the peers' P rows),
    // levels lrep.. are global and replicated on every rank once the global
    // level has <= rep_rows rows
    bool dist = false;
    int rep_rows = 250000;
    int dense_max = kAmgDenseMax;     // coarsest level: dense inverse at <= dense_max rows
    int fold_on = -1;                 // folded V(1,1) levels: 1 / 0, -1 = the XFK_AMG_FOLD default
    int col16 = -1;                   // 16-bit tile columns on level 0: 1 / 0, -1 = on unless XFK_NO_COL16
    int prec32 = -1;                  // f32 values of level 0's V-cycle operators: 1 / 0, -1 = on unless XFK_AMG_F32=0
    int lrep = 0;
    xfk_comm *comm = nullptr;
    int nranks = 1, rank = 0;
    std::vector<int> c0;              // first row of each rank's aggregates on level lrep (nranks + 1)
    int ncmax = 0;                    // largest per-rank aggregate count there (all-gather stride)
    DBuf<int> c0_dev;
    DBuf<int> span_dev, map_dev;      // peer spans of a sharded coarse level (setup scratch)
    DBuf<double> cb_loc, cb_all;      // restricted residual: own aggregates, all-gathered (padded)
    DBuf<int> pe_row, pe_col;         // P extended by the halo nodes' rows (global coarse columns)
    DBuf<double> pe_val, ebuf;
    DBuf<int> l_row, l_col, s_col;    // this rank's coarse rows (s_: padded send copy)
    DBuf<double> l_val, s_val;
    DBuf<int> g_row, g_col;           // all-gathered coarse rows (padded per rank)
    DBuf<double> g_val;
    DBuf<int> e0_dev;
    int *host_big = nullptr;          // pinned scratch for small device -> host reads
    int host_big_n = 0;
    double *part_gam_ = nullptr;      // vcycle's gamma partials, for vc_dist
    SideStream side;                  // sharded: halo exchanges overlapped with interior tiles
    // sharded, XFK_TIME_TAIL: event pairs around the replicated tail -- per
    // V-cycle the all-gather of the coarse right-hand side and the replicated
    // cycle (kind 0), in the setup the build of the replicated levels (kind 1)
    bool time_tail = false;
    std::vector<hipEvent_t> tail_ev;
    std::vector<char> tail_kind;      // per pair
    int tail_used = 0;                // events recorded (pairs * 2)
    int tail_begin(hipStream_t s, int kind);
    void tail_end(hipStream_t s, int at);
    // sum the recorded pairs per kind (after the stream is synchronised); resets
    int tail_read(double &ms_cycle, int &cycles, double &ms_setup);
    // single-device setup steps off the critical path -- R = P^T beside A P,
    // the folded transfers P~ / R~ beside the next level -- on a second
    // stream with scratch of its own (a: fork, b: R done / join, c: P~ done)
    SideStream sw;
    bool sw_used = false, rt_pending = false, fold_pending = false;
    DBuf<int> cnt2;
    DBuf<char> cub_tmp2;

    ~Amg();
    // wait for the hierarchy's own streams (overlap, setup side stream)
    void sync_streams()
    {
        if (side.cs) (void)hipStreamSynchronize(side.cs);
        if (sw.cs) (void)hipStreamSynchronize(sw.cs);
    }
    // Build the hierarchy for the n x n CSR on `s` (host-synchronising).
    // Columns >= ncol_lim (sharded halo) are ignored.  Returns XFK_OK, or
    // XFK_ERR_UNSUPPORTED when a SpGEMM row exceeds the LDS hash capacity.
    int setup(hipStream_t s, int n, int ncol_lim, const int *rowptr, const int *col, const double *val,
              long long nnz);
    // Sharded level 0: n owned rows, nh halo columns (local ids n.., filled by
    // comm->exchange(halo)).  Aggregation and P use the owned block; the
    // Galerkin product uses the full rows with the peers' P rows for the halo,
    // so the coarse operator carries every inter-rank coupling.  Collective.
    int setup_dist(hipStream_t s, xfk_comm *comm, const HaloPlan &halo, int n, int nh, const int *rowptr,
                   const int *col, const double *val, long long nnz);
    // u = M^-1 r (owned rows of level 0); kernels return early once *done != 0.
    // Sharded: collective (halo exchanges, one all-gather).
    // part_gam: the PCG's gamma = r.u partials (k_cg_spmv layout), produced by
    // the last level-0 sweep when the cycle's shape allows (gamma_done)
    int vcycle(hipStream_t s, const double *r, double *u, const int *done, double *part_gam = nullptr);
    bool gamma_done = false;
    // New values in the level-0 matrix (same pattern): refresh the fine-level
    // smoother (D^-1, rho_A); the coarse levels are kept.
    // fold: level 0 stays folded (P~ re-formed for the new values); false: it runs unfolded
    int refresh(hipStream_t s, bool fold = true);
    // the host read-back / staging buffers, taken when the problem is created
    // (from the process's pinned cache): a first setup pins no pages
    int reserve_host();

  private:
    int init(hipStream_t s);
    int build(hipStream_t s, int l0);
    int aggregate(hipStream_t s, int l, long long &nc, bool allow_stop);
    int joins_and_p_impl(hipStream_t s, int l);
    int galerkin_dist(hipStream_t s, int l, int st, bool &rep);
    int fold_dist_tiles(hipStream_t s, int l);
    double *vc_dist(hipStream_t s, int l, const double *b, double *out, const int *done, int &rc);
    int host_ints(int count);
    int nd_order(hipStream_t s, const AmgLevel &C, int &ld);
    int resolve_deferred(hipStream_t s, bool &overflow);
    int fetch_deferred(hipStream_t s);
    int wait_deferred(hipStream_t s, bool &overflow);
    int dense_inverse(hipStream_t s, const AmgLevel &C, int ld);
    int alloc_vectors();
    long long ap_nnz = 0;
};

}  // namespace xfk
