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

#include <cstdint>
#include <string>
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
    int LamType, BHpoints, bh_off, pad;
};

// Per-label parameters; the magnetisation direction is pre-evaluated on the
// host exactly as static2d.cpp:593-595 does (cos/sin of MagDir*PI/180).
struct DevLabel {
    double cos_m, sin_m;
    int blk, in_circuit, is_wound, pad;
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
    int done;
    int singular;
    long long iters;
};

struct NewtonScalars {
    double dx2;       // sum (V - Vold)^2
    double v2;        // sum V^2
};

// Small device buffer helper.
template <class T>
struct DBuf {
    T *p = nullptr;
    size_t n = 0;
    DBuf() = default;
    DBuf(const DBuf &) = delete;
    DBuf &operator=(const DBuf &) = delete;
    ~DBuf() { free(); }
    hipError_t alloc(size_t count) {
        if (count <= n && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        if (count == 0) return hipSuccess;
        hipError_t e = hipMalloc(&p, count * sizeof(T));
        if (e == hipSuccess) n = count;
        return e;
    }
    void free() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

}  // namespace xfk

// The opaque problem handle of the C-ABI.
struct xfk_problem {
    int device = 0;
    hipStream_t stream = nullptr;

    // sizes: N owned rows (= all nodes unless sharded), NL local nodes
    // (owned rows first, then the halo), NE local elements
    int N = 0, NL = 0, NE = 0;
    long long nnz = 0;
    int ncolors = 0;
    std::vector<int> color_off;      // ncolors + 1 (host)

    // sharded solve (xfk_problem_create_dist); comm == nullptr otherwise
    xfk_comm *comm = nullptr;
    int rank = 0, nranks = 1;
    int N_global = 0, row0 = 0;
    std::vector<int> l2g;            // local node -> global node
    xfk::HaloPlan halo;              // slices of the node vectors exchanged with peers
    int Gpart = 0;                   // length of each per-block partial array (agreed by all ranks)

    // host copies kept for host-side setup (periodic maps)
    std::vector<int> hp, hpbc;
    int length_units = 0, coords = 0;
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
    xfk::DBuf<double> mu1, mu2;      // colour order

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
    int nfix_cols = 0;
    // periodic map: dst <- sum_s w_s * src_s (values), and the same for b
    xfk::DBuf<int> pm_dst, pm_ptr, pm_src;
    xfk::DBuf<double> pm_w, pm_tmp;
    int pm_n = 0;
    xfk::DBuf<int> pb_dst, pb_ptr, pb_src;
    xfk::DBuf<double> pb_w, pb_tmp;
    int pb_n = 0;
    // fill-in entries requested by the periodic map (row, col) -> pattern
    std::vector<long long> pbc_fill;   // packed (row<<32)|col
    std::vector<std::vector<std::pair<long long, double>>> pbc_entry_terms;  // host form
    std::vector<long long> pbc_entry_key;
    std::vector<std::vector<std::pair<int, double>>> pbc_b_terms;
    std::vector<int> pbc_b_key;

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

    // preconditioner (xfk_set_option): XFK_PRECOND_AMG (default) or XFK_PRECOND_JACOBI
    int precond = XFK_PRECOND_AMG;
    int amg_sweeps = 2;
    double amg_theta = 0.08;
    xfk::Amg *amg = nullptr;         // hierarchy of the current matrix (xfk_amg.hip)
    int pc_used = XFK_PRECOND_JACOBI;  // preconditioner of the running solve

    // live SpMV launch timing (XFK_TIME_SPMV)
    bool time_spmv = false;
    std::vector<hipEvent_t> spmv_ev;   // pairs
    int spmv_used = 0;

    // last-solve statistics
    xfk_result last{};
};
