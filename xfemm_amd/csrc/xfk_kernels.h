// Launch wrappers of the device kernels (xfk_device.hip), used by xfk_api.hip.
#pragma once

#include "xfk_internal.h"

namespace xfk {

struct AssembleArgs {
    const int4 *erec;
    const int *ebits;
    const int *slot;
    const double *x, *y;
    const DevLabel *labels;
    const DevBlock *blocks;
    const DevLine *lines;
    const DevCirc *circs;
    const double *bhB, *bhH, *bhS;
    double *mu1, *mu2;
    const double *V;
    double *val, *b;
    int iter;
    int axi;                      // StaticAxisymmetric element matrices (staticaxi.cpp:172-632)
    double ext_ro, ext_ri, ext_zo;   // exterior region (cm)
    // row-gather assembly (k_assemble_rows): raw-order element data, node ->
    // element lists, the CSR pattern, permeability state out (mu1 / mu2 in)
    const int *p_raw, *lbl_raw, *ebits_raw, *n2e_ptr, *n2e, *rowptr, *col;
    double *mu1_out, *mu2_out;     // null: linear problem, no state kept
    int *miss;                      // set to 1 when an element entry has no slot in its row
    // planar Newton passes (iter > 0): each element's new state evaluated once
    // by k_planar_state into mu*_out, dv_el (dv of GetBHProps) and on_el (the
    // Newton terms apply), read by every row of the element; null: per row
    double *dv_el;
    unsigned char *on_el;
    int n_el;                       // elements (the state pass's range)
};

int grid_reduce(int N);

struct CgAxpyArgs {
    const double *W, *dinv;
    double *Z, *P, *V, *R, *U;
    const double *gam_in;            // gamma_i partials (Ggam), previous k_cg_axpy / init
    const double *del_in;            // delta_i partials (Gdel), previous k_cg_spmv
    const double *reso;              // (M^-1 b).b partials (Gdel), read at it == 0
    double *gam_out;                 // gamma_i+1 partials
    int Ggam, Gdel;
    CgState *S;
    long long it;
    int N;
    int amg;                         // u = M^-1 r comes from the AMG V-cycle (U), gamma from the SpMV
};

int cg_grid(int N);
int cg_axpy_grid(int N);
// r0 = b - A x0 (x0 = V when flag, else 0), u0 = M^-1 r0, z = p = 0; partials of
// (M^-1 b).b and gamma_0 (w0 = A u0 follows with launch_cg_spmv, S = nullptr)
void launch_cg_init_r(hipStream_t s, int N, int flag, const int *rowptr, const int *col, const double *val,
                      const double *b, double *V, double *R, double *U, double *Z, double *P, const double *dinv,
                      double *part_reso, double *part_gam0);
void launch_cg_axpy(hipStream_t s, const CgAxpyArgs &A);
// w = A u, partials of u.w (and of r.u into part_gam when R != nullptr)
// c16 / cbase: 16-bit column offsets per 512-row tile (AmgLevel::a16), or null
void launch_cg_spmv(hipStream_t s, int N, const int *rowptr, const int *col, const double *val, const double *U,
                    double *W, double *part_del, const CgState *S, const double *R = nullptr,
                    double *part_gam = nullptr, const int *tiles = nullptr, int ntiles = 0,
                    const unsigned short *c16 = nullptr, const int *cbase = nullptr);
void launch_cg_dot(hipStream_t s, int N, const double *a, const double *b, double *part);
void launch_cg_state_init(hipStream_t s, CgState *S, double tol, double tol_rel = 0.0);

void launch_count_incidence(hipStream_t s, int NE, const int *p, int *deg);
void launch_fill_n2e(hipStream_t s, int NE, const int *p, const int *ptr, int *cursor, int *n2e);
void launch_sort_segments(hipStream_t s, int N, const int *ptr, int *a);
void launch_slot_elements(hipStream_t s, int NE, int *v);
void launch_n2e_count(hipStream_t s, int NE, const int *p, int *deg);
void launch_n2e_fill(hipStream_t s, int NE, const int *p, const int *ptr, int *cursor, int *n2e);
void launch_n2e_sort(hipStream_t s, int v0, int NL, const int *ptr, int *n2e);
void launch_n2e_ptr(hipStream_t s, int NL, const int *keys, int n3, int *ptr);
long long row_tmp_size(int N, int NE, int nfill);   // ints of the row-build scratch
void launch_row_build(hipStream_t s, int N, const int *p, const int *n2e_ptr, const int *n2e, const int *fill_ptr,
                      const int *fill_col, int *tmp, int *rowcnt,
                      int *n2e_sort = nullptr);
void launch_row_copy(hipStream_t s, int N, const int *p, const int *n2e_ptr, const int *n2e, const int *fill_ptr,
                     const int *fill_col, const int *tmp, const int *rowptr, int *col, int *diag);
// one Jones-Plassmann round (node pass + element pass) over the full arrays
void launch_jp_round(hipStream_t s, int N, int NE, int round, unsigned char *active, int *pending_round,
                     const int *p, const int *n2e_ptr, const int *n2e, int *color, unsigned long long *maxkey,
                     unsigned long long *used);
void launch_color_hist(hipStream_t s, int NE, const int *color, int *hist, int maxc);
void launch_iota(hipStream_t s, int n, int *a);
void launch_build_erec(hipStream_t s, int NE, const int *perm, const int *p, const int *lbl, const int *ebits_raw,
                       int4 *erec, int *ebits, int *iperm);
void launch_build_slots(hipStream_t s, int NE, int nrows, const int *p, const int *iperm, const int *rowptr,
                        const int *col, int *slot, int *bad);
// data[slot[i]] += v[i] (unique slots: race-free)
void launch_add_at_slots(hipStream_t s, int n, const int *slot, const double *v, double *data);
void launch_lookup_slots(hipStream_t s, int n, const int *rc, const int *rowptr, const int *col, int *out);
void launch_mark_fix_adj(hipStream_t s, int N, const int *rowptr, const int *col, const unsigned char *fixed,
                         int *flag);
void launch_compact_flags(hipStream_t s, int N, const int *flag, int *cursor, int *out);
// one thread per owned row, contributions of the incident elements in element order
void launch_assemble_rows(hipStream_t s, int N, const AssembleArgs &A);
void launch_point_currents(hipStream_t s, int n, const int *nodes, const double *J, double *b);
// nadj < 0: the count of rows adjacent to fixed nodes is *nadj_dev (at most nadj_max)
void launch_dirichlet(hipStream_t s, int nrows, const int *rows, int nadj, const int *nadj_dev, int nadj_max,
                      const int *adj, const int *rowptr, const int *col, const int *diag, const unsigned char *fixed,
                      const double *fix_first, const double *fix_last, double *val, double *b);
void launch_map(hipStream_t s, int n, const int *dst, const int *ptr, const int *src, const double *w,
                double *data, double *tmp);
void launch_diag_inv(hipStream_t s, int N, const int *diag, const double *val, double *dinv, CgState *S);
void launch_newton_res(hipStream_t s, int N, const double *V, const double *Vold, double *partials,
                       unsigned *counter, NewtonScalars *S);
void launch_relax(hipStream_t s, int N, double relax, double *V, const double *Vold);
void launch_scale(hipStream_t s, int N, double sc, const double *V, double *out);

}  // namespace xfk
