// Smoothed-aggregation AMG preconditioner for the fsolver PCG on MI355X
// (gfx950).  Design and parameters: xfk_amg.h.  Replaces the reference's SSOR
// preconditioner (cfemm/libfemm/spars.cpp:186-236, CBigLinProb::MultPC) on the
// device; the PCG itself (and its stopping test, spars.cpp:259/313) is
// unchanged.
//
// Every setup kernel is deterministic: decisions read only the previous
// launch's state, floating-point sums run in a fixed order (the SpGEMM
// accumulates each output entry in product-enumeration order), and atomics
// are used only where the result does not depend on their order (set
// membership, counts, max of non-negative values, positions that are sorted
// afterwards).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "xfk_amg.h"
#include "xfk_comm.h"
#include "xfk_spmv.h"

namespace xfk {

namespace {

// --------------------------------------------------------------------------
// small helpers
// --------------------------------------------------------------------------

constexpr int kB = 256;
inline int nb(long long n) { return (int)((n + kB - 1) / kB); }

// MIS key: (state:2 | perm(i):30), perm a bijection of [0, 2^30) (odd
// multipliers and xor-shifts): unique per node, so the max over a
// neighbourhood picks an IN node first, then the undecided node of the
// largest pseudo-random priority -- 4-byte keys halve the gathers of the two
// max sweeps of every round
using MisKey = unsigned;
constexpr MisKey kStIn = 2u, kStUnd = 1u;   // OUT = 0
constexpr MisKey kKeyMask = 0x3FFFFFFFu;

__device__ __forceinline__ MisKey perm30(unsigned x)
{
    x &= kKeyMask;
    x = (x * 0x2C1B3C6Du) & kKeyMask;
    x ^= x >> 15;
    x = (x * 0x297A2D39u) & kKeyMask;
    x ^= x >> 12;
    x = (x * 0x7FEB352Du) & kKeyMask;
    x ^= x >> 15;
    return x;
}
__device__ __forceinline__ MisKey mis_key(MisKey st, int i) { return (st << 30) | perm30((unsigned)i); }
__device__ __forceinline__ MisKey key_st(MisKey k) { return k >> 30; }
__device__ __forceinline__ MisKey key_low(MisKey k) { return k & kKeyMask; }

// The columns of a level's CSR as the aggregation reads them: the int array,
// or (level 0) the 16-bit offsets from the row's 512-row tile base
// (xfk_spmv.h k_tile_col16; a tile without a base reads the int array)
struct ColView {
    const int *col;
    const unsigned short *c16;   // null: int columns only
    const int *cbase;
    __device__ __forceinline__ int base(int i) const { return c16 ? cbase[i / kCgBlock] : kNoColBase; }
    __device__ __forceinline__ int at(int cb, int k) const { return cb != kNoColBase ? cb + (int)c16[k] : col[k]; }
};

// entries of a row whose loads are issued together in the aggregation sweeps
// (per row; G lanes take kMisChunk / G each)
constexpr int kMisChunk = 8;

__device__ __forceinline__ double rho_of(const unsigned long long *p)
{
    return __longlong_as_double((long long)*p);
}

// max of two values over the workgroup (kB threads), result in thread 0
__device__ __forceinline__ void block_max2(double &a, double &b, double *red)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        a = fmax(a, __shfl_xor(a, off, 64));
        b = fmax(b, __shfl_xor(b, off, 64));
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        red[2 * wid] = a;
        red[2 * wid + 1] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0)
        for (int w = 1; w < kB / 64; ++w) {
            a = fmax(a, red[2 * w]);
            b = fmax(b, red[2 * w + 1]);
        }
}

constexpr int kMaxReduceT = 256;

// per-block maxima (2 arrays of nblk) -> rho[0..1] as ordered bit patterns;
// rho[0] (read only by the smoothers, weight 1 / rho[0]) is divided by the
// Jacobi weight factor omega
__global__ void __launch_bounds__(kMaxReduceT) k_max_reduce(int nblk, const double *__restrict__ part, double omega,
                                                     unsigned long long *rho)
{
    __shared__ double red[2 * 16];
    double a = 0.0, b = 0.0;
    // kMaxU partials per array per thread loaded before the first fmax: one
    // load latency per kMaxU * blockDim partials (level 0 has ~2e4 blocks).
    // Launched with 256 threads (kMaxReduceT), not 1024: a 16-wave workgroup
    // waits for 16 free wave slots on one CU, which the side stream's
    // k_fold_p (31k 4-wave blocks) did not leave until it drained -- up to
    // 50 us of the setup's critical path at level 1
    constexpr int kMaxU = 16;
    for (int i0 = threadIdx.x; i0 < nblk; i0 += kMaxU * blockDim.x) {
        double pa[kMaxU], pb[kMaxU];
#pragma unroll
        for (int q = 0; q < kMaxU; ++q) {
            const int i = i0 + q * (int)blockDim.x;
            pa[q] = i < nblk ? part[i] : 0.0;
            pb[q] = i < nblk ? part[nblk + i] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < kMaxU; ++q) {   // (fmax of non-negative bounds: any order, the same bits)
            a = fmax(a, pa[q]);
            b = fmax(b, pb[q]);
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        a = fmax(a, __shfl_xor(a, off, 64));
        b = fmax(b, __shfl_xor(b, off, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        red[2 * (threadIdx.x >> 6)] = a;
        red[2 * (threadIdx.x >> 6) + 1] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
            a = fmax(a, red[2 * w]);
            b = fmax(b, red[2 * w + 1]);
        }
        rho[0] = (unsigned long long)__double_as_longlong(a / omega);
        rho[1] = (unsigned long long)__double_as_longlong(b);
    }
}

// --------------------------------------------------------------------------
// setup: diagonal, strength, Gershgorin bounds
// --------------------------------------------------------------------------

__global__ void k_amg_diag(int n, const int *__restrict__ rowptr, const int *__restrict__ col,
                           const double *__restrict__ val, double *__restrict__ absd, double *__restrict__ dinv)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // the row's columns a chunk at a time, loads issued together; the first
    // match is the diagonal
    const int s = rowptr[i], e = rowptr[i + 1];
    int kd = -1;
    for (int k0 = s; k0 < e && kd < 0; k0 += kMisChunk) {
        int c[kMisChunk];
#pragma unroll
        for (int q = 0; q < kMisChunk; ++q) c[q] = k0 + q < e ? col[k0 + q] : -1;
#pragma unroll
        for (int q = kMisChunk - 1; q >= 0; --q)
            if (c[q] == i) kd = k0 + q;
    }
    const double d = kd >= 0 ? val[kd] : 0.0;
    absd[i] = fabs(d);
    dinv[i] = (d != 0.0) ? 1.0 / d : 0.0;
}

// strong flags per nonzero (1 strong off-diagonal, 2 diagonal, 0 weak or
// outside the block), strong degree per row, lumped filtered diagonal,
// Gershgorin bounds of D^-1 A (rho[0]) and D_F^-1 A_F (rho[1])
// kStrG lanes per row (consecutive entries of a row on consecutive lanes:
// coalesced col / val reads and flag writes, the row's sums by shuffles)
constexpr int kStrG = 4;
inline int nb_str(long long n) { return nb(n * kStrG); }

__global__ void __launch_bounds__(kB) k_amg_strength(int n, int ncl, double theta, const int *__restrict__ rowptr,
                                                     ColView cv, const double *__restrict__ val,
                                                     const double *__restrict__ absd,
                                                     const double *__restrict__ dinv,
                                                     unsigned char *__restrict__ sflag, int *__restrict__ sdeg,
                                                     double *__restrict__ dfinv, double *__restrict__ wF,
                                                     double *__restrict__ rho_part, bool sgnd)
{
    __shared__ double red[2 * (kB / 64)];
    const int i = (blockIdx.x * blockDim.x + threadIdx.x) / kStrG;
    const int g = threadIdx.x % kStrG;
    double rA = 0.0, rF = 0.0;
    double aii = 0.0, lump = 0.0, sumS = 0.0, sumA = 0.0;
    int deg = 0, hdeg = 0;
    if (i < n) {
        const double ai = absd[i];
        const int cb = cv.base(i);
        // signed strength: only couplings of the sign opposite to the
        // diagonal's are strong (-a_ij for a positive diagonal).  Couplings of
        // the diagonal's own sign -- the reference's AntiPeriodicity averaging
        // gives each seam node such couplings to its partner's neighbours, an
        // air-gap element gives a few -- are weak and lumped, so no aggregate
        // spans an antiperiodic seam with a constant tentative value.
        // The test follows the diagonal's sign: the static operators are SPD,
        // the harmonic surrogate (Re A + s Im A of FEMM's sign convention) is
        // negative definite -- the diagonal negative, the couplings positive.
        // (sgnd == 0: |a_ij|, the former test, XFK_AMG_ABS_STRENGTH=1)
        const double sg = dinv[i] < 0.0 ? -1.0 : 1.0;
        const int s = rowptr[i] + g, e = rowptr[i + 1];
        // a chunk of this lane's entries at a time: columns and values, then
        // their diagonals, loaded before the first use; the entries are then
        // taken in the same order as one at a time (same sums, same bits)
        constexpr int C = kMisChunk / kStrG;
        for (int k0 = s; k0 < e; k0 += C * kStrG) {
        int jc[C];
        double ac[C], dj[C];
#pragma unroll
        for (int q = 0; q < C; ++q) {
            const int k = k0 + q * kStrG;
            const bool ok = k < e;
            jc[q] = ok ? cv.at(cb, k) : i;
            ac[q] = ok ? val[k] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < C; ++q) dj[q] = absd[jc[q] < ncl ? jc[q] : i];
#pragma unroll
        for (int q = 0; q < C; ++q) {
            const int k = k0 + q * kStrG;
            if (k >= e) break;
            const int j = jc[q];
            const double a = ac[q];
            unsigned char f = 0;
            if (j == i) {
                aii = a;
                f = 2;   // the diagonal: not a neighbour, but kept by the prolongator smoothing
            } else if (j >= ncl) {
                // halo column: read by the smoother; for the rank-local P it is
                // lumped like a weak entry, so P keeps reproducing constants
                // (strong by the one-sided test -a_ij > theta |a_ii|: the
                // peer's diagonal is not known here)
                sumA += fabs(a);
                lump += a;
                hdeg += ((sgnd ? -sg * a : fabs(a)) > theta * ai);
            } else {
                sumA += fabs(a);
                if (a != 0.0 && (sgnd ? -sg * a : fabs(a)) > theta * sqrt(ai * dj[q])) {
                    f = 1;
                    ++deg;
                    sumS += fabs(a);
                } else {
                    lump += a;
                }
            }
            sflag[k] = f;
        }
        }
    }
#pragma unroll
    for (int off = 1; off < kStrG; off <<= 1) {   // fixed butterfly: the same bits on every run
        aii += __shfl_xor(aii, off, kStrG);
        lump += __shfl_xor(lump, off, kStrG);
        sumS += __shfl_xor(sumS, off, kStrG);
        sumA += __shfl_xor(sumA, off, kStrG);
        deg += __shfl_xor(deg, off, kStrG);
        hdeg += __shfl_xor(hdeg, off, kStrG);
    }
    if (i < n && g == 0) {
        const double dF = aii + lump;
        // -1: every strong coupling crosses to a peer -> a singleton aggregate
        sdeg[i] = (deg == 0 && hdeg > 0) ? -1 : deg;
        if (aii != 0.0) rA = (fabs(aii) + sumA) / fabs(aii);
        if (dF != 0.0) rF = (fabs(dF) + sumS) / fabs(dF);
        // prolongator smoothing weight per row, 4 / (3 max(rho_i, 2)) with
        // rho_i the row's Gershgorin bound of D_F^-1 A_F: one row whose
        // filtered diagonal nearly cancels no longer shrinks the weight of
        // every row of the level (a global Gershgorin maximum of 100-200 was
        // measured on coarse levels of the steel / air problem)
        // rows without strong couplings keep the tentative (injection) row
        dfinv[i] = (dF != 0.0) ? 1.0 / dF : 0.0;
        wF[i] = (dF != 0.0 && deg > 0) ? (4.0 / 3.0) / fmax(rF, 2.0) : 0.0;
    }
    block_max2(rA, rF, red);
    if (threadIdx.x == 0) {
        rho_part[blockIdx.x] = rA;
        rho_part[gridDim.x + blockIdx.x] = rF;
    }
}

// a Newton refresh (same aggregates, P and weights; new values): only the
// Gershgorin bound of D^-1 A, summed as k_amg_strength sums it (each lane's
// entries in order, the same butterfly: the same bits); rho[1] is not used
// after a setup and is left 0.  The row's diagonal found here also gives
// |a_ii| and D^-1 (k_amg_diag's values: the other lanes add 0.0 to it), so the
// refresh reads the matrix once
__global__ void __launch_bounds__(kB) k_amg_rho(int n, const int *__restrict__ rowptr, ColView cv,
                                                const double *__restrict__ val, double *__restrict__ rho_part,
                                                double *__restrict__ absd, double *__restrict__ dinv)
{
    __shared__ double red[2 * (kB / 64)];
    const int i = (blockIdx.x * blockDim.x + threadIdx.x) / kStrG;
    const int g = threadIdx.x % kStrG;
    double rA = 0.0, rF = 0.0, aii = 0.0, sumA = 0.0;
    if (i < n) {
        const int cb = cv.base(i);
        const int e = rowptr[i + 1];
        for (int k = rowptr[i] + g; k < e; k += kStrG) {
            const int j = cv.at(cb, k);
            const double a = val[k];
            if (j == i) aii = a;
            else sumA += fabs(a);
        }
    }
#pragma unroll
    for (int off = 1; off < kStrG; off <<= 1) {
        aii += __shfl_xor(aii, off, kStrG);
        sumA += __shfl_xor(sumA, off, kStrG);
    }
    if (i < n && g == 0) {
        if (aii != 0.0) rA = (fabs(aii) + sumA) / fabs(aii);
        absd[i] = fabs(aii);
        dinv[i] = (aii != 0.0) ? 1.0 / aii : 0.0;
    }
    block_max2(rA, rF, red);
    if (threadIdx.x == 0) {
        rho_part[blockIdx.x] = rA;
        rho_part[gridDim.x + blockIdx.x] = rF;
    }
}

// --------------------------------------------------------------------------
// setup: MIS-2 aggregation
// --------------------------------------------------------------------------

// also arms the round bookkeeping: "undecided" for the round before the
// first, no round run yet
__global__ void k_mis_init(int n, const int *__restrict__ sdeg, MisKey *__restrict__ key, int *und_prev,
                           int *run, unsigned char *__restrict__ act)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        *und_prev = 1;
        *run = 0;
    }
    if (i < n) {
        key[i] = mis_key(sdeg[i] > 0 ? kStUnd : (sdeg[i] < 0 ? kStIn : 0u), i);
        act[i] = 1;
    }
}

// Rounds are launched in batches without a host check in between: the
// undecided flag is double-buffered by round parity (prev = the last round's
// result, cur = this round's), and once a round leaves nothing undecided the
// later rounds of the batch exit at once (passing the 0 on).
// G lanes per row (coarse levels, 10-16 entries per row; 1 on the fine level):
// consecutive strong entries on consecutive lanes, the maximum by a butterfly.
// A row whose strong neighbourhood holds no undecided row any more keeps its
// maximum for good (decided rows never change): act[i] = 0 then, and later
// rounds skip the row -- after the first rounds most of the level.
template <int G>
__global__ void k_mis_max(int n, const int *__restrict__ rowptr, ColView cv,
                          const unsigned char *__restrict__ sflag, const MisKey *__restrict__ in,
                          MisKey *__restrict__ out, const int *prev, int *cur, int *run,
                          unsigned char *__restrict__ act, int xcd)
{
    // xcd: consecutive blocks on one XCD (xcd_tile): a block's neighbour rows
    // a mesh row away stay in that XCD's L2
    const int bx = xcd ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int t = bx * blockDim.x + threadIdx.x;
    const int i = t / G, g = t % G;
    if (blockIdx.x == 0 && threadIdx.x == 0) {   // k_mis_update of this round runs after this launch
        if (*prev != 0) *run += 1;   // rounds that did work (the next setup's batch size)
        *cur = 0;
    }
    if (i >= n || *prev == 0 || act[i] == 0) return;
    MisKey m = in[i];
    int any = key_st(m) == kStUnd;
    const int cb = cv.base(i);
    for (int k = rowptr[i] + g; k < rowptr[i + 1]; k += G)
        if (sflag[k] == 1) {
            const MisKey v = in[cv.at(cb, k)];
            m = max(m, v);
            any |= key_st(v) == kStUnd;
        }
#pragma unroll
    for (int off = 1; off < G; off <<= 1) {
        m = max(m, (MisKey)__shfl_xor((int)m, off, G));
        any |= __shfl_xor(any, off, G);
    }
    if (g == 0) {
        out[i] = m;
        if (!any) act[i] = 0;
    }
}

// second max sweep fused with the state update: an undecided node whose
// distance-2 maximum is itself joins the set; one that sees a set member
// within distance 2 leaves
// ROOTS (the last round of a batch): every row also writes its root flag
// (k_agg_roots folded in: one launch less per level)
template <int G, bool ROOTS = false>
__global__ void k_mis_update(int n, const int *__restrict__ rowptr, ColView cv,
                             const unsigned char *__restrict__ sflag, const MisKey *__restrict__ t1,
                             MisKey *__restrict__ key, const int *prev, int *undecided, int *__restrict__ flag,
                             int xcd)
{
    const int bx = xcd ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int t = bx * blockDim.x + threadIdx.x;
    const int i = t / G, g = t % G;
    if (i >= n) return;
    const MisKey k = key[i];
    if (*prev == 0 || key_st(k) != kStUnd) {   // uniform over the row's lanes
        if (ROOTS && g == 0) flag[i] = key_st(k) == kStIn;
        return;
    }
    MisKey m = t1[i];
    const int cb = cv.base(i);
    for (int q = rowptr[i] + g; q < rowptr[i + 1]; q += G)
        if (sflag[q] == 1) m = max(m, t1[cv.at(cb, q)]);
#pragma unroll
    for (int off = 1; off < G; off <<= 1) m = max(m, (MisKey)__shfl_xor((int)m, off, G));
    if (g != 0) return;
    int root = 0;
    if (key_low(m) == perm30((unsigned)i)) {
        key[i] = (kStIn << 30) | key_low(k);
        root = 1;
    } else if (key_st(m) == kStIn) {
        key[i] = key_low(k);
    } else {
        *undecided = 1;   // benign race: every writer stores 1
    }
    if (ROOTS) flag[i] = root;
}


// the aggregation's host check in one read: {roots, undecided flag, rounds that did work}
__global__ void k_mis_pack(const int *__restrict__ roots, const int *__restrict__ und, const int *__restrict__ run,
                           int *__restrict__ out)
{
    if (threadIdx.x == 0) {
        out[0] = *roots;
        out[1] = *und;
        out[2] = *run;
    }
}

// out = 1 when the pattern (rowptr[0..n], col[0..key_nnz)) differs from the
// key (rowptr, then col); equal row pointers make the lengths equal, so the
// first key_nnz columns decide (columns read only below the buffer capacity,
// checked by the caller)
__global__ void k_pattern_diff(int n, const int *__restrict__ rowptr, const int *__restrict__ col,
                               const int *__restrict__ key, int key_nnz, int *__restrict__ out)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    bool d = false;
    if (t <= n) d = rowptr[t] != key[t];
    if (t < key_nnz) d = d || col[t] != key[n + 1 + t];
    if (d) out[0] = 1;
}

// The joins take G lanes per row (consecutive entries on consecutive lanes,
// G = 1 on the fine level): each lane keeps its best candidate in its own
// (increasing) entry order and the lanes' candidates are combined by the
// same total order the one-thread loop applies -- the largest key, on a tie
// the earlier entry (joins 1, 2), the largest |a_ij| and then the larger j
// (join 3) -- so every G selects the same neighbour.  The coarse levels'
// rows hold 10-40 entries: one thread walking them took 30-40 us per level.
template <int G>
__device__ __forceinline__ void join_best_key(MisKey &best, int &bk, int &bj)
{
#pragma unroll
    for (int off = 1; off < G; off <<= 1) {
        const MisKey ob = __shfl_xor(best, off, G);
        const int obk = __shfl_xor(bk, off, G), obj = __shfl_xor(bj, off, G);
        if (obj >= 0 && (bj < 0 || ob > best || (ob == best && obk < bk))) {
            best = ob;
            bk = obk;
            bj = obj;
        }
    }
}

// distance 1: roots keep their aggregate, neighbours of roots join the root
// with the largest key
// rows left out that have (weak) couplings to aggregated owned rows join the
// aggregate of the largest |a_ij| (ties: larger j); their P row is the
// tentative injection (no strong couplings -> smoothing weight 0)
template <int G>
__global__ void __launch_bounds__(kB) k_agg_join3(int n, int ncl, const int *__restrict__ rowptr, ColView cv,
                                                  const double *__restrict__ val, const int *__restrict__ agg2,
                                                  int *__restrict__ agg)
{
    const int i = (blockIdx.x * blockDim.x + threadIdx.x) / G, l = threadIdx.x % G;
    if (i >= n) return;   // (whole groups)
    int a = agg2[i];
    if (a < 0) {
        double best = 0.0;
        int bj = -1;
        const int cb = cv.base(i);
        for (int k = rowptr[i] + l; k < rowptr[i + 1]; k += G) {
            const int j = cv.at(cb, k);
            if (j == i || j >= ncl || agg2[j] < 0) continue;
            const double v = fabs(val[k]);
            if (v > best || (v == best && v > 0.0 && j > bj)) {
                best = v;
                bj = j;
            }
        }
#pragma unroll
        for (int off = 1; off < G; off <<= 1) {
            const double ob = __shfl_xor(best, off, G);
            const int obj = __shfl_xor(bj, off, G);
            if (obj >= 0 && (ob > best || (ob == best && ob > 0.0 && obj > bj))) {
                best = ob;
                bj = obj;
            }
        }
        if (bj >= 0) a = agg2[bj];
    }
    if (l == 0) agg[i] = a;
}

template <int G>
__global__ void __launch_bounds__(kB) k_agg_join1(int n, const int *__restrict__ rowptr, ColView cv,
                                                  const unsigned char *__restrict__ sflag,
                                                  const MisKey *__restrict__ key, const int *__restrict__ rootid,
                                                  int *__restrict__ agg1)
{
    const int i = (blockIdx.x * blockDim.x + threadIdx.x) / G, l = threadIdx.x % G;
    if (i >= n) return;
    if (key_st(key[i]) == kStIn) {
        if (l == 0) agg1[i] = rootid[i];
        return;
    }
    int bj = -1, bk = INT_MAX;
    MisKey best = 0;
    const int cb = cv.base(i);
    for (int k = rowptr[i] + l; k < rowptr[i + 1]; k += G) {
        if (sflag[k] != 1) continue;
        const int j = cv.at(cb, k);
        const MisKey kj = key[j];
        if (key_st(kj) == kStIn && (bj < 0 || key_low(kj) > best)) {
            best = key_low(kj);
            bj = j;
            bk = k;
        }
    }
    join_best_key<G>(best, bk, bj);
    if (l == 0) agg1[i] = (bj >= 0) ? rootid[bj] : -1;
}

// distance 2: the rest join the aggregate of their largest-key neighbour
// that joined at distance 1
template <int G>
__global__ void __launch_bounds__(kB) k_agg_join2(int n, const int *__restrict__ rowptr, ColView cv,
                                                  const unsigned char *__restrict__ sflag,
                                                  const MisKey *__restrict__ key, const int *__restrict__ agg1,
                                                  int *__restrict__ agg)
{
    const int i = (blockIdx.x * blockDim.x + threadIdx.x) / G, l = threadIdx.x % G;
    if (i >= n) return;
    const int a = agg1[i];
    if (a >= 0) {
        if (l == 0) agg[i] = a;
        return;
    }
    int bj = -1, bk = INT_MAX;
    MisKey best = 0;
    const int cb = cv.base(i);
    for (int k = rowptr[i] + l; k < rowptr[i + 1]; k += G) {
        if (sflag[k] != 1) continue;
        const int j = cv.at(cb, k);
        if (agg1[j] < 0) continue;
        const MisKey kl = key_low(key[j]);
        if (bj < 0 || kl > best) {
            best = kl;
            bj = j;
            bk = k;
        }
    }
    join_best_key<G>(best, bk, bj);
    if (l == 0) agg[i] = (bj >= 0) ? agg1[bj] : -1;   // -1: isolated (or unreachable) -> no coarse dof
}

// lanes per row of the aggregation joins for rows of this average length
static int join_lanes(double per_row)
{
    const char *e = std::getenv("XFK_JOIN_LANES");   // (read per level: tests toggle it)
    const int v = e ? std::atoi(e) : 0;
    if (v == 1 || v == 4 || v == 8) return v;
    return per_row <= 8.0 ? 1 : (per_row <= 16.0 ? 4 : 8);
}

// --------------------------------------------------------------------------
// setup: R = P^T
// --------------------------------------------------------------------------

__global__ void k_rt_count(int n, const int *__restrict__ prow, const int *__restrict__ pcol, int *__restrict__ rcnt)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int k = prow[i]; k < prow[i + 1]; ++k) atomicAdd(&rcnt[pcol[k]], 1);
}

// the counts left by k_rt_count count down to each row's free slot (no
// zeroed cursor array needed)
__global__ void k_rt_fill(int n, const int *__restrict__ prow, const int *__restrict__ pcol,
                          const int *__restrict__ rrow, int *__restrict__ cnt, int *__restrict__ rcol)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int k = prow[i]; k < prow[i + 1]; ++k) {
        const int J = pcol[k];
        rcol[rrow[J] + atomicSub(&cnt[J], 1) - 1] = i;
    }
}

// Tiled transpose (XFK_RT_TILE, default on): a workgroup of 256 rows holds
// its entries' columns in a window [lo, hi] (a banded numbering: a few
// hundred columns), counts them in LDS and touches
// the global counts once per (workgroup, column) instead of once per entry.
// The fill reserves one chunk of each target row per workgroup (returning
// atomic on the count-down counter), places its entries there through LDS
// cursors and writes the values with the columns; the row sort restores the
// order.  A window wider than kRtWin falls back to per-entry atomics.
constexpr int kRtWin = 4096;
template <bool FILL>
__global__ void __launch_bounds__(256) k_rt_tile(int n, const int *__restrict__ mrow, const int *__restrict__ mcol,
                                                 const double *__restrict__ mval, const int *__restrict__ trow,
                                                 int *__restrict__ cnt, int *__restrict__ tcol,
                                                 double *__restrict__ tval)
{
    __shared__ int h[kRtWin];
    __shared__ int cur[FILL ? kRtWin : 1];
    __shared__ int red[8];
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int s = i < n ? mrow[i] : 0, e = i < n ? mrow[i + 1] : 0;
    int lo = INT_MAX, hi = INT_MIN;   // (every entry: the rows need not be sorted)
    for (int k = s; k < e; ++k) {
        const int c = mcol[k];
        lo = min(lo, c);
        hi = max(hi, c);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        lo = min(lo, __shfl_xor(lo, off, 64));
        hi = max(hi, __shfl_xor(hi, off, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6] = lo;
        red[4 + (threadIdx.x >> 6)] = hi;
    }
    __syncthreads();
    lo = min(min(red[0], red[1]), min(red[2], red[3]));
    hi = max(max(red[4], red[5]), max(red[6], red[7]));
    if (hi < lo) return;   // no entries in this tile
    if ((long long)hi - lo >= kRtWin) {   // wide window: one global atomic per entry
        for (int k = s; k < e; ++k) {
            const int J = mcol[k];
            if (!FILL) {
                atomicAdd(&cnt[J], 1);
            } else {
                const int pos = trow[J] + atomicSub(&cnt[J], 1) - 1;
                tcol[pos] = i;
                tval[pos] = mval[k];
            }
        }
        return;
    }
    const int w = hi - lo + 1;
    for (int c = threadIdx.x; c < w; c += 256) {
        h[c] = 0;
        if (FILL) cur[c] = 0;
    }
    __syncthreads();
    for (int k = s; k < e; ++k) atomicAdd(&h[mcol[k] - lo], 1);
    __syncthreads();
    if (!FILL) {
        for (int c = threadIdx.x; c < w; c += 256)
            if (h[c]) atomicAdd(&cnt[lo + c], h[c]);
        return;
    }
    for (int c = threadIdx.x; c < w; c += 256) {
        const int m = h[c];
        if (m) h[c] = trow[lo + c] + atomicSub(&cnt[lo + c], m) - m;   // this tile's chunk of row lo + c
    }
    __syncthreads();
    for (int k = s; k < e; ++k) {
        const int c = mcol[k] - lo;
        const int pos = h[c] + atomicAdd(&cur[c], 1);
        tcol[pos] = i;
        tval[pos] = mval[k];
    }
}

// sort each row's (column, value) pairs by column (the rows' entries are
// distinct).  A wavefront takes 4 consecutive rows: when all hold <= 64
// entries (the usual case) each 16-lane group ranks its row's columns in
// wave-private LDS (rank = number of smaller columns, <= 64 broadcast reads
// per entry) and writes every pair straight to its rank -- no compare-exchange
// network, values never shuffled; longer rows are taken one at a time by the
// whole wavefront (<= kRtLdsRow entries in LDS, else lane 0's insertion sort).
constexpr int kRtLdsRow = 1024;
__global__ void __launch_bounds__(256) k_rt_sort_pairs(int nc, const int *__restrict__ rrow, int *__restrict__ rcol,
                                                       double *__restrict__ rval)
{
    __shared__ int buf[4][kRtLdsRow];
    __shared__ double bufv[4][kRtLdsRow];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int J0 = ((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 4;
    if (J0 >= nc) return;
    int *b = buf[wv];
    double *bv = bufv[wv];
    auto wsync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // this group's row (groups past nc get an empty one)
    const int g = lane >> 4, gl = lane & 15, J = J0 + g;
    const int s = J < nc ? rrow[J] : 0, len = J < nc ? rrow[J + 1] - s : 0;
    int mx = len;
#pragma unroll
    for (int off = 16; off < 64; off <<= 1) mx = max(mx, __shfl_xor(mx, off, 64));
    if (mx <= 64) {
        int *gb = b + 64 * g;
        int kk[4];
        double vv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int a = gl + 16 * q;
            kk[q] = a < len ? rcol[s + a] : 0;
            vv[q] = a < len ? rval[s + a] : 0.0;
            if (a < len) gb[a] = kk[q];
        }
        wsync();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int a = gl + 16 * q;
            if (a < len) {
                int rk = 0;
                for (int t = 0; t < len; ++t) rk += gb[t] < kk[q];
                rcol[s + rk] = kk[q];
                rval[s + rk] = vv[q];
            }
        }
        return;
    }
    for (int r = 0; r < 4 && J0 + r < nc; ++r) {
        const int Jr = J0 + r;
        const int sr = rrow[Jr], er = rrow[Jr + 1], lr = er - sr;
        if (lr <= 1) continue;
        if (lr <= kRtLdsRow) {
            wsync();   // the previous row's reads of b are done
            for (int a = lane; a < lr; a += 64) {
                b[a] = rcol[sr + a];
                bv[a] = rval[sr + a];
            }
            wsync();
            for (int a = lane; a < lr; a += 64) {
                const int v = b[a];
                int rk = 0;
                for (int q = 0; q < lr; ++q) rk += b[q] < v;
                rcol[sr + rk] = v;
                rval[sr + rk] = bv[a];
            }
        } else if (lane == 0) {
            for (int a = sr + 1; a < er; ++a) {
                const int key = rcol[a];
                const double kv = rval[a];
                int q = a - 1;
                while (q >= sr && rcol[q] > key) {
                    rcol[q + 1] = rcol[q];
                    rval[q + 1] = rval[q];
                    --q;
                }
                rcol[q + 1] = key;
                rval[q + 1] = kv;
            }
        }
    }
}

// sort each R row (the atomic fill order is arbitrary), then look the values
// up in P.  One wavefront per row: rows of <= 64 entries are sorted by a
// register bitonic network, longer ones by lane 0 (insertion sort).
__global__ void __launch_bounds__(256) k_rt_sort_vals(int nc, const int *__restrict__ rrow, int *__restrict__ rcol,
                                                      const int *__restrict__ prow, const int *__restrict__ pcol,
                                                      const double *__restrict__ pval, double *__restrict__ rval)
{
    const int J = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (J >= nc) return;
    const int s = rrow[J], e = rrow[J + 1], len = e - s;
    if (len <= 64) {
        int v = (lane < len) ? rcol[s + lane] : INT_MAX;
#pragma unroll
        for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
            for (int j = k >> 1; j > 0; j >>= 1) {
                const int o = __shfl_xor(v, j, 64);
                const bool up = ((lane & k) == 0);
                const bool lower = ((lane & j) == 0);
                v = (lower == up) ? min(v, o) : max(v, o);
            }
        }
        if (lane < len) rcol[s + lane] = v;
    } else if (len <= kRtLdsRow) {
        // longer rows (the folded R~ of a coarse level: ~150 entries): the row
        // in LDS, every entry placed at its rank (the row indices are distinct)
        __shared__ int buf[4][kRtLdsRow];
        int *b = buf[threadIdx.x >> 6];
        for (int a = lane; a < len; a += 64) b[a] = rcol[s + a];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int a = lane; a < len; a += 64) {
            const int v = b[a];
            int rk = 0;
            for (int q = 0; q < len; ++q) rk += b[q] < v;
            rcol[s + rk] = v;
        }
    } else if (lane == 0) {
        for (int a = s + 1; a < e; ++a) {
            const int key = rcol[a];
            int b = a - 1;
            while (b >= s && rcol[b] > key) {
                rcol[b + 1] = rcol[b];
                --b;
            }
            rcol[b + 1] = key;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int a = s + lane; a < e; a += 64) {
        const int i = rcol[a];
        int lo = prow[i], hi = prow[i + 1] - 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (pcol[mid] < J) lo = mid + 1;
            else hi = mid;
        }
        rval[a] = pval[lo];
    }
}

// --------------------------------------------------------------------------
// setup: row-merge SpGEMM C = X Y, one wavefront per row
// --------------------------------------------------------------------------
//
// Products of row r are enumerated in a fixed order (X entries in row order,
// each Y row in column order), 64 at a time: a wave prefix sum of the Y-row
// lengths of up to 64 X entries maps lane products to (X entry, Y position).
// Pass COUNT inserts the output columns into an LDS hash set and returns the
// row length; pass FILL inserts them again, ranks them (sorted columns) and
// accumulates each product into its column in enumeration order: within a
// group of 64 products, the first lane of each column sums the group's
// products of that column in lane order, then adds the group sum to the LDS
// accumulator -- the same operation order on every run.
//
// PMODE builds the smoothed prolongator P = S P_tent directly: X is the level
// matrix masked to its strong entries and diagonal, with values
// S = I - omega D_F^-1 A_F, and Y = P_tent is given by the aggregate map
// (row k = {agg[k] : 1}, empty when k is not aggregated).

constexpr int kSgMax = 512;        // distinct output columns per row (COUNT pass hash: 2 kSgMax slots)

constexpr int ilog2(int v) { return v <= 1 ? 0 : 1 + ilog2(v >> 1); }

struct SgX {
    const int *rowptr, *col;
    const double *val;
    int col_lim;                   // X columns >= col_lim are skipped (sharded halo)
    const unsigned char *mask;     // PMODE: sflag (1 strong, 2 diagonal)
    const double *dfinv;           // PMODE: D_F^-1
    const double *wF;              // PMODE: per-row smoothing weight
    const unsigned short *c16 = nullptr;   // level 0: 16-bit tile columns (k_spgemm_sort reads them)
    const int *cbase = nullptr;
};
struct SgY {
    const int *rowptr, *col;
    const double *val;
    const int *agg;                // PMODE: P_tent
};

// CAP: distinct columns a row may have (FILL is launched with the smallest
// CAP that covers the longest row the COUNT pass found, so typical levels run
// with a few KiB of LDS per wave and full occupancy); hash slots = 2 CAP.
template <bool FILL, bool PMODE, int CAP>
__global__ void __launch_bounds__(64) k_spgemm(int nrows, SgX X, SgY Y, int *__restrict__ cnt_out,
                                               const int *__restrict__ crow, int *__restrict__ ccol,
                                               double *__restrict__ cval, int *overflow)
{
    constexpr int kSgHash = 2 * CAP;
    constexpr int kHashShift = 32 - ilog2(kSgHash);
    __shared__ int hk[kSgHash];
    __shared__ int hr[FILL ? kSgHash : 1];
    __shared__ int lst[FILL ? CAP : 1], lslot[FILL ? CAP : 1];
    __shared__ double acc[FILL ? CAP : 1];
    __shared__ int c_off[64], c_ys[64];
    __shared__ double c_xv[64];
    __shared__ __attribute__((aligned(16))) int s_rank[64];
    __shared__ double s_val[64];
    __shared__ int s_cnt, s_ovf, s_m;

    const int row = blockIdx.x;
    const int lane = threadIdx.x;
    if (row >= nrows) return;
    for (int t = lane; t < kSgHash; t += 64) hk[t] = -1;
    if (lane == 0) {
        s_cnt = 0;
        s_ovf = 0;
        s_m = 0;
    }
    __syncthreads();
    const int xs = X.rowptr[row], xe = X.rowptr[row + 1];
    double omega = 0.0, dfi = 0.0;
    if (PMODE) {
        omega = X.wF[row];
        dfi = X.dfinv[row];
    }

    auto insert = [&](int key) {
        unsigned h = ((unsigned)key * 2654435761u) >> kHashShift;
        for (int probe = 0; probe < kSgHash; ++probe) {
            const int old = atomicCAS(&hk[h], -1, key);
            if (old == -1) {
                atomicAdd(&s_cnt, 1);
                return;
            }
            if (old == key) return;
            h = (h + 1) & (kSgHash - 1);
        }
        s_ovf = 1;
    };
    auto lookup = [&](int key) -> int {
        unsigned h = ((unsigned)key * 2654435761u) >> kHashShift;
        for (int probe = 0; probe < kSgHash; ++probe) {
            const int k = hk[h];
            if (k == key) return (int)h;
            if (k == -1) return -1;
            h = (h + 1) & (kSgHash - 1);
        }
        return -1;
    };
    // stage up to 64 X entries of [e0, xe); returns the group's product count
    auto stage = [&](int e0) -> int {
        const int e = e0 + lane;
        int len = 0, ys = 0;
        double xv = 0.0;
        if (e < xe) {
            const int k = X.col[e];
            if (k < X.col_lim) {
                if (PMODE) {
                    const unsigned char f = X.mask[e];
                    if (f != 0 && Y.agg[k] >= 0) {
                        ys = k;
                        len = 1;
                        xv = (f == 2) ? 1.0 - omega : -omega * dfi * X.val[e];
                    }
                } else {
                    ys = Y.rowptr[k];
                    len = Y.rowptr[k + 1] - ys;
                    xv = X.val[e];
                }
            }
        }
        int incl = len;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int t = __shfl_up(incl, off, 64);
            if (lane >= off) incl += t;
        }
        const int total = __shfl(incl, 63, 64);
        c_off[lane] = incl - len;
        c_ys[lane] = ys;
        c_xv[lane] = xv;
        __syncthreads();
        return total;
    };
    // product p of the staged group -> (column, value)
    auto product = [&](int p, int &key, double &v) {
        int lo = 0, hi = 63;   // largest staged entry with c_off <= p
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (c_off[mid] <= p) lo = mid;
            else hi = mid - 1;
        }
        if (PMODE) {
            key = Y.agg[c_ys[lo]];
            v = c_xv[lo];
        } else {
            const int q = c_ys[lo] + (p - c_off[lo]);
            key = Y.col[q];
            if (FILL) v = c_xv[lo] * Y.val[q];
        }
    };

    // pass 1: the set of output columns
    for (int e0 = xs; e0 < xe; e0 += 64) {
        const int total = stage(e0);
        for (int p = lane; p < total; p += 64) {
            int key;
            double v;
            product(p, key, v);
            insert(key);
        }
        __syncthreads();
    }
    if (!FILL) {
        if (lane == 0) {
            cnt_out[row] = s_cnt;
            if (s_ovf || s_cnt > CAP) atomicOr(overflow, 1);
        }
        return;
    }
    // rank the columns (sorted order) and map hash slot -> rank
    for (int t = lane; t < kSgHash; t += 64)
        if (hk[t] != -1) {
            const int m = atomicAdd(&s_m, 1);
            if (m < CAP) {
                lst[m] = hk[t];
                lslot[m] = t;
            }
        }
    __syncthreads();
    const int cnt = min(s_m, CAP);
    const int cb = crow[row];
    for (int m = lane; m < cnt; m += 64) {
        const int key = lst[m];
        int rank = 0;
        for (int q = 0; q < cnt; ++q) rank += lst[q] < key;
        hr[lslot[m]] = rank;
        ccol[cb + rank] = key;
        acc[rank] = 0.0;
    }
    __syncthreads();
    // pass 2: values in enumeration order
    const int4 *r4 = reinterpret_cast<const int4 *>(s_rank);
    for (int e0 = xs; e0 < xe; e0 += 64) {
        const int total = stage(e0);
        for (int p0 = 0; p0 < total; p0 += 64) {
            const int p = p0 + lane;
            int rank = -1;
            double v = 0.0;
            if (p < total) {
                int key;
                product(p, key, v);
                const int h = lookup(key);
                rank = (h >= 0) ? hr[h] : -1;
            }
            s_rank[lane] = rank;
            s_val[lane] = v;
            __syncthreads();
            if (rank >= 0) {
                bool leader = true;
                double sum = 0.0;
#pragma unroll
                for (int m4 = 0; m4 < 16; ++m4) {
                    const int4 q = r4[m4];
                    const int m = 4 * m4;
                    if (q.x == rank) { leader &= (m < lane) ? false : true; sum += s_val[m]; }
                    if (q.y == rank) { leader &= (m + 1 < lane) ? false : true; sum += s_val[m + 1]; }
                    if (q.z == rank) { leader &= (m + 2 < lane) ? false : true; sum += s_val[m + 2]; }
                    if (q.w == rank) { leader &= (m + 3 < lane) ? false : true; sum += s_val[m + 3]; }
                }
                if (leader) acc[rank] += sum;
            }
            __syncthreads();
        }
    }
    for (int m = lane; m < cnt; m += 64) cval[cb + m] = acc[m];
}

// Products per row (upper bound of the output row length), for the choice
// between the sub-wave and the wave-per-row SpGEMM.
template <bool PMODE>
__global__ void k_spgemm_nprod(int nrows, SgX X, SgY Y, int *__restrict__ nprod)
{
    const int row = blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= nrows) return;
    int c = 0;
    for (int e = X.rowptr[row]; e < X.rowptr[row + 1]; ++e) {
        const int k = X.col[e];
        if (k >= X.col_lim) continue;
        if (PMODE) c += (X.mask[e] != 0 && Y.agg[k] >= 0);
        else c += Y.rowptr[k + 1] - Y.rowptr[k];
    }
    nprod[row] = c;
}

// Sub-wave SpGEMM (the fine levels: A P, the prolongator, R (A P)): G lanes
// per row, 64 / G rows per wavefront.  Groups of one wavefront advance
// independently; their LDS regions are private, and LDS traffic inside a
// wavefront is ordered, so no workgroup barriers are needed (wave_barrier
// keeps the compiler from reordering).
constexpr int kSortCap = 256;         // k_spgemm_sort: rows of at most this many products

__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Sort-based single-pass SpGEMM for rows of at most CAP products: a group of
// G lanes per row (64 / G rows per wavefront).  Lane l expands X entries
// l, l + G, ... (its Y row) into the row's product list in LDS -- the fixed
// enumeration order -- then the list is loaded as CAP virtual slots, S = CAP / G
// consecutive slots per lane in registers, and sorted by column with a bitonic
// network (in-lane compare-exchanges for distances < S, shuffles across the
// group for the others).  A segmented inclusive scan then sums each column's
// products and counts the distinct columns; the last slot of each column
// writes it at its rank.  The network and the scan are fixed, so the sums
// are the same bits on every run.  Only the product list (12 B per product)
// lives in LDS: several times more rows in flight than the hash kernels.
// The row is written padded (row * CAP) with its length; k_spgemm_compact
// moves it to its CSR place after the length scan.
template <bool PMODE, int G, int CAP>
__global__ void __launch_bounds__(64) k_spgemm_sort(int nrows, SgX X, SgY Y, int *__restrict__ cnt_out,
                                                    int *__restrict__ pcol, double *__restrict__ pval, int *ovf,
                                                    int *need = nullptr)
{
    constexpr int W = 64 / G;
    constexpr int S = CAP / G;
    static_assert(S >= 1 && S * G == CAP, "CAP must be a multiple of G");
    __shared__ int pk_all[W][CAP];
    __shared__ double pv_all[W][CAP];
    const int g = threadIdx.x / G, l = threadIdx.x % G;
    const int row = blockIdx.x * W + g;
    int *pk = pk_all[g];
    double *pv = pv_all[g];
    const bool live = row < nrows;
    int np = 0;
    if (live) {
        const int xs = X.rowptr[row], xe = X.rowptr[row + 1];
        const ColView xc{X.col, X.c16, X.cbase};
        const int cb = xc.base(row);
        double omega = 0.0, dfi = 0.0;
        if (PMODE) {
            omega = X.wF[row];
            dfi = X.dfinv[row];
        }
        for (int e0 = xs; e0 < xe; e0 += G) {
            const int e = e0 + l;
            int len = 0, ys = 0;
            double xv = 0.0;
            if (e < xe) {
                const int k = xc.at(cb, e);
                if (k < X.col_lim) {
                    if (PMODE) {
                        const unsigned char f = X.mask[e];
                        if (f != 0 && Y.agg[k] >= 0) {
                            ys = Y.agg[k];
                            len = 1;
                            xv = (f == 2) ? 1.0 - omega : -omega * dfi * X.val[e];
                        }
                    } else {
                        ys = Y.rowptr[k];
                        len = Y.rowptr[k + 1] - ys;
                        xv = X.val[e];
                    }
                }
            }
            int incl = len;
#pragma unroll
            for (int off = 1; off < G; off <<= 1) {
                const int t = __shfl_up(incl, off, G);
                if (l >= off) incl += t;
            }
            const int total = __shfl(incl, G - 1, G);
            const int o = np + incl - len;
            if (PMODE) {
                if (len && o < CAP) {
                    pk[o] = ys;
                    pv[o] = xv;
                }
            } else {
                // the first U entries of the Y row loaded together (rows of P
                // hold ~2.5, of A P ~5: one memory latency instead of one per entry)
                constexpr int U = CAP >= 128 ? 8 : 4;
                int yc[U];
                double yv[U];
#pragma unroll
                for (int q = 0; q < U; ++q)
                    if (q < len) {
                        yc[q] = Y.col[ys + q];
                        yv[q] = Y.val[ys + q];
                    }
#pragma unroll
                for (int q = 0; q < U; ++q)
                    if (q < len && o + q < CAP) {
                        pk[o + q] = yc[q];
                        pv[o + q] = xv * yv[q];
                    }
                for (int q = U; q < len && o + q < CAP; ++q) {
                    pk[o + q] = Y.col[ys + q];
                    pv[o + q] = xv * Y.val[ys + q];
                }
            }
            np += total;
        }
        // a capacity taken from another problem (need != null): some row must
        // need more than half of it, else a measurement would have taken a
        // smaller class (whose sort order -- and so whose bits -- differ)
        if (need && np > CAP / 2 && l == 0 && *(volatile int *)need == 0) *need = 1;
        // more products than slots (a capacity taken from an earlier setup):
        // the row is garbage, the host redoes the product with a measured capacity
        if (np > CAP) {
            if (l == 0) *ovf = 1;
            np = CAP;
        }
    }
    wave_lds_sync();
    int key[S];
    double val[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int v = l * S + s;
        key[s] = v < np ? pk[v] : INT_MAX;
        val[s] = v < np ? pv[v] : 0.0;
    }
    // bitonic sort of the CAP slots (slot v = l * S + s) by key
#pragma unroll
    for (int k = 2; k <= CAP; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j < S) {
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    const int t = s ^ j;
                    if (t > s) {
                        const bool up = ((l * S + s) & k) == 0;
                        if ((key[s] > key[t]) == up && key[s] != key[t]) {
                            const int tk = key[s];
                            key[s] = key[t];
                            key[t] = tk;
                            const double tv = val[s];
                            val[s] = val[t];
                            val[t] = tv;
                        }
                    }
                }
            } else {
                const int lm = j / S;
                const bool lower = (l & lm) == 0;
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    const int ok = __shfl_xor(key[s], lm, G);
                    const double ov = __shfl_xor(val[s], lm, G);
                    const bool up = ((l * S + s) & k) == 0;
                    // the lower slot of an ascending pair keeps the smaller key
                    const bool take = (lower == up) ? (ok < key[s]) : (ok > key[s]);
                    if (take) {
                        key[s] = ok;
                        val[s] = ov;
                    }
                }
            }
        }
    }
    // segmented inclusive scan: head = first slot of a column
    const int prev_last = __shfl_up(key[S - 1], 1, G);
    int head[S], nh = 0;
    double run[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int pk_ = s > 0 ? key[s - 1] : (l > 0 ? prev_last : -1);
        head[s] = (key[s] != INT_MAX && key[s] != pk_) ? 1 : 0;
        run[s] = (s > 0 && !head[s]) ? run[s - 1] + val[s] : val[s];
        nh += head[s];
    }
    // carry from earlier lanes into this lane's leading (headless) slots
    int seg_open = 1;   // no head in this lane yet: the lane continues the previous segment
#pragma unroll
    for (int s = 0; s < S; ++s) seg_open &= !head[s];
    double carry = run[S - 1];   // this lane's trailing partial
    int hpre = nh;
    int open = seg_open;
#pragma unroll
    for (int off = 1; off < G; off <<= 1) {
        const double oc = __shfl_up(carry, off, G);
        const int oo = __shfl_up(open, off, G);
        const int oh = __shfl_up(hpre, off, G);
        if (l >= off) {
            if (open) carry = oc + carry;
            open = open && oo;
            hpre += oh;
        }
    }
    // carry / head count of the lanes before this one
    double cin = __shfl_up(carry, 1, G);
    int hin = __shfl_up(hpre, 1, G);
    if (l == 0) {
        cin = 0.0;
        hin = 0;
    }
    const int cnt = __shfl(hpre, G - 1, G);
    if (!live) return;
    int h = hin;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        bool lead = true;   // slots before this lane's first head continue the incoming segment
#pragma unroll
        for (int q = 0; q <= s; ++q) lead = lead && !head[q];
        const double tot = lead ? cin + run[s] : run[s];
        h += head[s];
        const int nk = s + 1 < S ? key[s + 1] : __shfl_down(key[0], 1, G);
        const bool tail = key[s] != INT_MAX && (nk != key[s] || (s + 1 == S && l == G - 1));
        if (tail) {
            pcol[(size_t)row * CAP + h - 1] = key[s];
            pval[(size_t)row * CAP + h - 1] = tot;
        }
    }
    if (l == 0) cnt_out[row] = cnt;
}

// padded rows (row * cap) -> CSR; 16 lanes per row, so a row's reads and
// writes are contiguous runs
// nnz_out (optional): the product's length, for a deferred host read;
// L lanes per row (a quarter of the slot capacity: the rows hold about that many)
template <int L>
__global__ void k_spgemm_compact(int nrows, int cap, const int *__restrict__ crow, const int *__restrict__ pcol,
                                 const double *__restrict__ pval, int *__restrict__ ccol, double *__restrict__ cval,
                                 int *nnz_out)
{
    const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (t == 0 && nnz_out) *nnz_out = crow[nrows];
    const int row = (int)(t / L), l = (int)(t % L);
    if (row >= nrows) return;
    const int b = crow[row], n = crow[row + 1] - b;
    for (int m = l; m < n; m += L) {
        ccol[b + m] = pcol[(size_t)row * cap + m];
        cval[b + m] = pval[(size_t)row * cap + m];
    }
}

// --------------------------------------------------------------------------
// setup: coarsest level, dense inverse
// --------------------------------------------------------------------------

// The coarsest level (<= kAmgDenseMax rows) becomes a dense matrix padded to
// a multiple of kBj with an identity tail (ld = padded size), inverted in
// place by blocked Gauss-Jordan without pivoting (the level operators are
// symmetric positive semi-definite).  Step k of kBj-wide block columns
// (k_bgj_step, one launch):
//     D  = inv(M_kk)                      k_bgj_diag for k = 0, else workgroup 0
//                                         of step k-1 (once its tile is final)
//     M_kj = D M_kj          (j != k),    M_kk = D
//     M_ij -= M_ik (D M_kj)  (i, j != k)
//     M_ik = -M_ik D         (i != k)     (old values of row k / column k)
// The matrix is first scaled symmetrically to unit diagonal and the inverse
// unscaled at the end.  A pivot below 1e-11 of the (unit) scaled diagonal
// marks a null direction -- roundoff leaves the exact null pivot of a
// pure-Neumann operator near 1e-13 (tools/lab/gj_emul.py) -- and its row and
// column are zeroed (generalised inverse on the range).
constexpr int kBj = 64;

// the matrix has been zeroed (hipMemsetAsync); entries of row i, identity tail
// symmetric diagonal scaling sc_q = 1 / sqrt(a_qq) (1 for a zero diagonal
// and the padding rows): the scaled matrix has unit diagonal, so every
// Gauss-Jordan pivot (a Schur-complement diagonal) lies in (0, 1].
// perm / iperm (nested-dissection order, nullptr: identity): dense index of
// coarse row r is perm[r]; iperm[q] the coarse row of dense index q (-1: padding)
// kDsG lanes per dense row (consecutive entries on consecutive lanes): the
// row's column, permutation and scale loads of 16 entries in flight at once
// instead of one dependent chain per row (one thread per row took 11 + 26 us
// for the 1.6k-row coarsest level of configs[2]).  The coarse operator's rows
// hold distinct columns (SpGEMM output), so every entry is written once:
// 0 + v, the value the former accumulation into the zeroed matrix produced.
constexpr int kDsG = 16;
__global__ void k_dense_dscale(int n, int ld, const int *__restrict__ rowptr, const int *__restrict__ col,
                               const double *__restrict__ val, const int *__restrict__ iperm, double *__restrict__ sc)
{
    const int q = (blockIdx.x * blockDim.x + threadIdx.x) / kDsG, l = threadIdx.x % kDsG;
    if (q >= ld) return;   // (whole groups: ld * kDsG threads exactly cover the rows)
    const int i = iperm ? iperm[q] : (q < n ? q : -1);
    int kd = -1;
    if (i >= 0)
        for (int k = rowptr[i] + l; k < rowptr[i + 1]; k += kDsG)
            if (col[k] == i) kd = k;
#pragma unroll
    for (int off = 1; off < kDsG; off <<= 1) kd = max(kd, __shfl_xor(kd, off, kDsG));
    if (l != 0) return;
    const double d = kd >= 0 ? 0.0 + val[kd] : 0.0;
    sc[q] = d > 0.0 ? 1.0 / sqrt(d) : 1.0;
}
__global__ void k_dense_scatter(int n, int ld, const int *__restrict__ rowptr, const int *__restrict__ col,
                                const double *__restrict__ val, const int *__restrict__ perm,
                                const int *__restrict__ iperm, const double *__restrict__ sc, double *__restrict__ M)
{
    const int q = (blockIdx.x * blockDim.x + threadIdx.x) / kDsG, l = threadIdx.x % kDsG;
    if (q >= ld) return;
    const int i = iperm ? iperm[q] : (q < n ? q : -1);
    if (i < 0) {
        if (l == 0) M[(size_t)q * ld + q] = 1.0;
        return;
    }
    const double sq = sc[q];
    for (int k = rowptr[i] + l; k < rowptr[i + 1]; k += kDsG) {
        const int cj = col[k];
        if (cj >= n) continue;
        const int c = perm ? perm[cj] : cj;
        M[(size_t)q * ld + c] = 0.0 + val[k] * sq * sc[c];
    }
}

// The coarsest inverse the V-cycle applies, unpermuted: M is the inverse of
// the unit-diagonal scaled level (S A_c S)^-1, so A_c^-1 = S M S; the apply
// keeps S in f64 (osc, original order) and stores M symmetrised -- entries
// (i, j) and (j, i) both from the one value (M_qr + M_rq) / 2, rounded once --
// in f32 (V = float, the default: half the bytes of the per-iteration coarse
// solve) or f64.  Rounding the scaled, symmetrised inverse keeps the coarse
// correction exactly symmetric; the f32 perturbation is relative to the entries
// of a unit-diagonal matrix's inverse (not of A_c^-1 itself, whose entries span
// the coefficient contrast).  One 64 x 64 output tile per block, its mirror
// tile read through LDS.
template <class V>
__global__ void __launch_bounds__(256) k_dense_unperm(int n, int ld, int ldo, const double *__restrict__ M,
                                                      const double *__restrict__ sc, const int *__restrict__ iperm,
                                                      V *__restrict__ out, double *__restrict__ osc)
{
    __shared__ double t[64][65];
    const int bq = blockIdx.y * 64, br = blockIdx.x * 64;
    for (int k = threadIdx.x; k < 64 * 64; k += 256) {   // t[a][b] = M[br + b][bq + a]
        const int a = k & 63, b = k >> 6;
        t[a][b] = M[(size_t)(br + b) * ld + bq + a];
    }
    __syncthreads();
    for (int k = threadIdx.x; k < 64 * 64; k += 256) {
        const int a = k >> 6, b = k & 63, q = bq + a, r = br + b;
        const int i = iperm ? iperm[q] : (q < n ? q : -1), j = iperm ? iperm[r] : (r < n ? r : -1);
        if (i >= 0 && j >= 0) out[(size_t)i * ldo + j] = (V)(0.5 * (M[(size_t)q * ld + r] + t[a][b]));
    }
    if (blockIdx.x == 0)
        for (int a = threadIdx.x; a < 64; a += 256) {
            const int q = bq + a, i = iperm ? iperm[q] : (q < n ? q : -1);
            if (i >= 0) osc[i] = sc[q];
        }
}

__global__ void __launch_bounds__(1024) k_dense_maxdiag(int n, int ld, const double *__restrict__ M,
                                                        double *__restrict__ maxd)
{
    __shared__ double red[16];
    double m = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) m = fmax(m, fabs(M[(size_t)i * ld + i]));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) m = fmax(m, red[w]);
        *maxd = m;
    }
}

// D = inv(M_kk) by in-place Gauss-Jordan: 256 threads, thread t keeps the 16
// entries (rows 16 (t >> 6) + m, column t & 63) in registers for the whole
// inversion.  Pivots are taken four at a time: with P = {p0 .. p0+3},
// Dinv = inv(A_PP) (every thread inverts the 4 x 4 block in registers) and
//     c_i = A_iP,  r_j = Dinv A_Pj (j not in P),  r_j = e_t + Dinv[:, t] (j = p0 + t),
// one uniform rank-4 update a_ij -= c_i . r_j followed by a_sj += r_j[s] on
// the rows of P leaves Dinv A_Pj in rows P, -A_iP Dinv in columns P and Dinv
// in the pivot block; the scaled pivots lie in (0, 1], so no step cancels
// more than a few bits.  A pivot block with a vanishing pivot is eliminated
// by four scalar steps instead, which zero the row and column of a null
// direction.  Rows P and columns P go through LDS, double-buffered: one
// barrier per step.
__device__ __forceinline__ void gj_scalar_step(int p, double (&a)[16], double thr, double *slab, double *colk)
{
    const int j = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (w == (p >> 4))   // the wave holding row p publishes its slab
#pragma unroll
        for (int m = 0; m < 16; ++m) slab[m * kBj + j] = a[m];
    if (j == p)
#pragma unroll
        for (int m = 0; m < 16; ++m) colk[16 * w + m] = a[m];
    __syncthreads();
    const double *rowp = slab + (p & 15) * kBj;
    const double piv = rowp[p];
    if (!(fabs(piv) > thr)) {   // null direction: zero row p and column p
#pragma unroll
        for (int m = 0; m < 16; ++m)
            if (16 * w + m == p || j == p) a[m] = 0.0;
        return;
    }
    const double ip = 1.0 / piv;
    const double r = j == p ? 1.0 + ip : rowp[j] * ip;
#pragma unroll
    for (int m = 0; m < 16; ++m) a[m] -= (colk[16 * w + m] - (16 * w + m == p ? 1.0 : 0.0)) * r;
}

// lds: 2 * 16 * kBj + 2 * 4 * kBj doubles (16-byte aligned): the double-
// buffered 16-row slab holding P ([m][j]) and columns P ([i][t])
constexpr int kBjDiagLds = 2 * 16 * kBj + 2 * 4 * kBj;
__device__ __forceinline__ void bgj_diag_inv(double (&a)[16], double thr, double *lds)
{
    const int tid = threadIdx.x;
    const int j = tid & 63, w = tid >> 6;
    // (buffer pointers by arithmetic on lds: a runtime-indexed pointer array
    // would hide the LDS address space and turn every access into a flat op)
    int phase = 0;
    for (int p0 = 0; p0 < kBj; p0 += 4) {
        const int buf = phase & 1;
        const int mb = p0 & 15, wp = p0 >> 4;
        double *R4 = lds + buf * 16 * kBj, *C4 = lds + 32 * kBj + buf * 4 * kBj;
        if (w == wp)   // this wave holds rows P: publish its whole slab (no dynamic register index)
#pragma unroll
            for (int m = 0; m < 16; ++m) R4[m * kBj + j] = a[m];
        R4 += mb * kBj;   // rows P = slab rows mb .. mb+3
        if (j >= p0 && j < p0 + 4)   // these lanes hold columns P
#pragma unroll
            for (int m = 0; m < 16; ++m) C4[(16 * w + m) * 4 + (j - p0)] = a[m];
        __syncthreads();
        ++phase;
        // Dinv = inv(A_PP), in-place Gauss-Jordan in registers
        double Dv[4][4];
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
            for (int t = 0; t < 4; ++t) Dv[s2][t] = R4[s2 * kBj + p0 + t];
        bool ok = true;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const double piv = Dv[q][q];
            ok = ok && (fabs(piv) > thr);
            const double ip = 1.0 / piv;
            Dv[q][q] = 1.0;
#pragma unroll
            for (int t = 0; t < 4; ++t) Dv[q][t] *= ip;
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                if (s2 == q) continue;
                const double f = Dv[s2][q];
                Dv[s2][q] = 0.0;
#pragma unroll
                for (int t = 0; t < 4; ++t) Dv[s2][t] -= f * Dv[q][t];
            }
        }
        if (!ok) {   // a (near) null direction inside the block: scalar steps
            for (int p = p0; p < p0 + 4; ++p) {
                const int b2 = phase & 1;
                gj_scalar_step(p, a, thr, lds + b2 * 16 * kBj, lds + 32 * kBj + b2 * 4 * kBj);
                ++phase;
            }
            continue;
        }
        double r[4];
        if (j >= p0 && j < p0 + 4) {
            const int t = j - p0;
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                double d = Dv[s2][0];
#pragma unroll
                for (int tt = 1; tt < 4; ++tt)
                    if (tt == t) d = Dv[s2][tt];
                r[s2] = (s2 == t ? 1.0 : 0.0) + d;
            }
        } else {
            const double x0 = R4[j], x1 = R4[kBj + j], x2 = R4[2 * kBj + j], x3 = R4[3 * kBj + j];
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) r[s2] = Dv[s2][0] * x0 + Dv[s2][1] * x1 + Dv[s2][2] * x2 + Dv[s2][3] * x3;
        }
        const double4 *cr = reinterpret_cast<const double4 *>(&C4[16 * w * 4]);
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const double4 c = cr[m];
            a[m] -= c.x * r[0] + c.y * r[1] + c.z * r[2] + c.w * r[3];
        }
        if (w == wp)
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                const int s2 = m - mb;
                a[m] += (s2 == 0 ? r[0] : 0.0) + (s2 == 1 ? r[1] : 0.0) + (s2 == 2 ? r[2] : 0.0) +
                        (s2 == 3 ? r[3] : 0.0);
            }
    }
}

__global__ void __launch_bounds__(256) k_bgj_diag(int k, int ld, const double *__restrict__ M,
                                                  const double *__restrict__ maxd, double *__restrict__ D)
{
    __shared__ __attribute__((aligned(16))) double lds[kBjDiagLds];
    const int j = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t base = (size_t)k * kBj * ld + (size_t)k * kBj;
    double a[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) a[m] = M[base + (size_t)(16 * w + m) * ld + j];
    bgj_diag_inv(a, 1e-11 * (*maxd), lds);
#pragma unroll
    for (int m = 0; m < 16; ++m) D[(16 * w + m) * kBj + j] = a[m];
}

// C = X Y for 64 x 64 blocks staged in LDS on the f64 matrix cores: 4 waves,
// wave w computes the 32 x 32 quadrant (w >> 1, w & 1) as 2 x 2 tiles of
// v_mfma_f64_16x16x4_f64 (A[l & 15][k = l >> 4], B[k = l >> 4][l & 15];
// C/D col = l & 15, row = (l >> 4) + 4 r).  c[ti][tj][r] is element
// (32 (w >> 1) + 16 ti + (l >> 4) + 4 r, 32 (w & 1) + 16 tj + (l & 15)).
// LDS row strides (doubles) that make the operand reads conflict-free: a
// 32-lane half reads 16 rows x 2 k of X (stride 66 -> banks 4 li + 2 lk) and
// 2 k-rows x 16 columns of Y (stride 80 -> the two rows 32 banks apart).
typedef double dbl4 __attribute__((ext_vector_type(4)));
constexpr int kXs = 66, kYs = 80;

template <bool ZERO = true>
__device__ __forceinline__ void bgj_mm(const double *__restrict__ Xs, const double *__restrict__ Ys, dbl4 (&c)[2][2])
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = 32 * (w >> 1), c0 = 32 * (w & 1);
    const int li = lane & 15, lk = lane >> 4;
    if (ZERO)
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj) c[ti][tj] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
    for (int s = 0; s < kBj / 4; ++s) {
        double a[2], b[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            a[t] = Xs[(r0 + 16 * t + li) * kXs + 4 * s + lk];
            b[t] = Ys[(4 * s + lk) * kYs + c0 + 16 * t + li];
        }
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj)
                c[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ti], b[tj], c[ti][tj], 0, 0, 0);
    }
}

// (row, col) of element r of tile (ti, tj) of this thread
__device__ __forceinline__ int bgj_row(int ti, int r) { return 32 * ((threadIdx.x >> 6) >> 1) + 16 * ti + ((threadIdx.x & 63) >> 4) + 4 * r; }
__device__ __forceinline__ int bgj_col(int tj) { return 32 * ((threadIdx.x >> 6) & 1) + 16 * tj + (threadIdx.x & 15); }

// inv(A) of a 64 x 64 block held in bgj_mm's accumulator layout
// (c[ti][tj][r] = element (bgj_row(ti, r), bgj_col(tj))), in place: 16
// rank-4 Gauss-Jordan steps whose updates run on the f64 matrix cores.  Step
// s publishes rows and columns P = 4s .. 4s+3 to LDS; every lane forms
// D = inv(A_PP) in registers and its B operand r = D A_Pj (r = I + D on the
// pivot columns); then c -= A_iP r on the MFMA, and rows P += r -- the update
// of bgj_diag_inv without its 64 FMAs and 32 LDS reads per lane and step.
// A (near) null pivot (|piv| <= thr) zeroes its row and column, as there.
// lds: kBjInvLds doubles (two buffers of a 4 x 64 row slab and a 64 x 4 column slab).
constexpr int kBjInvLds = 2 * 8 * kBj;
static_assert(kBjInvLds <= kBjDiagLds && kBjInvLds <= kBj * kYs, "bgj_inv_mfma's LDS exceeds its callers' buffers");
__device__ __forceinline__ void bgj_inv_mfma(dbl4 (&c)[2][2], double thr, double *lds)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int R0 = 32 * (w >> 1), C0 = 32 * (w & 1);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const int p0 = 4 * s;
        const int tp = (p0 >> 4) & 1, rp = (p0 & 15) >> 2;   // tile / element index of rows (columns) P
        double *RS = lds + (s & 1) * 8 * kBj;   // RS[t][j] = A(p0 + t, j)
        double *CS = RS + 4 * kBj;              // CS[i][t] = A(i, p0 + t)
        const bool rowhold = (w >> 1) == (p0 >> 5);
        if (rowhold)   // this lane holds row p0 + lk
#pragma unroll
            for (int tj = 0; tj < 2; ++tj) RS[lk * kBj + C0 + 16 * tj + li] = c[tp][tj][rp];
        if ((w & 1) == (p0 >> 5) && li >= (p0 & 15) && li < (p0 & 15) + 4)   // ... column p0 + li - (p0 & 15)
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                for (int r = 0; r < 4; ++r) CS[(R0 + 16 * ti + lk + 4 * r) * 4 + li - (p0 & 15)] = c[ti][tp][r];
        __syncthreads();
        double W[4][4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int t = 0; t < 4; ++t) W[q][t] = RS[q * kBj + p0 + t];
        // a null pivot takes ip = 0: its row of D becomes 0 and the
        // elimination leaves the other rows alone, i.e. D is the inverse on
        // the other directions; the update then zeroes column p0 + q of the
        // block by itself (r = e_q there), and row p0 + q is zeroed below
        unsigned nul = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const double piv = W[q][q];
            const bool ok = fabs(piv) > thr;
            nul |= ok ? 0u : 1u << q;
            double ip = __builtin_amdgcn_rcp(piv);   // 1 / piv: v_rcp_f64 + two Newton steps
            ip = fma(fma(-piv, ip, 1.0), ip, ip);
            ip = fma(fma(-piv, ip, 1.0), ip, ip);
            ip = ok ? ip : 0.0;
            W[q][q] = 1.0;
#pragma unroll
            for (int t = 0; t < 4; ++t) W[q][t] *= ip;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                if (t == q) continue;
                const double f = W[t][q];
                W[t][q] = 0.0;
#pragma unroll
                for (int u = 0; u < 4; ++u) W[t][u] -= f * W[q][u];
            }
        }
        // row lk of D: this lane's B operand row
        double Dk[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) Dk[t] = lk == 0 ? W[0][t] : lk == 1 ? W[1][t] : lk == 2 ? W[2][t] : W[3][t];
        double bop[2], aop[2];
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) {
            const int jj = C0 + 16 * tj + li, tc = jj - p0;
            if (tc >= 0 && tc < 4) {
                const double d = tc == 0 ? Dk[0] : tc == 1 ? Dk[1] : tc == 2 ? Dk[2] : Dk[3];
                bop[tj] = (lk == tc ? 1.0 : 0.0) + d;
            } else {
                bop[tj] = Dk[0] * RS[jj] + Dk[1] * RS[kBj + jj] + Dk[2] * RS[2 * kBj + jj] + Dk[3] * RS[3 * kBj + jj];
            }
        }
#pragma unroll
        for (int ti = 0; ti < 2; ++ti) aop[ti] = -CS[(R0 + 16 * ti + li) * 4 + lk];
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj) c[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(aop[ti], bop[tj], c[ti][tj], 0, 0, 0);
        if (rowhold) {
            const bool zr = (nul >> lk) & 1u;   // row p0 + lk of a null pivot
#pragma unroll
            for (int tj = 0; tj < 2; ++tj) c[tp][tj][rp] = zr ? 0.0 : c[tp][tj][rp] + bop[tj];
        }
    }
}

// XFK_BGJ_INV=0: the pivot-block inverse by bgj_diag_inv (FMA updates)
static int bgj_inv_mode()
{
    static const int v = [] {
        const char *e = std::getenv("XFK_BGJ_INV");
        return e ? std::atoi(e) : 1;
    }();
    return v;
}

template <int S>
__device__ __forceinline__ void bgj_load(double *__restrict__ dst, const double *__restrict__ src, size_t ld)
{
    // 2048 double2 per tile, 8 per thread, all issued before the first use
    double2 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int e = threadIdx.x + 256 * q, r = e >> 5, c = 2 * (e & 31);
        v[q] = *reinterpret_cast<const double2 *>(src + (size_t)r * ld + c);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int e = threadIdx.x + 256 * q, r = e >> 5, c = 2 * (e & 31);
        dst[r * S + c] = v[q].x;
        dst[r * S + c + 1] = v[q].y;
    }
}

// One launch per block step k.
// Step k reads only snapshots written by step k-1 (or the prologue), so every
// tile is finalised in the same launch with no ordering between workgroups:
//     D    = inv(M_kk)                               Dk
//     R[j] = M_kj after step k-1 (row k, unscaled)    Rk + j T2
//     C[i] = M_ik after step k-1 (column k)           Ck + i T2
// tile (i, j):  i == k:  M_kj = D R[j]          (j == k: M_kk = D)
//               j == k:  M_ik = -C[i] D
//               else:    M_ij -= C[i] (D R[j])  (T_kj = D R[j] recomputed per
//                                                tile: no row launch, no wait)
// Row k+1 of the result goes to Rn, column k+1 to Cn; workgroup 0 takes tile
// (k+1, k+1) -- the next pivot block -- and inverts it into Dn once written.
// The chain per step is one launch: the pivot workgroup's two tile GEMMs and
// the 64 x 64 inversion.
// snapshots of row k (R[j] = M_kj) and column k (C[i] = M_ik) before step k
__global__ void __launch_bounds__(256) k_bgj_snap(int k, int nbk, int ld, const double *__restrict__ M,
                                                  double *__restrict__ R, double *__restrict__ C)
{
    const int t = blockIdx.x % nbk;
    const bool row = blockIdx.x < nbk;
    const double *src = row ? M + (size_t)k * kBj * ld + (size_t)t * kBj : M + (size_t)t * kBj * ld + (size_t)k * kBj;
    double *dst = (row ? R : C) + (size_t)t * kBj * kBj;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int e = threadIdx.x + 256 * q, r = e >> 5, c = 2 * (e & 31);
        *reinterpret_cast<double2 *>(dst + r * kBj + c) = *reinterpret_cast<const double2 *>(src + (size_t)r * ld + c);
    }
}

__global__ void __launch_bounds__(256) k_bgj_step(int k, int nbk, int ld, double *__restrict__ M,
                                                  const double *__restrict__ Dk, const double *__restrict__ Rk,
                                                  const double *__restrict__ Ck, double *__restrict__ Dn,
                                                  double *__restrict__ Rn, double *__restrict__ Cn,
                                                  const double *__restrict__ maxd, int inv_mode)
{
    const int nt = nbk * nbk, kn = k + 1 < nbk ? k + 1 : 0;
    const int b = (int)((blockIdx.x + (unsigned)(kn * nbk + kn)) % (unsigned)nt);
    const int i = b / nbk, j = b % nbk;
    const bool piv = k + 1 < nbk && blockIdx.x == 0;
    const size_t T2 = (size_t)kBj * kBj;
    __shared__ __attribute__((aligned(16))) double Xs[kBj * kXs];
    __shared__ __attribute__((aligned(16))) double Ys[kBj * kYs];
    double *Mij = M + (size_t)i * kBj * ld + (size_t)j * kBj;
    if (i == k && j == k) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = threadIdx.x + 256 * q, r = e >> 5, c = 2 * (e & 31);
            *reinterpret_cast<double2 *>(Mij + (size_t)r * ld + c) = *reinterpret_cast<const double2 *>(Dk + r * kBj + c);
        }
        return;
    }
    dbl4 c[2][2];
    double sgn = 1.0;
    bool rmw = false;
    if (i == k) {   // T = D R[j]
        bgj_load<kXs>(Xs, Dk, kBj);
        bgj_load<kYs>(Ys, Rk + j * T2, kBj);
        __syncthreads();
        bgj_mm(Xs, Ys, c);
    } else if (j == k) {   // -C[i] D
        bgj_load<kXs>(Xs, Ck + i * T2, kBj);
        bgj_load<kYs>(Ys, Dk, kBj);
        __syncthreads();
        bgj_mm(Xs, Ys, c);
        sgn = -1.0;
    } else {   // M_ij - C[i] (D R[j])
        double2 pre[8];   // C[i], in flight during the first product
        const double *Ci = Ck + i * T2;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = threadIdx.x + 256 * q, r = e >> 5, cc = 2 * (e & 31);
            pre[q] = *reinterpret_cast<const double2 *>(Ci + r * kBj + cc);
        }
        bgj_load<kXs>(Xs, Dk, kBj);
        bgj_load<kYs>(Ys, Rk + j * T2, kBj);
        __syncthreads();
        bgj_mm(Xs, Ys, c);
        __syncthreads();
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj)
#pragma unroll
                for (int r = 0; r < 4; ++r) Ys[bgj_row(ti, r) * kYs + bgj_col(tj)] = c[ti][tj][r];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = threadIdx.x + 256 * q, r = e >> 5, cc = 2 * (e & 31);
            Xs[r * kXs + cc] = pre[q].x;
            Xs[r * kXs + cc + 1] = pre[q].y;
        }
        __syncthreads();
        bgj_mm(Xs, Ys, c);
        sgn = -1.0;
        rmw = true;
    }
    double *rn = (i == k + 1) ? Rn + j * T2 : nullptr;
    double *cn = (j == k + 1) ? Cn + i * T2 : nullptr;
    const bool fast = piv && inv_mode != 0;
    if (piv) __syncthreads();   // Xs / Ys are reused below
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = bgj_row(ti, r), col = bgj_col(tj);
                double *e = &Mij[(size_t)row * ld + col];
                const double v = rmw ? *e - c[ti][tj][r] : sgn * c[ti][tj][r];
                *e = v;
                if (rn) rn[row * kBj + col] = v;
                if (cn) cn[row * kBj + col] = v;
                if (fast) c[ti][tj][r] = v;
                else if (piv) Xs[row * kBj + col] = v;
            }
    if (!piv) return;
    if (fast) {
        bgj_inv_mfma(c, 1e-11 * (*maxd), Ys);
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj)
#pragma unroll
                for (int r = 0; r < 4; ++r) Dn[bgj_row(ti, r) * kBj + bgj_col(tj)] = c[ti][tj][r];
        return;
    }
    __syncthreads();
    const int jl = threadIdx.x & 63, w = threadIdx.x >> 6;
    double a[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) a[m] = Xs[(16 * w + m) * kBj + jl];
    bgj_diag_inv(a, 1e-11 * (*maxd), Ys);
#pragma unroll
    for (int m = 0; m < 16; ++m) Dn[(16 * w + m) * kBj + jl] = a[m];
}

// Nested-dissection steps.  The coarsest operator is reordered by a
// recursive bisection: leaves (parts that share no entry), then their
// separators, the top separator last.  Gauss-Jordan keeps distinct leaves
// decoupled: eliminating a block column of a leaf touches only the tiles of
// its region -- the leaf plus its ancestor separators -- and the updates of
// different leaves commute.  So the leaves' block columns are eliminated side
// by side, one pivot chain per leaf in each launch (up to four), then the
// separators of the next tree level the same way (region: their subtree plus
// ancestors), the top separator last.  Each tile applies the update of every
// chain whose region holds it (separator tiles: several, summed on the MFMA
// in chain order); per block, bit c of `mask` marks chain c's region.
constexpr int kNdChains = 8;
struct BgjStep {
    int n;                                             // chains of this step
    int k[kNdChains];                                  // their pivot blocks
    const double *D[kNdChains], *R[kNdChains], *C[kNdChains];   // inv(M_kk), row / column snapshots
    int nn;                                            // distinct next pivot blocks
    int nx[kNdChains];
    double *Dn[kNdChains], *Rn[kNdChains], *Cn[kNdChains];
};

// (chain fields are selected by unrolled comparisons: a dynamically indexed
// by-value kernel argument would be placed in scratch memory)
__global__ void __launch_bounds__(256, 2) k_bgj_multi(int nbk, int ld, double *__restrict__ M, BgjStep st,
                                                      const unsigned char *__restrict__ mask,
                                                      const int *__restrict__ tiles, const double *maxd, int inv_mode)
{
    const size_t T2 = (size_t)kBj * kBj;
    int i, j;
    double *Dpiv = nullptr;
    if ((int)blockIdx.x < st.nn) {   // workgroups 0 .. nn-1 finalise and invert the next pivot blocks
#pragma unroll
        for (int t = 0; t < kNdChains; ++t)
            if (t == (int)blockIdx.x) {
                i = j = st.nx[t];
                Dpiv = st.Dn[t];
            }
    } else {
        const int t = tiles[blockIdx.x - st.nn];
        i = t / nbk;
        j = t % nbk;
        if (i == j)
#pragma unroll
            for (int u = 0; u < kNdChains; ++u)
                if (u < st.nn && st.nx[u] == i) return;   // taken by a pivot workgroup
    }
    const unsigned act = (unsigned)mask[i] & (unsigned)mask[j];
    int pc = -1;
    const double *pD = nullptr, *pR = nullptr, *pC = nullptr;
    int pk = -1;
#pragma unroll
    for (int c = 0; c < kNdChains; ++c)
        if (c < st.n && ((act >> c) & 1u) && (i == st.k[c] || j == st.k[c])) {
            pc = c;
            pk = st.k[c];
            pD = st.D[c];
            pR = st.R[c];
            pC = st.C[c];
        }
    __shared__ __attribute__((aligned(16))) double Xs[kBj * kXs];
    __shared__ __attribute__((aligned(16))) double Ys[kBj * kYs];
    double *Mij = M + (size_t)i * kBj * ld + (size_t)j * kBj;
    if (pc >= 0 && i == pk && j == pk) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = threadIdx.x + 256 * q, r = e >> 5, c = 2 * (e & 31);
            *reinterpret_cast<double2 *>(Mij + (size_t)r * ld + c) = *reinterpret_cast<const double2 *>(pD + r * kBj + c);
        }
        return;
    }
    dbl4 acc[2][2];
    double sgn = 1.0;
    bool rmw = false;
    if (pc >= 0 && i == pk) {   // row of a pivot: D R[j]
        bgj_load<kXs>(Xs, pD, kBj);
        bgj_load<kYs>(Ys, pR + j * T2, kBj);
        __syncthreads();
        bgj_mm(Xs, Ys, acc);
    } else if (pc >= 0) {       // column of a pivot: -C[i] D
        bgj_load<kXs>(Xs, pC + i * T2, kBj);
        bgj_load<kYs>(Ys, pD, kBj);
        __syncthreads();
        bgj_mm(Xs, Ys, acc);
        sgn = -1.0;
    } else {                    // M_ij - sum over the chains holding the tile of C[i] (D R[j])
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj) acc[ti][tj] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int c = 0; c < kNdChains; ++c) {
            if (!(c < st.n && ((act >> c) & 1u))) continue;
            double2 pre[8];
            const double *Ci = st.C[c] + i * T2;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = threadIdx.x + 256 * u, r = e >> 5, cc = 2 * (e & 31);
                pre[u] = *reinterpret_cast<const double2 *>(Ci + r * kBj + cc);
            }
            __syncthreads();   // the LDS of the previous chain's product is free
            bgj_load<kXs>(Xs, st.D[c], kBj);
            bgj_load<kYs>(Ys, st.R[c] + j * T2, kBj);
            __syncthreads();
            dbl4 t[2][2];
            bgj_mm(Xs, Ys, t);
            __syncthreads();
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                for (int tj = 0; tj < 2; ++tj)
#pragma unroll
                    for (int r = 0; r < 4; ++r) Ys[bgj_row(ti, r) * kYs + bgj_col(tj)] = t[ti][tj][r];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = threadIdx.x + 256 * u, r = e >> 5, cc = 2 * (e & 31);
                Xs[r * kXs + cc] = pre[u].x;
                Xs[r * kXs + cc + 1] = pre[u].y;
            }
            __syncthreads();
            bgj_mm<false>(Xs, Ys, acc);
        }
        rmw = true;
    }
    // row / column snapshots of the next pivot blocks this tile belongs to
    double *rs[kNdChains], *cs[kNdChains];
#pragma unroll
    for (int t = 0; t < kNdChains; ++t) {
        rs[t] = (t < st.nn && i == st.nx[t]) ? st.Rn[t] + j * T2 : nullptr;
        cs[t] = (t < st.nn && j == st.nx[t]) ? st.Cn[t] + i * T2 : nullptr;
    }
    const bool fast = Dpiv && inv_mode != 0;
    if (Dpiv) __syncthreads();   // Xs / Ys are reused below
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = bgj_row(ti, r), col = bgj_col(tj);
                double *e = &Mij[(size_t)row * ld + col];
                const double v = rmw ? *e - acc[ti][tj][r] : sgn * acc[ti][tj][r];
                *e = v;
#pragma unroll
                for (int t = 0; t < kNdChains; ++t) {
                    if (rs[t]) rs[t][row * kBj + col] = v;
                    if (cs[t]) cs[t][row * kBj + col] = v;
                }
                if (fast) acc[ti][tj][r] = v;
                else if (Dpiv) Xs[row * kBj + col] = v;
            }
    if (!Dpiv) return;
    if (fast) {
        bgj_inv_mfma(acc, 1e-11 * (*maxd), Ys);
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj)
#pragma unroll
                for (int r = 0; r < 4; ++r) Dpiv[bgj_row(ti, r) * kBj + bgj_col(tj)] = acc[ti][tj][r];
        return;
    }
    __syncthreads();
    const int jl = threadIdx.x & 63, w = threadIdx.x >> 6;
    double a[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) a[m] = Xs[(16 * w + m) * kBj + jl];
    bgj_diag_inv(a, 1e-11 * (*maxd), Ys);
#pragma unroll
    for (int m = 0; m < 16; ++m) Dpiv[(16 * w + m) * kBj + jl] = a[m];
}

// first step of the first phase: pivot-block inverses (workgroups 0 .. n-1)
// and row / column snapshots of the chains' first pivot blocks
__global__ void __launch_bounds__(256) k_bgj_init(int nbk, int ld, const double *__restrict__ M, BgjStep st,
                                                  const double *__restrict__ maxd, int inv_mode)
{
    const int b = blockIdx.x;
    if (b < st.nn) {
        __shared__ __attribute__((aligned(16))) double lds[kBjDiagLds];
        int k = 0;
        double *D = nullptr;
#pragma unroll
        for (int t = 0; t < kNdChains; ++t)
            if (t == b) {
                k = st.nx[t];
                D = st.Dn[t];
            }
        const int jl = threadIdx.x & 63, w = threadIdx.x >> 6;
        const size_t base = (size_t)k * kBj * ld + (size_t)k * kBj;
        if (inv_mode != 0) {
            dbl4 c[2][2];
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                for (int tj = 0; tj < 2; ++tj)
#pragma unroll
                    for (int r = 0; r < 4; ++r) c[ti][tj][r] = M[base + (size_t)bgj_row(ti, r) * ld + bgj_col(tj)];
            bgj_inv_mfma(c, 1e-11 * (*maxd), lds);
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                for (int tj = 0; tj < 2; ++tj)
#pragma unroll
                    for (int r = 0; r < 4; ++r) D[bgj_row(ti, r) * kBj + bgj_col(tj)] = c[ti][tj][r];
            return;
        }
        double a[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) a[m] = M[base + (size_t)(16 * w + m) * ld + jl];
        bgj_diag_inv(a, 1e-11 * (*maxd), lds);
#pragma unroll
        for (int m = 0; m < 16; ++m) D[(16 * w + m) * kBj + jl] = a[m];
        return;
    }
    const int e0 = b - st.nn, ch = e0 / (2 * nbk), rem = e0 % (2 * nbk);
    const int t = rem % nbk;
    const bool row = rem < nbk;
    int k = 0;
    double *dst = nullptr;
#pragma unroll
    for (int u = 0; u < kNdChains; ++u)
        if (u == ch) {
            k = st.nx[u];
            dst = (row ? st.Rn[u] : st.Cn[u]) + (size_t)t * kBj * kBj;
        }
    const double *src = row ? M + (size_t)k * kBj * ld + (size_t)t * kBj : M + (size_t)t * kBj * ld + (size_t)k * kBj;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int e = threadIdx.x + 256 * q, r = e >> 5, c = 2 * (e & 31);
        *reinterpret_cast<double2 *>(dst + r * kBj + c) = *reinterpret_cast<const double2 *>(src + (size_t)r * ld + c);
    }
}

// --------------------------------------------------------------------------
// V-cycle kernels
// --------------------------------------------------------------------------

enum SmoothMode {
    kSweepFromZero = 0,   // x1 = w D^-1 b implicit, out = x1 + w D^-1 (b - A x1)
    kSweep = 1,           // out = x + w D^-1 (b - A x)
    kResid = 2,           // r = b - A x
    kResidFromZero = 3    // x1 = w D^-1 b (written to out), r = b - A x1
};

template <int MODE>
__device__ __forceinline__ void smooth_finish(int i, double ax, double w, const double *__restrict__ dinv,
                                              const double *__restrict__ b, const double *__restrict__ x,
                                              double *__restrict__ out, double *__restrict__ rout)
{
    constexpr bool implicit = (MODE == kSweepFromZero || MODE == kResidFromZero);
    const double bi = b[i], di = dinv[i];
    const double xi = implicit ? w * di * bi : x[i];
    const double res = bi - ax;
    if constexpr (MODE == kSweepFromZero || MODE == kSweep) out[i] = xi + w * di * res;
    if constexpr (MODE == kResid || MODE == kResidFromZero) rout[i] = res;
    if constexpr (MODE == kResidFromZero)
        if (out) out[i] = xi;   // (a folded level-0 post-step recomputes x_pre: not written)
}

// smooth_finish with the row's b, D^-1 and x already loaded; returns out[i]
template <int MODE>
__device__ __forceinline__ double smooth_finish_v(int i, double ax, double w, double di, double bi, double xv,
                                                  double *__restrict__ out, double *__restrict__ rout)
{
    constexpr bool implicit = (MODE == kSweepFromZero || MODE == kResidFromZero);
    const double xi = implicit ? w * di * bi : xv;
    const double res = bi - ax;
    double o = xi;
    if constexpr (MODE == kSweepFromZero || MODE == kSweep) {
        o = xi + w * di * res;
        out[i] = o;
    }
    if constexpr (MODE == kResid || MODE == kResidFromZero) rout[i] = res;
    if constexpr (MODE == kResidFromZero)
        if (out) out[i] = xi;   // (a folded level-0 post-step recomputes x_pre: not written)
    return o;
}

// CSR-stream tile SpMV (the PCG's kernel shape): B = 1024 on level 0, 256 on
// large coarse levels (more workgroups than CUs)
// part_gam (the PCG's last level-0 sweep only): per-tile partials of
// b . out, i.e. gamma = r . u of the CG, in the layout and summation order of
// k_cg_spmv's (same tiles, same workgroup sum), so the SpMV need not read r
template <int MODE, int B, int SLOTS = 2, class V = double>
__global__ void __launch_bounds__(B) k_amg_smooth(int n, int ncl, const int *__restrict__ rowptr,
                                                         const int *__restrict__ col, const V *__restrict__ val,
                                                         const double *__restrict__ dinv,
                                                         const unsigned long long *rho, const double *__restrict__ b,
                                                         const double *__restrict__ x, double *__restrict__ out,
                                                         double *__restrict__ rout, const int *done,
                                                         double *__restrict__ part_gam, const int *__restrict__ tl,
                                                         const unsigned short *__restrict__ c16 = nullptr,
                                                         const int *__restrict__ cbase = nullptr)
{
    // the convergence flag, rho, the tile's row range and this row's b,
    // D^-1, x are loaded together before the first branch
    const int dn = load_flag_v(done);
    __shared__ __attribute__((aligned(16))) double lds[4 * SLOTS * B];
    const double ra = rho_of(rho);
    const int t = tl ? tl[xcd_tile(blockIdx.x, gridDim.x)] : xcd_tile(blockIdx.x, gridDim.x);
    const int r0 = t * B;
    const int i = r0 + threadIdx.x;
    constexpr bool implicit = (MODE == kSweepFromZero || MODE == kResidFromZero);
    const TileRows tr = tile_rows<B>(r0, n, rowptr);
    const int cb = load_col_base(cbase, t);
    const double bi = i < n ? b[i] : 0.0, di = i < n ? dinv[i] : 0.0;
    const double xv = (!implicit && i < n) ? x[i] : 0.0;
    if (dn) return;
    const double w = ra > 0.0 ? 1.0 / ra : 0.0;
    double ax;
    if constexpr (implicit)
        ax = cg_tile_spmv16<B, SLOTS>(tr, c16, cb, col, val,
                                      [&](int j) { return j < ncl ? w * dinv[j] * b[j] : 0.0; }, lds);
    else
        ax = cg_tile_spmv16<B, SLOTS>(tr, c16, cb, col, val, [&](int j) { return j < ncl ? x[j] : 0.0; }, lds);
    double oi = 0.0;
    if (i < n) oi = smooth_finish_v<MODE>(i, ax, w, di, bi, xv, out, rout);
    if constexpr (MODE == kSweep) {
        if (part_gam) {   // uniform per launch
            __shared__ double red[2 * (B / 64)];
            double g = 0.0, zero = 0.0;
            if (i < n) g = bi * oi;
            cg_block_sum2(zero, g, red);
            if (threadIdx.x == 0) part_gam[t] = g;
        }
    }
}

// G lanes per row, strided over the row, butterfly sum inside the group
template <int G, class XF>
__device__ __forceinline__ double group_row_dot(int i, int n, const int *__restrict__ rowptr,
                                                const int *__restrict__ col, const double *__restrict__ val, XF X)
{
    const int g = threadIdx.x & (G - 1);
    double s = 0.0;
    if (i < n)
        for (int k = rowptr[i] + g; k < rowptr[i + 1]; k += G) s += val[k] * X(col[k]);
#pragma unroll
    for (int off = G >> 1; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    return s;
}

// coarse levels: G lanes per row
template <int MODE, int G>
__global__ void __launch_bounds__(256) k_amg_smooth_g(int n, int ncl, const int *__restrict__ rowptr,
                                                      const int *__restrict__ col, const double *__restrict__ val,
                                                      const double *__restrict__ dinv, const unsigned long long *rho,
                                                      const double *__restrict__ b, const double *__restrict__ x,
                                                      double *__restrict__ out, double *__restrict__ rout,
                                                      const int *done)
{
    if (done && *done) return;
    const double ra = rho_of(rho);
    const double w = ra > 0.0 ? 1.0 / ra : 0.0;
    const int i = (xcd_tile(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x) / G;
    constexpr bool implicit = (MODE == kSweepFromZero || MODE == kResidFromZero);
    double ax;
    if constexpr (implicit)
        ax = group_row_dot<G>(i, n, rowptr, col, val, [&](int j) { return j < ncl ? w * dinv[j] * b[j] : 0.0; });
    else
        ax = group_row_dot<G>(i, n, rowptr, col, val, [&](int j) { return j < ncl ? x[j] : 0.0; });
    if (i < n && (threadIdx.x & (G - 1)) == 0) smooth_finish<MODE>(i, ax, w, dinv, b, x, out, rout);
}

// y = M x (ACC: y += M x), tile form (large transfer operators)
template <int B, bool ACC, int SLOTS = 2, class V = double>
__global__ void __launch_bounds__(B) k_csr_mv_tile(int n, const int *__restrict__ rowptr, const int *__restrict__ col,
                                                   const V *__restrict__ val, const double *__restrict__ x,
                                                   double *__restrict__ y, const int *done,
                                                   const unsigned short *__restrict__ c16 = nullptr,
                                                   const int *__restrict__ cbase = nullptr)
{
    const int dn = load_flag_v(done);
    __shared__ __attribute__((aligned(16))) double lds[4 * SLOTS * B];
    const int t = xcd_tile(blockIdx.x, gridDim.x);
    const int r0 = t * B;
    const int i = r0 + threadIdx.x;
    const TileRows tr = tile_rows<B>(r0, n, rowptr);
    const int cb = load_col_base(cbase, t);
    const double y0 = (ACC && i < n) ? y[i] : 0.0;
    if (dn) return;
    const double s = cg_tile_spmv16<B, SLOTS>(tr, c16, cb, col, val, [&](int j) { return x[j]; }, lds);
    if (i < n) y[i] = ACC ? y0 + s : s;
}

// y = M x (ACC: y += M x), G lanes per row (restriction R r, prolongation x += P xc)
template <int G, bool ACC>
__global__ void __launch_bounds__(256) k_csr_mv_g(int n, const int *__restrict__ rowptr, const int *__restrict__ col,
                                                  const double *__restrict__ val, const double *__restrict__ x,
                                                  double *__restrict__ y, const int *done)
{
    if (done && *done) return;
    const int i = (xcd_tile(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x) / G;
    const double s = group_row_dot<G>(i, n, rowptr, col, val, [&](int j) { return x[j]; });
    if (i < n && (threadIdx.x & (G - 1)) == 0) y[i] = ACC ? y[i] + s : s;
}

// Folded coarse level (V(1,1) with one Jacobi sweep, x_pre = w D^-1 b):
//   pre   y  = x_pre + w D^-1 (b - A x_pre),  b_c = P~^T b
//   post  x  = y + P~ x_c,                     P~ = (I - w D^-1 A) P
// equal in exact arithmetic to sweep-from-0 + residual, R r, x += P x_c and
// the post-sweep (R r' = P^T (I - w A D^-1) b = P~^T b for symmetric A), in
// two launches instead of four.  P~ is formed over the pattern of A P (which
// holds P's, the diagonal of A being nonzero).
// kFoldLanes lanes per row of A P, each entry's P_ij found by a scan of the
// (short: 2-3 entries) P row
constexpr int kFoldLanes = 8;
__global__ void __launch_bounds__(256) k_fold_p(int n, const unsigned long long *rho, const double *__restrict__ dinv,
                                                const int *__restrict__ aprow, const int *__restrict__ apcol,
                                                const double *__restrict__ apval, const int *__restrict__ prow,
                                                const int *__restrict__ pcol, const double *__restrict__ pval,
                                                int *__restrict__ fcol, double *__restrict__ fval)
{
    const int i = (int)(((long long)blockIdx.x * blockDim.x + threadIdx.x) / kFoldLanes);
    if (i >= n) return;
    const int g = threadIdx.x & (kFoldLanes - 1);
    const double ra = rho_of(rho);
    const double wd = (ra > 0.0 ? 1.0 / ra : 0.0) * dinv[i];
    const int pb = prow[i], pe = prow[i + 1];
    for (int k = aprow[i] + g; k < aprow[i + 1]; k += kFoldLanes) {
        const int c = apcol[k];
        double pij = 0.0;
        for (int q = pb; q < pe; ++q)
            if (pcol[q] == c) pij = pval[q];
        fcol[k] = c;
        fval[k] = pij - wd * apval[k];
    }
}

// A Newton refresh (new level-0 values, same pattern, same P): P~ re-formed
// numerically over its own pattern, P~_ic = P_ic - w d_i sum_j a_ij P_jc, no
// SpGEMM (the pattern of A P is the pattern of P~, which the setup formed).
// kFoldLanes lanes per row: the row's products a_ij x (c, P_jc) -- A's row in
// column order, each P row j in its stored order -- are staged in LDS once
// (the lanes' P-row lengths prefix-summed by shuffles); then one lane per P~
// entry c sums the products of column c in that order (P rows hold a column
// once, so the sum is the one over j in A's column order).  Rows of more than
// kRfA entries or kRfP products read A and P from memory in the same order.
// f32 (optional): the f32 copy of P~ written alongside.  stage = 0 reads
// every row from memory (XFK_REFOLD_STAGE=0: the test of the staged order).
constexpr int kRfA = 16, kRfP = 64, kRfRows = 256 / kFoldLanes;
static_assert(kRfA == 2 * kFoldLanes, "k_refold_p stages two A entries per lane");
__global__ void __launch_bounds__(256) k_refold_p(int n, const unsigned long long *rho, const double *__restrict__ dinv,
                                                  const int *__restrict__ rowptr, const int *__restrict__ col,
                                                  const double *__restrict__ val, const int *__restrict__ prow,
                                                  const int *__restrict__ pcol, const double *__restrict__ pval,
                                                  const int *__restrict__ frow, const int *__restrict__ fcol,
                                                  double *__restrict__ fval, float *__restrict__ f32, int stage)
{
    // (rows padded by one element: the 8 rows of a wave read one e at a time)
    __shared__ int s_pc[kRfRows][kRfP + 1];
    __shared__ double s_av[kRfRows][kRfP + 1], s_pv[kRfRows][kRfP + 1];
    const int lr = threadIdx.x / kFoldLanes, g = threadIdx.x & (kFoldLanes - 1);
    const int i = (int)blockIdx.x * kRfRows + lr;
    const bool live = i < n;   // (every thread reaches the barrier)
    const int ab = live ? rowptr[i] : 0, na = live ? rowptr[i + 1] - ab : 0;
    // lane g: A entries u = g and u = g + kFoldLanes, their P rows
    int pb[2] = {0, 0}, len[2] = {0, 0};
    double av[2] = {0.0, 0.0};
    if (na <= kRfA)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int u = g + h * kFoldLanes;
            if (u < na) {
                const int j = col[ab + u];
                pb[h] = prow[j];
                len[h] = prow[j + 1] - pb[h];
                av[h] = val[ab + u];
            }
        }
    int off[2], tot = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // exclusive prefix over u = 0 .. 15
        int inc = len[h];
#pragma unroll
        for (int d = 1; d < kFoldLanes; d <<= 1) {
            const int v = __shfl_up(inc, d, kFoldLanes);
            if (g >= d) inc += v;
        }
        off[h] = tot + inc - len[h];
        tot += __shfl(inc, kFoldLanes - 1, kFoldLanes);
    }
    const bool staged = stage && na <= kRfA && tot <= kRfP;
    if (staged)
#pragma unroll
        for (int h = 0; h < 2; ++h)
            for (int q = 0; q < len[h]; ++q) {
                s_pc[lr][off[h] + q] = pcol[pb[h] + q];
                s_pv[lr][off[h] + q] = pval[pb[h] + q];
                s_av[lr][off[h] + q] = av[h];
            }
    __syncthreads();
    if (!live) return;
    const double ra = rho_of(rho);
    const double wd = (ra > 0.0 ? 1.0 / ra : 0.0) * dinv[i];
    const int qb = prow[i], qe = prow[i + 1];
    for (int k = frow[i] + g; k < frow[i + 1]; k += kFoldLanes) {
        const int c = fcol[k];
        double ap = 0.0, pic = 0.0;
        for (int q = qb; q < qe; ++q)
            if (pcol[q] == c) pic = pval[q];
        if (staged) {
            for (int e = 0; e < tot; ++e)
                if (s_pc[lr][e] == c) ap = fma(s_av[lr][e], s_pv[lr][e], ap);
        } else {
            for (int t = ab; t < ab + na; ++t) {
                const int j = col[t];
                for (int q = prow[j]; q < prow[j + 1]; ++q)
                    if (pcol[q] == c) ap = fma(val[t], pval[q], ap);
            }
        }
        const double v = pic - wd * ap;
        fval[k] = v;
        if (f32) f32[k] = (float)v;
    }
}

// level 0, folded post-step (the pre-step stays sweep-from-0 + residual and
// R r'): u = x_pre + w D^-1 r' + P~ x_c, i.e. the prolongation and the
// post-sweep in one pass over P~ instead of P and A.  Tile shape and r.u
// partials as k_amg_smooth's last sweep (the SpMV's tiles and summation order).
template <int B, int SLOTS, class V>
__global__ void __launch_bounds__(B) k_fold_post0(int n, const int *__restrict__ frow, const int *__restrict__ fcol,
                                                  const V *__restrict__ fval, const double *__restrict__ xc,
                                                  const double *__restrict__ dinv, const unsigned long long *rho,
                                                  const double *__restrict__ rres,
                                                  const double *__restrict__ b, double *__restrict__ out,
                                                  const int *done, double *__restrict__ part_gam,
                                                  const unsigned short *__restrict__ c16,
                                                  const int *__restrict__ cbase)
{
    const int dn = load_flag_v(done);
    __shared__ __attribute__((aligned(16))) double lds[4 * SLOTS * B];
    const double ra = rho_of(rho);
    const int t = xcd_tile(blockIdx.x, gridDim.x);
    const int r0 = t * B;
    const int i = r0 + threadIdx.x;
    const TileRows tr = tile_rows<B>(r0, n, frow);
    const int cb = load_col_base(cbase, t);
    const double di = i < n ? dinv[i] : 0.0, bi = i < n ? b[i] : 0.0, ri = i < n ? rres[i] : 0.0;
    if (dn) return;
    const double w = ra > 0.0 ? 1.0 / ra : 0.0;
    const double pc = cg_tile_spmv16<B, SLOTS>(tr, c16, cb, fcol, fval, [&](int j) { return xc[j]; }, lds);
    double u = 0.0;
    if (i < n) {
        u = (w * di * bi + w * di * ri) + pc;
        out[i] = u;
    }
    if (part_gam) {   // uniform per launch
        __shared__ double red[2 * (B / 64)];
        double g = 0.0, zero = 0.0;
        if (i < n) g = bi * u;
        cg_block_sum2(zero, g, red);
        if (threadIdx.x == 0) part_gam[t] = g;
    }
}

// the folded pre-step: workgroups [0, blocks_a) form y (GA lanes per fine
// row), the rest b_c = P~^T b (GB lanes per coarse row)
template <int GA, int GB>
__global__ void __launch_bounds__(256) k_fold_pre(int n, int ncl, const int *__restrict__ rowptr,
                                                  const int *__restrict__ col, const double *__restrict__ val,
                                                  const double *__restrict__ dinv, const unsigned long long *rho,
                                                  const double *__restrict__ b, double *__restrict__ y, int nc,
                                                  const int *__restrict__ rrow, const int *__restrict__ rcol,
                                                  const double *__restrict__ rval, double *__restrict__ bc,
                                                  int blocks_a, const int *done, const double *__restrict__ yadd)
{
    if (done && *done) return;
    // XCD-contiguous row blocks in each range (blocks_a is a multiple of 8):
    // an XCD's L2 serves the vector entries its neighbouring rows share
    if ((int)blockIdx.x < blocks_a) {
        const double ra = rho_of(rho);
        const double w = ra > 0.0 ? 1.0 / ra : 0.0;
        const int i = (xcd_tile(blockIdx.x, blocks_a) * blockDim.x + threadIdx.x) / GA;
        const double ax =
            group_row_dot<GA>(i, n, rowptr, col, val, [&](int j) { return j < ncl ? w * dinv[j] * b[j] : 0.0; });
        if (i < n && (threadIdx.x & (GA - 1)) == 0) {
            const double di = dinv[i], bi = b[i], xi = w * di * bi;
            const double yi = xi + w * di * (bi - ax);
            y[i] = yadd ? yadd[i] + yi : yi;   // (a W-cycle's second correction adds onto the first)
        }
    } else {
        const int c = (xcd_tile(blockIdx.x - blocks_a, gridDim.x - blocks_a) * blockDim.x + threadIdx.x) / GB;
        const double sc = group_row_dot<GB>(c, nc, rrow, rcol, rval, [&](int j) { return b[j]; });
        if (c < nc && (threadIdx.x & (GB - 1)) == 0) bc[c] = sc;
    }
}

// x = M b, one 256-thread workgroup per row of the f32 inverse (ld a multiple
// of 64, padding columns zero): every thread issues its 16-B loads (4 floats)
// of the row at once, so the whole inverse is in flight (one wave per row
// left a 1.6k-row inverse at 2.3 TB/s: 6 waves per CU, each walking its row
// in dependent batches); products and sums in f64
constexpr int kDmvLoads = 2;
template <class V>
struct DmvVec;
template <>
struct DmvVec<float> {
    using T = float4;
};
template <>
struct DmvVec<double> {
    struct T {
        double x, y, z, w;
    };
};
// x = S M S b: row i of the symmetrised scaled inverse M (f32 or f64), the
// scale osc in f64, products and sums in f64
template <class V>
__global__ void __launch_bounds__(256) k_dense_mv(int n, int ld, const V *__restrict__ M,
                                                  const double *__restrict__ osc, const double *__restrict__ b,
                                                  double *__restrict__ x, const int *done)
{
    if (done && *done) return;
    using V4 = typename DmvVec<V>::T;
    __shared__ double red[4];
    const int i = blockIdx.x;
    const V4 *Mi = reinterpret_cast<const V4 *>(M + (size_t)i * ld);
    const int n4 = ld >> 2;
    double s0 = 0.0, s1 = 0.0;
    for (int j0 = 0; j0 < n4; j0 += 256 * kDmvLoads) {
        V4 m[kDmvLoads];
#pragma unroll
        for (int q = 0; q < kDmvLoads; ++q) {
            const int j = j0 + threadIdx.x + 256 * q;
            if (j < n4) m[q] = Mi[j];
            else m[q] = V4{0, 0, 0, 0};
        }
#pragma unroll
        for (int q = 0; q < kDmvLoads; ++q) {
            const int c = 4 * (j0 + threadIdx.x + 256 * q);
            if (c + 3 < n) {
                const double2 b0 = *reinterpret_cast<const double2 *>(b + c);
                const double2 b1 = *reinterpret_cast<const double2 *>(b + c + 2);
                const double2 c0 = *reinterpret_cast<const double2 *>(osc + c);
                const double2 c1 = *reinterpret_cast<const double2 *>(osc + c + 2);
                s0 += (double)m[q].x * (c0.x * b0.x) + (double)m[q].z * (c1.x * b1.x);
                s1 += (double)m[q].y * (c0.y * b0.y) + (double)m[q].w * (c1.y * b1.y);
            } else {
                if (c < n) s0 += (double)m[q].x * (osc[c] * b[c]);
                if (c + 1 < n) s1 += (double)m[q].y * (osc[c + 1] * b[c + 1]);
                if (c + 2 < n) s0 += (double)m[q].z * (osc[c + 2] * b[c + 2]);
            }
        }
    }
    const double w = cg_wave_sum(s0 + s1);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = w;
    __syncthreads();
    if (threadIdx.x == 0) x[i] = osc[i] * ((red[0] + red[1]) + (red[2] + red[3]));
}

// diagnostics (XFK_AMG_DEBUG): rows left without an aggregate, split by
// whether they have strong (owned) couplings / any off-diagonal coupling
__global__ void k_setup_zero(int *__restrict__ a, int na, unsigned long long *__restrict__ b, int nb_)
{
    for (int k = threadIdx.x; k < na; k += blockDim.x) a[k] = 0;
    for (int k = threadIdx.x; k < nb_; k += blockDim.x) b[k] = 0ull;
}

__global__ void k_debug_unagg(int n, const int *__restrict__ rowptr, const int *__restrict__ col,
                              const int *__restrict__ sdeg, const int *__restrict__ agg, int *out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || agg[i] >= 0) return;
    int offd = 0;
    for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) offd += (col[k] != i);
    atomicAdd(&out[sdeg[i] > 0 ? 0 : (offd > 0 ? 1 : 2)], 1);
}

// --------------------------------------------------------------------------
// sharded level 0: helpers of the distributed Galerkin product and V-cycle
// --------------------------------------------------------------------------

// x = w D^-1 b: the first Jacobi sweep from zero, written out (its halo is
// exchanged before the residual)
__global__ void k_jacobi_first(int n, const unsigned long long *rho, const double *__restrict__ dinv,
                               const double *__restrict__ b, double *__restrict__ x, const int *done)
{
    if (done && *done) return;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double ra = rho_of(rho);
    x[i] = (ra > 0.0 ? 1.0 / ra : 0.0) * dinv[i] * b[i];
}
__global__ void k_row_len_d(int n, const int *__restrict__ rowptr, double *__restrict__ len)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) len[i] = (double)(rowptr[i + 1] - rowptr[i]);
}
__global__ void k_dbl2int(long long n, const double *__restrict__ a, int *__restrict__ b)
{
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i < n) b[i] = (int)a[i];
}
__global__ void k_int2dbl(long long n, const int *__restrict__ a, double *__restrict__ b)
{
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i < n) b[i] = (double)a[i];
}
// b = (float) a over the rowptr[n] entries of a CSR (the length read on the
// device: the host may only hold an upper bound); fixed grid, grid-stride
__global__ void k_d2f(int n, const int *__restrict__ rowptr, const double *__restrict__ a, float *__restrict__ b)
{
    const long long m = rowptr[n];
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < m; i += (long long)gridDim.x * blockDim.x)
        b[i] = (float)a[i];
}

__global__ void k_add_int(long long n, int *__restrict__ a, int v)
{
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i < n) a[i] += v;
}
// row pointer of P extended by the halo rows: owned rows, then pnnz + hrow
__global__ void k_pe_row(int n, int nh, long long pnnz, const int *__restrict__ prow, const int *__restrict__ hrow,
                         int *__restrict__ out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= n) out[i] = prow[i];
    else if (i <= n + nh) out[i] = (int)pnnz + hrow[i - n];
}
// global coarse row pointer from the all-gathered per-rank row pointers
// (stride ld per rank); c0 / e0: first row / entry of each rank (nranks + 1)
__global__ void k_concat_rowptr(int NC, int nranks, const int *__restrict__ c0, const int *__restrict__ e0,
                                const int *__restrict__ grow, int ld, int *__restrict__ out)
{
    const int I = blockIdx.x * blockDim.x + threadIdx.x;
    if (I > NC) return;
    if (I == NC) {
        out[I] = e0[nranks];
        return;
    }
    int q = 0;
    while (c0[q + 1] <= I) ++q;
    out[I] = e0[q] + grow[(size_t)q * ld + (I - c0[q])];
}
// global coarse vector from the padded all-gather (stride ld per rank)
__global__ void k_unpad(int NC, int nranks, const int *__restrict__ c0, const double *__restrict__ all, int ld,
                        double *__restrict__ out, const int *done)
{
    if (done && *done) return;
    const int I = blockIdx.x * blockDim.x + threadIdx.x;
    if (I >= NC) return;
    int q = 0;
    while (c0[q + 1] <= I) ++q;
    out[I] = all[(size_t)q * ld + (I - c0[q])];
}

}  // namespace

// --------------------------------------------------------------------------
// host side
// --------------------------------------------------------------------------

Amg::~Amg()
{
    pinned_free(nd_stage);   // (to the process cache when the problem is destroyed)
    pinned_free(def_host);
    pinned_free(host_int);
    pinned_free(host_big);
    if (ev_host) (void)hipEventDestroy(ev_host);
    for (hipEvent_t e : tail_ev) (void)hipEventDestroy(e);
}

#define AMG_CHECK(call)                                                          \
    do {                                                                         \
        hipError_t _e = (call);                                                  \
        if (_e != hipSuccess) {                                                  \
            ::xfk::set_error(std::string(#call) + ": " + hipGetErrorString(_e)); \
            return XFK_ERR_HIP;                                                  \
        }                                                                        \
    } while (0)

namespace {

// out[0..n] = exclusive scan of in[0..n-1], out[n] = total; returns total
// Short scans (coarse levels: <= kScanLds entries) in one workgroup, one
// launch instead of hipcub's memset + state init + scan: each of 1024 threads
// loads 16 consecutive entries at once (four 16-B loads), scans them in
// registers, a workgroup scan of the thread sums gives the offsets, and the
// prefixes are stored -- one memory round trip each way.
constexpr int kScanLds = 16384;

// XFK_NO_SCAN_LDS=1: every scan through hipcub
bool scan_lds_on(int n)
{
    static const bool v = [] {
        const char *e = std::getenv("XFK_NO_SCAN_LDS");
        return !(e && std::atoi(e) != 0);
    }();
    return v && n <= kScanLds;
}

__global__ void __launch_bounds__(1024) k_scan_lds(int n, const int *__restrict__ in, int *__restrict__ out)
{
    __shared__ int wsum[16];
    const int b = 16 * threadIdx.x;
    int v[16];
    if (b + 16 <= n && (reinterpret_cast<uintptr_t>(in) & 15) == 0) {
        const int4 *p = reinterpret_cast<const int4 *>(in + b);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int4 x = p[q];
            v[4 * q] = x.x;
            v[4 * q + 1] = x.y;
            v[4 * q + 2] = x.z;
            v[4 * q + 3] = x.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = b + q < n ? in[b + q] : 0;
    }
#pragma unroll
    for (int q = 1; q < 16; ++q) v[q] += v[q - 1];
    const int loc = v[15];
    // exclusive scan of the thread sums over the workgroup
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int x = loc;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int t = __shfl_up(x, off, 64);
        if (lane >= off) x += t;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    int before = x - loc;
#pragma unroll
    for (int w = 0; w < 16; ++w)
        if (w < wid) before += wsum[w];
#pragma unroll
    for (int q = 0; q < 16; ++q)
        if (b + q < n) out[b + q + 1] = before + v[q];
    if (threadIdx.x == 0) out[0] = 0;
}

int scan_total(Amg &A, hipStream_t s, const int *in, int *out, int n, long long &total)
{
    if (scan_lds_on(n)) {
        k_scan_lds<<<1, 1024, 0, s>>>(n, in, out);
        AMG_CHECK(hipGetLastError());
    } else {
        size_t bytes = 0;
        AMG_CHECK(hipcub::DeviceScan::InclusiveSum(nullptr, bytes, in, out + 1, n, s));
        AMG_CHECK(A.cub_tmp.alloc(bytes ? bytes : 1));
        AMG_CHECK(hipMemsetAsync(out, 0, sizeof(int), s));
        if (n > 0) AMG_CHECK(hipcub::DeviceScan::InclusiveSum(A.cub_tmp.p, bytes, in, out + 1, n, s));
    }
    AMG_CHECK(hipMemcpyAsync(A.host_int, out + n, sizeof(int), hipMemcpyDeviceToHost, s));
    AMG_CHECK(hipStreamSynchronize(s));
    total = A.host_int[0];
    return XFK_OK;
}

// the same without reading the total back (no host synchronisation), with
// the given temporary storage.  `in` must hold n + 1 readable entries: the
// long scans are exclusive over n + 1 (out[0] = 0 without a memset; in[n]
// only fills the unused last slot)
int scan_only(DBuf<char> &tmp, hipStream_t s, const int *in, int *out, int n)
{
    if (scan_lds_on(n)) {
        k_scan_lds<<<1, 1024, 0, s>>>(n, in, out);
        AMG_CHECK(hipGetLastError());
        return XFK_OK;
    }
    size_t bytes = 0;
    AMG_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, n + 1, s));
    AMG_CHECK(tmp.alloc(bytes ? bytes : 1));
    AMG_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp.p, bytes, in, out, n + 1, s));
    return XFK_OK;
}
int scan_only(Amg &A, hipStream_t s, const int *in, int *out, int n) { return scan_only(A.cub_tmp, s, in, out, n); }

int read_flag(Amg &A, hipStream_t s, int idx, int &v)
{
    AMG_CHECK(hipMemcpyAsync(A.host_int + 1, A.dev_int.p + idx, sizeof(int), hipMemcpyDeviceToHost, s));
    AMG_CHECK(hipStreamSynchronize(s));
    v = A.host_int[1];
    return XFK_OK;
}

// C = X Y (rowptr/col/val allocated here); XFK_ERR_UNSUPPORTED on LDS overflow
void launch_compact(hipStream_t s, int nrows, int cap, const int *crow, const int *pc, const double *pv, int *ccol,
                    double *cval, int *nnz_out)
{
    if (cap <= 16)
        k_spgemm_compact<4><<<(unsigned)(((long long)nrows * 4 + kB - 1) / kB), kB, 0, s>>>(nrows, cap, crow, pc, pv,
                                                                                             ccol, cval, nnz_out);
    else if (cap <= 32)
        k_spgemm_compact<8><<<(unsigned)(((long long)nrows * 8 + kB - 1) / kB), kB, 0, s>>>(nrows, cap, crow, pc, pv,
                                                                                             ccol, cval, nnz_out);
    else
        k_spgemm_compact<16><<<(unsigned)(((long long)nrows * 16 + kB - 1) / kB), kB, 0, s>>>(nrows, cap, crow, pc,
                                                                                               pv, ccol, cval, nnz_out);
}

template <bool PMODE>
int spgemm(Amg &M, hipStream_t s, int nrows, const SgX &X, const SgY &Y, DBuf<int> &crow, DBuf<int> &ccol,
           DBuf<double> &cval, long long &cnnz, int key = -1, bool defer = true)
{
    AMG_CHECK(M.cnt.alloc((size_t)nrows + 1));
    AMG_CHECK(crow.alloc((size_t)nrows + 1));
    // single pass into padded rows of `cap` slots (sort-based), then scan +
    // compaction; returns the overflow flag (rows with more products than
    // slots), read back with the scan's own synchronisation
    int *sovf = M.dev_int.p + 6;
    auto launch_sort = [&](int cap, int *ovf, int *need = nullptr) {
        int *pc = M.pad_col.p;
        double *pv = M.pad_val.p;
        if (nrows > 0) {
            // few lanes per row, 4-8 sorted slots per lane: many rows per
            // wavefront to overlap their dependent gathers
            if (cap == 16)
                k_spgemm_sort<PMODE, 4, 16><<<(nrows + 15) / 16, 64, 0, s>>>(nrows, X, Y, M.cnt.p, pc, pv, ovf, need);
            else if (cap == 32)
                k_spgemm_sort<PMODE, 8, 32><<<(nrows + 7) / 8, 64, 0, s>>>(nrows, X, Y, M.cnt.p, pc, pv, ovf, need);
            else if (cap == 64)
                k_spgemm_sort<PMODE, 8, 64><<<(nrows + 7) / 8, 64, 0, s>>>(nrows, X, Y, M.cnt.p, pc, pv, ovf, need);
            else if (cap == 128)
                k_spgemm_sort<PMODE, 16, 128><<<(nrows + 3) / 4, 64, 0, s>>>(nrows, X, Y, M.cnt.p, pc, pv, ovf, need);
            else
                k_spgemm_sort<PMODE, 32, 256><<<(nrows + 1) / 2, 64, 0, s>>>(nrows, X, Y, M.cnt.p, pc, pv, ovf, need);
        }
    };
    // single pass into padded rows of `cap` slots (sort-based), then scan +
    // compaction; returns the overflow flag (rows with more products than
    // slots), read back with the scan's own synchronisation
    auto sort_pass = [&](int cap, bool &overflow) -> int {
        AMG_CHECK(M.pad_col.alloc((size_t)nrows * cap));
        AMG_CHECK(M.pad_val.alloc((size_t)nrows * cap));
        AMG_CHECK(hipMemsetAsync(sovf, 0, sizeof(int), s));
        launch_sort(cap, sovf);
        AMG_CHECK(hipMemcpyAsync(M.host_int + 4, sovf, sizeof(int), hipMemcpyDeviceToHost, s));
        int rc = scan_total(M, s, M.cnt.p, crow.p, nrows, cnnz);   // synchronises
        if (rc != XFK_OK) return rc;
        overflow = M.host_int[4] != 0;
        if (overflow) return XFK_OK;
        AMG_CHECK(ccol.alloc((size_t)std::max(1LL, cnnz)));
        AMG_CHECK(cval.alloc((size_t)std::max(1LL, cnnz)));
        if (nrows > 0)
            launch_compact(s, nrows, cap, crow.p, M.pad_col.p, M.pad_val.p, ccol.p, cval.p, nullptr);
        return XFK_OK;
    };
    // the slot capacity this product needed in the previous setup (same
    // call site): taken without measuring the longest product list first,
    // and without any host synchronisation -- the output is sized for
    // nrows x cap, its length and the kernel's overflow flag land in a
    // deferred slot that the setup reads once at its end (an overflow there
    // rebuilds the hierarchy with measured capacities)
    auto deferred_pass = [&](int cap, bool verify = false) -> int {
        int *slot = M.def_dev.p + M.def_n;
        // (a capacity from another problem: its class is checked on the device)
        int *need = (verify && cap > 16) ? M.def_dev.p + kAmgDeferSlots + M.def_n / 2 : nullptr;
        M.def_verify[M.def_n / 2] = need ? cap : 0;
        AMG_CHECK(M.pad_col.alloc((size_t)nrows * cap));
        AMG_CHECK(M.pad_val.alloc((size_t)nrows * cap));
        AMG_CHECK(ccol.alloc((size_t)std::max(1LL, (long long)nrows * cap)));
        AMG_CHECK(cval.alloc((size_t)std::max(1LL, (long long)nrows * cap)));
        launch_sort(cap, slot, need);
        int rc = scan_only(M, s, M.cnt.p, crow.p, nrows);
        if (rc != XFK_OK) return rc;
        if (nrows > 0)
            launch_compact(s, nrows, cap, crow.p, M.pad_col.p, M.pad_val.p, ccol.p, cval.p, slot + 1);
        else
            AMG_CHECK(hipMemsetAsync(slot + 1, 0, sizeof(int), s));
        M.def_target[M.def_n / 2] = &cnnz;
        M.def_n += 2;
        cnnz = (long long)nrows * cap;   // an upper bound until the deferred read
        return XFK_OK;
    };
    if (key >= 0) {
        auto hint = M.cap_hint.find(key);
        if (hint != M.cap_hint.end()) {
            if (defer && M.def_n + 2 <= kAmgDeferSlots) return deferred_pass(hint->second, M.foreign);
            if (M.foreign) {   // (no slot to check another problem's capacity in: measure)
                M.cap_hint.erase(hint);
                hint = M.cap_hint.end();
            }
        }
        if (hint != M.cap_hint.end()) {
            bool overflow = false;
            int rc = sort_pass(hint->second, overflow);
            if (rc != XFK_OK || !overflow) return rc;
            M.cap_hint.erase(hint);
        }
    }
    // longest product list -> sub-wave (<= 64 products per row) or wave-per-row kernels
    int maxprod = 0;
    if (nrows > 0) {
        k_spgemm_nprod<PMODE><<<nb(nrows), kB, 0, s>>>(nrows, X, Y, M.cnt.p);
        size_t bytes = 0;
        AMG_CHECK(hipcub::DeviceReduce::Max(nullptr, bytes, M.cnt.p, M.dev_int.p + 3, nrows, s));
        AMG_CHECK(M.cub_tmp.alloc(bytes ? bytes : 1));
        AMG_CHECK(hipcub::DeviceReduce::Max(M.cub_tmp.p, bytes, M.cnt.p, M.dev_int.p + 3, nrows, s));
        int rc = read_flag(M, s, 3, maxprod);
        if (rc != XFK_OK) return rc;
    }
    if (maxprod <= kSortCap) {
        const int cap = maxprod <= 16 ? 16 : maxprod <= 32 ? 32 : maxprod <= 64 ? 64 : maxprod <= 128 ? 128 : 256;
        int rc = XFK_OK;
        if (defer && key >= 0 && M.def_n + 2 <= kAmgDeferSlots) {
            // the measured capacity (no overflow possible) through the
            // deferred slot as a hinted one: the same kernels, so the same
            // bits, without the host check for the length (~20 us per call
            // site of a first setup)
            rc = deferred_pass(cap);
        } else {
            bool overflow = false;
            rc = sort_pass(cap, overflow);
            if (rc == XFK_OK && overflow) {
                set_error("AMG: internal SpGEMM capacity error");
                return XFK_ERR_HIP;
            }
        }
        if (rc != XFK_OK) return rc;
        if (key >= 0) {
            // XFK_AMG_TEST_SMALL_HINT=1 (tests only): store a too-small capacity so
            // the next setup takes the overflow-and-rebuild path
            const bool small = std::getenv("XFK_AMG_TEST_SMALL_HINT") != nullptr;
            M.cap_hint[key] = small ? 16 : cap;   // (16: the smallest capacity the kernels have)
        }
        return XFK_OK;
    }
    AMG_CHECK(hipMemsetAsync(M.dev_int.p + 2, 0, 2 * sizeof(int), s));
    if (nrows > 0)
        k_spgemm<false, PMODE, kSgMax><<<nrows, 64, 0, s>>>(nrows, X, Y, M.cnt.p, nullptr, nullptr, nullptr,
                                                            M.dev_int.p + 2);
    if (nrows > 0) {   // longest row -> LDS capacity of the FILL pass
        size_t bytes = 0;
        AMG_CHECK(hipcub::DeviceReduce::Max(nullptr, bytes, M.cnt.p, M.dev_int.p + 3, nrows, s));
        AMG_CHECK(M.cub_tmp.alloc(bytes ? bytes : 1));
        AMG_CHECK(hipcub::DeviceReduce::Max(M.cub_tmp.p, bytes, M.cnt.p, M.dev_int.p + 3, nrows, s));
    }
    AMG_CHECK(hipMemcpyAsync(M.host_int + 2, M.dev_int.p + 2, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
    int rc = scan_total(M, s, M.cnt.p, crow.p, nrows, cnnz);   // synchronises
    if (rc != XFK_OK) return rc;
    const int ovf = M.host_int[2], maxrow = M.host_int[3];
    if (ovf) {
        set_error("AMG: a SpGEMM row exceeds the LDS hash capacity");
        return XFK_ERR_UNSUPPORTED;
    }
    AMG_CHECK(ccol.alloc((size_t)std::max(1LL, cnnz)));
    AMG_CHECK(cval.alloc((size_t)std::max(1LL, cnnz)));
    if (nrows > 0) {
        int *of = M.dev_int.p + 2;
        if (maxrow <= 32)
            k_spgemm<true, PMODE, 32><<<nrows, 64, 0, s>>>(nrows, X, Y, nullptr, crow.p, ccol.p, cval.p, of);
        else if (maxrow <= 128)
            k_spgemm<true, PMODE, 128><<<nrows, 64, 0, s>>>(nrows, X, Y, nullptr, crow.p, ccol.p, cval.p, of);
        else
            k_spgemm<true, PMODE, kSgMax><<<nrows, 64, 0, s>>>(nrows, X, Y, nullptr, crow.p, ccol.p, cval.p, of);
    }
    return XFK_OK;
}

// levels / transfer operators with at least this many rows use the tile kernels
// (XFK_TILE_MIN_ROWS overrides, for experiments)
static int tile_min_rows()
{
    static const int v = [] {
        const char *e = std::getenv("XFK_TILE_MIN_ROWS");
        return e ? std::atoi(e) : 16384;
    }();
    return v;
}
#define kTileMinRows tile_min_rows()

// folded coarse levels (k_fold_pre); XFK_AMG_FOLD=0 keeps the four-launch form
static bool fold_levels()
{
    static const bool v = [] {
        const char *e = std::getenv("XFK_AMG_FOLD");
        return !e || std::atoi(e) != 0;
    }();
    return v;
}

// lanes per row for a CSR with this many nonzeros per row on average
int lanes_for(double per_row)
{
    return per_row <= 6.0 ? 4 : (per_row <= 20.0 ? 8 : 16);
}

// lab switch for the long-row transfer operators (R of level 0): 0 = tile of
// 256 rows with 6 slots (48 KiB LDS), 1 = G lanes per row, 2 = tile of 128
// rows with 6 slots (24 KiB), 3 = tile of 256 rows with 3 slots (24 KiB)
static int rmv_mode()
{
    static const int v = [] {
        const char *e = std::getenv("XFK_RMV");
        return e ? std::atoi(e) : 0;
    }();
    return v;
}

// level 0 with f32 values: the 256-row tile kernels (level 0 always has >= kTileMinRows rows)
// (128- and 64-row tiles for R's ~25-entry rows were measured slower: 14.4 -> 15.0 / 15.6 us,
// profiles/r04_experiments/r04h_XFK_R0_TILE_*.json)
// XFK_R0_SLOTS (lab): staging slots per lane for the long rows (6 = 6144
// products per pass; R's ~27-entry rows fill 256-row tiles with ~6900);
// 8 / 7 (one pass, 64 / 56 KiB of LDS) measured 20.3 / 20.2 us vs 14.7 us
static int r0_slots()
{
    static const int v = [] {
        const char *e = std::getenv("XFK_R0_SLOTS");
        return e ? std::atoi(e) : 6;
    }();
    return v;
}

void launch_mv32(hipStream_t s, int n, const int *rowptr, const int *col, const float *val, const double *x,
                 double *y, bool acc, int G, const int *done, const unsigned short *c16, const int *cbase)
{
    if (n <= 0) return;
    const int g = (n + 255) / 256;
    if (G > 4 && r0_slots() != 6 && !acc) {
        const int v = r0_slots();
        if (v == 8) k_csr_mv_tile<256, false, 8><<<g, 256, 0, s>>>(n, rowptr, col, val, x, y, done, c16, cbase);
        else if (v == 4) k_csr_mv_tile<256, false, 4><<<g, 256, 0, s>>>(n, rowptr, col, val, x, y, done, c16, cbase);
        else if (v == 3) k_csr_mv_tile<256, false, 3><<<g, 256, 0, s>>>(n, rowptr, col, val, x, y, done, c16, cbase);
        else k_csr_mv_tile<256, false, 2><<<g, 256, 0, s>>>(n, rowptr, col, val, x, y, done, c16, cbase);
        return;
    }
    if (G <= 4) {
        if (acc) k_csr_mv_tile<256, true, 2><<<g, 256, 0, s>>>(n, rowptr, col, val, x, y, done, c16, cbase);
        else k_csr_mv_tile<256, false, 2><<<g, 256, 0, s>>>(n, rowptr, col, val, x, y, done, c16, cbase);
    } else {
        if (acc) k_csr_mv_tile<256, true, 6><<<g, 256, 0, s>>>(n, rowptr, col, val, x, y, done, c16, cbase);
        else k_csr_mv_tile<256, false, 6><<<g, 256, 0, s>>>(n, rowptr, col, val, x, y, done, c16, cbase);
    }
}

// c16 / cbase: 16-bit column offsets in 256-row tiles (used by the 256-row tile kernels only)
void launch_mv(hipStream_t s, int n, const int *rowptr, const int *col, const double *val, const double *x, double *y,
               bool acc, int G, const int *done, const unsigned short *c16 = nullptr, const int *cbase = nullptr)
{
    if (n <= 0) return;
    if (n >= kTileMinRows && G == 8 && rmv_mode() == 2) {
        const int g = (n + 127) / 128;
        if (acc) k_csr_mv_tile<128, true, 6><<<g, 128, 0, s>>>(n, rowptr, col, val, x, y, done);
        else k_csr_mv_tile<128, false, 6><<<g, 128, 0, s>>>(n, rowptr, col, val, x, y, done);
        return;
    }
    if (n >= kTileMinRows && G == 8 && rmv_mode() == 3) {
        const int g = (n + 255) / 256;
        if (acc) k_csr_mv_tile<256, true, 3><<<g, 256, 0, s>>>(n, rowptr, col, val, x, y, done);
        else k_csr_mv_tile<256, false, 3><<<g, 256, 0, s>>>(n, rowptr, col, val, x, y, done);
        return;
    }
    if (n >= kTileMinRows && G <= 8 && !(G == 8 && rmv_mode() == 1)) {
        // G = 8: 7..20 entries per row -> 6 slots per lane, one staging pass per tile
        const int g = (n + 255) / 256;
        if (G <= 4) {
            if (acc) k_csr_mv_tile<256, true, 2><<<g, 256, 0, s>>>(n, rowptr, col, val, x, y, done, c16, cbase);
            else k_csr_mv_tile<256, false, 2><<<g, 256, 0, s>>>(n, rowptr, col, val, x, y, done, c16, cbase);
        } else {
            if (acc) k_csr_mv_tile<256, true, 6><<<g, 256, 0, s>>>(n, rowptr, col, val, x, y, done, c16, cbase);
            else k_csr_mv_tile<256, false, 6><<<g, 256, 0, s>>>(n, rowptr, col, val, x, y, done, c16, cbase);
        }
        return;
    }
    const int g = (int)(((long long)n * G + 255) / 256);
#define XFK_MV(GG)                                                                                        \
    if (acc) k_csr_mv_g<GG, true><<<g, 256, 0, s>>>(n, rowptr, col, val, x, y, done);                    \
    else k_csr_mv_g<GG, false><<<g, 256, 0, s>>>(n, rowptr, col, val, x, y, done);
    if (G == 4) { XFK_MV(4) } else if (G == 8) { XFK_MV(8) } else { XFK_MV(16) }
#undef XFK_MV
}

}  // namespace

// tile t reads a halo column (>= n) in one of its rows
__global__ void k_tile_halo_flags(int n, int B, const int *__restrict__ rowptr, const int *__restrict__ col,
                                  int *__restrict__ flag)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    bool h = false;
    for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) h = h || col[k] >= n;
    if (h) flag[i / B] = 1;   // benign race: every writer stores 1
}

int build_tile_split(hipStream_t s, int n, int B, const int *rowptr, const int *col, TileSplit &ts)
{
    const int nt = (n + B - 1) / B;
    ts.B = 0;
    ts.n_in = ts.n_bd = 0;
    if (nt == 0) {
        ts.B = B;
        return XFK_OK;
    }
    DBuf<int> flag;
    AMG_CHECK(flag.alloc(nt));
    AMG_CHECK(hipMemsetAsync(flag.p, 0, sizeof(int) * nt, s));
    k_tile_halo_flags<<<nb(n), kB, 0, s>>>(n, B, rowptr, col, flag.p);
    std::vector<int> h(nt), list;
    list.reserve(nt);
    AMG_CHECK(hipMemcpyAsync(h.data(), flag.p, sizeof(int) * nt, hipMemcpyDeviceToHost, s));
    AMG_CHECK(hipStreamSynchronize(s));
    for (int t = 0; t < nt; ++t)
        if (!h[t]) list.push_back(t);
    ts.n_in = (int)list.size();
    for (int t = 0; t < nt; ++t)
        if (h[t]) list.push_back(t);
    ts.n_bd = nt - ts.n_in;
    AMG_CHECK(ts.tiles.alloc(nt));
    AMG_CHECK(hipMemcpyAsync(ts.tiles.p, list.data(), sizeof(int) * nt, hipMemcpyHostToDevice, s));
    AMG_CHECK(hipStreamSynchronize(s));   // `list` is a host temporary
    ts.B = B;
    return XFK_OK;
}

namespace {
std::mutex g_pool_mu;
std::map<hipStream_t, int> g_pool_dev;                 // every pooled stream -> its device
std::map<int, std::vector<hipStream_t>> g_pool_free;   // idle streams per device
}  // namespace

hipError_t stream_acquire(hipStream_t *s)
{
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        auto &f = g_pool_free[dev];
        if (!f.empty()) {
            *s = f.back();
            f.pop_back();
            return hipSuccess;
        }
    }
    e = hipStreamCreateWithFlags(s, hipStreamNonBlocking);
    if (e == hipSuccess) {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        g_pool_dev[*s] = dev;
    }
    return e;
}

void stream_release(hipStream_t s)
{
    if (!s) return;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    auto it = g_pool_dev.find(s);
    if (it == g_pool_dev.end()) {
        (void)hipStreamDestroy(s);
        return;
    }
    g_pool_free[it->second].push_back(s);
}

void stream_pool_drain()
{
    std::vector<hipStream_t> idle;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (auto &kv : g_pool_free)
            for (hipStream_t q : kv.second) {
                idle.push_back(q);
                g_pool_dev.erase(q);
            }
        g_pool_free.clear();
    }
    for (hipStream_t q : idle) (void)hipStreamDestroy(q);
}

long long stream_pool_idle()
{
    std::lock_guard<std::mutex> lk(g_pool_mu);
    long long n = 0;
    for (auto &kv : g_pool_free) n += (long long)kv.second.size();
    return n;
}

int SideStream::init()
{
    if (cs) return XFK_OK;
    AMG_CHECK(stream_acquire(&cs));
    AMG_CHECK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
    AMG_CHECK(hipEventCreateWithFlags(&b, hipEventDisableTiming));
    AMG_CHECK(hipEventCreateWithFlags(&c, hipEventDisableTiming));
    return XFK_OK;
}

SideStream::~SideStream()
{
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
    if (c) (void)hipEventDestroy(c);
    if (cs) {
        (void)hipStreamSynchronize(cs);
        stream_release(cs);
    }
}

// The folded coarse level that runs a W-cycle (two coarse corrections): by
// default the level above the last V-cycle level (nlev - 3: on configs[2]
// level 1, whose coarse level of 14k rows costs a few launches per visit;
// 21 -> 18 PCG iterations), in single-device and replicated hierarchies
// alike.  wlevel when set (-1: none), else XFK_AMG_W (-1: none).
int Amg::wcycle_level() const
{
    static const int v = [] {
        const char *e = std::getenv("XFK_AMG_W");
        return e ? std::atoi(e) : -2;
    }();
    const int w = wlevel != -2 ? wlevel : v;
    if (w != -2) return w;
    return nlev >= 4 ? nlev - 3 : -1;
}

// W-cycle at level l: l is the W level, or between XFK_AMG_W_LO and it
// (experiments with W over several levels; default: the W level alone)
bool Amg::w_at(int l) const
{
    static const int lo_env = [] {
        const char *e = std::getenv("XFK_AMG_W_LO");
        return e ? std::atoi(e) : -1;
    }();
    const int w = wcycle_level();
    if (w < 0 || l > w || l + 1 >= nlev - 1) return false;
    return l == w || (lo_env >= 0 && l >= lo_env);
}

// XFK_NO_COL16=1: level 0 reads 32-bit column indices
static bool col16_on()
{
    static const bool v = [] {
        const char *e = std::getenv("XFK_NO_COL16");
        return !(e && std::atoi(e) != 0);
    }();
    return v;
}

// XFK_NO_SIDE_SETUP=1: every setup step on the main stream
static bool side_setup_on()
{
    static const bool v = [] {
        const char *e = std::getenv("XFK_NO_SIDE_SETUP");
        return !(e && std::atoi(e) != 0);
    }();
    return v;
}

// XFK_AMG_F32=0: level 0's V-cycle operators keep f64 values
// signed strength (k_amg_strength); XFK_AMG_ABS_STRENGTH=1: |a_ij|
static bool signed_strength()
{
    static const bool v = std::getenv("XFK_AMG_ABS_STRENGTH") == nullptr;
    return v;
}

static bool f32_on()
{
    static const bool v = [] {
        const char *e = std::getenv("XFK_AMG_F32");
        return !(e && std::atoi(e) == 0);
    }();
    return v;
}

// XFK_AMG_F32_SWEEP=1: the level-0 sweeps read the f32 copy of A too (measured
// slower: the sweep's two gathers per entry, not its value stream, bound it)
static bool f32_sweep_on()
{
    static const bool v = [] {
        const char *e = std::getenv("XFK_AMG_F32_SWEEP");
        return e && std::atoi(e) != 0;
    }();
    return v;
}

// f32 copy of a CSR's values (cap: an upper bound of its length, for the allocation)
static int to_f32(hipStream_t s, int n, const int *rowptr, long long cap, const double *a, DBuf<float> &b)
{
    if (b.alloc((size_t)std::max(1LL, cap)) != hipSuccess) return XFK_ERR_HIP;
    if (n > 0) k_d2f<<<2048, 256, 0, s>>>(n, rowptr, a, b.p);
    return XFK_OK;
}

// XFK_MIS_XCD=0: MIS-2 sweeps with round-robin blocks (measurement)
static bool mis_xcd_on()
{
    static const bool v = [] {
        const char *e = std::getenv("XFK_MIS_XCD");
        return !(e && std::atoi(e) == 0);
    }();
    return v;
}

// XFK_NO_SPEC=1: no setup work enqueued ahead of a host check
static bool spec_on()
{
    static const bool v = [] {
        const char *e = std::getenv("XFK_NO_SPEC");
        return !(e && std::atoi(e) != 0);
    }();
    return v;
}

// Off by default: on MI355X each cross-stream hop (side stream waits for the
// main stream, main waits for the exchange) costs more than the interior
// tiles it overlaps -- configs[4] rank 0 of 8, compute only, 469 vs 304 us
// per PCG iteration (profiles/r04c_rank0_overlap.txt).  XFK_OVERLAP=1 turns
// it on (XFK_NO_OVERLAP=1 keeps it off).
bool overlap_enabled()
{
    const char *n = std::getenv("XFK_NO_OVERLAP");
    if (n && std::atoi(n) != 0) return false;
    const char *e = std::getenv("XFK_OVERLAP");
    return e && std::atoi(e) != 0;
}

int Amg::resolve_deferred(hipStream_t s, bool &overflow)
{
    int rc = fetch_deferred(s);
    if (rc != XFK_OK) return rc;
    return wait_deferred(s, overflow);
}

// the deferred slots' read, enqueued (the host waits for it in wait_deferred;
// work enqueued in between runs meanwhile)
int Amg::fetch_deferred(hipStream_t s)
{
    if (def_n == 0) return XFK_OK;
    AMG_CHECK(hipMemcpyAsync(def_host, def_dev.p, sizeof(int) * kAmgDeferTotal, hipMemcpyDeviceToHost, s));
    AMG_CHECK(hipEventRecord(ev_host, s));
    return XFK_OK;
}

int Amg::wait_deferred(hipStream_t s, bool &overflow)
{
    overflow = false;
    if (def_n == 0) return XFK_OK;
    AMG_CHECK(hipEventSynchronize(ev_host));
    for (int q = 0; q < def_n / 2; ++q) {
        if (def_host[2 * q]) overflow = true;
        else if (def_verify[q] && !def_host[kAmgDeferSlots + q]) overflow = true;   // another class measured
        else *def_target[q] = def_host[2 * q + 1];
        def_verify[q] = 0;
    }
    def_n = 0;
    AMG_CHECK(hipMemsetAsync(def_dev.p, 0, sizeof(int) * kAmgDeferTotal, s));
    return XFK_OK;
}

int Amg::host_ints(int count)
{
    if (host_big_n >= count) return XFK_OK;
    pinned_free(host_big);   // (outside a destroy: hipHostFree)
    host_big = nullptr;
    host_big_n = 0;
    AMG_CHECK(pinned_malloc((void **)&host_big, sizeof(int) * std::max(count, 1)));
    host_big_n = count;
    return XFK_OK;
}

int Amg::reserve_host()
{
    if (!host_int) AMG_CHECK(pinned_malloc((void **)&host_int, 16 * sizeof(int)));
    if (!def_host) AMG_CHECK(pinned_malloc((void **)&def_host, kAmgDeferTotal * sizeof(int)));
    if (!ev_host) AMG_CHECK(hipEventCreateWithFlags(&ev_host, hipEventDisableTiming));
    constexpr int kHostBig = 64 << 10;   // ints: a coarsest pattern of ~1600 rows x 40
    if (host_big_n < kHostBig) {
        const int rc = host_ints(kHostBig);
        if (rc != XFK_OK) return rc;
    }
    constexpr size_t kStage = 64 << 10;  // bytes: a nested-dissection plan of ~1600 rows
    if (nd_stage_n < kStage) {
        pinned_free(nd_stage);
        nd_stage = nullptr;
        nd_stage_n = 0;
        AMG_CHECK(pinned_malloc((void **)&nd_stage, kStage));
        nd_stage_n = kStage;
    }
    return XFK_OK;
}

int Amg::init(hipStream_t s)
{
    if (!host_int) AMG_CHECK(pinned_malloc((void **)&host_int, 16 * sizeof(int)));
    if (!ev_host) AMG_CHECK(hipEventCreateWithFlags(&ev_host, hipEventDisableTiming));
    if (!def_host) AMG_CHECK(pinned_malloc((void **)&def_host, kAmgDeferTotal * sizeof(int)));
    AMG_CHECK(dev_int.alloc(8));
    AMG_CHECK(def_dev.alloc(kAmgDeferTotal));
    def_n = 0;
    for (int &v : def_verify) v = 0;
    AMG_CHECK(rho.alloc(2 * kAmgMaxLevels));
    k_setup_zero<<<1, 64, 0, s>>>(def_dev.p, kAmgDeferTotal, rho.p, 2 * kAmgMaxLevels);   // (one launch, not two fills)
    if (L.empty()) L.emplace_back(new AmgLevel());
    for (auto &lv : L) {   // levels are rebuilt: none sharded until setup_dist says so
        lv->dist = false;
        lv->has16 = false;
        lv->has32 = false;
        lv->plan = HaloPlan();
        lv->ts.B = 0;
    }
    stats = AmgStats();
    dense_coarse = false;
    return XFK_OK;
}

// Hints of a fresh hierarchy, a priori from the longest fine row m (one int
// read with the pattern's length, no host check):
//   P = (I - W D^-1 A_F) P_tent on level 0: one product per entry of A's row,
//     at most m -- exact, so it is the capacity a measurement would choose;
//   MIS-2: 12 rounds per level (11-12 measured on configs[1] / configs[2]).
// The other products are measured in the first setup (a host check each):
// an a priori bound for them is 2x oversized, and a capacity carried over
// from an oversized first setup would stay so (the sort kernels over twice
// the padded rows: round 4 measured the warm setup 2.24 -> 2.64 ms with
// seeded A P and R (A P) capacities), while a capacity that changes between
// setups changes the Galerkin products' summation order, so repeated solves
// would no longer be bit-identical.  XFK_AMG_NO_SEED=1: measure everything.

// Hints across problems.  A fresh problem has no hints of its own; the last
// single-device setup of the process leaves its SpGEMM capacities, MIS-2
// round counts and the coarsest nested-dissection plan here, keyed by the
// fine level's size (the next rotor angle, the next analysis of a session:
// the same mesh family).  A fresh hierarchy of the same size takes them as
// speculation, checked on the device, never trusted: a capacity must show no
// overflow AND some row needing more than half of it (else a measurement
// would have chosen a smaller class, with another sort order: the setup is
// redone with measured capacities, so the bits are always those of the
// measured class); the round counts only size the MIS-2 batches; the plan is
// used only if the coarsest pattern equals its key (k_pattern_diff).
// XFK_AMG_NO_FOREIGN=1: fresh problems measure everything.
namespace {
struct HintStore {
    std::mutex mu;
    bool valid = false;
    int n0 = 0;
    long long nnz0 = 0;
    std::map<int, int> cap, mis;
    std::vector<int> nd_key;
    std::vector<Amg::NdPhase> nd_phases;
    int nd_ld = 0, nd_key_n = -1;
    long long nd_key_nnz = 0;
    std::vector<char> nd_plan;   // perm, iperm, tiles, masks as nd_order uploads them
    size_t nd_tl_n = 0, nd_mask_n = 0;
};
HintStore &hint_store()
{
    static HintStore *h = new HintStore();   // (never destroyed, like the device caches)
    return *h;
}
bool foreign_on()
{
    static const bool v = std::getenv("XFK_AMG_NO_FOREIGN") == nullptr;
    return v;
}
}  // namespace

}  // namespace xfk

extern "C" int xfk_amg_forget_hints(void)
{
    xfk::HintStore &h = xfk::hint_store();
    std::lock_guard<std::mutex> g(h.mu);
    h.valid = false;
    h.cap.clear();
    h.mis.clear();
    h.nd_key.clear();
    h.nd_phases.clear();
    h.nd_plan.clear();
    h.nd_key_n = -1;
    return XFK_OK;
}

namespace xfk {

void Amg::save_hints(int n0, long long nnz0)
{
    if (!foreign_on() || cap_hint.empty()) return;
    HintStore &h = hint_store();
    std::lock_guard<std::mutex> g(h.mu);
    h.valid = true;
    h.n0 = n0;
    h.nnz0 = nnz0;
    h.cap = cap_hint;
    // XFK_AMG_TEST_FOREIGN_BIG=1 (tests only): store one class too large, so
    // the next problem's device check must refuse it and rebuild
    if (std::getenv("XFK_AMG_TEST_FOREIGN_BIG"))
        for (auto &c : h.cap) c.second = std::min(2 * c.second, (int)kSortCap);
    h.mis = mis_hint;
    h.nd_key = nd_key;
    h.nd_phases = nd_phases_key;
    h.nd_ld = nd_ld;
    h.nd_key_n = nd_key_n;
    h.nd_key_nnz = nd_key_nnz;
    h.nd_plan = nd_plan;
    h.nd_tl_n = nd_tl_n;
    h.nd_mask_n = nd_mask_n;
}

int Amg::load_hints(hipStream_t s, int n0, long long nnz0)
{
    foreign = false;
    if (!foreign_on() || !cap_hint.empty() || !mis_hint.empty()) return XFK_OK;
    HintStore &h = hint_store();
    std::lock_guard<std::mutex> g(h.mu);
    if (!h.valid || h.n0 != n0 || h.nnz0 != nnz0) return XFK_OK;
    cap_hint = h.cap;
    mis_hint = h.mis;
    foreign = true;
    const size_t plan_bytes = sizeof(int) * ((size_t)h.nd_key_n + h.nd_ld + h.nd_tl_n) + h.nd_mask_n;
    if (h.nd_key_n > 0 && !h.nd_key.empty() && !h.nd_phases.empty() && h.nd_plan.size() == plan_bytes) {
        const int n = h.nd_key_n, ld = h.nd_ld;
        AMG_CHECK(cinv_perm.alloc(n));
        AMG_CHECK(cinv_iperm.alloc(ld));
        AMG_CHECK(nd_mask.alloc(h.nd_mask_n));
        AMG_CHECK(nd_tiles.alloc(h.nd_tl_n));
        const char *q = h.nd_plan.data();
        AMG_CHECK(hipMemcpyAsync(cinv_perm.p, q, sizeof(int) * n, hipMemcpyHostToDevice, s));
        AMG_CHECK(hipMemcpyAsync(cinv_iperm.p, q + sizeof(int) * n, sizeof(int) * ld, hipMemcpyHostToDevice, s));
        AMG_CHECK(hipMemcpyAsync(nd_tiles.p, q + sizeof(int) * ((size_t)n + ld), sizeof(int) * h.nd_tl_n,
                                 hipMemcpyHostToDevice, s));
        AMG_CHECK(hipMemcpyAsync(nd_mask.p, q + sizeof(int) * ((size_t)n + ld + h.nd_tl_n), h.nd_mask_n,
                                 hipMemcpyHostToDevice, s));
        nd_plan = h.nd_plan;
        nd_tl_n = h.nd_tl_n;
        nd_mask_n = h.nd_mask_n;
        nd_key = h.nd_key;
        nd_phases_key = h.nd_phases;
        nd_ld = h.nd_ld;
        nd_key_n = h.nd_key_n;
        nd_key_nnz = h.nd_key_nnz;
        AMG_CHECK(nd_key_dev.alloc(nd_key.size()));
        AMG_CHECK(hipMemcpyAsync(nd_key_dev.p, nd_key.data(), sizeof(int) * nd_key.size(), hipMemcpyHostToDevice, s));
        AMG_CHECK(hipStreamSynchronize(s));   // (the host vector is the staging buffer; a first setup only)
    }
    return XFK_OK;
}

void Amg::seed_hints()
{
    static const bool off = std::getenv("XFK_AMG_NO_SEED") != nullptr;
    if (off || row_max0 <= 0 || !cap_hint.empty() || !mis_hint.empty()) return;
    auto cap = [](long long v) { return v <= 16 ? 16 : v <= 32 ? 32 : v <= 64 ? 64 : v <= 128 ? 128 : 256; };
    if (row_max0 <= kSortCap) cap_hint[0] = cap(row_max0);
    for (int l = 0; l < kAmgMaxLevels; ++l) mis_hint[l] = 12;
}

double Amg::theta_at(int l) const
{
    static const double env = [] {
        const char *e = std::getenv("XFK_AMG_THETA_COARSE");
        return e ? std::atof(e) : -1.0;
    }();
    if (l == 0) return theta;
    if (env >= 0.0) return env;
    return theta_coarse >= 0.0 ? theta_coarse : theta;
}

int Amg::setup(hipStream_t s, int n0, int ncl0, const int *rowptr0, const int *col0, const double *val0,
               long long nnz0)
{
    dist = false;
    comm = nullptr;
    lrep = 0;
    int rc = load_hints(s, n0, nnz0);
    if (rc != XFK_OK) return rc;
    seed_hints();
    rc = init(s);
    if (rc != XFK_OK) return rc;
    AmgLevel &F = *L[0];
    F.n = n0;
    F.nnz = nnz0;
    F.ncol_lim = ncl0;
    F.ncol_smooth = ncl0;
    F.rowptr = rowptr0;
    F.col = col0;
    F.val = val0;
    rc = build(s, 0);
    if (rc == XFK_OK) {
        foreign = false;   // (verified, or rebuilt with measured capacities)
        save_hints(n0, nnz0);
    }
    return rc;
}

// MIS-2 aggregation of level l, P = (I - omega D_F^-1 A_F) P_tent and R = P^T
// (strength flags and rho_F already computed).  nc = 0 when the level does
// not coarsen usefully (allow_stop) or has no aggregate.
// T = M^T of an n x nc CSR whose rows are sorted by column (T's rows come
// out sorted by row): counting transpose, the fill counting the row counts
// back down, rows sorted by a wave bitonic network, values looked up in M.
// T's arrays hold as many entries as M (no read-back of the scan).
// cnt / tmp: scratch of the stream it runs on (the setup's side stream has its own)
// XFK_RT_TILE=0: the per-entry transpose (global atomics, values looked up after the sort)
static bool rt_tile_on()
{
    static const bool v = [] {
        const char *e = std::getenv("XFK_RT_TILE");
        return !(e && std::atoi(e) == 0);
    }();
    return v;
}

static int transpose_csr(DBuf<int> &cnt, DBuf<char> &tmp, hipStream_t s, int n, int nc, const int *mrow,
                         const int *mcol, const double *mval, int *trow, int *tcol, double *tval)
{
    AMG_CHECK(cnt.alloc((size_t)std::max(n, nc) + 1));
    AMG_CHECK(hipMemsetAsync(cnt.p, 0, sizeof(int) * ((size_t)nc + 1), s));
    const bool tiled = rt_tile_on();
    if (n > 0) {
        if (tiled) k_rt_tile<false><<<nb(n), 256, 0, s>>>(n, mrow, mcol, mval, trow, cnt.p, tcol, tval);
        else k_rt_count<<<nb(n), kB, 0, s>>>(n, mrow, mcol, cnt.p);
    }
    int rc = scan_only(tmp, s, cnt.p, trow, nc);
    if (rc != XFK_OK) return rc;
    if (tiled) {
        if (n > 0) k_rt_tile<true><<<nb(n), 256, 0, s>>>(n, mrow, mcol, mval, trow, cnt.p, tcol, tval);
        if (nc > 0) k_rt_sort_pairs<<<(int)((((long long)nc + 3) / 4 * 64 + 255) / 256), 256, 0, s>>>(nc, trow, tcol, tval);
        AMG_CHECK(hipGetLastError());
        return XFK_OK;
    }
    if (n > 0) k_rt_fill<<<nb(n), kB, 0, s>>>(n, mrow, mcol, trow, cnt.p, tcol);
    if (nc > 0)
        k_rt_sort_vals<<<(int)(((long long)nc * 64 + 255) / 256), 256, 0, s>>>(nc, trow, tcol, mrow, mcol, mval, tval);
    AMG_CHECK(hipGetLastError());
    return XFK_OK;
}

// 16-bit tile columns (xfk_spmv.h) of an n-row CSR in tiles of B rows, on st
template <int B>
static int build_col16(hipStream_t st, int n, const int *rowptr, const int *col, long long nnz,
                       DBuf<unsigned short> &c16, DBuf<int> &base)
{
    const int nt = (n + B - 1) / B;
    AMG_CHECK(c16.alloc((size_t)std::max(1LL, nnz)));
    AMG_CHECK(base.alloc((size_t)std::max(1, nt)));
    if (nt > 0) k_tile_col16<B><<<nt, 256, 0, st>>>(n, rowptr, col, c16.p, base.p);
    AMG_CHECK(hipGetLastError());
    return XFK_OK;
}

int Amg::aggregate(hipStream_t s, int l, long long &nc, bool allow_stop)
{
    AmgLevel &A = *L[l];
    const int n = A.n;
    const ColView cv{A.col, A.has16 ? A.a16.p : nullptr, A.has16 ? A.a16b.p : nullptr};
    nc = 0;
    A.nc = 0;
    AMG_CHECK(key.alloc(n));
    AMG_CHECK(t1.alloc(n));
    const std::string lv = g_prof ? "setup L" + std::to_string(l) + " " : std::string();
    if (g_prof) g_prof->begin(lv + "MIS-2 aggregation", 0.0);
    int rounds = 0;
    int *und2 = dev_int.p + 4;   // undecided flag of rounds of parity 0 / 1
    int *run = dev_int.p + 7;    // rounds that did work
    AMG_CHECK(act.alloc(n));
    k_mis_init<<<std::max(1, nb(n)), kB, 0, s>>>(n, cnt.p, key.p, und2 + 1, run, act.p);
    AMG_CHECK(flag.alloc((size_t)n + 1));
    AMG_CHECK(cursor.alloc((size_t)n + 1));
    // Batches of rounds without a host check; the first batch is the round
    // count this level needed in the last setup (the same matrix family
    // needs the same count: one host check in the usual case, no idle
    // rounds), 12 without one.  Roots and their numbering are formed
    // speculatively after each batch and read back in the same host check.
    auto hint = mis_hint.find(l);
    // speculative joins and P need a round hint and a hinted (non-synchronising) P
    // (levels of a sharded hierarchy replicated on every rank speculate like a
    // single device's: every rank holds the same level and hints, so every
    // rank takes the same decisions; sharded levels keep their host checks)
    const bool spec = spec_on() && !g_prof && !A.dist && hint != mis_hint.end() && cap_hint.count(4 * l) &&
                      def_n + 4 <= kAmgDeferSlots && !std::getenv("XFK_AMG_DEBUG");
    bool joined = false;
    auto joins_and_p = [&]() { return joins_and_p_impl(s, l); };
    AMG_CHECK(mis_out.alloc(4));
    for (int batch = hint != mis_hint.end() ? std::max(1, hint->second) : 12;; batch = 2) {
        for (int b = 0; b < batch; ++b, ++rounds) {
            int *cur = und2 + (rounds & 1), *prev = und2 + ((rounds + 1) & 1);
            const bool last = b + 1 == batch;   // its update also writes the root flags
            const int xc = mis_xcd_on() ? 1 : 0;
            if (A.nnz > 9LL * n) {
                k_mis_max<4><<<nb(4LL * n), kB, 0, s>>>(n, A.rowptr, cv, sflag.p, key.p, t1.p, prev, cur, run,
                                                         act.p, xc);
                if (last)
                    k_mis_update<4, true><<<nb(4LL * n), kB, 0, s>>>(n, A.rowptr, cv, sflag.p, t1.p, key.p, prev, cur,
                                                                      flag.p, xc);
                else
                    k_mis_update<4><<<nb(4LL * n), kB, 0, s>>>(n, A.rowptr, cv, sflag.p, t1.p, key.p, prev, cur,
                                                                nullptr, xc);
            } else {
                k_mis_max<1><<<nb(n), kB, 0, s>>>(n, A.rowptr, cv, sflag.p, key.p, t1.p, prev, cur, run, act.p, xc);
                if (last)
                    k_mis_update<1, true><<<nb(n), kB, 0, s>>>(n, A.rowptr, cv, sflag.p, t1.p, key.p, prev, cur,
                                                                flag.p, xc);
                else
                    k_mis_update<1><<<nb(n), kB, 0, s>>>(n, A.rowptr, cv, sflag.p, t1.p, key.p, prev, cur, nullptr,
                                                          xc);
            }
        }
        int rc = scan_only(*this, s, flag.p, cursor.p, n);   // cursor = root ids
        if (rc != XFK_OK) return rc;
        k_mis_pack<<<1, 64, 0, s>>>(cursor.p + n, und2 + ((rounds - 1) & 1), run, mis_out.p);
        AMG_CHECK(hipMemcpyAsync(host_int + 8, mis_out.p, 3 * sizeof(int), hipMemcpyDeviceToHost, s));
        AMG_CHECK(hipEventRecord(ev_host, s));
        // while the host waits for the check, the device goes on with the
        // joins and P (correct when the check finds the MIS complete -- the
        // usual case with a round hint; otherwise redone after more rounds)
        joined = spec;
        if (spec && (rc = joins_and_p()) != XFK_OK) return rc;
        AMG_CHECK(hipEventSynchronize(ev_host));
        if (!host_int[9]) break;
        joined = false;
        if (rounds > 4096) {
            set_error("AMG: MIS-2 aggregation did not terminate");
            return XFK_ERR_NOCONV;
        }
    }
    mis_hint[l] = host_int[10];
    nc = host_int[8];
    stats.mis_rounds[l] = host_int[10];
    int rc = XFK_OK;
    if (allow_stop && (nc == 0 || nc > (long long)(0.9 * n))) {   // no useful coarsening: smoother-only coarsest
        nc = 0;
        return XFK_OK;
    }
    if (!joined && (rc = joins_and_p()) != XFK_OK) return rc;
    A.nc = (int)nc;
    if (std::getenv("XFK_AMG_DEBUG")) std::fprintf(stderr, "[amg] level %d P nnz %lld\n", l, A.pnnz);
    // R = P^T: on the side stream (single-device levels) while the main
    // stream forms A P; the Galerkin product R (A P) waits for it
    AMG_CHECK(A.rrow.alloc((size_t)nc + 1));
    AMG_CHECK(A.rcol.alloc((size_t)std::max(1LL, A.pnnz)));
    AMG_CHECK(A.rval.alloc((size_t)std::max(1LL, A.pnnz)));
    const bool off = side_setup_on() && !A.dist && !dist;
    hipStream_t ts = s;
    if (off) {
        if ((rc = sw.init()) != XFK_OK) return rc;
        AMG_CHECK(hipEventRecord(sw.a, s));
        AMG_CHECK(hipStreamWaitEvent(sw.cs, sw.a, 0));
        ts = sw.cs;
        sw_used = true;
    }
    if ((rc = transpose_csr(off ? cnt2 : cnt, off ? cub_tmp2 : cub_tmp, ts, n, (int)nc, A.prow.p, A.pcol.p,
                            A.pval.p, A.rrow.p, A.rcol.p, A.rval.p)) != XFK_OK)
        return rc;
    if (off) {   // R (A P) waits for R itself; R's V-cycle forms below are joined at the end of the build
        AMG_CHECK(hipEventRecord(sw.b, sw.cs));
        rt_pending = true;
    }
    if (l == 0 && A.has16 && (rc = build_col16<256>(ts, (int)nc, A.rrow.p, A.rcol.p, A.pnnz, A.r16, A.r16b)) != XFK_OK)
        return rc;
    if (l == 0 && A.has32 &&
        ((rc = to_f32(ts, (int)nc, A.rrow.p, A.pnnz, A.rval.p, A.r32)) != XFK_OK ||
         (f32_sweep_on() && (rc = to_f32(ts, n, A.rowptr, A.nnz, A.val, A.a32)) != XFK_OK)))
        return rc;
    if (l == 0 && A.has32 && A.dist &&   // the sharded level 0 prolongs through P itself (no fold)
        ((rc = to_f32(ts, n, A.prow.p, A.pnnz, A.pval.p, A.p32)) != XFK_OK ||
         (rc = build_col16<256>(ts, n, A.prow.p, A.pcol.p, A.pnnz, A.p16, A.p16b)) != XFK_OK))
        return rc;
    if (g_prof) g_prof->end();
    return XFK_OK;
}

// joins of the MIS-2 roots' neighbourhoods (agg), then P = (I - omega D_F^-1 A_F) P_tent
int Amg::joins_and_p_impl(hipStream_t s, int l)
{
    AmgLevel &A = *L[l];
    const int n = A.n;
    const ColView cv{A.col, A.has16 ? A.a16.p : nullptr, A.has16 ? A.a16b.p : nullptr};
    const std::string lv = g_prof ? "setup L" + std::to_string(l) + " " : std::string();
    AMG_CHECK(agg1.alloc(n));
    AMG_CHECK(agg.alloc(n));
    // lanes per row for the joins (XFK_JOIN_LANES: 1 = one thread per row)
    const int jg = join_lanes((double)A.nnz / std::max(1, n));
    auto joins = [&](auto g) {
        constexpr int G = decltype(g)::value;
        const int blocks = nb((long long)n * G);
        k_agg_join1<G><<<blocks, kB, 0, s>>>(n, A.rowptr, cv, sflag.p, key.p, cursor.p, agg1.p);
        k_agg_join2<G><<<blocks, kB, 0, s>>>(n, A.rowptr, cv, sflag.p, key.p, agg1.p, agg.p);
        k_agg_join3<G><<<blocks, kB, 0, s>>>(n, A.ncol_lim, A.rowptr, cv, A.val, agg.p, agg1.p);
    };
    if (jg == 8) joins(std::integral_constant<int, 8>{});
    else if (jg == 4) joins(std::integral_constant<int, 4>{});
    else joins(std::integral_constant<int, 1>{});
    std::swap(agg.p, agg1.p);   // agg = the joined map
    std::swap(agg.n, agg1.n);
    if (g_prof) g_prof->end();
    if (std::getenv("XFK_AMG_DEBUG")) {
        DBuf<int> d;
        AMG_CHECK(d.alloc(3));
        AMG_CHECK(hipMemsetAsync(d.p, 0, 3 * sizeof(int), s));
        k_debug_unagg<<<nb(n), kB, 0, s>>>(n, A.rowptr, A.col, cnt.p, agg.p, d.p);
        int h[3];
        unsigned long long r2[2];
        AMG_CHECK(hipMemcpyAsync(h, d.p, sizeof(h), hipMemcpyDeviceToHost, s));
        AMG_CHECK(hipMemcpyAsync(r2, rho.p + 2 * l, sizeof(r2), hipMemcpyDeviceToHost, s));
        AMG_CHECK(hipStreamSynchronize(s));
        double ra, rf;
        std::memcpy(&ra, &r2[0], 8);
        std::memcpy(&rf, &r2[1], 8);
        std::fprintf(stderr, "[amg] rank %d level %d n %d nnz %lld nc %lld unaggregated: strong %d weak-only %d isolated %d "
                     "rhoA/omega %.4g rhoF %.4g mis_rounds %d\n", dist ? rank : 0, l, n, A.nnz, (long long)host_int[8], h[0], h[1],
                     h[2], ra, rf, host_int[10]);
    }
    // P = (I - omega D_F^-1 A_F) P_tent
    SgX XS{A.rowptr, A.col, A.val, A.ncol_lim, sflag.p, dfinv.p, wF.p, cv.c16, cv.cbase};
    SgY YT{nullptr, nullptr, nullptr, agg.p};
    if (g_prof) g_prof->begin(lv + "P = (I - w D^-1 A) P_tent, R = P^T", 0.0);
    // (a sharded level needs P's length on the host at once -- the halo rows'
    // plan -- so it takes its capacity hint without deferring the length)
    return spgemm<true>(*this, s, n, XS, YT, A.prow, A.pcol, A.pval, A.pnnz, 4 * l, !A.dist);
}

// Nested-dissection order of the coarsest level for the dense inverse: a
// recursive bisection -- left = the first half of the rows (the levels are
// numbered along the fine level's Cuthill-McKee order, so the halves are
// banded slabs), right = the other rows without an entry in the left half,
// separator = those with one (about one grid line).  Two tree levels give
// four leaves (four pivot chains per launch), then their two separators,
// then the top separator; one level two leaves.  Groups are padded with
// identity rows to whole blocks, the groups of one phase to equal block
// counts.  Falls back to one level, then to the plain order, when a
// separator would be empty or hold more than a quarter of the rows.
// Host-synchronising (the coarsest level has <= dense_max rows).
namespace {
void nd_split_at(const std::vector<int> &rp, const std::vector<int> &cl, const std::vector<int> &rows, size_t h,
                 std::vector<char> &inl, std::vector<int> &L, std::vector<int> &R, std::vector<int> &S)
{
    L.assign(rows.begin(), rows.begin() + h);
    R.clear();
    S.clear();
    for (int r : L) inl[r] = 1;
    for (size_t t = h; t < rows.size(); ++t) {
        const int r = rows[t];
        bool cross = false;
        for (int k = rp[r]; k < rp[r + 1] && !cross; ++k) cross = inl[cl[k]] != 0;
        (cross ? S : R).push_back(r);
    }
    for (int r : L) inl[r] = 0;
}
// split position chosen so that the two parts (not counting the separator)
// come out about equal: the chain length of a phase is its largest part
void nd_bisect(const std::vector<int> &rp, const std::vector<int> &cl, const std::vector<int> &rows,
               std::vector<char> &inl, std::vector<int> &L, std::vector<int> &R, std::vector<int> &S)
{
    nd_split_at(rp, cl, rows, rows.size() / 2, inl, L, R, S);
    const size_t h = (rows.size() - S.size()) / 2;
    if (h > 0 && h != rows.size() / 2) nd_split_at(rp, cl, rows, h, inl, L, R, S);
}
}  // namespace

int Amg::nd_order(hipStream_t s, const AmgLevel &C, int &ld)
{
    const int n = C.n;
    nd_phases.clear();
    ld = ((n + kBj - 1) / kBj) * kBj;
    if (n < 8 * kBj || std::getenv("XFK_NO_ND")) {
        nd_key_n = -1;
        return XFK_OK;
    }
    // the pattern through pinned memory; an unchanged pattern (the next setup
    // of the same matrix family) keeps the plan and its device arrays
    const size_t npat = (size_t)n + 1 + (size_t)C.nnz;
    {
        int rc = host_ints((int)npat);
        if (rc != XFK_OK) return rc;
        AMG_CHECK(hipMemcpyAsync(host_big, C.rowptr, sizeof(int) * (n + 1), hipMemcpyDeviceToHost, s));
        AMG_CHECK(hipMemcpyAsync(host_big + n + 1, C.col, sizeof(int) * C.nnz, hipMemcpyDeviceToHost, s));
        AMG_CHECK(hipStreamSynchronize(s));
    }
    if (nd_key.size() == npat && std::equal(nd_key.begin(), nd_key.end(), host_big)) {
        nd_phases = nd_phases_key;
        ld = nd_ld;
        return XFK_OK;
    }
    nd_key.assign(host_big, host_big + npat);
    // the device copy of the key: the next setup compares its coarsest
    // pattern on the device and applies this plan without a host read
    AMG_CHECK(nd_key_dev.alloc(npat));
    AMG_CHECK(hipMemcpyAsync(nd_key_dev.p, C.rowptr, sizeof(int) * (n + 1), hipMemcpyDeviceToDevice, s));
    AMG_CHECK(hipMemcpyAsync(nd_key_dev.p + n + 1, C.col, sizeof(int) * C.nnz, hipMemcpyDeviceToDevice, s));
    nd_key_n = n;
    nd_key_nnz = C.nnz;
    nd_phases_key.clear();
    nd_ld = ld;
    std::vector<int> rp(host_big, host_big + n + 1), cl(host_big + n + 1, host_big + npat);
    for (int r = 0; r < n; ++r)   // columns >= n (none on a level built here) are dropped by the scatter
        for (int k = rp[r]; k < rp[r + 1]; ++k) cl[k] = std::min(cl[k], n);
    std::vector<char> inl(n + 1, 0);
    std::vector<int> all(n);
    for (int r = 0; r < n; ++r) all[r] = r;
    // groups: rows, phase, slot in the phase, parent separator group, subtree groups
    struct G {
        std::vector<int> rows;
        int phase, slot, parent;
        std::vector<int> sub;
    };
    std::vector<G> g;
    // the deepest bisection (3, 2, then 1 level) whose groups are all non-empty,
    // whose separators hold at most a quarter of the rows, and whose leaves
    // keep >= 1 block; leaves are phase 0 (slots = leaf index), the
    // separators of bisection level lev are phase D - lev
    // The bisection levels are computed once: nd_bisect is a function of its
    // set, so the first D levels of a deeper bisection are the D-level one and
    // every depth reads the same splits (no recomputation per depth tried)
    const int Dmax = n >= 24 * kBj ? 3 : (n >= 16 * kBj ? 2 : 1);
    std::vector<std::vector<std::vector<int>>> lev_sets(Dmax + 1), lev_seps(Dmax);
    std::vector<size_t> lev_nsep(Dmax, 0);
    int lev_done = 0;   // levels computed, each with all its groups non-empty
    lev_sets[0].push_back(all);
    for (int lev = 0; lev < Dmax; ++lev) {
        bool okl = true;
        for (const auto &x : lev_sets[lev]) {
            std::vector<int> L, R, S;
            nd_bisect(rp, cl, x, inl, L, R, S);
            okl = okl && !L.empty() && !R.empty() && !S.empty();
            lev_nsep[lev] += S.size();
            lev_sets[lev + 1].push_back(std::move(L));
            lev_sets[lev + 1].push_back(std::move(R));
            lev_seps[lev].push_back(std::move(S));
        }
        if (!okl) break;
        lev_done = lev + 1;
    }
    for (int D = Dmax; D >= 1 && g.empty(); --D) {
        bool ok = lev_done >= D;
        size_t nsep = 0;
        for (int lev = 0; lev < D && lev < Dmax; ++lev) nsep += lev_nsep[lev];
        const std::vector<std::vector<int>> &sets = lev_sets[std::min(D, lev_done + 1)];
        const std::vector<std::vector<std::vector<int>>> &seps = lev_seps;
        if (std::getenv("XFK_AMG_DEBUG")) {
            std::fprintf(stderr, "[amg] nested dissection depth %d: ok %d separators %zu, sets", D, (int)ok, nsep);
            for (const auto &x : sets) std::fprintf(stderr, " %zu", x.size());
            std::fprintf(stderr, "\n");
        }
        // (XFK_ND_DEPTH: this depth whatever its separators -- measurement hook)
        const char *fd = std::getenv("XFK_ND_DEPTH");
        if (fd && std::atoi(fd) != D) continue;
        if (!ok || (!fd && 3 * nsep > (size_t)n)) continue;
        if (D > 1)
            for (const auto &x : sets) ok = ok && x.size() >= (size_t)kBj;
        if (!ok) continue;
        // group indices: leaves 0 .. 2^D - 1, then separators by level, deepest first
        const int nl = 1 << D;
        std::vector<int> sep_at(D);   // first group index of level lev's separators
        int q = nl;
        for (int lev = D - 1; lev >= 0; --lev) {
            sep_at[lev] = q;
            q += 1 << lev;
        }
        g.resize(q);
        for (int k = 0; k < nl; ++k)
            g[k] = {sets[k], 0, k, sep_at[D - 1] + (k >> 1), {k}};
        for (int lev = D - 1; lev >= 0; --lev)
            for (int m = 0; m < (1 << lev); ++m) {
                G &x = g[sep_at[lev] + m];
                x.rows = seps[lev][m];
                x.phase = D - lev;
                x.slot = m;
                x.parent = lev > 0 ? sep_at[lev - 1] + (m >> 1) : -1;
                // subtree: leaves and deeper separators under this one, and itself
                for (int k = 0; k < nl; ++k)
                    if ((k >> (D - lev)) == m) x.sub.push_back(k);
                for (int l2 = lev + 1; l2 < D; ++l2)
                    for (int m2 = 0; m2 < (1 << l2); ++m2)
                        if ((m2 >> (l2 - lev)) == m) x.sub.push_back(sep_at[l2] + m2);
                x.sub.push_back(sep_at[lev] + m);
            }
    }
    if (g.empty()) return XFK_OK;
    if (std::getenv("XFK_AMG_DEBUG")) {
        std::fprintf(stderr, "[amg] coarsest %d rows: nested dissection, %d groups:", n, (int)g.size());
        for (const G &x : g) std::fprintf(stderr, " %d/%d", (int)x.rows.size(), x.phase);
        std::fprintf(stderr, "\n");
    }
    const int nph = g.back().phase + 1;
    // blocks: each phase's groups padded to the phase's largest group
    std::vector<int> pblk(nph, 0), b0(g.size());
    for (const G &x : g) pblk[x.phase] = std::max(pblk[x.phase], (int)((x.rows.size() + kBj - 1) / kBj));
    int nbk = 0;
    for (size_t q = 0; q < g.size(); ++q) {
        b0[q] = nbk;
        nbk += pblk[g[q].phase];
    }
    ld = nbk * kBj;
    std::vector<int> perm(n), iperm(ld, -1);
    for (size_t q = 0; q < g.size(); ++q)
        for (size_t t = 0; t < g[q].rows.size(); ++t) {
            perm[g[q].rows[t]] = b0[q] * kBj + (int)t;
            iperm[b0[q] * kBj + (int)t] = g[q].rows[t];
        }
    // per phase: region masks (bit = slot) and the tiles some chain holds
    std::vector<unsigned char> mask((size_t)nph * nbk, 0);
    std::vector<int> tl;
    for (int ph = 0; ph < nph; ++ph) {
        unsigned char *m = mask.data() + (size_t)ph * nbk;
        NdPhase P{};
        P.steps = pblk[ph];
        for (size_t q = 0; q < g.size(); ++q) {
            if (g[q].phase != ph) continue;
            P.base[g[q].slot] = b0[q];
            P.nch = std::max(P.nch, g[q].slot + 1);
            P.next_slot[g[q].slot] = g[q].parent >= 0 ? g[g[q].parent].slot : -1;
            std::vector<int> reg = g[q].sub;
            for (int a = g[q].parent; a >= 0; a = g[a].parent) reg.push_back(a);
            for (int x : reg)
                for (int bb = 0; bb < pblk[g[x].phase]; ++bb) m[b0[x] + bb] |= (unsigned char)(1u << g[q].slot);
        }
        P.tiles_off = (int)tl.size();
        for (int i = 0; i < nbk; ++i)
            for (int j = 0; j < nbk; ++j)
                if (m[i] & m[j]) tl.push_back(i * nbk + j);
        P.ntiles = (int)tl.size() - P.tiles_off;
        nd_phases.push_back(P);
    }
    AMG_CHECK(cinv_perm.alloc(n));
    AMG_CHECK(cinv_iperm.alloc(ld));
    AMG_CHECK(nd_mask.alloc(mask.size()));
    AMG_CHECK(nd_tiles.alloc(tl.size()));
    // uploads from a pinned staging copy (no host check: the staging buffer
    // is rewritten only after the next setup's synchronising pattern read)
    const size_t bytes = sizeof(int) * ((size_t)n + ld + tl.size()) + mask.size();
    if (nd_stage_n < bytes) {
        pinned_free(nd_stage);   // (outside a destroy: hipHostFree)
        nd_stage = nullptr;
        nd_stage_n = 0;
        AMG_CHECK(pinned_malloc((void **)&nd_stage, bytes));
        nd_stage_n = bytes;
    }
    char *h = nd_stage;
    std::memcpy(h, perm.data(), sizeof(int) * n);
    std::memcpy(h + sizeof(int) * n, iperm.data(), sizeof(int) * ld);
    std::memcpy(h + sizeof(int) * ((size_t)n + ld), tl.data(), sizeof(int) * tl.size());
    std::memcpy(h + sizeof(int) * ((size_t)n + ld + tl.size()), mask.data(), mask.size());
    if (foreign_on()) {   // (the plan's device arrays for the next fresh problem of this size)
        nd_plan.assign(h, h + bytes);
        nd_tl_n = tl.size();
        nd_mask_n = mask.size();
    }
    AMG_CHECK(hipMemcpyAsync(cinv_perm.p, h, sizeof(int) * n, hipMemcpyHostToDevice, s));
    AMG_CHECK(hipMemcpyAsync(cinv_iperm.p, h + sizeof(int) * n, sizeof(int) * ld, hipMemcpyHostToDevice, s));
    AMG_CHECK(hipMemcpyAsync(nd_tiles.p, h + sizeof(int) * ((size_t)n + ld), sizeof(int) * tl.size(),
                             hipMemcpyHostToDevice, s));
    AMG_CHECK(hipMemcpyAsync(nd_mask.p, h + sizeof(int) * ((size_t)n + ld + tl.size()), mask.size(),
                             hipMemcpyHostToDevice, s));
    nd_phases_key = nd_phases;
    nd_ld = ld;
    return XFK_OK;
}

// the dense coarsest inverse of C in the order nd_phases / cinv_perm give
// (ld: the padded size of that order)
int Amg::dense_inverse(hipStream_t s, const AmgLevel &C, int ld)
{
    const bool nd = !nd_phases.empty();
    const int nbk = ld / kBj;
    cinv_ld = ld;
    AMG_CHECK(cinv.alloc((size_t)ld * ld));
    const size_t T2 = (size_t)kBj * kBj;
    // per chain slot and parity: row / column snapshots and the pivot inverse
    const size_t per = 2 * (size_t)nbk * T2 + T2;
    AMG_CHECK(bgj_tmp.alloc(2 * kNdChains * per + 1 + ld));
    auto Rb = [&](int c, int q) { return bgj_tmp.p + (size_t)(2 * c + q) * per; };
    auto Cb = [&](int c, int q) { return Rb(c, q) + (size_t)nbk * T2; };
    auto Db = [&](int c, int q) { return Rb(c, q) + 2 * (size_t)nbk * T2; };
    double *maxd = bgj_tmp.p + 2 * kNdChains * per, *sc = maxd + 1;
    const int *pm = nd ? cinv_perm.p : nullptr, *ipm = nd ? cinv_iperm.p : nullptr;
    AMG_CHECK(hipMemsetAsync(cinv.p, 0, sizeof(double) * (size_t)ld * ld, s));
    k_dense_dscale<<<nb((long long)ld * kDsG), kB, 0, s>>>(C.n, ld, C.rowptr, C.col, C.val, ipm, sc);
    k_dense_scatter<<<nb((long long)ld * kDsG), kB, 0, s>>>(C.n, ld, C.rowptr, C.col, C.val, pm, ipm, sc, cinv.p);
    k_dense_maxdiag<<<1, 1024, 0, s>>>(ld, ld, cinv.p, maxd);
    // (a lookahead variant -- block column k+1 first, its pivot block
    // inverted on a second stream during the rest of the update -- was
    // measured slower: the two cross-stream waits cost ~15 us per step,
    // more than the 25 us pivot-block inversion it hides)
    if (nd) {
        int par = 0;
        BgjStep st{};
        st.nn = nd_phases[0].nch;
        for (int c = 0; c < st.nn; ++c) {
            st.nx[c] = nd_phases[0].base[c];
            st.Dn[c] = Db(c, 0);
            st.Rn[c] = Rb(c, 0);
            st.Cn[c] = Cb(c, 0);
        }
        k_bgj_init<<<st.nn * (1 + 2 * nbk), 256, 0, s>>>(nbk, ld, cinv.p, st, maxd, bgj_inv_mode());
        for (size_t ph = 0; ph < nd_phases.size(); ++ph) {
            const NdPhase &P = nd_phases[ph];
            for (int t = 0; t < P.steps; ++t) {
                const int pp = par, qq = par ^ 1;
                BgjStep x{};
                x.n = P.nch;
                for (int c = 0; c < P.nch; ++c) {
                    x.k[c] = P.base[c] + t;
                    x.D[c] = Db(c, pp);
                    x.R[c] = Rb(c, pp);
                    x.C[c] = Cb(c, pp);
                }
                if (t + 1 < P.steps) {
                    x.nn = P.nch;
                    for (int c = 0; c < P.nch; ++c) x.nx[c] = P.base[c] + t + 1;
                } else if (ph + 1 < nd_phases.size()) {
                    const NdPhase &Q = nd_phases[ph + 1];
                    x.nn = Q.nch;
                    for (int c = 0; c < Q.nch; ++c) x.nx[c] = Q.base[c];
                }
                for (int c = 0; c < x.nn; ++c) {
                    x.Dn[c] = Db(c, qq);
                    x.Rn[c] = Rb(c, qq);
                    x.Cn[c] = Cb(c, qq);
                }
                k_bgj_multi<<<P.ntiles + x.nn, 256, 0, s>>>(nbk, ld, cinv.p, x, nd_mask.p + ph * (size_t)nbk,
                                                            nd_tiles.p + P.tiles_off, maxd, bgj_inv_mode());
                par = qq;
            }
        }
    } else {
        BgjStep st{};
        st.nn = 1;
        st.nx[0] = 0;
        st.Dn[0] = Db(0, 0);
        st.Rn[0] = Rb(0, 0);
        st.Cn[0] = Cb(0, 0);
        k_bgj_init<<<1 + 2 * nbk, 256, 0, s>>>(nbk, ld, cinv.p, st, maxd, bgj_inv_mode());
        for (int k = 0; k < nbk; ++k) {
            const int p = k & 1, q = (k + 1) & 1;
            k_bgj_step<<<nbk * nbk, 256, 0, s>>>(k, nbk, ld, cinv.p, Db(0, p), Rb(0, p), Cb(0, p), Db(0, q),
                                                 Rb(0, q), Cb(0, q), maxd, bgj_inv_mode());
        }
    }
    {
        const int ldo = ((C.n + kBj - 1) / kBj) * kBj;
        const dim3 g(ld / 64, ld / 64);
        AMG_CHECK(cinv_sc.alloc((size_t)ldo));
        cinv_f64 = !(prec32 < 0 ? f32_on() : prec32 != 0);   // (f64 transfers: the f64 inverse too)
        if (cinv_f64) {
            AMG_CHECK(cinv_o64.alloc((size_t)ldo * ldo));
            AMG_CHECK(hipMemsetAsync(cinv_o64.p, 0, sizeof(double) * (size_t)ldo * ldo, s));   // (padding columns)
            k_dense_unperm<double><<<g, 256, 0, s>>>(C.n, ld, ldo, cinv.p, sc, nd ? cinv_iperm.p : nullptr,
                                                     cinv_o64.p, cinv_sc.p);
        } else {
            AMG_CHECK(cinv_o.alloc((size_t)ldo * ldo));
            AMG_CHECK(hipMemsetAsync(cinv_o.p, 0, sizeof(float) * (size_t)ldo * ldo, s));
            k_dense_unperm<float><<<g, 256, 0, s>>>(C.n, ld, ldo, cinv.p, sc, nd ? cinv_iperm.p : nullptr, cinv_o.p,
                                                    cinv_sc.p);
        }
        cinv_apply = cinv_o.p;
        cinv_ld = ldo;
    }
    return XFK_OK;
}

// the V-cycle's per-level vectors
int Amg::alloc_vectors()
{
    for (int k = 0; k < nlev; ++k) {
        AmgLevel &A = *L[k];
        const size_t nv = (size_t)std::max(1, std::max(A.n, A.ncol_smooth));
        AMG_CHECK(A.xa.alloc(nv));
        AMG_CHECK(A.xb.alloc(nv));
        AMG_CHECK(A.r.alloc((size_t)std::max(1, A.n)));
        if (k > 0) AMG_CHECK(A.b.alloc((size_t)std::max(1, A.n)));
    }
    return XFK_OK;
}

// levels l0.. of the hierarchy (L[l0] set up by the caller), then the
// smoother vectors and the dense coarsest inverse
int Amg::build(hipStream_t s, int l0)
{
    int l = l0;
    for (;; ++l) {
        AmgLevel &A = *L[l];
        const int n = A.n;
        stats.n[l] = n;
        stats.nnz[l] = A.nnz;
        A.nc = 0;
        AMG_CHECK(A.dinv.alloc(n));
        AMG_CHECK(absd.alloc(n));
        AMG_CHECK(dfinv.alloc(n));
        AMG_CHECK(wF.alloc(n));
        AMG_CHECK(cnt.alloc((size_t)n + 1));
        const std::string lv = g_prof ? "setup L" + std::to_string(l) + " " : std::string();
        if (g_prof) g_prof->begin(lv + "diagonal, strength, rho", 0.0);
        k_amg_diag<<<nb(n), kB, 0, s>>>(n, A.rowptr, A.col, A.val, absd.p, A.dinv.p);
        if (n <= dense_max) {
            if (g_prof) g_prof->end();
            dense_coarse = true;
            break;
        }
        // level 0 (single device): 16-bit tile columns of A for the SpMV and
        // the sweeps, built off the critical path (they are read from the
        // first V-cycle on, after the join at the end of the build)
        A.has16 = l == 0 && !A.dist && !dist && (col16 < 0 ? col16_on() : col16 != 0);
        A.has32 = A.has16 && (prec32 < 0 ? f32_on() : prec32 != 0);
        if (A.has16) {   // (on the main stream: the aggregation reads them too)
            int rc0 = build_col16<kCgBlock>(s, n, A.rowptr, A.col, A.nnz, A.a16, A.a16b);
            if (rc0 != XFK_OK) return rc0;
        }
        AMG_CHECK(sflag.alloc((size_t)A.nnz));
        AMG_CHECK(rho_part.alloc(2 * (size_t)nb_str(n)));
        k_amg_strength<<<nb_str(n), kB, 0, s>>>(n, A.ncol_lim, theta_at(l), A.rowptr,
                                                ColView{A.col, A.has16 ? A.a16.p : nullptr, A.has16 ? A.a16b.p : nullptr},
                                                A.val, absd.p, A.dinv.p, sflag.p, cnt.p,
                                                dfinv.p, wF.p, rho_part.p, signed_strength());
        k_max_reduce<<<1, kMaxReduceT, 0, s>>>(nb_str(n), rho_part.p, omega, rho.p + 2 * l);
        if (g_prof) g_prof->end();
        if (l == kAmgMaxLevels - 1) break;   // smoother-only coarsest level
        long long nc = 0;
        int rc = aggregate(s, l, nc, true);
        if (rc != XFK_OK) return rc;
        if (nc == 0) break;
        // AP = A P, then A_c = R (A P)
        SgX XA{A.rowptr, A.col, A.val, A.ncol_lim, nullptr, nullptr, nullptr, A.has16 ? A.a16.p : nullptr,
               A.has16 ? A.a16b.p : nullptr};
        SgY YP{A.prow.p, A.pcol.p, A.pval.p, nullptr};
        if (fold_pending) {   // the previous level's folded transfer still reads A P's buffers
            AMG_CHECK(hipStreamWaitEvent(s, sw.c, 0));
            fold_pending = false;
        }
        if (g_prof) g_prof->begin(lv + "SpGEMM A P", 0.0);
        // A P's row pointers go straight to the level (they are P~'s when it
        // folds): no copy before the next level reuses the A P buffers
        rc = spgemm<false>(*this, s, n, XA, YP, A.ftrow, ap_col, ap_val, ap_nnz, 4 * l + 1);
        if (g_prof) g_prof->end();
        if (rc != XFK_OK) return rc;
        if ((int)L.size() <= l + 1) L.emplace_back(new AmgLevel());
        AmgLevel &C = *L[l + 1];
        SgX XR{A.rrow.p, A.rcol.p, A.rval.p, INT_MAX, nullptr, nullptr, nullptr};
        SgY YAP{A.ftrow.p, ap_col.p, ap_val.p, nullptr};
        if (rt_pending) {   // R = P^T from the side stream
            AMG_CHECK(hipStreamWaitEvent(s, sw.b, 0));
            rt_pending = false;
        }
        if (g_prof) g_prof->begin(lv + "SpGEMM R (A P)", 0.0);
        rc = spgemm<false>(*this, s, (int)nc, XR, YAP, C.rowptr_o, C.col_o, C.val_o, C.nnz, 4 * l + 2);
        if (g_prof) g_prof->end();
        if (rc != XFK_OK) return rc;
        // folded level (l >= 1): P~ from A P before the next level reuses its buffers
        A.fold = (fold_on < 0 ? fold_levels() : fold_on != 0) && sweeps == 1 && !A.dist;
        A.fold_formed = A.fold;
        if (A.fold) {
            if (g_prof) g_prof->begin(lv + "folded transfer P~ = (I - w D^-1 A) P, R~ = P~^T", 0.0);
            A.fnnz = ap_nnz;   // an upper bound while the A P length is deferred
            AMG_CHECK(A.ftrow.alloc((size_t)n + 1));
            AMG_CHECK(A.ftcol.alloc((size_t)std::max(1LL, ap_nnz)));
            AMG_CHECK(A.ftval.alloc((size_t)std::max(1LL, ap_nnz)));
            if (l > 0) {
                AMG_CHECK(A.frrow.alloc((size_t)nc + 1));
                AMG_CHECK(A.frcol.alloc((size_t)std::max(1LL, ap_nnz)));
                AMG_CHECK(A.frval.alloc((size_t)std::max(1LL, ap_nnz)));
            }
            // P~ and R~ on the side stream: only the V-cycle reads them; the
            // next level's A P (which reuses A P's buffers) waits for P~
            const bool off = side_setup_on();
            hipStream_t fs = s;
            if (off) {
                if ((rc = sw.init()) != XFK_OK) return rc;
                AMG_CHECK(hipEventRecord(sw.a, s));
                AMG_CHECK(hipStreamWaitEvent(sw.cs, sw.a, 0));
                fs = sw.cs;
                sw_used = true;
            }
            if (n > 0)
                k_fold_p<<<(int)(((long long)n * kFoldLanes + 255) / 256), 256, 0, fs>>>(
                    n, rho.p + 2 * l, A.dinv.p, A.ftrow.p, ap_col.p, ap_val.p, A.prow.p, A.pcol.p, A.pval.p, A.ftcol.p,
                    A.ftval.p);
            if (l == 0 && A.has16 &&
                (rc = build_col16<kCgBlock>(fs, n, A.ftrow.p, A.ftcol.p, ap_nnz, A.f16, A.f16b)) != XFK_OK)
                return rc;
            if (l == 0 && A.has32 && (rc = to_f32(fs, n, A.ftrow.p, ap_nnz, A.ftval.p, A.f32v)) != XFK_OK) return rc;
            if (off) {
                AMG_CHECK(hipEventRecord(sw.c, sw.cs));
                fold_pending = true;
            }
            // level 0 folds only its post-step (its pre-step keeps R r'): no R~
            if (l > 0)
                rc = transpose_csr(off ? cnt2 : cnt, off ? cub_tmp2 : cub_tmp, fs, n, (int)nc, A.ftrow.p, A.ftcol.p,
                                   A.ftval.p, A.frrow.p, A.frcol.p, A.frval.p);
            if (rc != XFK_OK) return rc;
            // the exact length picks the V-cycle's lanes per row (and so the
            // summation order): from a deferred slot when A P's length is
            // deferred too, so hinted and measured setups agree bit for bit
            if (def_n > 0 && def_n + 2 <= kAmgDeferSlots) {
                AMG_CHECK(hipMemcpyAsync(def_dev.p + def_n + 1, A.ftrow.p + n, sizeof(int), hipMemcpyDeviceToDevice, s));
                def_target[def_n / 2] = &A.fnnz;
                def_n += 2;
            } else if (def_n > 0) {
                int len = 0;
                AMG_CHECK(hipMemcpyAsync(&len, A.ftrow.p + n, sizeof(int), hipMemcpyDeviceToHost, s));
                AMG_CHECK(hipStreamSynchronize(s));
                A.fnnz = len;
            }
            if (g_prof) g_prof->end();
        }
        C.n = (int)nc;
        C.ncol_lim = (int)nc;
        C.ncol_smooth = (int)nc;
        C.rowptr = C.rowptr_o.p;
        C.col = C.col_o.p;
        C.val = C.val_o.p;
    }
    nlev = l + 1;
    {
        // the SpGEMM lengths taken without a host check (capacity hints); an
        // overflow means a hint was too small: rebuild with measured capacities.
        // The dense coarsest inverse needs the nested-dissection plan, which
        // the host makes from the coarsest pattern; when the pattern equals
        // the one the cached plan was made for (compared on the device, read
        // with the deferred lengths), the inverse launched ahead of that read
        // stands -- otherwise (or on overflow) it is redone
        AmgLevel &C = *L[nlev - 1];
        const bool nd_spec = dense_coarse && spec_on() && !g_prof && def_n > 0 && nlev - 1 > l0 &&
                             C.n >= 8 * kBj && nd_key_n == C.n && C.col == C.col_o.p &&
                             (size_t)nd_key_nnz <= C.col_o.n && !std::getenv("XFK_NO_ND");
        if (nd_spec) {
            AMG_CHECK(mis_out.alloc(4));
            AMG_CHECK(hipMemsetAsync(mis_out.p + 3, 0, sizeof(int), s));
            const int nt = (int)std::max((long long)C.n + 1, nd_key_nnz);
            k_pattern_diff<<<nb(nt), kB, 0, s>>>(C.n, C.rowptr, C.col, nd_key_dev.p, (int)nd_key_nnz, mis_out.p + 3);
            AMG_CHECK(hipMemcpyAsync(host_int + 11, mis_out.p + 3, sizeof(int), hipMemcpyDeviceToHost, s));
        }
        int rc = fetch_deferred(s);
        if (rc != XFK_OK) return rc;
        if (nd_spec) {
            rc = alloc_vectors();
            if (rc != XFK_OK) return rc;
            nd_phases = nd_phases_key;
            if ((rc = dense_inverse(s, C, nd_ld)) != XFK_OK) return rc;
        }
        bool overflow = false;
        rc = wait_deferred(s, overflow);
        if (rc != XFK_OK) return rc;
        if (overflow) {
            if (sw_used) {   // nothing of this attempt may still run on the side stream
                AMG_CHECK(hipStreamSynchronize(sw.cs));
                sw_used = rt_pending = fold_pending = false;
            }
            cap_hint.clear();
            return build(s, l0);
        }
        for (int k = l0; k < nlev; ++k) stats.nnz[k] = L[k]->nnz;
        if (std::getenv("XFK_AMG_HINTS_PRINT")) {   // lab: the capacities / MIS rounds a setup measured
            std::fprintf(stderr, "[amg hints] levels %d:", nlev);
            for (auto &h : cap_hint) std::fprintf(stderr, " cap[%d.%d]=%d", h.first / 4, h.first % 4, h.second);
            for (auto &h : mis_hint) std::fprintf(stderr, " mis[%d]=%d", h.first, h.second);
            for (int k = 0; k < nlev; ++k) std::fprintf(stderr, " n%d=%d/%lld", k, L[k]->n, L[k]->nnz);
            std::fprintf(stderr, "\n");
        }
        stats.levels = nlev;
        double tot = 0;
        for (int k = 0; k < nlev; ++k) tot += (double)stats.nnz[k];
        stats.op_complexity = stats.nnz[0] > 0 ? tot / (double)stats.nnz[0] : 0.0;
        rc = alloc_vectors();
        if (rc != XFK_OK) return rc;
        if (dense_coarse && !(nd_spec && host_int[11] == 0)) {
            if (g_prof) g_prof->begin("setup L" + std::to_string(nlev - 1) + " dense inverse (blocked Gauss-Jordan)", 0.0);
            int ld = 0;
            if ((rc = nd_order(s, C, ld)) != XFK_OK) return rc;
            if ((rc = dense_inverse(s, C, ld)) != XFK_OK) return rc;
            if (g_prof) g_prof->end();
        }
    }
    if (sw_used) {   // the V-cycle reads R, P~, R~: join the side stream (after the dense inverse's launches)
        // by the time the host gets here (after the deferred read) the side
        // stream has usually drained: its work is complete and visible, and
        // the cross-stream wait -- ~15 us of barrier packet on the main
        // queue between the dense inverse and the PCG -- is skipped
        const hipError_t q = hipStreamQuery(sw.cs);
        if (q == hipErrorNotReady) {
            AMG_CHECK(hipEventRecord(sw.b, sw.cs));
            AMG_CHECK(hipStreamWaitEvent(s, sw.b, 0));
        } else {
            AMG_CHECK(q);
        }
        sw_used = rt_pending = fold_pending = false;
    }
    AMG_CHECK(hipGetLastError());   // no host check: nothing on the host waits for the device here
    return XFK_OK;
}


// ---------------------------------------------------------------------------
// sharded level 0
// ---------------------------------------------------------------------------

namespace {

// every rank's k doubles -> host (rank-major); collective
int gather_host(Amg &M, xfk_comm *comm, hipStream_t s, const double *vals, int k, std::vector<double> &out)
{
    DBuf<double> d;
    AMG_CHECK(d.alloc((size_t)k * (comm->size + 1)));
    AMG_CHECK(hipMemcpyAsync(d.p, vals, sizeof(double) * k, hipMemcpyHostToDevice, s));
    int rc = comm->allgather(d.p, d.p + k, (size_t)k, s);
    if (rc != XFK_OK) return rc;
    out.assign((size_t)k * comm->size, 0.0);
    AMG_CHECK(hipMemcpyAsync(out.data(), d.p + k, sizeof(double) * k * comm->size, hipMemcpyDeviceToHost, s));
    AMG_CHECK(hipStreamSynchronize(s));
    (void)M;
    return XFK_OK;
}

}  // namespace

// XFK_AMG_FOLD_DIST=0: sharded levels keep the unfolded post-step
// (prolongation, halo exchange, sweep); read per setup
static bool dist_fold_on()
{
    const char *e = std::getenv("XFK_AMG_FOLD_DIST");
    return !(e && std::atoi(e) == 0);
}

// a folded sharded level 0: P~ in f32 with 16-bit columns in the V-cycle's
// 512-row tiles (a tile reaching the halo columns may keep the int columns,
// decided per tile), as the single-device level 0's
int Amg::fold_dist_tiles(hipStream_t s, int l)
{
    AmgLevel &A = *L[l];
    if (!A.fold || l != 0) return XFK_OK;
    int rc = XFK_OK;
    if (A.has16 && (rc = build_col16<kCgBlock>(s, A.n, A.ftrow.p, A.ftcol.p, A.fnnz, A.f16, A.f16b)) != XFK_OK)
        return rc;
    if (A.has32 && (rc = to_f32(s, A.n, A.ftrow.p, A.fnnz, A.ftval.p, A.f32v)) != XFK_OK) return rc;
    return XFK_OK;
}

int Amg::setup_dist(hipStream_t s, xfk_comm *comm_, const HaloPlan &halo_, int n, int nh, const int *rowptr,
                    const int *col, const double *val, long long nnz)
{
    dist = true;
    comm = comm_;
    nranks = comm->size;
    rank = comm->rank;
    int rc = init(s);
    if (rc != XFK_OK) return rc;
    {
        AmgLevel &A = *L[0];
        A.n = n;
        A.nnz = nnz;
        A.ncol_lim = n;            // aggregation and P: the owned block
        A.ncol_smooth = n + nh;    // smoother and residual: the full rows
        A.rowptr = rowptr;
        A.col = col;
        A.val = val;
        A.dist = true;
        A.plan = halo_;
        // 16-bit tile columns of the owned rows (the overlapped PCG SpMV and the
        // level-0 sweeps read them; a boundary tile reaching the halo ids spans
        // more than 65535 columns and keeps the int columns, decided per tile)
        A.has16 = col16 < 0 ? col16_on() : col16 != 0;
        if (A.has16 && (rc = build_col16<kCgBlock>(s, n, rowptr, col, nnz, A.a16, A.a16b)) != XFK_OK) return rc;
        // f32 restriction / prolongation (converted after the aggregation)
        A.has32 = A.has16 && (prec32 < 0 ? f32_on() : prec32 != 0);
    }
    for (int l = 0;; ++l) {
        AmgLevel &A = *L[l];
        const int nl = A.n;
        stats.n[l] = nl;
        stats.nnz[l] = A.nnz;
        AMG_CHECK(A.dinv.alloc(std::max(1, nl)));
        AMG_CHECK(absd.alloc(std::max(1, nl)));
        AMG_CHECK(dfinv.alloc(std::max(1, nl)));
        AMG_CHECK(wF.alloc(std::max(1, nl)));
        AMG_CHECK(cnt.alloc((size_t)nl + 1));
        AMG_CHECK(sflag.alloc((size_t)std::max(1LL, A.nnz)));
        AMG_CHECK(rho_part.alloc(2 * (size_t)std::max(1, nb_str(nl))));
        k_amg_diag<<<nb(nl), kB, 0, s>>>(nl, A.rowptr, A.col, A.val, absd.p, A.dinv.p);
        k_amg_strength<<<nb_str(nl), kB, 0, s>>>(nl, nl, theta_at(l), A.rowptr, ColView{A.col, nullptr, nullptr}, A.val,
                                                 absd.p, A.dinv.p, sflag.p, cnt.p, dfinv.p, wF.p, rho_part.p,
                                                 signed_strength());
        k_max_reduce<<<1, kMaxReduceT, 0, s>>>(nb_str(nl), rho_part.p, omega, rho.p + 2 * l);
        long long nc = 0;
        rc = aggregate(s, l, nc, false);
        if (rc != XFK_OK && rc != XFK_ERR_UNSUPPORTED) return rc;
        // test hook: this rank reports an aggregation failure at level 0, so
        // every rank must agree on the Jacobi fallback through the collectives
        if (const char *fr = std::getenv("XFK_TEST_AMG_FAIL_RANK"))
            if (l == 0 && std::atoi(fr) == rank) rc = XFK_ERR_UNSUPPORTED;
        bool rep = false;
        if ((rc = galerkin_dist(s, l, rc == XFK_OK ? 0 : 1, rep)) != XFK_OK) return rc;
        if (rep) {
            lrep = l + 1;
            const int te = tail_begin(s, 1);
            rc = build(s, l + 1);
            tail_end(s, te);
            return rc;
        }
    }
}

namespace {

// per peer: the smallest and largest of its ids this rank's columns reference
// (reduced per workgroup in LDS first: the entries of one peer all hit the
// same two words, and one global atomic per entry serialised ~150 us per call
// at configs[4] / 8 ranks)
constexpr int kSpanRanks = 64;
__global__ void __launch_bounds__(kB) k_peer_span(long long nnz, const int *__restrict__ col, int own0, int own1,
                                                  const int *__restrict__ c0, int nranks, int *lo, int *hi)
{
    __shared__ int slo[kSpanRanks], shi[kSpanRanks];
    for (int q = threadIdx.x; q < kSpanRanks; q += blockDim.x) {
        slo[q] = INT_MAX;
        shi[q] = -1;
    }
    __syncthreads();
    const long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (e < nnz) {
        const int J = col[e];
        if (J < own0 || J >= own1) {
            int q = 0;
            while (c0[q + 1] <= J) ++q;
            atomicMin(&slo[q], J);
            atomicMax(&shi[q], J);
        }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < nranks; q += blockDim.x)
        if (shi[q] >= 0) {
            atomicMin(&lo[q], slo[q]);
            atomicMax(&hi[q], shi[q]);
        }
}
// global ids -> local: own rows first, then the peers' spans in peer order
__global__ void k_localize(long long nnz, int *__restrict__ col, int own0, int own1, int n,
                           const int *__restrict__ c0, int nranks, const int *__restrict__ lo,
                           const int *__restrict__ off)
{
    const long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (e >= nnz) return;
    const int J = col[e];
    if (J >= own0 && J < own1) {
        col[e] = J - own0;
        return;
    }
    int q = 0;
    while (c0[q + 1] <= J) ++q;
    col[e] = n + off[q] + (J - lo[q]);
}
__global__ void k_fill_int(int n, int *a, int v)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = v;
}

}  // namespace

// A_{l+1} = R (A P_ext) on every rank for its own aggregates (P_ext: P plus
// the peers' P rows of the halo nodes, global coarse ids).  The result either
// stays sharded (own rows, halo spans and an exchange plan built here) or, once
// the global level has <= rep_rows rows, is all-gathered into the replicated
// level l+1 (rep = true).  st: this rank's status so far -- every rank makes
// the same collective calls whatever its status.
int Amg::galerkin_dist(hipStream_t s, int l, int st, bool &rep)
{
    AmgLevel &A = *L[l];
    const int n = A.n, nh = A.ncol_smooth - A.n;
    const int nc = st ? 0 : A.nc;
    std::vector<double> all;
    if (nranks > kSpanRanks) {   // (same on every rank)
        set_error("AMG: a sharded hierarchy of more than 64 ranks");
        return XFK_ERR_UNSUPPORTED;
    }
    // 1. aggregate counts and status of every rank
    {
        const double mine[2] = {(double)nc, (double)st};
        int rc = gather_host(*this, comm, s, mine, 2, all);
        if (rc != XFK_OK) return rc;
    }
    std::vector<int> cn(nranks + 1, 0);
    int cmax = 1, cmin = INT_MAX;
    bool fail = false;
    for (int q = 0; q < nranks; ++q) {
        cn[q + 1] = cn[q] + (int)all[2 * q];
        cmax = std::max(cmax, (int)all[2 * q]);
        cmin = std::min(cmin, (int)all[2 * q]);
        fail |= all[2 * q + 1] != 0.0;
    }
    const int NC = cn[nranks];
    if (fail || NC == 0) {
        set_error("AMG: a rank could not aggregate its rows");
        return XFK_ERR_UNSUPPORTED;
    }
    // replicate small levels (and never leave a rank without rows)
    rep = NC <= rep_rows || cmin == 0 || l + 2 >= kAmgMaxLevels;
    AMG_CHECK(c0_dev.alloc(nranks + 1));
    AMG_CHECK(hipMemcpyAsync(c0_dev.p, cn.data(), sizeof(int) * (nranks + 1), hipMemcpyHostToDevice, s));
    // 2. P rows of the halo nodes: lengths through the level's plan, then the
    //    entries through a plan over the P arrays (a peer's rows for one halo
    //    range are one contiguous run of its P entries)
    const long long pnnz = A.pnnz;
    const int ncl = n + nh;
    AMG_CHECK(ebuf.alloc((size_t)std::max(1, ncl)));
    if (n > 0) k_row_len_d<<<nb(n), kB, 0, s>>>(n, A.prow.p, ebuf.p);
    int rc = comm->exchange(A.plan, ebuf.p, s);
    if (rc != XFK_OK) return rc;
    AMG_CHECK(cnt.alloc((size_t)std::max(n, nh) + 1));
    AMG_CHECK(flag.alloc((size_t)nh + 1));
    if (nh > 0) k_dbl2int<<<nb(nh), kB, 0, s>>>(nh, ebuf.p + n, cnt.p);
    // flag = halo row pointer (its total, the halo rows' P entries, read with
    // the ranges' pointers below: one host check)
    if ((rc = scan_only(*this, s, cnt.p, flag.p, nh)) != XFK_OK) return rc;
    AMG_CHECK(pe_row.alloc((size_t)ncl + 1));
    k_pe_row<<<nb(ncl + 1), kB, 0, s>>>(n, nh, pnnz, A.prow.p, flag.p, pe_row.p);
    const HaloPlan &hp = A.plan;
    const int nsr = (int)(hp.send.size() + hp.recv.size());
    if ((rc = host_ints(2 * nsr + 1)) != XFK_OK) return rc;
    long long nhe = 0;
    {
        int k = 0;
        for (const HaloRange &t : hp.send) {
            AMG_CHECK(hipMemcpyAsync(host_big + k++, A.prow.p + t.off, sizeof(int), hipMemcpyDeviceToHost, s));
            AMG_CHECK(hipMemcpyAsync(host_big + k++, A.prow.p + t.off + t.len, sizeof(int), hipMemcpyDeviceToHost, s));
        }
        for (const HaloRange &r : hp.recv) {
            AMG_CHECK(hipMemcpyAsync(host_big + k++, flag.p + (r.off - n), sizeof(int), hipMemcpyDeviceToHost, s));
            AMG_CHECK(hipMemcpyAsync(host_big + k++, flag.p + (r.off - n) + r.len, sizeof(int),
                                     hipMemcpyDeviceToHost, s));
        }
        AMG_CHECK(hipMemcpyAsync(host_big + k, flag.p + nh, sizeof(int), hipMemcpyDeviceToHost, s));
        AMG_CHECK(hipStreamSynchronize(s));
        nhe = host_big[k];
    }
    HaloPlan ep;
    {
        int k = 0;
        for (const HaloRange &t : hp.send) {
            const int b0 = host_big[k++], b1 = host_big[k++];
            ep.send.push_back(HaloRange{t.peer, b0, b1 - b0, t.g0});
        }
        for (const HaloRange &r : hp.recv) {
            const int b0 = host_big[k++], b1 = host_big[k++];
            ep.recv.push_back(HaloRange{r.peer, (int)pnnz + b0, b1 - b0, r.g0});
        }
    }
    const size_t ne = (size_t)std::max(1LL, pnnz + nhe);
    AMG_CHECK(pe_val.alloc(ne));
    if (pnnz > 0)
        AMG_CHECK(hipMemcpyAsync(pe_val.p, A.pval.p, sizeof(double) * pnnz, hipMemcpyDeviceToDevice, s));
    if ((rc = comm->exchange(ep, pe_val.p, s)) != XFK_OK) return rc;
    // columns in global coarse ids (A.pcol itself stays rank-local: the
    // prolongation reads the own aggregates only)
    AMG_CHECK(pe_col.alloc(ne));
    if (pnnz > 0) {
        AMG_CHECK(hipMemcpyAsync(pe_col.p, A.pcol.p, sizeof(int) * pnnz, hipMemcpyDeviceToDevice, s));
        k_add_int<<<nb(pnnz), kB, 0, s>>>(pnnz, pe_col.p, cn[rank]);
    }
    AMG_CHECK(ebuf.alloc(ne));
    if (pnnz > 0) k_int2dbl<<<nb(pnnz), kB, 0, s>>>(pnnz, pe_col.p, ebuf.p);
    if ((rc = comm->exchange(ep, ebuf.p, s)) != XFK_OK) return rc;
    if (nhe > 0) k_dbl2int<<<nb(nhe), kB, 0, s>>>(nhe, ebuf.p + pnnz, pe_col.p + pnnz);
    // 3. AP over the full rows, then this rank's coarse rows R (AP)
    long long lnnz = 0, apnnz = 0;
    AMG_CHECK(l_row.alloc((size_t)cmax + 1));
    {
        SgX XA{A.rowptr, A.col, A.val, ncl, nullptr, nullptr, nullptr};
        SgY YP{pe_row.p, pe_col.p, pe_val.p, nullptr};
        // (the lengths are needed on the host at once: capacity hints of the
        // last setup, rank-local, taken without deferring -- one host check
        // per product instead of two)
        rc = spgemm<false>(*this, s, n, XA, YP, ap_row, ap_col, ap_val, apnnz, 4 * l + 1, false);
        if (rc == XFK_OK) {
            SgX XR{A.rrow.p, A.rcol.p, A.rval.p, INT_MAX, nullptr, nullptr, nullptr};
            SgY YAP{ap_row.p, ap_col.p, ap_val.p, nullptr};
            rc = spgemm<false>(*this, s, nc, XR, YAP, l_row, l_col, l_val, lnnz, 4 * l + 2, false);
        }
        if (rc != XFK_OK && rc != XFK_ERR_UNSUPPORTED) return rc;
    }
    // 4. folded post-step of this sharded level (V(1,1)): P~ = (I - w D^-1 A) P_ext
    //    over the pattern of A P_ext -- own rows, global coarse columns (the
    //    peers' aggregates next to the halo included); formed before the next
    //    level reuses A P's buffers.  The V-cycle's prolongation and post-sweep
    //    become one pass over P~ reading x_c with its coarse halo (a sharded
    //    next level: the columns are localised with its plan below; a
    //    replicated one: the global coarse vector every rank holds).
    const bool ok3 = rc == XFK_OK;
    A.fold = A.fold_formed =
        ok3 && sweeps == 1 && dist_fold_on() && (fold_on < 0 ? fold_levels() : fold_on != 0);
    if (A.fold) {
        A.fnnz = apnnz;
        AMG_CHECK(A.ftrow.alloc((size_t)n + 1));
        AMG_CHECK(A.ftcol.alloc((size_t)std::max(1LL, apnnz)));
        AMG_CHECK(A.ftval.alloc((size_t)std::max(1LL, apnnz)));
        AMG_CHECK(hipMemcpyAsync(A.ftrow.p, ap_row.p, sizeof(int) * ((size_t)n + 1), hipMemcpyDeviceToDevice, s));
        if (n > 0)
            k_fold_p<<<(int)(((long long)n * kFoldLanes + 255) / 256), 256, 0, s>>>(
                n, rho.p + 2 * l, A.dinv.p, ap_row.p, ap_col.p, ap_val.p, pe_row.p, pe_col.p, pe_val.p, A.ftcol.p,
                A.ftval.p);
    }
    // 5. entry counts, status and -- the next level staying sharded -- the
    //    spans of the peers' aggregate ids this rank's A_{l+1} and P~ columns
    //    reference (what each peer must send): one all-gather, one host check
    const int own0 = cn[rank], own1 = cn[rank + 1];
    const int RW = 2 + 2 * nranks;   // per rank: lnnz, status, lo[nranks], hi[nranks]
    DBuf<double> recs;
    AMG_CHECK(recs.alloc((size_t)RW * (nranks + 1)));
    const double mine[2] = {(double)lnnz, ok3 ? 0.0 : 1.0};   // (read before the host check below)
    AMG_CHECK(hipMemcpyAsync(recs.p, mine, sizeof(mine), hipMemcpyHostToDevice, s));
    AMG_CHECK(span_dev.alloc(2 * (size_t)nranks));
    k_fill_int<<<1, 64, 0, s>>>(nranks, span_dev.p, INT_MAX);
    k_fill_int<<<1, 64, 0, s>>>(nranks, span_dev.p + nranks, -1);
    if (!rep && ok3) {
        if (lnnz > 0)
            k_peer_span<<<nb(lnnz), kB, 0, s>>>(lnnz, l_col.p, own0, own1, c0_dev.p, nranks, span_dev.p,
                                                 span_dev.p + nranks);
        if (A.fold && apnnz > 0)
            k_peer_span<<<nb(apnnz), kB, 0, s>>>(apnnz, A.ftcol.p, own0, own1, c0_dev.p, nranks, span_dev.p,
                                                  span_dev.p + nranks);
    }
    k_int2dbl<<<1, 256, 0, s>>>(2LL * nranks, span_dev.p, recs.p + 2);
    if ((rc = comm->allgather(recs.p, recs.p + RW, (size_t)RW, s)) != XFK_OK) return rc;
    all.assign((size_t)RW * nranks, 0.0);
    AMG_CHECK(hipMemcpyAsync(all.data(), recs.p + RW, sizeof(double) * RW * nranks, hipMemcpyDeviceToHost, s));
    AMG_CHECK(hipStreamSynchronize(s));
    std::vector<int> e0(nranks + 1, 0);
    long long nnzmax = 1;
    for (int q = 0; q < nranks; ++q) {
        e0[q + 1] = e0[q] + (int)all[(size_t)RW * q];
        nnzmax = std::max(nnzmax, (long long)all[(size_t)RW * q]);
        fail |= all[(size_t)RW * q + 1] != 0.0;
    }
    if (fail) {
        set_error("AMG: a SpGEMM row exceeds the LDS hash capacity");
        return XFK_ERR_UNSUPPORTED;
    }
    if ((int)L.size() <= l + 1) L.emplace_back(new AmgLevel());
    AmgLevel &C = *L[l + 1];
    if (!rep) {
        // 5a. stay sharded: own rows with local columns, halo spans per peer
        //     (what I need: my spans; what each peer needs from me: its spans
        //     of my ids)
        auto span_of = [&](int r, int q, bool hi) { return (int)all[(size_t)RW * r + 2 + (hi ? nranks : 0) + q]; };
        std::vector<int> span(2 * nranks);
        for (int q = 0; q < nranks; ++q) {
            span[q] = span_of(rank, q, false);
            span[nranks + q] = span_of(rank, q, true);
        }
        HaloPlan cp;
        std::vector<int> off(nranks, 0);
        int nhc = 0;
        for (int q = 0; q < nranks; ++q) {
            if (q == rank || span[q] > span[nranks + q]) continue;
            const int len = span[nranks + q] - span[q] + 1;
            off[q] = nhc;
            cp.recv.push_back(HaloRange{q, nc + nhc, len, span[q]});
            nhc += len;
        }
        for (int r = 0; r < nranks; ++r) {
            if (r == rank) continue;
            const int lo = span_of(r, rank, false), hi = span_of(r, rank, true);
            if (lo > hi) continue;
            cp.send.push_back(HaloRange{r, lo - own0, hi - lo + 1, lo});
        }
        AMG_CHECK(map_dev.alloc(nranks));
        AMG_CHECK(hipMemcpyAsync(map_dev.p, off.data(), sizeof(int) * nranks, hipMemcpyHostToDevice, s));
        AMG_CHECK(C.rowptr_o.alloc((size_t)nc + 1));
        AMG_CHECK(C.col_o.alloc((size_t)std::max(1LL, lnnz)));
        AMG_CHECK(C.val_o.alloc((size_t)std::max(1LL, lnnz)));
        AMG_CHECK(hipMemcpyAsync(C.rowptr_o.p, l_row.p, sizeof(int) * (nc + 1), hipMemcpyDeviceToDevice, s));
        if (lnnz > 0) {
            AMG_CHECK(hipMemcpyAsync(C.col_o.p, l_col.p, sizeof(int) * lnnz, hipMemcpyDeviceToDevice, s));
            AMG_CHECK(hipMemcpyAsync(C.val_o.p, l_val.p, sizeof(double) * lnnz, hipMemcpyDeviceToDevice, s));
            k_localize<<<nb(lnnz), kB, 0, s>>>(lnnz, C.col_o.p, own0, own1, nc, c0_dev.p, nranks, span_dev.p,
                                                map_dev.p);
        }
        if (A.fold && apnnz > 0)
            k_localize<<<nb(apnnz), kB, 0, s>>>(apnnz, A.ftcol.p, own0, own1, nc, c0_dev.p, nranks, span_dev.p,
                                                 map_dev.p);
        if ((rc = fold_dist_tiles(s, l)) != XFK_OK) return rc;
        C.n = nc;
        C.nnz = lnnz;
        C.ncol_lim = nc;
        C.ncol_smooth = nc + nhc;
        C.rowptr = C.rowptr_o.p;
        C.col = C.col_o.p;
        C.val = C.val_o.p;
        C.dist = true;
        C.plan = cp;
        AMG_CHECK(hipStreamSynchronize(s));
        return XFK_OK;
    }
    // 5b. all-gather the coarse rows (padded per rank) into the replicated level
    if ((rc = fold_dist_tiles(s, l)) != XFK_OK) return rc;
    c0 = cn;
    ncmax = cmax;
    AMG_CHECK(s_col.alloc((size_t)nnzmax));
    AMG_CHECK(s_val.alloc((size_t)nnzmax));
    if (lnnz > 0) {
        AMG_CHECK(hipMemcpyAsync(s_col.p, l_col.p, sizeof(int) * lnnz, hipMemcpyDeviceToDevice, s));
        AMG_CHECK(hipMemcpyAsync(s_val.p, l_val.p, sizeof(double) * lnnz, hipMemcpyDeviceToDevice, s));
    }
    AMG_CHECK(g_row.alloc((size_t)nranks * (ncmax + 1)));
    AMG_CHECK(g_col.alloc((size_t)nranks * nnzmax));
    AMG_CHECK(g_val.alloc((size_t)nranks * nnzmax));
    if ((rc = comm->allgather_bytes(l_row.p, g_row.p, sizeof(int) * (ncmax + 1), s)) != XFK_OK) return rc;
    if ((rc = comm->allgather_bytes(s_col.p, g_col.p, sizeof(int) * nnzmax, s)) != XFK_OK) return rc;
    if ((rc = comm->allgather(s_val.p, g_val.p, (size_t)nnzmax, s)) != XFK_OK) return rc;
    const long long NNZ = e0[nranks];
    AMG_CHECK(C.rowptr_o.alloc((size_t)NC + 1));
    AMG_CHECK(C.col_o.alloc((size_t)std::max(1LL, NNZ)));
    AMG_CHECK(C.val_o.alloc((size_t)std::max(1LL, NNZ)));
    AMG_CHECK(e0_dev.alloc(nranks + 1));
    AMG_CHECK(hipMemcpyAsync(e0_dev.p, e0.data(), sizeof(int) * (nranks + 1), hipMemcpyHostToDevice, s));
    k_concat_rowptr<<<nb(NC + 1), kB, 0, s>>>(NC, nranks, c0_dev.p, e0_dev.p, g_row.p, ncmax + 1, C.rowptr_o.p);
    for (int q = 0; q < nranks; ++q) {
        const long long cq = e0[q + 1] - e0[q];
        if (cq == 0) continue;
        AMG_CHECK(hipMemcpyAsync(C.col_o.p + e0[q], g_col.p + (size_t)q * nnzmax, sizeof(int) * cq,
                                 hipMemcpyDeviceToDevice, s));
        AMG_CHECK(hipMemcpyAsync(C.val_o.p + e0[q], g_val.p + (size_t)q * nnzmax, sizeof(double) * cq,
                                 hipMemcpyDeviceToDevice, s));
    }
    C.n = NC;
    C.nnz = NNZ;
    C.ncol_lim = NC;
    C.ncol_smooth = NC;
    C.rowptr = C.rowptr_o.p;
    C.col = C.col_o.p;
    C.val = C.val_o.p;
    C.dist = false;
    C.plan = HaloPlan();
    if (std::getenv("XFK_AMG_DEBUG") && rank == 0) {   // symmetry of the gathered A_1
        std::vector<int> hr(NC + 1), hc(NNZ);
        std::vector<double> hv(NNZ);
        AMG_CHECK(hipMemcpyAsync(hr.data(), C.rowptr, sizeof(int) * (NC + 1), hipMemcpyDeviceToHost, s));
        AMG_CHECK(hipMemcpyAsync(hc.data(), C.col, sizeof(int) * NNZ, hipMemcpyDeviceToHost, s));
        AMG_CHECK(hipMemcpyAsync(hv.data(), C.val, sizeof(double) * NNZ, hipMemcpyDeviceToHost, s));
        AMG_CHECK(hipStreamSynchronize(s));
        std::vector<std::pair<int, double>> row;
        std::vector<std::vector<std::pair<int, double>>> R(NC);
        double amax = 0, dmax = 0;
        long long missing = 0;
        for (int i = 0; i < NC; ++i) {
            for (int k = hr[i]; k < hr[i + 1]; ++k) R[i].push_back({hc[k], hv[k]});
            std::sort(R[i].begin(), R[i].end());
        }
        for (int i = 0; i < NC; ++i)
            for (auto &e : R[i]) {
                amax = std::max(amax, std::fabs(e.second));
                auto &Rj = R[e.first];
                auto it = std::lower_bound(Rj.begin(), Rj.end(), std::make_pair(i, -1e300));
                if (it == Rj.end() || it->first != i) {
                    ++missing;
                    dmax = std::max(dmax, std::fabs(e.second));
                } else {
                    dmax = std::max(dmax, std::fabs(e.second - it->second));
                }
            }
        std::fprintf(stderr, "[amg] A_1 %d rows %lld nnz: max|A - A^T| / max|A| = %.3e, %lld entries without a mirror\n",
                     NC, NNZ, dmax / amax, missing);
    }
    AMG_CHECK(cb_loc.alloc((size_t)ncmax));
    AMG_CHECK(cb_all.alloc((size_t)nranks * ncmax));
    return XFK_OK;
}

namespace {

// which: 0 every row; 1 / 2 the interior / boundary tiles of A.ts (tile levels)
template <int MODE>
void launch_smooth_t(hipStream_t s, int l, const AmgLevel &A, const unsigned long long *rho, const double *b,
                     const double *x, double *out, double *rout, const int *done, double *part_gam, int which)
{
    const int *tl = nullptr;
    int nt = 0;
    if (which) {
        tl = A.ts.tiles.p + (which == 2 ? A.ts.n_in : 0);
        nt = which == 1 ? A.ts.n_in : A.ts.n_bd;
        if (nt == 0) return;
    }
    if (l == 0) {
        const int g = tl ? nt : (A.n + kCgBlock - 1) / kCgBlock;
        if (A.has32 && f32_sweep_on())
            k_amg_smooth<MODE, kCgBlock><<<g, kCgBlock, 0, s>>>(A.n, A.ncol_smooth, A.rowptr, A.col, A.a32.p,
                                                                A.dinv.p, rho, b, x, out, rout, done, part_gam, tl,
                                                                A.has16 ? A.a16.p : nullptr,
                                                                A.has16 ? A.a16b.p : nullptr);
        else
            k_amg_smooth<MODE, kCgBlock><<<g, kCgBlock, 0, s>>>(A.n, A.ncol_smooth, A.rowptr, A.col, A.val, A.dinv.p,
                                                                rho, b, x, out, rout, done, part_gam, tl,
                                                                A.has16 ? A.a16.p : nullptr,
                                                                A.has16 ? A.a16b.p : nullptr);
        return;
    }
    if (A.n >= kTileMinRows) {
        // coarse levels carry 10-16 entries per row: 4 slots per lane, one pass per tile
        const int g = tl ? nt : (A.n + 255) / 256;
        if ((double)A.nnz <= 8.0 * A.n)
            k_amg_smooth<MODE, 256, 2><<<g, 256, 0, s>>>(A.n, A.ncol_smooth, A.rowptr, A.col, A.val, A.dinv.p, rho, b,
                                                         x, out, rout, done, nullptr, tl);
        else
            k_amg_smooth<MODE, 256, 4><<<g, 256, 0, s>>>(A.n, A.ncol_smooth, A.rowptr, A.col, A.val, A.dinv.p, rho, b,
                                                         x, out, rout, done, nullptr, tl);
        return;
    }
    const int G = lanes_for(A.n > 0 ? (double)A.nnz / A.n : 1.0);
    const int g = (int)(((long long)A.n * G + 255) / 256);
    if (G == 4)
        k_amg_smooth_g<MODE, 4><<<g, 256, 0, s>>>(A.n, A.ncol_smooth, A.rowptr, A.col, A.val, A.dinv.p, rho, b, x, out,
                                                 rout, done);
    else if (G == 8)
        k_amg_smooth_g<MODE, 8><<<g, 256, 0, s>>>(A.n, A.ncol_smooth, A.rowptr, A.col, A.val, A.dinv.p, rho, b, x, out,
                                                 rout, done);
    else
        k_amg_smooth_g<MODE, 16><<<g, 256, 0, s>>>(A.n, A.ncol_smooth, A.rowptr, A.col, A.val, A.dinv.p, rho, b, x,
                                                  out, rout, done);
}

void launch_smooth(hipStream_t s, int mode, int l, const AmgLevel &A, const unsigned long long *rho, const double *b,
                   const double *x, double *out, double *rout, const int *done, double *part_gam = nullptr,
                   int which = 0)
{
    switch (mode) {
    case kSweepFromZero: launch_smooth_t<kSweepFromZero>(s, l, A, rho, b, x, out, rout, done, nullptr, which); break;
    case kSweep: launch_smooth_t<kSweep>(s, l, A, rho, b, x, out, rout, done, part_gam, which); break;
    case kResid: launch_smooth_t<kResid>(s, l, A, rho, b, x, out, rout, done, nullptr, which); break;
    default: launch_smooth_t<kResidFromZero>(s, l, A, rho, b, x, out, rout, done, nullptr, which); break;
    }
}

// lanes per row of the long R~ rows (up to one wavefront)
int lanes_wide(double per_row)
{
    return per_row <= 6.0 ? 4 : (per_row <= 20.0 ? 8 : (per_row <= 40.0 ? 16 : (per_row <= 80.0 ? 32 : 64)));
}

template <int GA>
void launch_fold_pre_a(hipStream_t s, const AmgLevel &A, const unsigned long long *rho, const double *b, double *y,
                       double *bc, const int *done, const double *yadd)
{
    const int GB = lanes_wide(A.nc > 0 ? (double)A.fnnz / A.nc : 1.0);
    // (the first range padded to whole rounds of the 8 XCDs, so both ranges
    // take the XCD-contiguous block order)
    const int ga = (int)(((((long long)A.n * GA + 255) / 256) + 7) & ~7LL);
    const int gb = (int)(((long long)A.nc * GB + 255) / 256);
#define XFK_FOLD(GG)                                                                                               \
    k_fold_pre<GA, GG><<<ga + gb, 256, 0, s>>>(A.n, A.ncol_smooth, A.rowptr, A.col, A.val, A.dinv.p, rho, b, y,   \
                                               A.nc, A.frrow.p, A.frcol.p, A.frval.p, bc, ga, done, yadd)
    switch (GB) {
    case 4: XFK_FOLD(4); break;
    case 8: XFK_FOLD(8); break;
    case 16: XFK_FOLD(16); break;
    case 32: XFK_FOLD(32); break;
    default: XFK_FOLD(64); break;
    }
#undef XFK_FOLD
}

void launch_fold_pre(hipStream_t s, const AmgLevel &A, const unsigned long long *rho, const double *b, double *y,
                     double *bc, const int *done, const double *yadd = nullptr)
{
    if (A.n <= 0) return;
    const int GA = lanes_for((double)A.nnz / A.n);
    if (GA == 4) launch_fold_pre_a<4>(s, A, rho, b, y, bc, done, yadd);
    else if (GA == 8) launch_fold_pre_a<8>(s, A, rho, b, y, bc, done, yadd);
    else launch_fold_pre_a<16>(s, A, rho, b, y, bc, done, yadd);
}

// tile size of the level's smoother launches (0: sub-wave kernels, no split)
int smooth_tile(int l, const AmgLevel &A) { return l == 0 ? kCgBlock : (A.n >= kTileMinRows ? 256 : 0); }

}  // namespace

// algorithmic bytes of one smoother launch (mode as launch_smooth): the
// matrix stream, the gathered operand once, b / D^-1, the written vectors
static double smooth_bytes(const AmgLevel &A, int mode)
{
    const double n = A.n, base = ((A.has16 ? 2.0 : 4.0) + (A.has32 && f32_sweep_on() ? 4.0 : 8.0)) * (double)A.nnz +
                                 4.0 * (n + 1);
    const bool implicit = mode == kSweepFromZero || mode == kResidFromZero;
    const double rd = (implicit ? 2.0 : 3.0) * 8.0 * n;
    const double wr = (mode == kResidFromZero && !A.fold ? 2.0 : 1.0) * 8.0 * n;
    return base + rd + wr;
}

static const char *smooth_name(int mode)
{
    switch (mode) {
    case kResidFromZero: return "sweep from 0 + residual";
    case kSweepFromZero: return "sweep from 0";
    case kResid: return "residual";
    default: return "sweep";
    }
}

static void smooth_ph(hipStream_t s, int mode, int l, const AmgLevel &A, const unsigned long long *rho,
                      const double *b, const double *x, double *out, double *rout, const int *done,
                      double *part_gam = nullptr)
{
    if (g_prof)
        XFK_PHASE("L" + std::to_string(l) + " " + smooth_name(mode) + (part_gam ? " (+ r.u partials)" : ""),
                  smooth_bytes(A, mode), launch_smooth(s, mode, l, A, rho, b, x, out, rout, done, part_gam));
    else
        launch_smooth(s, mode, l, A, rho, b, x, out, rout, done, part_gam);
}

// Symmetric V-cycle; returns the buffer holding the level's result.  Level 0
// writes its result to `out0`.
// (coarse folded / dense levels: yout = the result buffer instead of xa,
// yadd = a vector the result is added onto -- the W-cycle's second correction)
static double *vcycle_level(Amg &M, hipStream_t s, int l, const double *b, double *out0, const int *done,
                            double *part_gam = nullptr, double *yout = nullptr, const double *yadd = nullptr)
{
    AmgLevel &A = *M.L[l];
    const unsigned long long *rho = M.rho.p + 2 * l;
    const int nu = M.sweeps;
    auto other = [&](double *c) { return c == A.xa.p ? A.xb.p : A.xa.p; };
    const std::string lv = g_prof ? "L" + std::to_string(l) + " " : std::string();
    if (l == M.nlev - 1) {
        double *dst = (l == 0) ? out0 : (yout ? yout : A.xa.p);
        if (M.dense_coarse) {
            if (M.cinv_f64)
                XFK_PHASE(lv + "dense inverse x b", 8.0 * A.n * M.cinv_ld + 8.0 * (2 * M.cinv_ld + A.n),
                          (k_dense_mv<double><<<A.n, 256, 0, s>>>(A.n, M.cinv_ld, M.cinv_o64.p, M.cinv_sc.p, b, dst,
                                                                  done)));
            else
                XFK_PHASE(lv + "dense inverse x b", 4.0 * A.n * M.cinv_ld + 8.0 * (2 * M.cinv_ld + A.n),
                          (k_dense_mv<float><<<A.n, 256, 0, s>>>(A.n, M.cinv_ld, M.cinv_apply, M.cinv_sc.p, b, dst,
                                                                 done)));
            return dst;
        }
        // smoother-only coarsest level: 2 nu sweeps from zero
        double *cur = A.xa.p;
        smooth_ph(s, kSweepFromZero, l, A, rho, b, nullptr, cur, nullptr, done);
        for (int k = 2; k < 2 * nu; ++k) {
            double *nx = (k == 2 * nu - 1 && l == 0) ? out0 : other(cur);
            smooth_ph(s, kSweep, l, A, rho, b, cur, nx, nullptr, done);
            cur = nx;
        }
        if (l == 0 && cur != out0)
            (void)hipMemcpyAsync(out0, cur, sizeof(double) * A.n, hipMemcpyDeviceToDevice, s);
        return cur;
    }
    if (A.fold && l > 0) {
        // two launches: y and the coarse right-hand side, then x = y + P~ x_c
        AmgLevel &C = *M.L[l + 1];
        double *y = yout ? yout : A.xa.p;
        const double n = A.n, nc = A.nc, f = (double)A.fnnz;
        XFK_PHASE(lv + "folded pre: y, R~ r", 12.0 * A.nnz + 4.0 * (n + 1) + 24.0 * n + 12.0 * f + 4.0 * (nc + 1) +
                                                   8.0 * nc + (yadd ? 8.0 * n : 0.0),
                  launch_fold_pre(s, A, rho, b, y, C.b.p, done, yadd));
        const double *xc;
        if (M.w_at(l)) {
            // W-cycle at this level: a second coarse correction from the
            // coarse residual after the first, b_c' = b_c - A_c x_c (Galerkin:
            // R (b - A (x_pre + P x_c)) = b_c - A_c x_c), x_c += V(b_c'); the
            // second visit adds its result onto the first (its folded
            // pre-step starts from x_c), so the post-step prolongs the sum.
            // Symmetric like the V-cycle; three launches more than it.
            const double *x1 = vcycle_level(M, s, l + 1, C.b.p, nullptr, done, nullptr, C.xb.p);
            smooth_ph(s, kResid, l + 1, C, M.rho.p + 2 * (l + 1), C.b.p, x1, nullptr, C.r.p, done);
            xc = vcycle_level(M, s, l + 1, C.r.p, nullptr, done, nullptr, C.xa.p, x1);
        } else {
            xc = vcycle_level(M, s, l + 1, C.b.p, nullptr, done);
        }
        XFK_PHASE(lv + "folded post: x = y + P~ xc", 12.0 * f + 4.0 * (n + 1) + 8.0 * nc + 16.0 * n,
                  launch_mv(s, A.n, A.ftrow.p, A.ftcol.p, A.ftval.p, xc, y, true, lanes_for(f / n), done));
        return y;
    }
    // pre-smoothing (nu sweeps from zero) and residual
    double *cur = A.xa.p;
    if (nu == 1) {
        // (a folded level 0 recomputes x_pre = w D^-1 b in its post-step)
        smooth_ph(s, kResidFromZero, l, A, rho, b, nullptr, (A.fold && l == 0) ? nullptr : cur, A.r.p, done);
    } else {
        smooth_ph(s, kSweepFromZero, l, A, rho, b, nullptr, cur, nullptr, done);
        for (int k = 2; k < nu; ++k) {
            double *nx = other(cur);
            smooth_ph(s, kSweep, l, A, rho, b, cur, nx, nullptr, done);
            cur = nx;
        }
        smooth_ph(s, kResid, l, A, rho, b, cur, nullptr, A.r.p, done);
    }
    AmgLevel &C = *M.L[l + 1];
    const long long rnnz = A.pnnz;
    XFK_PHASE(lv + "restriction R r", A.nz_bytes() * rnnz + 4.0 * (A.nc + 1) + 8.0 * A.n + 8.0 * A.nc,
              (A.has32 ? launch_mv32(s, A.nc, A.rrow.p, A.rcol.p, A.r32.p, A.r.p, C.b.p, false,
                                     lanes_for((double)rnnz / A.nc), done, A.r16.p, A.r16b.p)
                       : launch_mv(s, A.nc, A.rrow.p, A.rcol.p, A.rval.p, A.r.p, C.b.p, false,
                                   lanes_for((double)rnnz / A.nc), done, A.has16 ? A.r16.p : nullptr,
                                   A.has16 ? A.r16b.p : nullptr)));
    const double *xc = vcycle_level(M, s, l + 1, C.b.p, nullptr, done);
    if (A.fold && l == 0 && nu == 1) {
        const double n = A.n, f = (double)A.fnnz;
        XFK_PHASE(lv + "folded post: u = x + w D^-1 r + P~ xc" + (part_gam ? " (+ r.u partials)" : ""),
                  A.nz_bytes() * f + 4.0 * (n + 1) + 8.0 * A.nc + 32.0 * n,
                  (A.has32 ? k_fold_post0<kCgBlock, 2><<<(A.n + kCgBlock - 1) / kCgBlock, kCgBlock, 0, s>>>(
                                 A.n, A.ftrow.p, A.ftcol.p, A.f32v.p, xc, A.dinv.p, rho, A.r.p, b, out0, done,
                                 part_gam, A.f16.p, A.f16b.p)
                           : k_fold_post0<kCgBlock, 2><<<(A.n + kCgBlock - 1) / kCgBlock, kCgBlock, 0, s>>>(
                                 A.n, A.ftrow.p, A.ftcol.p, A.ftval.p, xc, A.dinv.p, rho, A.r.p, b, out0, done,
                                 part_gam, A.has16 ? A.f16.p : nullptr, A.has16 ? A.f16b.p : nullptr)));
        if (part_gam) M.gamma_done = true;
        return out0;
    }
    XFK_PHASE(lv + "prolongation x += P xc", 12.0 * rnnz + 4.0 * (A.n + 1) + 8.0 * A.nc + 16.0 * A.n,
              launch_mv(s, A.n, A.prow.p, A.pcol.p, A.pval.p, xc, cur, true, lanes_for((double)rnnz / A.n), done));
    for (int k = 0; k < nu; ++k) {
        const bool last0 = k == nu - 1 && l == 0;
        double *nx = last0 ? out0 : other(cur);
        smooth_ph(s, kSweep, l, A, rho, b, cur, nx, nullptr, done, last0 ? part_gam : nullptr);
        if (last0 && part_gam) M.gamma_done = true;
        cur = nx;
    }
    return cur;
}

// sharded level l: every sweep reads the peers' halo values of the iterate;
// the restriction / prolongation stay rank-local (P rows reference the own
// aggregates only).  Returns the buffer holding the result (`out` if given).
double *Amg::vc_dist(hipStream_t s, int l, const double *b, double *out, const int *done, int &rc)
{
    AmgLevel &A = *L[l];
    const unsigned long long *rh = rho.p + 2 * l;
    double *cur = A.xa.p, *oth = A.xb.p;
    rc = XFK_OK;
    // tile levels: the halo exchange of the iterate overlaps the interior tiles
    const int B = smooth_tile(l, A);
    const bool ov = B > 0 && overlap_enabled();
    if (ov && !A.ts.ready()) {
        if ((rc = side.init()) != XFK_OK) return nullptr;
        if ((rc = build_tile_split(s, A.n, B, A.rowptr, A.col, A.ts)) != XFK_OK) return nullptr;
    }
    // halo of x, then mode over the level's rows (interior tiles during the exchange)
    auto smooth_after_exchange = [&](int mode, double *x, double *o, double *ro, double *pg) -> int {
        if (!ov) {
            const int r = comm->exchange(A.plan, x, s);
            if (r != XFK_OK) return r;
            launch_smooth(s, mode, l, A, rh, b, x, o, ro, done, pg);
            return XFK_OK;
        }
        return exchange_overlapped(
            s, side, [&](hipStream_t cs) { return comm->exchange(A.plan, x, cs); },
            [&] { launch_smooth(s, mode, l, A, rh, b, x, o, ro, done, pg, 1); },
            [&] { launch_smooth(s, mode, l, A, rh, b, x, o, ro, done, pg, 2); });
    };
    if (A.n > 0) k_jacobi_first<<<nb(A.n), kB, 0, s>>>(A.n, rh, A.dinv.p, b, cur, done);
    for (int k = 1; k < sweeps; ++k) {
        if ((rc = smooth_after_exchange(kSweep, cur, oth, nullptr, nullptr)) != XFK_OK) return nullptr;
        std::swap(cur, oth);
    }
    if ((rc = smooth_after_exchange(kResid, cur, nullptr, A.r.p, nullptr)) != XFK_OK) return nullptr;
    AmgLevel &C = *L[l + 1];
    const int GR = lanes_for(A.nc > 0 ? (double)A.pnnz / A.nc : 1.0);
    const double *xc;
    // level 0 with f32 transfers: R and P in f32 with 16-bit tile columns
    auto restrict_to = [&](double *dst) {
        if (A.has32)
            launch_mv32(s, A.nc, A.rrow.p, A.rcol.p, A.r32.p, A.r.p, dst, false, GR, done, A.r16.p, A.r16b.p);
        else
            launch_mv(s, A.nc, A.rrow.p, A.rcol.p, A.rval.p, A.r.p, dst, false, GR, done);
    };
    const bool fold = A.fold && sweeps == 1;
    const double *xfull = nullptr;   // folded: x_c with the columns P~ reads (coarse halo / global)
    if (C.dist) {
        restrict_to(C.b.p);
        xc = vc_dist(s, l + 1, C.b.p, nullptr, done, rc);
        if (rc != XFK_OK) return nullptr;
        if (fold) {   // the coarse halo P~ reads (the next level's plan covers P~'s columns)
            double *xh = const_cast<double *>(xc);
            if ((rc = comm->exchange(C.plan, xh, s)) != XFK_OK) return nullptr;
            xfull = xh;
        }
    } else {
        // the replicated levels: gather the global right-hand side, solve the
        // same coarse problem on every rank, read the own aggregates back
        restrict_to(cb_loc.p);
        const int te = tail_begin(s, 0);
        if ((rc = comm->allgather(cb_loc.p, cb_all.p, (size_t)ncmax, s)) != XFK_OK) return nullptr;
        k_unpad<<<nb(C.n), kB, 0, s>>>(C.n, nranks, c0_dev.p, cb_all.p, ncmax, C.b.p, done);
        xfull = vcycle_level(*this, s, l + 1, C.b.p, nullptr, done);
        xc = xfull + c0[rank];
        tail_end(s, te);
    }
    if (fold) {
        // u = w D^-1 b + w D^-1 r' + P~ x_c over the own rows: the prolongation
        // and the post-sweep (whose halo exchange it replaces) in one pass
        double *o = out ? out : oth;
        if (A.n > 0) {
            double *pg = (l == 0 && out) ? part_gam_ : nullptr;
            if (l == 0) {
                const int g = (A.n + kCgBlock - 1) / kCgBlock;
                if (A.has32)
                    k_fold_post0<kCgBlock, 2><<<g, kCgBlock, 0, s>>>(A.n, A.ftrow.p, A.ftcol.p, A.f32v.p, xfull,
                                                                     A.dinv.p, rh, A.r.p, b, o, done, pg,
                                                                     A.has16 ? A.f16.p : nullptr,
                                                                     A.has16 ? A.f16b.p : nullptr);
                else
                    k_fold_post0<kCgBlock, 2><<<g, kCgBlock, 0, s>>>(A.n, A.ftrow.p, A.ftcol.p, A.ftval.p, xfull,
                                                                     A.dinv.p, rh, A.r.p, b, o, done, pg,
                                                                     A.has16 ? A.f16.p : nullptr,
                                                                     A.has16 ? A.f16b.p : nullptr);
            } else {
                const int g = (A.n + 255) / 256;
                const unsigned short *no16 = nullptr;
                const int *nob = nullptr;
                if ((double)A.fnnz <= 8.0 * A.n)
                    k_fold_post0<256, 2><<<g, 256, 0, s>>>(A.n, A.ftrow.p, A.ftcol.p, A.ftval.p, xfull, A.dinv.p, rh,
                                                           A.r.p, b, o, done, pg, no16, nob);
                else
                    k_fold_post0<256, 4><<<g, 256, 0, s>>>(A.n, A.ftrow.p, A.ftcol.p, A.ftval.p, xfull, A.dinv.p, rh,
                                                           A.r.p, b, o, done, pg, no16, nob);
            }
        }
        if (l == 0 && out && part_gam_) gamma_done = true;
        return o;
    }
    if (A.n > 0) {
        const int GP = lanes_for((double)A.pnnz / A.n);
        if (A.has32)
            launch_mv32(s, A.n, A.prow.p, A.pcol.p, A.p32.p, xc, cur, true, GP, done, A.p16.p, A.p16b.p);
        else
            launch_mv(s, A.n, A.prow.p, A.pcol.p, A.pval.p, xc, cur, true, GP, done);
    }
    for (int k = 0; k < sweeps; ++k) {
        const bool last0 = k == sweeps - 1 && out && l == 0;
        double *nx = (k == sweeps - 1 && out) ? out : oth;
        if ((rc = smooth_after_exchange(kSweep, cur, nx, nullptr, last0 ? part_gam_ : nullptr)) != XFK_OK)
            return nullptr;
        if (last0 && part_gam_) gamma_done = true;
        oth = cur;
        cur = nx;
    }
    return cur;
}

int Amg::tail_begin(hipStream_t s, int kind)
{
    if (!time_tail) return -1;
    const int at = tail_used;
    while ((int)tail_ev.size() < at + 2) {
        hipEvent_t e = nullptr;
        if (hipEventCreate(&e) != hipSuccess) return -1;
        tail_ev.push_back(e);
    }
    if (hipEventRecord(tail_ev[at], s) != hipSuccess) return -1;
    tail_kind.resize(at / 2 + 1);
    tail_kind[at / 2] = (char)kind;
    tail_used = at + 2;
    return at;
}

void Amg::tail_end(hipStream_t s, int at)
{
    if (at >= 0) (void)hipEventRecord(tail_ev[at + 1], s);
}

int Amg::tail_read(double &ms_cycle, int &cycles, double &ms_setup)
{
    ms_cycle = ms_setup = 0;
    cycles = 0;
    for (int k = 0; k + 1 < tail_used; k += 2) {
        float m = 0;
        AMG_CHECK(hipEventElapsedTime(&m, tail_ev[k], tail_ev[k + 1]));
        if (tail_kind[k / 2] == 0) {
            ms_cycle += m;
            ++cycles;
        } else {
            ms_setup += m;
        }
    }
    tail_used = 0;
    return XFK_OK;
}

// XFK_AMG_REFOLD=0: a Newton refresh runs level 0 unfolded (the former way)
static bool refold_on()
{
    const char *e = std::getenv("XFK_AMG_REFOLD");   // (read per refresh: tests toggle it)
    return !(e && std::atoi(e) == 0);
}

static int refold_stage()
{
    const char *e = std::getenv("XFK_REFOLD_STAGE");   // (read per refresh: tests toggle it)
    return (e && std::atoi(e) == 0) ? 0 : 1;
}

int Amg::refresh(hipStream_t s, bool fold)
{
    AmgLevel &A = *L[0];
    const int n = A.n;
    // level 0's P~ belongs to the matrix it was formed from: re-formed below
    // for the new values (k_refold_p), or level 0 runs unfolded; a refresh
    // that unfolds keeps P~'s arrays, so a later one may fold again
    const bool refold = fold && A.fold_formed && !dist && refold_on() && A.fnnz > 0;
    A.fold = refold;
    AMG_CHECK(absd.alloc(std::max(1, n)));
    AMG_CHECK(rho_part.alloc(2 * (size_t)std::max(1, nb_str(n))));
    if (n > 0) {
        k_amg_rho<<<nb_str(n), kB, 0, s>>>(n, A.rowptr,
                                           ColView{A.col, A.has16 ? A.a16.p : nullptr, A.has16 ? A.a16b.p : nullptr},
                                           A.val, rho_part.p, absd.p, A.dinv.p);
        k_max_reduce<<<1, kMaxReduceT, 0, s>>>(nb_str(n), rho_part.p, omega, rho.p);
    }
    if (A.has32 && f32_sweep_on()) {   // the sweeps' f32 copy of the new values
        int rc = to_f32(s, n, A.rowptr, A.nnz, A.val, A.a32);
        if (rc != XFK_OK) return rc;
    }
    if (refold && n > 0) {   // P~ = (I - w D^-1 A_new) P over its own pattern (new D^-1 and rho above)
        if (A.has32) AMG_CHECK(A.f32v.alloc((size_t)std::max(1LL, A.fnnz)));   // (the setup's copy: same pattern)
        k_refold_p<<<(n + kRfRows - 1) / kRfRows, 256, 0, s>>>(n, rho.p, A.dinv.p, A.rowptr, A.col, A.val, A.prow.p,
                                                                A.pcol.p, A.pval.p, A.ftrow.p, A.ftcol.p, A.ftval.p,
                                                                A.has32 ? A.f32v.p : nullptr, refold_stage());
    }
    AMG_CHECK(hipGetLastError());
    return XFK_OK;
}

int Amg::vcycle(hipStream_t s, const double *r, double *u, const int *done, double *part_gam)
{
    gamma_done = false;
    if (!dist) {
        vcycle_level(*this, s, 0, r, u, done, part_gam);
        return XFK_OK;
    }
    int rc = XFK_OK;
    part_gam_ = part_gam;
    vc_dist(s, 0, r, u, done, rc);
    part_gam_ = nullptr;
    if (rc != XFK_OK) return rc;
    AMG_CHECK(hipGetLastError());
    return XFK_OK;
}

}  // namespace xfk

// xfk_device_init: loads this translation unit's code object onto the device
// (the first use of any of its kernels would otherwise do it inside a solve)
hipError_t xfk::warm_module_amg()
{
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&k_max_reduce));
}
