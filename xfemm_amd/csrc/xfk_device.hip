// HIP kernels of the fsolver static-2D hot path for MI355X (gfx950, CDNA4).
//
// Reference behaviour (temudschin/xfemm): FSolver::Static2D
// (cfemm/fsolver/static2d.cpp:53-1033) and CBigLinProb (cfemm/libfemm/spars.cpp).
// Design notes are in DESIGN.md; the host driver is xfk_api.hip.
//
// Conventions: 256-thread workgroups (4 waves of 64), f64 arithmetic (the
// reference is double), grid-wide reductions are deterministic two-level sums
// (wave shuffle -> LDS -> per-block partial -> last-arriving block sums the
// partials in block order).  The last-block hand-off follows the
// sc1-store / relaxed-ticket / sc1-load form of cdna_hip_programming.md
// Guideline 16 (no L2 write-back fences on the hot path).
#include "xfk_kernels.h"
#include "xfk_axi.h"
#include "xfk_spmv.h"

namespace xfk {

// --------------------------------------------------------------------------
// reduction helpers
// --------------------------------------------------------------------------

__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Sum over the workgroup; result valid in thread 0.  `lds` holds >= 4 doubles.
__device__ __forceinline__ double block_sum(double v, double *lds)
{
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) lds[wid] = v;
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x == 0) {
        const int nw = (blockDim.x + 63) >> 6;
        for (int w = 0; w < nw; ++w) r += lds[w];
    }
    return r;
}

// Publish NV per-block partial sums and decide whether this block arrived
// last.  Returns true in every thread of the last block, which may then read
// all partials with sc1 loads (ticket form, Guideline 16 table row 1).
template <int NV>
__device__ __forceinline__ bool publish_partials(const double (&v)[NV], double *partials,
                                                 unsigned *counter, int *lds_flag)
{
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k)
            __hip_atomic_store(&partials[k * gridDim.x + blockIdx.x], v[k], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *lds_flag = (t == gridDim.x - 1) ? 1 : 0;
    }
    __syncthreads();
    return *lds_flag != 0;
}

// In the last block: sum partials k of all blocks in block order (result in thread 0).
__device__ __forceinline__ double gather_partials(const double *partials, int k, double *lds)
{
    double s = 0.0;
    const int G = gridDim.x;
    // fixed per-thread strided order -> deterministic
    for (int i = threadIdx.x; i < G; i += blockDim.x)
        s += __hip_atomic_load(&partials[k * G + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return block_sum(s, lds);
}

__device__ __forceinline__ void reset_counter(unsigned *counter)
{
    __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// --------------------------------------------------------------------------
// symbolic phase: node->element lists, CSR pattern, colouring, slot maps
// --------------------------------------------------------------------------

__global__ void k_count_incidence(int NE, const int *__restrict__ p, int *__restrict__ deg)
{
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= NE) return;
    atomicAdd(&deg[p[3 * e + 0]], 1);
    atomicAdd(&deg[p[3 * e + 1]], 1);
    atomicAdd(&deg[p[3 * e + 2]], 1);
}

__global__ void k_fill_n2e(int NE, const int *__restrict__ p, const int *__restrict__ ptr,
                           int *__restrict__ cursor, int *__restrict__ n2e)
{
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= NE) return;
    for (int j = 0; j < 3; ++j) {
        int v = p[3 * e + j];
        int pos = atomicAdd(&cursor[v], 1);
        n2e[ptr[v] + pos] = e;
    }
}

// Node -> element lists by counting: per-node counts (atomic increments, order-
// free), an exclusive scan, a fill at atomically taken positions (arbitrary
// order within a node's list), then every node's short list sorted in
// registers -- each node's elements come out ascending, the order the radix
// sort below produced (the reference's AddTo order), in ~1/3 of its time
// (three 8-bit passes over 3 NE pairs)
__global__ void k_n2e_count(long long n3, const int *__restrict__ p, int *__restrict__ deg)
{
    const long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (k < n3) atomicAdd(&deg[p[k]], 1);
}

__global__ void k_n2e_fill(long long n3, const int *__restrict__ p, const int *__restrict__ ptr,
                           int *__restrict__ cursor, int *__restrict__ n2e)
{
    const long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (k >= n3) return;
    const int v = p[k];
    n2e[ptr[v] + atomicAdd(&cursor[v], 1)] = (int)(k / 3);
}

// The same counts and fill through LDS: a workgroup of 256 elements touches
// the nodes of a narrow window (element and node numberings are both banded),
// counts its incidences there and touches the global counters once per
// (workgroup, node) instead of once per incidence; the fill reserves one
// chunk of each node's list per workgroup and places its elements there
// through LDS cursors (the per-node sort below fixes the order).  A window
// wider than kN2eWin falls back to one global atomic per incidence.
constexpr int kN2eWin = 4096;
template <bool FILL>
__global__ void __launch_bounds__(256) k_n2e_tile(int NE, const int *__restrict__ p, const int *__restrict__ ptr,
                                                  int *__restrict__ cnt, int *__restrict__ n2e)
{
    __shared__ int h[kN2eWin];
    __shared__ int cur[FILL ? kN2eWin : 1];
    __shared__ int red[8];
    const int e = blockIdx.x * 256 + threadIdx.x;
    int v[3] = {0, 0, 0};
    int lo = INT_MAX, hi = INT_MIN;
    if (e < NE) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            v[j] = p[3 * e + j];
            lo = min(lo, v[j]);
            hi = max(hi, v[j]);
        }
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
    if (hi < lo) return;   // no element in this tile
    if ((long long)hi - lo >= kN2eWin) {   // wide window: one global atomic per incidence
        if (e < NE)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                if (!FILL) atomicAdd(&cnt[v[j]], 1);
                else n2e[ptr[v[j]] + atomicAdd(&cnt[v[j]], 1)] = e;
            }
        return;
    }
    const int w = hi - lo + 1;
    for (int c = threadIdx.x; c < w; c += 256) {
        h[c] = 0;
        if (FILL) cur[c] = 0;
    }
    __syncthreads();
    if (e < NE)
#pragma unroll
        for (int j = 0; j < 3; ++j) atomicAdd(&h[v[j] - lo], 1);
    __syncthreads();
    if (!FILL) {
        for (int c = threadIdx.x; c < w; c += 256)
            if (h[c]) atomicAdd(&cnt[lo + c], h[c]);
        return;
    }
    for (int c = threadIdx.x; c < w; c += 256) {
        const int m = h[c];
        if (m) h[c] = ptr[lo + c] + atomicAdd(&cnt[lo + c], m);   // this tile's chunk of node lo + c
    }
    __syncthreads();
    if (e < NE)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int c = v[j] - lo;
            n2e[h[c] + atomicAdd(&cur[c], 1)] = e;
        }
}

// lists of <= 16 elements: a register bitonic network (padding INT_MAX);
// longer ones (rare high-valence nodes): insertion sort in place
__device__ __forceinline__ void sort_node_list(int s, int e, int *__restrict__ n2e)
{
    const int len = e - s;
    if (len <= 1) return;
    if (len <= 16) {
        int a[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) a[q] = q < len ? n2e[s + q] : INT_MAX;
#pragma unroll
        for (int k = 2; k <= 16; k <<= 1)
#pragma unroll
            for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int o = q ^ j;
                    if (o > q) {
                        const bool up = (q & k) == 0;
                        const int x = a[q], y = a[o];
                        a[q] = up ? min(x, y) : max(x, y);
                        a[o] = up ? max(x, y) : min(x, y);
                    }
                }
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if (q < len) n2e[s + q] = a[q];
        return;
    }
    for (int i = s + 1; i < e; ++i) {
        const int key = n2e[i];
        int j = i - 1;
        while (j >= s && n2e[j] > key) {
            n2e[j + 1] = n2e[j];
            --j;
        }
        n2e[j + 1] = key;
    }
}

// nodes v0 <= v < NL (the row-length pass sorts the lists of the rows it builds)
__global__ void k_n2e_sort(int v0, int NL, const int *__restrict__ ptr, int *__restrict__ n2e)
{
    const int v = v0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= NL) return;
    sort_node_list(ptr[v], ptr[v + 1], n2e);
}

// Node -> element lists by a stable radix sort of the (node, element)
// incidence pairs (xfk_api.hip: build_symbolic): values k / 3 of the
// element-major incidence slots, then each node's first slot by a lower
// bound in the sorted keys (nodes of no element get an empty range)
__global__ void k_slot_elements(long long n3, int *__restrict__ v)
{
    const long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (k < n3) v[k] = (int)(k / 3);
}

__global__ void k_n2e_ptr(int NL, const int *__restrict__ keys, int n3, int *__restrict__ ptr)
{
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n > NL) return;
    int lo = 0, hi = n3;   // first slot with key >= n
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (keys[mid] < n) lo = mid + 1;
        else hi = mid;
    }
    ptr[n] = lo;
}

// Deterministic order of each node's element list (insertion sort, lists are short).
__global__ void k_sort_segments(int N, const int *__restrict__ ptr, int *__restrict__ a)
{
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= N) return;
    int s = ptr[v], e = ptr[v + 1];
    for (int i = s + 1; i < e; ++i) {
        int key = a[i];
        int j = i - 1;
        while (j >= s && a[j] > key) {
            a[j + 1] = a[j];
            --j;
        }
        a[j + 1] = key;
    }
}

// CSR row v = sorted unique {vertices of the elements incident to v} u
// {periodic fill-in columns of v} u {v}.  One thread per row gathers its
// candidates into LDS (or, for rows with more than kRowLds candidates, into
// its own region of `tmp`), sorts and de-duplicates them there, and leaves the
// row at tmp[cand_base(v)]; k_row_copy moves it to its CSR place after the
// row-length scan.
constexpr int kRowLds = 32;

struct RowCands {
    const int *p, *n2e_ptr, *n2e, *fill_ptr, *fill_col;
    __device__ __forceinline__ int count(int v) const
    {
        int ne = n2e_ptr[v + 1] - n2e_ptr[v];
        int nf = fill_ptr ? (fill_ptr[v + 1] - fill_ptr[v]) : 0;
        return 3 * ne + nf + 1;
    }
    __device__ __forceinline__ long long base(int v) const
    {
        return 3LL * n2e_ptr[v] + (fill_ptr ? fill_ptr[v] : 0) + v;
    }
};

__global__ void __launch_bounds__(kBlock) k_row_build(int N, RowCands rc, int *__restrict__ tmp,
                                                      int *__restrict__ rowcnt)
{
    __shared__ int s_c[kBlock * (kRowLds + 1)];
    const int v = blockIdx.x * kBlock + threadIdx.x;
    if (v >= N) return;
    const int m = rc.count(v);
    int *out = tmp + rc.base(v);
    int *c = (m <= kRowLds) ? &s_c[threadIdx.x * (kRowLds + 1)] : out;
    int k = 0;
    const int t1 = rc.n2e_ptr[v + 1];
    for (int t = rc.n2e_ptr[v]; t < t1; ++t) {
        const int f = rc.n2e[t];
        c[k++] = rc.p[3 * f];
        c[k++] = rc.p[3 * f + 1];
        c[k++] = rc.p[3 * f + 2];
    }
    if (rc.fill_ptr)
        for (int t = rc.fill_ptr[v]; t < rc.fill_ptr[v + 1]; ++t) c[k++] = rc.fill_col[t];
    c[k++] = v;
    // insertion sort, then unique
    for (int i = 1; i < m; ++i) {
        const int key = c[i];
        int j = i - 1;
        while (j >= 0 && c[j] > key) {
            c[j + 1] = c[j];
            --j;
        }
        c[j + 1] = key;
    }
    int u = 0;
    for (int i = 0; i < m; ++i)
        if (u == 0 || c[i] != c[u - 1]) c[u++] = c[i];
    if (c != out)
        for (int i = 0; i < u; ++i) out[i] = c[i];
    rowcnt[v] = u;
}

// Rows of up to kRowRegElems incident elements and no periodic fill-in (all
// but a few rows of a triangle mesh): the candidates -- v and the two other
// vertices of each incident element -- are sorted by a register bitonic
// network of 16 or 32 and de-duplicated there, twice: once for the row
// length, once (after the scan) writing the row in place.  No temporary rows,
// no copy pass.  Other rows take k_row_build / k_row_copy's path through tmp.
constexpr int kRowRegElems = 15;

template <int W>
__device__ __forceinline__ void bitonic_regs(int (&a)[W])
{
#pragma unroll
    for (int k = 2; k <= W; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
            for (int q = 0; q < W; ++q) {
                const int o = q ^ j;
                if (o > q) {
                    const bool up = (q & k) == 0;
                    const int x = a[q], y = a[o];
                    a[q] = up ? min(x, y) : max(x, y);
                    a[o] = up ? max(x, y) : min(x, y);
                }
            }
}

// candidates of row v (ne incident elements) into a[0 .. W): v, then two per
// element; unused slots INT_MAX
template <int W>
__device__ __forceinline__ void row_regs(int v, int s, int ne, const RowCands &rc, int (&a)[W])
{
    a[0] = v;
    int f[(W - 1) / 2];
#pragma unroll
    for (int q = 0; q < (W - 1) / 2; ++q) f[q] = q < ne ? rc.n2e[s + q] : -1;
#pragma unroll
    for (int q = 0; q < (W - 1) / 2; ++q) {
        int x = INT_MAX, y = INT_MAX, z = INT_MAX;
        if (f[q] >= 0) {
            x = rc.p[3 * f[q]];
            y = rc.p[3 * f[q] + 1];
            z = rc.p[3 * f[q] + 2];
        }
        a[1 + 2 * q] = x == v ? y : x;
        a[2 + 2 * q] = (x == v || y == v) ? z : y;
    }
#pragma unroll
    for (int q = 2 * ((W - 1) / 2) + 1; q < W; ++q) a[q] = INT_MAX;
    bitonic_regs(a);
}

__device__ __forceinline__ bool row_reg_ok(const RowCands &rc, int v, int ne)
{
    return ne <= kRowRegElems && !(rc.fill_ptr && rc.fill_ptr[v + 1] > rc.fill_ptr[v]);
}

template <int W>
__device__ __forceinline__ int row_regs_len(int v, int s, int ne, const RowCands &rc)
{
    int a[W];
    row_regs<W>(v, s, ne, rc, a);
    int u = 0;
#pragma unroll
    for (int q = 0; q < W; ++q) u += (a[q] != INT_MAX && (q == 0 || a[q] != a[q - 1])) ? 1 : 0;
    return u;
}

template <int W>
__device__ __forceinline__ void row_regs_write(int v, int s, int ne, const RowCands &rc, int r0,
                                               int *__restrict__ col, int *__restrict__ diag)
{
    int a[W];
    row_regs<W>(v, s, ne, rc, a);
    int u = 0;
#pragma unroll
    for (int q = 0; q < W; ++q)
        if (a[q] != INT_MAX && (q == 0 || a[q] != a[q - 1])) {
            col[r0 + u] = a[q];
            if (a[q] == v) diag[v] = r0 + u;
            ++u;
        }
}

// n2e_sort is rc.n2e itself (sorted in place, then read through rc.n2e): no
// __restrict__ on it, so the reads below stay ordered after the sort's stores
__global__ void __launch_bounds__(kBlock) k_row_len_reg(int N, RowCands rc, int *__restrict__ tmp,
                                                        int *__restrict__ rowcnt, int *n2e_sort)
{
    __shared__ int s_c[kBlock * (kRowLds + 1)];
    const int v = blockIdx.x * kBlock + threadIdx.x;
    if (v >= N) return;
    const int s = rc.n2e_ptr[v], ne = rc.n2e_ptr[v + 1] - s;
    // this row's element list into ascending order (the assembly's summation
    // order) -- the candidates below do not depend on it
    if (n2e_sort) sort_node_list(s, s + ne, n2e_sort);
    if (row_reg_ok(rc, v, ne)) {
        rowcnt[v] = ne <= 7 ? row_regs_len<16>(v, s, ne, rc) : row_regs_len<32>(v, s, ne, rc);
        return;
    }
    // long or periodic rows: candidates through LDS / tmp (k_row_build)
    const int m = rc.count(v);
    int *out = tmp + rc.base(v);
    int *c = (m <= kRowLds) ? &s_c[threadIdx.x * (kRowLds + 1)] : out;
    int k = 0;
    for (int t = s; t < s + ne; ++t) {
        const int f = rc.n2e[t];
        c[k++] = rc.p[3 * f];
        c[k++] = rc.p[3 * f + 1];
        c[k++] = rc.p[3 * f + 2];
    }
    if (rc.fill_ptr)
        for (int t = rc.fill_ptr[v]; t < rc.fill_ptr[v + 1]; ++t) c[k++] = rc.fill_col[t];
    c[k++] = v;
    for (int i = 1; i < m; ++i) {
        const int key = c[i];
        int j = i - 1;
        while (j >= 0 && c[j] > key) {
            c[j + 1] = c[j];
            --j;
        }
        c[j + 1] = key;
    }
    int u = 0;
    for (int i = 0; i < m; ++i)
        if (u == 0 || c[i] != c[u - 1]) c[u++] = c[i];
    if (c != out)
        for (int i = 0; i < u; ++i) out[i] = c[i];
    rowcnt[v] = u;
}

__global__ void k_row_fill_reg(int N, RowCands rc, const int *__restrict__ tmp, const int *__restrict__ rowptr,
                               int *__restrict__ col, int *__restrict__ diag)
{
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= N) return;
    const int s = rc.n2e_ptr[v], ne = rc.n2e_ptr[v + 1] - s;
    const int r0 = rowptr[v];
    if (row_reg_ok(rc, v, ne)) {
        if (ne <= 7) row_regs_write<16>(v, s, ne, rc, r0, col, diag);
        else row_regs_write<32>(v, s, ne, rc, r0, col, diag);
        return;
    }
    const int *src = tmp + rc.base(v);
    const int len = rowptr[v + 1] - r0;
    for (int i = 0; i < len; ++i) {
        const int c = src[i];
        col[r0 + i] = c;
        if (c == v) diag[v] = r0 + i;
    }
}

__global__ void k_row_copy(int N, RowCands rc, const int *__restrict__ tmp, const int *__restrict__ rowptr,
                           int *__restrict__ col, int *__restrict__ diag)
{
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= N) return;
    const int *src = tmp + rc.base(v);
    const int r0 = rowptr[v], len = rowptr[v + 1] - r0;
    for (int i = 0; i < len; ++i) {
        const int c = src[i];
        col[r0 + i] = c;
        if (c == v) diag[v] = r0 + i;
    }
}

__device__ __forceinline__ unsigned hash_u32(unsigned x)
{
    x ^= x >> 16; x *= 0x7feb352dU;
    x ^= x >> 15; x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// Jones-Plassmann colouring of the element conflict graph (two elements
// conflict when they share a node), expressed through the nodes.  Round r:
//   k_jp_nodes: for every node that still has a pending incident element,
//               the largest priority key among those elements and the mask
//               of colours its coloured incident elements hold;
//   k_jp_elems: a pending element whose key is the largest at all three of its
//               nodes (a local maximum: the winners of one round share no
//               node) takes the smallest colour absent from the three masks.
// Both passes read only the state left by the previous launch, so the
// colouring is deterministic.  They sweep the full arrays in mesh order with
// an early exit for finished items (an inactive node costs one byte read):
// compacted worklists needed atomics and scrambled the spatial order, both of
// which cost more than the sweep.  A workgroup with a pending element left
// after round r stores r + 1 into *pending_round (plain store, one per
// workgroup); the host stops when a round leaves it unchanged.
__device__ __forceinline__ unsigned long long jp_key(int e)
{
    return ((unsigned long long)hash_u32((unsigned)e) << 32) | (unsigned)e;
}

__global__ void __launch_bounds__(kBlock) k_jp_nodes(int N, unsigned char *__restrict__ active,
                                                     const int *__restrict__ n2e_ptr, const int *__restrict__ n2e,
                                                     const int *__restrict__ color,
                                                     unsigned long long *__restrict__ maxkey,
                                                     unsigned long long *__restrict__ used)
{
    const int v = blockIdx.x * kBlock + threadIdx.x;
    if (v >= N || !active[v]) return;
    unsigned long long mk = 0, u0 = 0, u1 = 0;
    bool pending = false;
    const int t1 = n2e_ptr[v + 1];
    for (int t = n2e_ptr[v]; t < t1; ++t) {
        const int f = n2e[t];
        const int c = color[f];
        if (c < 0) {
            const unsigned long long k = jp_key(f);
            mk = k > mk ? k : mk;
            pending = true;
        } else if (c < 64) {
            u0 |= 1ull << c;
        } else if (c < 128) {
            u1 |= 1ull << (c - 64);
        }
    }
    if (pending) {
        maxkey[v] = mk;
        used[2 * v] = u0;
        used[2 * v + 1] = u1;
    } else {
        active[v] = 0;
    }
}

__global__ void __launch_bounds__(kBlock) k_jp_elems(int NE, int round, int *__restrict__ pending_round,
                                                     const int *__restrict__ p,
                                                     const unsigned long long *__restrict__ maxkey,
                                                     const unsigned long long *__restrict__ used,
                                                     int *__restrict__ color)
{
    const int e = blockIdx.x * kBlock + threadIdx.x;
    bool lose = false;
    if (e < NE && color[e] < 0) {
        const unsigned long long k = jp_key(e);
        const int v0 = p[3 * e], v1 = p[3 * e + 1], v2 = p[3 * e + 2];
        lose = (maxkey[v0] != k) || (maxkey[v1] != k) || (maxkey[v2] != k);
        if (!lose) {
            const unsigned long long u0 = used[2 * v0] | used[2 * v1] | used[2 * v2];
            const unsigned long long u1 = used[2 * v0 + 1] | used[2 * v1 + 1] | used[2 * v2 + 1];
            int c;
            if (~u0) c = __ffsll((long long)~u0) - 1;
            else if (~u1) c = 64 + __ffsll((long long)~u1) - 1;
            else c = 255;  // > 128 colours: flagged by the host
            color[e] = c;
        }
    }
    if (__syncthreads_or(lose) && threadIdx.x == 0) *pending_round = round + 1;
}

// Count elements per colour (LDS-private histogram, one global atomic per bin
// per block).
__global__ void __launch_bounds__(kBlock) k_color_hist(int NE, const int *__restrict__ color, int *__restrict__ hist,
                                                       int maxc)
{
    __shared__ int h[256];
    for (int k = threadIdx.x; k < 256; k += kBlock) h[k] = 0;
    __syncthreads();
    for (int e = blockIdx.x * kBlock + threadIdx.x; e < NE; e += gridDim.x * kBlock) {
        const int c = color[e];
        atomicAdd(&h[c < maxc ? c : maxc], 1);
    }
    __syncthreads();
    for (int k = threadIdx.x; k <= maxc; k += kBlock)
        if (h[k]) atomicAdd(&hist[k], h[k]);
}

__global__ void k_iota(int n, int *__restrict__ a)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = i;
}

__global__ void k_build_erec(int NE, const int *__restrict__ perm, const int *__restrict__ p,
                             const int *__restrict__ lbl, const int *__restrict__ ebits_raw,
                             int4 *__restrict__ erec, int *__restrict__ ebits, int *__restrict__ iperm)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= NE) return;
    int e = perm[i];
    iperm[e] = i;
    erec[i] = make_int4(p[3 * e], p[3 * e + 1], p[3 * e + 2], lbl[e]);
    ebits[i] = ebits_raw[e];
}

__device__ __forceinline__ int find_slot(const int *__restrict__ rowptr, const int *__restrict__ col,
                                         int r, int c)
{
    int lo = rowptr[r], hi = rowptr[r + 1] - 1;
    while (lo <= hi) {
        int mid = (lo + hi) >> 1;
        int v = col[mid];
        if (v == c) return mid;
        if (v < c) lo = mid + 1;
        else hi = mid - 1;
    }
    return -1;
}

// slot[9 i + 3 j + k] = CSR position of (n_j, n_k) of the element at colour
// position i (-1 for the rows of halo nodes, which a sharded rank does not own).  Threads walk the elements in their raw (mesh, spatially
// coherent) order so that the row gathers hit in cache, one linear scan per
// row (independent loads; rows are short), and scatter the 9 slots to the
// element's colour position.
__global__ void k_build_slots(int NE, int nrows, const int *__restrict__ p, const int *__restrict__ iperm,
                              const int *__restrict__ rowptr, const int *__restrict__ col, int *__restrict__ slot,
                              int *__restrict__ bad)
{
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= NE) return;
    const int n[3] = {p[3 * e], p[3 * e + 1], p[3 * e + 2]};
    int *dst = slot + 9LL * iperm[e];
    int missing = 0;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        int s[3] = {-1, -1, -1};
        if (n[j] >= nrows) {          // halo row of a sharded problem: not assembled here
#pragma unroll
            for (int q = 0; q < 3; ++q) dst[3 * j + q] = -1;
            continue;
        }
        const int k1 = rowptr[n[j] + 1];
        for (int k = rowptr[n[j]]; k < k1; ++k) {
            const int c = col[k];
#pragma unroll
            for (int q = 0; q < 3; ++q) s[q] = (c == n[q]) ? k : s[q];
        }
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            missing |= (s[q] < 0);
            dst[3 * j + q] = s[q];
        }
    }
    if (missing) atomicAdd(bad, 1);
}

// (row, col) pairs -> CSR slots (periodic-map preparation)
__global__ void k_lookup_slots(int n, const int *__restrict__ rc, const int *__restrict__ rowptr,
                               const int *__restrict__ col, int *__restrict__ out)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = find_slot(rowptr, col, rc[2 * i], rc[2 * i + 1]);
}

// rows that hold a fixed (Dirichlet) column but are not fixed themselves
__global__ void k_mark_fix_adj(int N, const int *__restrict__ rowptr, const int *__restrict__ col,
                               const unsigned char *__restrict__ fixed, int *__restrict__ flag)
{
    int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= N) return;
    int f = 0;
    if (!fixed[r])
        for (int k = rowptr[r]; k < rowptr[r + 1]; ++k) f |= fixed[col[k]];
    flag[r] = f;
}

__global__ void k_compact_flags(int N, const int *__restrict__ flag, int *__restrict__ cursor,
                                int *__restrict__ out)
{
    int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= N || !flag[r]) return;
    out[atomicAdd(cursor, 1)] = r;
}

// --------------------------------------------------------------------------
// numeric assembly (static2d.cpp:352-816), one launch per colour
// --------------------------------------------------------------------------

// CMSolverMaterialProp::GetBHProps (CMaterialProp.cpp:997-1057), real axis.
__device__ void get_bh_props(const DevBlock &m, const double *__restrict__ Bt, const double *__restrict__ Ht,
                             const double *__restrict__ St, double B, double &v, double &dv)
{
    const double b = fabs(B);
    const int n = m.BHpoints;
    const double *Bd = Bt + m.bh_off, *Hd = Ht + m.bh_off, *sl = St + m.bh_off;
    if (b == 0) { v = sl[0]; dv = 0; return; }
    if (b > Bd[n - 1]) {
        double h = (Hd[n - 1] + sl[n - 1] * (b - Bd[n - 1]));
        double dh = sl[n - 1];
        v = h / b;
        dv = 0.5 * (dh / (b * b) - h / (b * b * b));
        return;
    }
    // the first knot interval with Bd[i] <= b <= Bd[i + 1], as the reference's
    // scan finds it; on a non-decreasing table that is the first i with
    // Bd[i + 1] >= b (b <= Bd[n - 1] here) if Bd[i] <= b, else none -- found
    // by bisection (~6 dependent loads instead of a scan of ~25 on M-19)
    int lo = -1;
    if (m.bh_sorted) {
        int l = 0, h = n - 2;
        while (l < h) {
            const int mid = (l + h) >> 1;
            if (Bd[mid + 1] >= b) h = mid;
            else l = mid + 1;
        }
        if (b >= Bd[l]) lo = l;
    } else {
        for (int i = 0; i < n - 1; ++i)
            if ((b >= Bd[i]) && (b <= Bd[i + 1])) {
                lo = i;
                break;
            }
    }
    if (lo < 0) return;
    const int i = lo;
    double l = (Bd[i + 1] - Bd[i]);
    double z = (b - Bd[i]) / l;
    double z2 = z * z;
    double h = (1. - 3. * z2 + 2. * z2 * z) * Hd[i] + z * (1. - 2. * z + z2) * l * sl[i] +
               z2 * (3. - 2. * z) * Hd[i + 1] + z2 * (z - 1.) * l * sl[i + 1];
    double dh = 6. * z * (z - 1.) * Hd[i] / l + (1. - 4. * z + 3. * z * z) * sl[i] +
                6. * z * (1. - z) * Hd[i + 1] / l + z * (3. * z - 2.) * sl[i + 1];
    v = h / b;
    dv = 0.5 * (dh / (b * b) - h / (b * b * b));
}

// FSolver::StaticAxisymmetric element (staticaxi.cpp:172-636): x is r, y is
// z.  Flux-formulation matrices with the logarithmic mean radius R_hat, r-
// weighted sources and boundary terms, B from the element energy, the
// exterior-region permeability warp.  Me / be are the element's contribution
// before the sign of the global assembly (as in the planar path).
template <bool FIRST>
__device__ __forceinline__ void axi_element(int eb, const AssembleArgs &A, const int (&n)[3], const double (&X)[3],
                            const double (&Y)[3], const DevLabel &lab, const DevBlock &bp, double &m1, double &m2,
                            double (&Me)[3][3], double (&be)[3])
{
    AxiGeom Gm;
    axi_geometry(X, Y, Gm);
    double Mn[3][3];
    const double(&Mx)[3][3] = Gm.Mx;
    const double(&My)[3][3] = Gm.My;
    const double a = Gm.a, R = Gm.R, vol = Gm.vol;
    for (int j = 0; j < 3; ++j) {
        for (int k = 0; k < 3; ++k) { Me[j][k] = 0.; Mn[j][k] = 0.; }
        be[j] = 0.;
    }
    // mixed boundary conditions (staticaxi.cpp:298-320)
    if (eb)
        for (int j = 0; j < 3; ++j) {
            const int ej = ((eb >> (10 * j)) & 1023) - 1;
            if (ej < 0) continue;
            const DevLine ln = A.lines[ej];
            if (ln.format != 2) continue;
            const int k = (j + 1) % 3;
            const double lj = sqrt(pow(X[k] - X[j], 2.) + pow(Y[k] - Y[j], 2.));
            const double r = (X[j] + X[k]) / 2.;
            double Kb = -0.0001 * kC * 2. * r * ln.c0 * lj / 6.;
            Me[j][j] += Kb * 2.;
            Me[k][k] += Kb * 2.;
            Me[j][k] += Kb;
            Me[k][j] += Kb;
            Kb = (ln.c1 * lj / 2.) * 0.0001 * 2 * r;
            be[j] += Kb;
            be[k] += Kb;
        }
    // source current density (staticaxi.cpp:322-337)
    double t = 0;
    if (lab.in_circuit >= 0) {
        const DevCirc C = A.circs[lab.in_circuit];
        if (C.ccase == 1) t = C.J;
        if (C.ccase == 0) t = -100. * C.dV * bp.Cduct / R;
    }
    const double Ks = -2. * R * (bp.J_re + t) * a / 3.;
    be[0] += Ks; be[1] += Ks; be[2] += Ks;
    // magnetisation (staticaxi.cpp:396-407)
    if (bp.H_c != 0.0)
        for (int j = 0; j < 3; ++j) {
            const int k = (j + 1) % 3;
            const double r = (X[j] + X[k]) / 2.;
            const double Km = -0.0001 * r * bp.H_c * (lab.cos_m * (X[k] - X[j]) + lab.sin_m * (Y[k] - Y[j]));
            be[j] += Km;
            be[k] += Km;
        }
    // permeability (staticaxi.cpp:409-632); m1 / m2 in: the element's Newton
    // state (iter > 0), out: its new state
    const double Vn[3] = {A.V[n[0]], A.V[n[1]], A.V[n[2]]};
    if (FIRST) {   // iter == 0: the blocks' linear permeabilities
        const double f = bp.LamFill;
        if (bp.LamType == 0) { m1 = bp.mu_x * f; m2 = bp.mu_y * f; }
        else if (bp.LamType == 1) { m1 = bp.mu_x * f + (1. - f); m2 = bp.mu_x / (f + bp.mu_x * (1. - f)); }
        else if (bp.LamType == 2) { m1 = bp.mu_y * f + (1. - f); m2 = bp.mu_y / (f + bp.mu_y * (1. - f)); }
        else { m1 = 1; m2 = 1; }
        if (lab.external) {
            const double Z = (Y[0] + Y[1] + Y[2]) / 3. - A.ext_zo;
            const double kludge = (R * R + Z * Z) * A.ext_ri / (A.ext_ro * A.ext_ro * A.ext_ro);
            m1 /= kludge;
            m2 /= kludge;
        }
    } else {
        if (bp.BHpoints > 0 && bp.LamType <= 2 && (bp.LamType != 0 || m1 == m2)) {
            const double f = bp.LamFill;
            const double sx = (bp.LamType == 2) ? 1. / (f * f) : 1., sy = (bp.LamType == 1) ? 1. / (f * f) : 1.;
            double v[3], u[3], dv = 0;
            for (int j = 0; j < 3; ++j) {
                v[j] = 0;
                for (int w = 0; w < 3; ++w) v[j] += (Mx[j][w] * sx + My[j][w] * sy) * Vn[w];
            }
            for (int j = 0; j < 3; ++j) dv += Vn[j] * v[j];
            dv *= (10000. * kC * kC / vol);
            const double B = sqrt(fabs(dv));
            double mu = 0;
            get_bh_props(bp, A.bhB, A.bhH, A.bhS, B, mu, dv);
            mu = 1. / (kMUO * mu);
            if (bp.LamType == 0) {
                m1 = mu; m2 = mu;
                for (int j = 0; j < 3; ++j) {
                    v[j] = 0;
                    for (int w = 0; w < 3; ++w) v[j] += (Mx[j][w] + My[j][w]) * Vn[w];
                }
                const double Kn = -200. * kC * kC * kC * dv / vol;
                for (int j = 0; j < 3; ++j)
                    for (int w = 0; w < 3; ++w) Mn[j][w] = Kn * v[j] * v[w];
            } else {
                if (bp.LamType == 1) { m1 = mu * f; m2 = mu / (f + mu * (1. - f)); }
                else { m2 = mu * f; m1 = mu / (f + mu * (1. - f)); }
                for (int j = 0; j < 3; ++j) {
                    v[j] = 0; u[j] = 0;
                    for (int w = 0; w < 3; ++w) {
                        if (bp.LamType == 1) {
                            v[j] += (My[j][w] / f + Mx[j][w]) * Vn[w];
                            u[j] += (My[j][w] / f + f * Mx[j][w]) * Vn[w];
                        } else {
                            v[j] += (Mx[j][w] / f + My[j][w]) * Vn[w];
                            u[j] += (Mx[j][w] / f + f * My[j][w]) * Vn[w];
                        }
                    }
                }
                const double Kn = -100. * kC * kC * kC * dv / (vol);
                for (int j = 0; j < 3; ++j)
                    for (int w = 0; w < 3; ++w) Mn[j][w] = Kn * (v[j] * u[w] + v[w] * u[j]);
            }
        }
    }
    // (two reciprocals instead of 18 f64 divisions: within an ulp of the
    // reference's Mx / m2 + My / m1, far inside the assembly tolerance)
    const double im1 = 1.0 / m1, im2 = 1.0 / m2;
    for (int j = 0; j < 3; ++j)
        for (int k = 0; k < 3; ++k) {
            Me[j][k] += (Mx[j][k] * im2 + My[j][k] * im1 + Mn[j][k]);
            be[j] += Mn[j][k] * Vn[k];
        }
}

// The Newton state of a planar element (static2d.cpp:600-640): B from the
// element's A, GetBHProps, the new permeabilities by lamination type; false
// (m1 / m2 kept) when the element's material is linear or its state says so.
// p / q / a: the element's geometry as planar_element forms it.
__device__ __forceinline__ bool planar_newton_state(const AssembleArgs &A, const DevBlock &bp, const double (&p)[3],
                                                    const double (&q)[3], double a, const double (&Vn)[3], double &m1,
                                                    double &m2, double &dv)
{
    dv = 0;
    if (!(bp.BHpoints > 0 && bp.LamType <= 2 && (bp.LamType != 0 || m1 == m2))) return false;
    const double f = bp.LamFill;
    double B1 = 0., B2 = 0.;
    if (bp.LamType == 0) {
        for (int j = 0; j < 3; ++j) { B1 += Vn[j] * q[j]; B2 += Vn[j] * p[j]; }
    } else if (bp.LamType == 1) {
        for (int j = 0; j < 3; ++j) { B1 += Vn[j] * q[j]; B2 += Vn[j] * p[j] / f; }
    } else {
        for (int j = 0; j < 3; ++j) { B1 += (Vn[j] * q[j]) / f; B2 += Vn[j] * p[j]; }
    }
    const double B = kC * sqrt(B1 * B1 + B2 * B2) / (0.02 * a);
    double mu = 0;
    get_bh_props(bp, A.bhB, A.bhH, A.bhS, B, mu, dv);
    mu = 1. / (kMUO * mu);
    if (bp.LamType == 0) { m1 = mu; m2 = mu; }
    else if (bp.LamType == 1) { m1 = mu * f; m2 = mu / (f + mu * (1. - f)); }
    else { m2 = mu * f; m1 = mu / (f + mu * (1. - f)); }
    return true;
}

// the Newton terms Mn of a planar element in the state above (static2d.cpp:640-797)
__device__ __forceinline__ void planar_newton_terms(const DevBlock &bp, const double (&Mx)[3][3],
                                                    const double (&My)[3][3], double a, const double (&Vn)[3],
                                                    double dv, double (&Mn)[3][3])
{
    const double f = bp.LamFill;
    double v[3], u[3];
    if (bp.LamType == 0) {
        for (int j = 0; j < 3; ++j) {
            v[j] = 0;
            for (int w = 0; w < 3; ++w) v[j] += (Mx[j][w] + My[j][w]) * Vn[w];
        }
        const double Kn = -200. * kC * kC * kC * dv / a;
        for (int j = 0; j < 3; ++j)
            for (int w = 0; w < 3; ++w) Mn[j][w] = Kn * v[j] * v[w];
    } else {
        for (int j = 0; j < 3; ++j) {
            v[j] = 0; u[j] = 0;
            for (int w = 0; w < 3; ++w) {
                if (bp.LamType == 1) {
                    v[j] += (My[j][w] / f + Mx[j][w]) * Vn[w];
                    u[j] += (My[j][w] / f + f * Mx[j][w]) * Vn[w];
                } else {
                    v[j] += (Mx[j][w] / f + My[j][w]) * Vn[w];
                    u[j] += (Mx[j][w] / f + f * My[j][w]) * Vn[w];
                }
            }
        }
        const double Kn = -100. * kC * kC * kC * dv / (a);
        for (int j = 0; j < 3; ++j)
            for (int w = 0; w < 3; ++w) Mn[j][w] = Kn * (v[j] * u[w] + v[w] * u[j]);
    }
}

// the element geometry of planar_element: p, q and the signed area a
__device__ __forceinline__ double planar_geometry(const double (&X)[3], const double (&Y)[3], double (&p)[3],
                                                  double (&q)[3])
{
    p[0] = Y[1] - Y[2]; p[1] = Y[2] - Y[0]; p[2] = Y[0] - Y[1];
    q[0] = X[2] - X[1]; q[1] = X[0] - X[2]; q[2] = X[1] - X[0];
    return (p[0] * q[1] - p[1] * q[0]) / 2.;
}

// FSolver::Static2D element (static2d.cpp:352-805): Me / be before the sign
// of the global assembly, m1 / m2 the element's permeability state.  PRE (a
// Newton pass, iter > 0): m1 / m2 are already the new state and pre_dv /
// pre_on its dv and whether the Newton terms apply (k_planar_state).
template <bool FIRST, bool PRE = false>
__device__ __forceinline__ void planar_element(int eb, const AssembleArgs &A, const int (&n)[3],
                                               const double (&X)[3], const double (&Y)[3], const DevLabel &lab,
                                               const DevBlock &bp, double &m1, double &m2, double (&Me)[3][3],
                                               double (&be)[3], double pre_dv = 0.0, bool pre_on = false)
{
    double p[3], q[3];
    const double a = planar_geometry(X, Y, p, q);
    const double K = (-1. / (4. * a));
    double Mx[3][3], My[3][3], Mn[3][3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            Mx[j][k] = K * p[j] * p[k];
            My[j][k] = K * q[j] * q[k];
            Me[j][k] = 0.;
            Mn[j][k] = 0.;
        }
        be[j] = 0.;
    }

    // mixed boundary conditions on the element's edges (static2d.cpp:459-480)
    if (eb) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            int ej = ((eb >> (10 * j)) & 1023) - 1;
            if (ej < 0) continue;
            const DevLine ln = A.lines[ej];
            if (ln.format != 2) continue;
            int k = (j + 1) % 3;
            double lj = sqrt(pow(X[k] - X[j], 2.) + pow(Y[k] - Y[j], 2.));
            double Kb = -0.0001 * kC * ln.c0 * lj / 6.;
            Me[j][j] += Kb * 2.;
            Me[k][k] += Kb * 2.;
            Me[j][k] += Kb;
            Me[k][j] += Kb;
            Kb = (ln.c1 * lj / 2.) * 0.0001;
            be[j] += Kb;
            be[k] += Kb;
        }
    }

    // source current density (static2d.cpp:482-507)
    double t = 0;
    if (lab.in_circuit >= 0) {
        const DevCirc C = A.circs[lab.in_circuit];
        if (C.ccase == 1) t = C.J;
        if (C.ccase == 0) t = -C.dV * bp.Cduct;
    }
    const double Ks = -(bp.J_re + t) * a / 3.;
    be[0] += Ks; be[1] += Ks; be[2] += Ks;

    // magnetisation (static2d.cpp:584-598)
    if (bp.H_c != 0.0) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            int k = (j + 1) % 3;
            double Km = 0.0001 * bp.H_c * (lab.cos_m * (X[k] - X[j]) + lab.sin_m * (Y[k] - Y[j])) / 2.;
            be[j] += Km;
            be[k] += Km;
        }
    }

    // permeability (static2d.cpp:600-797); m1 / m2 in: the element's Newton
    // state (iter > 0), out: its new state
    const double Vn[3] = {A.V[n[0]], A.V[n[1]], A.V[n[2]]};
    if (FIRST) {   // iter == 0: the blocks' linear permeabilities
        const double f = bp.LamFill;
        if (bp.LamType == 0) { m1 = bp.mu_x * f + (1. - f); m2 = bp.mu_y * f + (1. - f); }
        else if (bp.LamType == 1) { m1 = bp.mu_x * f + (1. - f); m2 = bp.mu_x / (f + bp.mu_x * (1. - f)); }
        else if (bp.LamType == 2) { m2 = bp.mu_y * f + (1. - f); m1 = bp.mu_y / (f + bp.mu_y * (1. - f)); }
        else { m1 = 1; m2 = 1; }
    } else {
        double dv = pre_dv;
        const bool on = PRE ? pre_on : planar_newton_state(A, bp, p, q, a, Vn, m1, m2, dv);
        if (on) planar_newton_terms(bp, Mx, My, a, Vn, dv, Mn);
    }

    // element matrix, v12 == 0 outside incremental problems (static2d.cpp:799-805)
    // (two reciprocals instead of 18 f64 divisions: within an ulp of the
    // reference's Mx / m2 + My / m1, far inside the assembly tolerance)
    const double im1 = 1.0 / m1, im2 = 1.0 / m2;
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            Me[j][k] += (Mx[j][k] * im2 + My[j][k] * im1 + Mn[j][k]);
            be[j] += Mn[j][k] * Vn[k];
        }

}

// Row-gather assembly (static planar / axisymmetric): one thread per owned CSR
// row i sums the contributions of the elements incident on node i, in
// ascending element order -- the order the reference's AddTo accumulates each
// entry in -- so no colouring, no element -> slot maps and no zeroing pass are
// needed, and every row is written exactly once.  Each element is evaluated
// once per vertex (3x the arithmetic of a scatter, none of its random
// read-modify-writes).  Rows of <= kRowAcc entries accumulate in LDS, longer
// ones (air-gap rings, periodic corners) in place in val (the row is private
// to its thread).  The element's permeability state is read from mu*_in and
// written to mu*_out by the thread of its first owned vertex.
constexpr int kRowBlock = 128;
constexpr int kRowAcc = 12;

// XCD: consecutive row blocks on one XCD (xcd_tile), so the coordinates and
// element data a block shares with the blocks a mesh row away stay in that
// XCD's L2 (round-robin blocks fetched them once per XCD: 470 MB of HBM
// traffic per launch for ~100 MB of algorithmic bytes on configs[2])
template <bool AXI, bool FIRST, bool XCD, bool PRE>
__device__ __forceinline__ void assemble_rows(int N, const AssembleArgs &A)
{
    __shared__ double s_acc[kRowAcc * kRowBlock];
    __shared__ int s_col[kRowAcc * kRowBlock];
    const int i0 = (XCD ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x) * kRowBlock;
    const int i = i0 + threadIdx.x;
    const bool live = i < N;   // (every thread reaches the barriers below)
    const int rs = live ? A.rowptr[i] : 0, L = live ? A.rowptr[i + 1] - rs : 0;
    const bool lds = L <= kRowAcc;
    double *acc = lds ? s_acc + threadIdx.x : A.val + rs;
    const int stride = lds ? kRowBlock : 1;
    const int *cols = lds ? s_col + threadIdx.x : A.col + rs;
    for (int k = 0; k < L; ++k) {
        acc[k * stride] = 0.;
        if (lds) s_col[k * kRowBlock + threadIdx.x] = A.col[rs + k];
    }
    double bi = 0.;
    bool miss = false;
    const int t1 = live ? A.n2e_ptr[i + 1] : 0;
    for (int t = live ? A.n2e_ptr[i] : 0; t < t1; ++t) {
        const int e = A.n2e[t];
        const int n[3] = {A.p_raw[3 * e], A.p_raw[3 * e + 1], A.p_raw[3 * e + 2]};
        const int j = (n[0] == i) ? 0 : ((n[1] == i) ? 1 : 2);
        const DevLabel lab = A.labels[A.lbl_raw[e]];
        const DevBlock bp = A.blocks[lab.blk];
        const double X[3] = {A.x[n[0]], A.x[n[1]], A.x[n[2]]};
        const double Y[3] = {A.y[n[0]], A.y[n[1]], A.y[n[2]]};
        double m1 = 0., m2 = 0., Me[3][3], be[3];
        if (PRE) {   // the new state, from k_planar_state
            m1 = A.mu1_out[e];
            m2 = A.mu2_out[e];
        } else if (!FIRST) {
            m1 = A.mu1[e];
            m2 = A.mu2[e];
        }
        if (AXI) axi_element<FIRST>(A.ebits_raw[e], A, n, X, Y, lab, bp, m1, m2, Me, be);
        else if (PRE) planar_element<false, true>(A.ebits_raw[e], A, n, X, Y, lab, bp, m1, m2, Me, be, A.dv_el[e], A.on_el[e] != 0);
        else planar_element<FIRST>(A.ebits_raw[e], A, n, X, Y, lab, bp, m1, m2, Me, be);
        const int w = (n[0] < N) ? 0 : ((n[1] < N) ? 1 : 2);
        if (!PRE && w == j && A.mu1_out) {   // (linear problems keep no permeability state)
            A.mu1_out[e] = m1;
            A.mu2_out[e] = m2;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            // row j of Me, upper values (exact symmetry), selected without
            // dynamic register indexing
            const double m = (j == 0) ? Me[0][k] : ((j == 1) ? ((k >= 1) ? Me[1][k] : Me[0][1])
                                                             : ((k == 2) ? Me[2][2] : Me[k][2]));
            int pos = 0;
            while (pos < L - 1 && cols[pos * stride] != n[k]) ++pos;
            miss |= cols[pos * stride] != n[k];
            acc[pos * stride] -= m;
        }
        bi -= (j == 0) ? be[0] : ((j == 1) ? be[1] : be[2]);
    }
    if (miss && A.miss) *A.miss = 1;   // an element entry outside the row's pattern (read with the PCG's first poll)
    // The block's rows are one contiguous run of val: when every row sat in
    // LDS, the values are laid out linearly in LDS and written with
    // consecutive lanes on consecutive entries (whole cache lines), instead of
    // each lane storing its own row (64 partial lines per store).
    if (__syncthreads_and(lds)) {
        double r[kRowAcc];
#pragma unroll
        for (int k = 0; k < kRowAcc; ++k) r[k] = k < L ? s_acc[k * kRowBlock + threadIdx.x] : 0.;
        const int rb0 = A.rowptr[i0], rb1 = A.rowptr[min(i0 + kRowBlock, N)];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kRowAcc; ++k)
            if (k < L) s_acc[rs - rb0 + k] = r[k];
        __syncthreads();
        for (int m = threadIdx.x; m < rb1 - rb0; m += kRowBlock) A.val[rb0 + m] = s_acc[m];
    } else if (lds) {
        for (int k = 0; k < L; ++k) A.val[rs + k] = s_acc[k * kRowBlock + threadIdx.x];
    }
    if (live) A.b[i] = bi;
}

template <bool AXI, bool FIRST, bool XCD = true>
__global__ void __launch_bounds__(kRowBlock) k_assemble_rows(int N, AssembleArgs A)
{
    assemble_rows<AXI, FIRST, XCD, false>(N, A);
}

// the planar Newton pass after k_planar_state: 4 waves per SIMD (132 VGPRs
// unbounded, 3 waves)
__global__ void __launch_bounds__(kRowBlock, 4) k_assemble_rows_pre(int N, AssembleArgs A)
{
    assemble_rows<false, false, true, true>(N, A);
}

// A planar Newton pass: each element's new state once (planar_newton_state),
// for the three rows that gather it (k_assemble_rows<PRE>)
__global__ void __launch_bounds__(256) k_planar_state(int NE, AssembleArgs A)
{
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= NE) return;
    const DevLabel lab = A.labels[A.lbl_raw[e]];
    const DevBlock bp = A.blocks[lab.blk];
    double m1 = A.mu1[e], m2 = A.mu2[e], dv = 0;
    bool on = false;
    if (bp.BHpoints > 0 && bp.LamType <= 2 && (bp.LamType != 0 || m1 == m2)) {
        const int n[3] = {A.p_raw[3 * e], A.p_raw[3 * e + 1], A.p_raw[3 * e + 2]};
        const double X[3] = {A.x[n[0]], A.x[n[1]], A.x[n[2]]};
        const double Y[3] = {A.y[n[0]], A.y[n[1]], A.y[n[2]]};
        const double Vn[3] = {A.V[n[0]], A.V[n[1]], A.V[n[2]]};
        double p[3], q[3];
        const double a = planar_geometry(X, Y, p, q);
        on = planar_newton_state(A, bp, p, q, a, Vn, m1, m2, dv);
    }
    A.mu1_out[e] = m1;
    A.mu2_out[e] = m2;
    A.dv_el[e] = dv;
    A.on_el[e] = on ? 1 : 0;
}

// point currents (static2d.cpp:818-825)
__global__ void k_point_currents(int n, const int *__restrict__ nodes, const double *__restrict__ J,
                                 double *__restrict__ b)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[nodes[i]] += J[i];
}

// CBigLinProb::SetValue (spars.cpp:318-346) for every fixed node: its row
// keeps only the diagonal, b = diag * value (last value set wins)
__global__ void k_dirichlet_rows(int n, const int *__restrict__ rows, const int *__restrict__ rowptr,
                                 const int *__restrict__ diag, double *__restrict__ val,
                                 double *__restrict__ b, const double *__restrict__ fix_last)
{
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    int r = rows[t];
    int d = diag[r];
    for (int k = rowptr[r]; k < rowptr[r + 1]; ++k)
        if (k != d) val[k] = 0.0;
    b[r] = val[d] * fix_last[r];
}

// the column half of SetValue: b[k] -= A(k,i)*x_i, A(k,i) = 0 (first value set)
__device__ __forceinline__ void dirichlet_col_row(int r, const int *__restrict__ rowptr, const int *__restrict__ col,
                                                  const unsigned char *__restrict__ fixed,
                                                  const double *__restrict__ fix_first, double *__restrict__ val,
                                                  double *__restrict__ b)
{
    double br = b[r];
    for (int k = rowptr[r]; k < rowptr[r + 1]; ++k) {
        int c = col[k];
        if (fixed[c]) {
            double z = val[k];
            if (z != 0) {
                br = br - (z * fix_first[c]);
                val[k] = 0.0;
            }
        }
    }
    b[r] = br;
}
__global__ void k_dirichlet_cols(int n, const int *__restrict__ rows, const int *__restrict__ rowptr,
                                 const int *__restrict__ col, const unsigned char *__restrict__ fixed,
                                 const double *__restrict__ fix_first, double *__restrict__ val,
                                 double *__restrict__ b)
{
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    dirichlet_col_row(rows[t], rowptr, col, fixed, fix_first, val, b);
}
// the same with the row count on the device (left there by the symbolic
// phase: no host read-back), grid-stride
__global__ void k_dirichlet_cols_d(const int *__restrict__ count, const int *__restrict__ rows,
                                   const int *__restrict__ rowptr, const int *__restrict__ col,
                                   const unsigned char *__restrict__ fixed, const double *__restrict__ fix_first,
                                   double *__restrict__ val, double *__restrict__ b)
{
    const int n = *count;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x)
        dirichlet_col_row(rows[t], rowptr, col, fixed, fix_first, val, b);
}

// (anti)periodic averaging map (CBigLinProb::Periodicity / AntiPeriodicity,
// spars.cpp:366-474, composed on the host): dst <- sum w * src, two phases
__global__ void k_map_gather(int n, const int *__restrict__ ptr, const int *__restrict__ src,
                             const double *__restrict__ w, const double *__restrict__ data,
                             double *__restrict__ tmp)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double s = 0.0;
    for (int k = ptr[i]; k < ptr[i + 1]; ++k) s += w[k] * data[src[k]];
    tmp[i] = s;
}

// air-gap element values at their CSR slots (one thread per unique slot)
__global__ void k_add_at_slots(int n, const int *__restrict__ slot, const double *__restrict__ v,
                               double *__restrict__ data)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) data[slot[i]] += v[i];
}

__global__ void k_map_scatter(int n, const int *__restrict__ dst, const double *__restrict__ tmp,
                              double *__restrict__ data)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) data[dst[i]] = tmp[i];
}

// Jacobi preconditioner + the reference's singularity check (spars.cpp:245)
__global__ void k_diag_inv(int N, const int *__restrict__ diag, const double *__restrict__ val,
                           double *__restrict__ dinv, CgState *__restrict__ S)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    double d = val[diag[i]];
    if (d == 0.0) {
        S->singular = 1;
        dinv[i] = 0.0;
    } else {
        dinv[i] = 1.0 / d;
    }
}

// nonlinear residual sums (static2d.cpp:953-970)
__global__ void __launch_bounds__(kBlock) k_newton_res(int N, const double *__restrict__ V,
                                                       const double *__restrict__ Vold, double *partials,
                                                       unsigned *counter, NewtonScalars *S)
{
    __shared__ double red[8];
    __shared__ int last;
    double dx = 0.0, vv = 0.0;
    // two rows per lane and step (16-B loads; V, Vold hipMalloc'd), the odd
    // last row by the lane that would hold its pair
    const int np = N >> 1;
    for (int q = blockIdx.x * kBlock + threadIdx.x; q < np; q += gridDim.x * kBlock) {
        const double2 v = reinterpret_cast<const double2 *>(V)[q], o = reinterpret_cast<const double2 *>(Vold)[q];
        const double d0 = v.x - o.x, d1 = v.y - o.y;
        dx += d0 * d0;
        dx += d1 * d1;
        vv += v.x * v.x;
        vv += v.y * v.y;
    }
    if ((N & 1) && blockIdx.x * kBlock + threadIdx.x == np % (gridDim.x * kBlock)) {
        const double v = V[N - 1], d = v - Vold[N - 1];
        dx += d * d;
        vv += v * v;
    }
    double v[2];
    v[0] = block_sum(dx, red);
    v[1] = block_sum(vv, red);
    if (publish_partials<2>(v, partials, counter, &last)) {
        double a0 = gather_partials(partials, 0, red);
        double a1 = gather_partials(partials, 1, red);
        if (threadIdx.x == 0) {
            S->dx2 = a0;
            S->v2 = a1;
            reset_counter(counter);
        }
    }
}

__global__ void k_relax(int N, double relax, double *__restrict__ V, const double *__restrict__ Vold)
{
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < N; r += gridDim.x * blockDim.x)
        V[r] = relax * V[r] + (1.0 - relax) * Vold[r];
}

__global__ void k_scale(int N, double s, const double *__restrict__ V, double *__restrict__ out)
{
    int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < N) out[r] = V[r] * s;
}

// --------------------------------------------------------------------------
// launch wrappers (host side)
// --------------------------------------------------------------------------

static inline int nblk(long long n) { return (int)((n + kBlock - 1) / kBlock); }

int grid_reduce(int N)
{
    int t = (N + kBlock - 1) / kBlock;
    return t < kRedGrid ? (t > 0 ? t : 1) : kRedGrid;
}

void launch_count_incidence(hipStream_t s, int NE, const int *p, int *deg)
{
    if (NE) k_count_incidence<<<nblk(NE), kBlock, 0, s>>>(NE, p, deg);
}
void launch_fill_n2e(hipStream_t s, int NE, const int *p, const int *ptr, int *cursor, int *n2e)
{
    if (NE) k_fill_n2e<<<nblk(NE), kBlock, 0, s>>>(NE, p, ptr, cursor, n2e);
}
// XFK_N2E_TILE=0: one global atomic per incidence (measurement)
static bool n2e_tile_on()
{
    static const bool v = [] {
        const char *e = std::getenv("XFK_N2E_TILE");
        return !(e && std::atoi(e) == 0);
    }();
    return v;
}
void launch_n2e_count(hipStream_t s, int NE, const int *p, int *deg)
{
    const long long n3 = 3LL * NE;
    if (NE && n2e_tile_on()) k_n2e_tile<false><<<(NE + 255) / 256, 256, 0, s>>>(NE, p, nullptr, deg, nullptr);
    else if (NE) k_n2e_count<<<(unsigned)((n3 + kBlock - 1) / kBlock), kBlock, 0, s>>>(n3, p, deg);
}
void launch_n2e_fill(hipStream_t s, int NE, const int *p, const int *ptr, int *cursor, int *n2e)
{
    const long long n3 = 3LL * NE;
    if (NE && n2e_tile_on()) k_n2e_tile<true><<<(NE + 255) / 256, 256, 0, s>>>(NE, p, ptr, cursor, n2e);
    else if (NE) k_n2e_fill<<<(unsigned)((n3 + kBlock - 1) / kBlock), kBlock, 0, s>>>(n3, p, ptr, cursor, n2e);
}
void launch_n2e_sort(hipStream_t s, int v0, int NL, const int *ptr, int *n2e)
{
    if (NL > v0) k_n2e_sort<<<nblk(NL - v0), kBlock, 0, s>>>(v0, NL, ptr, n2e);
}
void launch_slot_elements(hipStream_t s, int NE, int *v)
{
    const long long n3 = 3LL * NE;
    if (NE) k_slot_elements<<<(unsigned)((n3 + kBlock - 1) / kBlock), kBlock, 0, s>>>(n3, v);
}
void launch_n2e_ptr(hipStream_t s, int NL, const int *keys, int n3, int *ptr)
{
    k_n2e_ptr<<<nblk(NL + 1), kBlock, 0, s>>>(NL, keys, n3, ptr);
}
void launch_sort_segments(hipStream_t s, int N, const int *ptr, int *a)
{
    if (N) k_sort_segments<<<nblk(N), kBlock, 0, s>>>(N, ptr, a);
}
// XFK_ROW_REG=0: every CSR row through k_row_build / k_row_copy (measurement)
static bool row_reg_on()
{
    static const bool v = [] {
        const char *e = std::getenv("XFK_ROW_REG");
        return !(e && std::atoi(e) == 0);
    }();
    return v;
}
long long row_tmp_size(int N, int NE, int nfill) { return 9LL * NE + nfill + N; }
void launch_row_build(hipStream_t s, int N, const int *p, const int *n2e_ptr, const int *n2e, const int *fill_ptr,
                      const int *fill_col, int *tmp, int *rowcnt, int *n2e_sort)
{
    if (n2e_sort && !row_reg_on()) launch_n2e_sort(s, 0, N, n2e_ptr, n2e_sort);   // (the LDS path sorts nothing)
    RowCands rc{p, n2e_ptr, n2e, fill_ptr, fill_col};
    if (N && row_reg_on()) k_row_len_reg<<<nblk(N), kBlock, 0, s>>>(N, rc, tmp, rowcnt, n2e_sort);
    else if (N) k_row_build<<<nblk(N), kBlock, 0, s>>>(N, rc, tmp, rowcnt);
}
void launch_row_copy(hipStream_t s, int N, const int *p, const int *n2e_ptr, const int *n2e, const int *fill_ptr,
                     const int *fill_col, const int *tmp, const int *rowptr, int *col, int *diag)
{
    RowCands rc{p, n2e_ptr, n2e, fill_ptr, fill_col};
    if (N && row_reg_on()) k_row_fill_reg<<<nblk(N), kBlock, 0, s>>>(N, rc, tmp, rowptr, col, diag);
    else if (N) k_row_copy<<<nblk(N), kBlock, 0, s>>>(N, rc, tmp, rowptr, col, diag);
}
void launch_jp_round(hipStream_t s, int N, int NE, int round, unsigned char *active, int *pending_round,
                     const int *p, const int *n2e_ptr, const int *n2e, int *color, unsigned long long *maxkey,
                     unsigned long long *used)
{
    if (N) k_jp_nodes<<<nblk(N), kBlock, 0, s>>>(N, active, n2e_ptr, n2e, color, maxkey, used);
    if (NE) k_jp_elems<<<nblk(NE), kBlock, 0, s>>>(NE, round, pending_round, p, maxkey, used, color);
}
void launch_color_hist(hipStream_t s, int NE, const int *color, int *hist, int maxc)
{
    if (NE) k_color_hist<<<std::min(nblk(NE), 2048), kBlock, 0, s>>>(NE, color, hist, maxc);
}
void launch_iota(hipStream_t s, int n, int *a)
{
    if (n) k_iota<<<nblk(n), kBlock, 0, s>>>(n, a);
}
void launch_build_erec(hipStream_t s, int NE, const int *perm, const int *p, const int *lbl, const int *ebits_raw,
                       int4 *erec, int *ebits, int *iperm)
{
    if (NE) k_build_erec<<<nblk(NE), kBlock, 0, s>>>(NE, perm, p, lbl, ebits_raw, erec, ebits, iperm);
}
void launch_build_slots(hipStream_t s, int NE, int nrows, const int *p, const int *iperm, const int *rowptr,
                        const int *col, int *slot, int *bad)
{
    if (NE) k_build_slots<<<nblk(NE), kBlock, 0, s>>>(NE, nrows, p, iperm, rowptr, col, slot, bad);
}
void launch_lookup_slots(hipStream_t s, int n, const int *rc, const int *rowptr, const int *col, int *out)
{
    if (n) k_lookup_slots<<<nblk(n), kBlock, 0, s>>>(n, rc, rowptr, col, out);
}
void launch_mark_fix_adj(hipStream_t s, int N, const int *rowptr, const int *col, const unsigned char *fixed,
                         int *flag)
{
    if (N) k_mark_fix_adj<<<nblk(N), kBlock, 0, s>>>(N, rowptr, col, fixed, flag);
}
void launch_compact_flags(hipStream_t s, int N, const int *flag, int *cursor, int *out)
{
    if (N) k_compact_flags<<<nblk(N), kBlock, 0, s>>>(N, flag, cursor, out);
}
void launch_assemble_rows(hipStream_t s, int N, const AssembleArgs &A)
{
    if (N <= 0) return;
    const int g = (N + kRowBlock - 1) / kRowBlock;
    // XFK_ASM_XCD=0: round-robin row blocks (measurement)
    static const bool xcd = [] {
        const char *e = std::getenv("XFK_ASM_XCD");
        return !(e && std::atoi(e) == 0);
    }();
    if (!xcd && !A.axi) {
        if (A.iter == 0) k_assemble_rows<false, true, false><<<g, kRowBlock, 0, s>>>(N, A);
        else k_assemble_rows<false, false, false><<<g, kRowBlock, 0, s>>>(N, A);
        return;
    }
    if (A.axi) {
        if (A.iter == 0) k_assemble_rows<true, true><<<g, kRowBlock, 0, s>>>(N, A);
        else k_assemble_rows<true, false><<<g, kRowBlock, 0, s>>>(N, A);
    } else {
        if (A.iter == 0) {
            k_assemble_rows<false, true><<<g, kRowBlock, 0, s>>>(N, A);
        } else if (A.dv_el && A.mu1_out) {
            if (A.n_el > 0) k_planar_state<<<(A.n_el + 255) / 256, 256, 0, s>>>(A.n_el, A);
            k_assemble_rows_pre<<<g, kRowBlock, 0, s>>>(N, A);
        } else {
            k_assemble_rows<false, false><<<g, kRowBlock, 0, s>>>(N, A);
        }
    }
}

void launch_point_currents(hipStream_t s, int n, const int *nodes, const double *J, double *b)
{
    if (n) k_point_currents<<<nblk(n), kBlock, 0, s>>>(n, nodes, J, b);
}
void launch_dirichlet(hipStream_t s, int nrows, const int *rows, int nadj, const int *nadj_dev, int nadj_max,
                      const int *adj, const int *rowptr, const int *col, const int *diag, const unsigned char *fixed,
                      const double *fix_first, const double *fix_last, double *val, double *b)
{
    if (nadj < 0) {   // count on the device, at most nadj_max
        if (nadj_max > 0)
            k_dirichlet_cols_d<<<std::min(nblk(nadj_max), 1024), kBlock, 0, s>>>(nadj_dev, adj, rowptr, col, fixed,
                                                                              fix_first, val, b);
    } else if (nadj) {
        k_dirichlet_cols<<<nblk(nadj), kBlock, 0, s>>>(nadj, adj, rowptr, col, fixed, fix_first, val, b);
    }
    if (nrows) k_dirichlet_rows<<<nblk(nrows), kBlock, 0, s>>>(nrows, rows, rowptr, diag, val, b, fix_last);
}
void launch_add_at_slots(hipStream_t s, int n, const int *slot, const double *v, double *data)
{
    if (n) k_add_at_slots<<<nblk(n), kBlock, 0, s>>>(n, slot, v, data);
}
void launch_map(hipStream_t s, int n, const int *dst, const int *ptr, const int *src, const double *w,
                double *data, double *tmp)
{
    if (!n) return;
    k_map_gather<<<nblk(n), kBlock, 0, s>>>(n, ptr, src, w, data, tmp);
    k_map_scatter<<<nblk(n), kBlock, 0, s>>>(n, dst, tmp, data);
}
void launch_diag_inv(hipStream_t s, int N, const int *diag, const double *val, double *dinv, CgState *S)
{
    if (N) k_diag_inv<<<nblk(N), kBlock, 0, s>>>(N, diag, val, dinv, S);
}
void launch_newton_res(hipStream_t s, int N, const double *V, const double *Vold, double *partials,
                       unsigned *counter, NewtonScalars *S)
{
    // (256 workgroups: the last-workgroup ticket is one atomic per workgroup
    // on one counter -- 1024 of them cost ~15 us of a 21 us launch at 1M rows)
    k_newton_res<<<std::min(grid_reduce(N), 256), kBlock, 0, s>>>(N, V, Vold, partials, counter, S);
}
void launch_relax(hipStream_t s, int N, double relax, double *V, const double *Vold)
{
    k_relax<<<grid_reduce(N), kBlock, 0, s>>>(N, relax, V, Vold);
}
void launch_scale(hipStream_t s, int N, double sc, const double *V, double *out)
{
    if (N) k_scale<<<nblk(N), kBlock, 0, s>>>(N, sc, V, out);
}

}  // namespace xfk

// xfk_device_init: loads this translation unit's code object onto the device
// (the first use of any of its kernels would otherwise do it inside a solve)
hipError_t xfk::warm_module_device()
{
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&k_count_incidence));
}
