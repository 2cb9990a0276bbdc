// Device helpers shared by the PCG (xfk_pcg.hip) and the AMG V-cycle
// (xfk_amg.hip): wavefront/workgroup sums and the CSR-stream tile SpMV.
#pragma once

#include <hip/hip_runtime.h>

namespace xfk {

constexpr int kCgBlock = 512;             // 8 waves; one row tile per workgroup
constexpr int kCgCap = 8 * kCgBlock;      // products staged per LDS pass (64 KiB)

__device__ __forceinline__ double cg_wave_sum(double v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// two simultaneous workgroup sums, results broadcast to every thread
__device__ __forceinline__ void cg_block_sum2(double &a, double &b, double *red)
{
    a = cg_wave_sum(a);
    b = cg_wave_sum(b);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) {
        red[2 * wid] = a;
        red[2 * wid + 1] = b;
    }
    __syncthreads();
    double sa = 0.0, sb = 0.0;
    const int nw = blockDim.x >> 6;
    for (int w = 0; w < nw; ++w) {
        sa += red[2 * w];
        sb += red[2 * w + 1];
    }
    a = sa;
    b = sb;
}

// deterministic sum of G partials (pairs) of the previous launch, in every block
__device__ __forceinline__ void cg_reduce_partials(const double *__restrict__ part, int G, double &a, double &b,
                                                   double *red)
{
    double sa = 0.0, sb = 0.0;
    for (int i = threadIdx.x; i < G; i += blockDim.x) {
        sa += part[i];
        sb += part[G + i];
    }
    cg_block_sum2(sa, sb, red);
    a = sa;
    b = sb;
}

// XCD-aware tile order: workgroup b is dispatched to XCD b % 8, so XCD x gets
// the contiguous run of tiles [x q + min(x, r), ...) (q = nb / 8, r = nb % 8)
// and its L2 serves the x-vector reuse between neighbouring tiles of a banded
// matrix instead of every XCD fetching every tile's halo of x
__device__ __forceinline__ int xcd_tile(int b, int nb)
{
    const int q = nb >> 3, r = nb & 7, x = b & 7, k = b >> 3;
    return x * q + min(x, r) + k;
}

// a device flag read as a per-lane (vector) load: a scalar load would be
// waited for together with the kernel arguments (the scalar cache's counter
// is waited to zero), before any other load is issued; as a vector load it
// is in flight with the tile's first loads and the branch on it waits for it
// alone.  The empty asm makes the zero index opaque to the compiler.
// (p == nullptr reads a zero flag; selecting the pointer instead of
// branching keeps the load in straight-line code: a branch around it would
// be closed by a wait for it)
static __device__ int xfk_zero_flag = 0;
__device__ __forceinline__ int load_flag_v(const int *p)
{
    int z = 0;
    asm volatile("" : "+v"(z));
    const int *q = p ? p : &xfk_zero_flag;
    return q[z];
}

// a tile's column base (kNoColBase without 16-bit offsets), read like a flag
static __device__ int xfk_no_col_base = -2147483647 - 1;
__device__ __forceinline__ int load_col_base(const int *base, int t)
{
    int z = 0;
    asm volatile("" : "+v"(z));
    const int *q = base ? base + t : &xfk_no_col_base;
    return q[z];
}

// the tile's row range and this thread's row: loaded first, so a kernel can
// have them in flight together with its other early loads (the convergence
// flag, its own row's vector entries) before it branches on any of them
struct TileRows {
    int s, e, my_s, my_e;
};
// (the tile's bounds are read by vector loads too -- a scalar load would be
// sunk below the kernel's first branch -- and moved to scalar registers by
// cg_tile_spmv)
template <int B = kCgBlock>
__device__ __forceinline__ TileRows tile_rows(int r0, int N, const int *__restrict__ rowptr)
{
    const int r = r0 + threadIdx.x;
    const int rend = min(r0 + B, N);
    int z = 0;
    asm volatile("" : "+v"(z));
    TileRows t;
    t.s = rowptr[r0 + z];
    t.e = rowptr[rend + z];
    t.my_s = (r < N) ? rowptr[r] : 0;
    t.my_e = (r < N) ? rowptr[r + 1] : 0;
    return t;
}

// y = sum_k val[k] * X(col[k]) for the B rows of one tile (B threads, one
// row each); CSR-stream: the tile's products are staged through LDS by
// coalesced 16-B reads -- each lane takes 4 consecutive nonzeros per slot (one
// int4 of col, two double2 of val; the stream realigned to 4 entries, the
// partial quads at its ends read per entry), 2 slots per lane per pass -- then
// each thread sums its own row in order.  Measured on the configs[2] matrix
// (tools/lab/spmv_lab.hip): 16.5 us vs 19.9 us for one 4/8-B entry per lane,
// bit-identical sums.  col / val must be 16-B aligned (hipMalloc'd arrays).
// SLOTS: 4-entry slots per lane per pass (CAP = 4 SLOTS B products staged per
// pass, lds holds CAP doubles): 2 for the ~7 entries per row of the fine
// level, more for the longer rows of coarse levels and of R, so that a tile
// takes one pass (each pass is a load / barrier / sum / barrier round trip)
// Columns come either as the CSR's int array or as 16-bit offsets from a
// per-tile base (TileCols16: 2 B instead of 4 B per nonzero, the same column
// indices, so the same bits); a tile whose columns span more than 65535
// carries kNoColBase and reads the int array.
constexpr int kNoColBase = -2147483647 - 1;

// V: the stored value type -- double, or float for the AMG's level-0 transfer
// and smoother operators (products and sums in double either way)
template <int B, int SLOTS, class V, class C4, class C1, class XF>
__device__ __forceinline__ double tile_spmv_impl(const TileRows &tr, C4 cols4, C1 col1,
                                                 const V *__restrict__ val, XF X, double *lds)
{
    constexpr int CAP = 4 * SLOTS * B;
    const int s = __builtin_amdgcn_readfirstlane(tr.s), e = __builtin_amdgcn_readfirstlane(tr.e);
    const int my_s = tr.my_s, my_e = tr.my_e;
    double acc = 0.0;
    for (int c0 = s & ~3; c0 < e; c0 += CAP) {
        const int c1 = min(e, c0 + CAP);
#pragma unroll
        for (int m = 0; m < SLOTS; ++m) {
            const int k = c0 + 4 * (threadIdx.x + m * B);
            if (k >= s && k + 3 < c1) {
                const int4 c = cols4(k);
                if constexpr (sizeof(V) == 8) {
                    const double2 v0 = *reinterpret_cast<const double2 *>(val + k);
                    const double2 v1 = *reinterpret_cast<const double2 *>(val + k + 2);
                    lds[k - c0] = v0.x * X(c.x);
                    lds[k + 1 - c0] = v0.y * X(c.y);
                    lds[k + 2 - c0] = v1.x * X(c.z);
                    lds[k + 3 - c0] = v1.y * X(c.w);
                } else {
                    const float4 v = *reinterpret_cast<const float4 *>(val + k);
                    lds[k - c0] = (double)v.x * X(c.x);
                    lds[k + 1 - c0] = (double)v.y * X(c.y);
                    lds[k + 2 - c0] = (double)v.z * X(c.z);
                    lds[k + 3 - c0] = (double)v.w * X(c.w);
                }
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (k + q >= s && k + q < c1) lds[k + q - c0] = (double)val[k + q] * X(col1(k + q));
            }
        }
        __syncthreads();
        const int a = max(my_s, c0), z = min(my_e, c1);
        for (int k = a; k < z; ++k) acc += lds[k - c0];
        __syncthreads();
    }
    return acc;
}

template <int B = kCgBlock, int SLOTS = 2, class V, class XF>
__device__ __forceinline__ double cg_tile_spmv(const TileRows &tr, const int *__restrict__ col,
                                               const V *__restrict__ val, XF X, double *lds)
{
    return tile_spmv_impl<B, SLOTS>(
        tr, [&](int k) { return *reinterpret_cast<const int4 *>(col + k); }, [&](int k) { return col[k]; }, val, X,
        lds);
}

// the same with 16-bit column offsets when the tile has a base (cb)
template <int B = kCgBlock, int SLOTS = 2, class V, class XF>
__device__ __forceinline__ double cg_tile_spmv16(const TileRows &tr, const unsigned short *__restrict__ c16, int cb,
                                                 const int *__restrict__ col, const V *__restrict__ val, XF X,
                                                 double *lds)
{
    cb = __builtin_amdgcn_readfirstlane(cb);
    if (cb == kNoColBase) return cg_tile_spmv<B, SLOTS>(tr, col, val, X, lds);
    return tile_spmv_impl<B, SLOTS>(
        tr,
        [&](int k) {
            const uint2 u = *reinterpret_cast<const uint2 *>(c16 + k);
            return make_int4(cb + (int)(u.x & 0xffffu), cb + (int)(u.x >> 16), cb + (int)(u.y & 0xffffu),
                             cb + (int)(u.y >> 16));
        },
        [&](int k) { return cb + (int)c16[k]; }, val, X, lds);
}

template <int B = kCgBlock, int SLOTS = 2, class XF>
__device__ __forceinline__ double cg_tile_spmv(int r0, int N, const int *__restrict__ rowptr,
                                               const int *__restrict__ col, const double *__restrict__ val,
                                               XF X, double *lds)
{
    return cg_tile_spmv<B, SLOTS>(tile_rows<B>(r0, N, rowptr), col, val, X, lds);
}

// Per-tile 16-bit column offsets of a CSR (tiles of B rows): base[t] = the
// tile's smallest column, c16[k] = col[k] - base[t]; kNoColBase when the
// tile's columns span more than 65535.  One workgroup per tile.
template <int B>
__global__ void __launch_bounds__(256) k_tile_col16(int n, const int *__restrict__ rowptr,
                                                    const int *__restrict__ col, unsigned short *__restrict__ c16,
                                                    int *__restrict__ base)
{
    __shared__ int red[2 * 4];
    const int t = blockIdx.x, r0 = t * B, r1 = min(n, r0 + B);
    const int s = rowptr[r0], e = rowptr[r1];
    int lo = 2147483647, hi = -2147483647 - 1;
    for (int k = s + threadIdx.x; k < e; k += 256) {
        const int c = col[k];
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
    const bool fits = e == s || (long long)hi - lo <= 65535;
    if (threadIdx.x == 0) base[t] = fits ? (e == s ? 0 : lo) : kNoColBase;
    if (!fits) return;
    for (int k = s + threadIdx.x; k < e; k += 256) c16[k] = (unsigned short)(col[k] - lo);
}

}  // namespace xfk
