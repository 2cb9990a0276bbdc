// FEASolver::SortElements (cfemm/libfemm/cuthill.cpp:39-86 of the reference)
// on the device: the comb sort of the elements by p0 + p1 + p2, pass for
// pass, with the reference's gap sequence (gap * 10 / 13, 9 and 10 -> 11), its
// strict-decrease swap test and its stop rule -- `while ((gap > 1) && (i > 0))`:
// the sort ends after the first pass that swaps nothing, or after the first
// gap-1 pass, so its result need not be sorted -- an unstable sort whose order
// is the one the reference's swaps leave, so every pass is simulated.  The
// host enqueues the whole gap sequence; a pass that swapped nothing sets a
// device stop flag that turns the later passes into copies (no host round
// trip per pass).
//
// One pass with gap g compares (j, j + g) for j ascending.  Positions form g
// classes (j mod g); a pass over one class is a bubble pass: the entry carried
// into position k is c_k = op(c_{k-1}, x_k), op(c, x) = c if score(c) >
// score(x) else x (max over (score, position)), and position k receives
// score(c_k) > score(x_{k+1}) ? x_{k+1} : c_k -- an associative scan.  With the
// array seen as rows of g positions (class = column), a pass is a column
// scan: per chunk of kRows rows the op-reduction of each column, the
// exclusive scan of those over the chunks (the carries), then each chunk
// rescanned from its carry, writing the pass's output out of place.  The
// all-zero key (score 0) is op's identity from the left.
//
// Keys: score << 32 | element index (scores < 2^32 for meshes < 1.4G nodes).
// HBM traffic per pass: ~3 x 8 B per element; 52 passes on a 2M-element mesh
// take ~1-2 ms against ~45 ms for the host comb sort on 16 cores.
#include "xfk_internal.h"

namespace xfk {
namespace {

constexpr int kRows = 16;

__device__ __forceinline__ unsigned long long sort_op(unsigned long long c, unsigned long long x)
{
    return (c >> 32) > (x >> 32) ? c : x;
}

__global__ void k_sort_keys(int n, const unsigned *score, unsigned long long *key)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) key[i] = ((unsigned long long)score[i] << 32) | (unsigned)i;
}

__global__ void k_sort_perm(int n, const unsigned long long *key, int *perm)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) perm[i] = (int)(key[i] & 0xffffffffULL);
}

// red[b g + c] = op over rows [b kRows, (b + 1) kRows) of column c, b < nb - 1
// (every such chunk holds whole rows)
__global__ void k_comb_reduce(long long total, int g, const unsigned long long *__restrict__ key,
                              unsigned long long *__restrict__ red, const int *__restrict__ stop)
{
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total || *stop) return;
    const long long b = t / g;
    const int c = (int)(t - b * g);
    const unsigned long long *k = key + b * kRows * (long long)g + c;
    unsigned long long x[kRows];
#pragma unroll
    for (int i = 0; i < kRows; ++i) x[i] = k[(long long)i * g];
    unsigned long long r = 0;
#pragma unroll
    for (int i = 0; i < kRows; ++i) r = sort_op(r, x[i]);
    red[t] = r;
}

// carries, few chunks per column: one thread per column, cin[b g + c] =
// op(red[0 .. b - 1][c]) for b in [1, nb)
__global__ void k_comb_carry_seq(int g, long long nb, const unsigned long long *__restrict__ red,
                                 unsigned long long *__restrict__ cin, const int *__restrict__ stop)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= g || *stop) return;
    unsigned long long acc = 0;
    for (long long b = 1; b < nb; ++b) {
        acc = sort_op(acc, red[(b - 1) * g + c]);
        cin[b * g + c] = acc;
    }
}

// carries, many chunks per column: one workgroup per column, each thread a
// contiguous segment of the column's m = nb - 1 chunk reductions
__global__ __launch_bounds__(256) void k_comb_carry_wg(int g, long long nb, const unsigned long long *__restrict__ red,
                                                       unsigned long long *__restrict__ cin,
                                                       const int *__restrict__ stop)
{
    __shared__ unsigned long long sh[256];
    if (*stop) return;   // (uniform over the workgroup)
    const int c = blockIdx.x;
    const long long m = nb - 1;
    const long long seg = (m + 255) / 256;
    const long long b0 = threadIdx.x * seg, b1 = b0 + seg < m ? b0 + seg : m;
    unsigned long long r = 0;
    for (long long b = b0; b < b1; ++b) r = sort_op(r, red[b * g + c]);
    sh[threadIdx.x] = r;
    __syncthreads();
    // inclusive scan over the 256 segment reductions (Hillis-Steele; op is
    // associative, later segments on the right)
    for (int d = 1; d < 256; d <<= 1) {
        const unsigned long long v = threadIdx.x >= d ? sh[threadIdx.x - d] : 0ULL;
        __syncthreads();
        if (threadIdx.x >= d) sh[threadIdx.x] = sort_op(v, sh[threadIdx.x]);
        __syncthreads();
    }
    unsigned long long acc = threadIdx.x ? sh[threadIdx.x - 1] : 0ULL;
    for (long long b = b0; b < b1; ++b) {
        acc = sort_op(acc, red[b * g + c]);
        cin[(b + 1) * g + c] = acc;
    }
}

// the pass: thread (b, c) rescans rows [b kRows, ...) of column c from its
// carry and writes the pass's output; flag[0] = 1 when some entry moved.
// After the stop (flag[1]) the pass is a copy.
__global__ void k_comb_scan(long long n, int g, long long nb, const unsigned long long *__restrict__ key,
                            const unsigned long long *__restrict__ cin, unsigned long long *__restrict__ out,
                            int *__restrict__ flag)
{
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nb * (long long)g) return;
    const long long b = t / g;
    const int c = (int)(t - b * g);
    int *any = flag;
    if (flag[1]) {
        long long q = b * kRows * (long long)g + c;
        for (int i = 0; i < kRows && q < n; ++i, q += g) out[q] = key[q];
        return;
    }
    unsigned long long car = b ? cin[t] : 0ULL;
    long long q = b * kRows * (long long)g + c;
    bool moved = false;
    for (int i = 0; i < kRows && q < n; ++i, q += g) {
        const unsigned long long cc = sort_op(car, key[q]);   // c_k
        car = cc;
        if (q + g < n) {
            const unsigned long long nx = key[q + g];          // x_{k+1}
            const bool sw = (cc >> 32) > (nx >> 32);
            out[q] = sw ? nx : cc;
            moved |= sw;
        } else {
            out[q] = cc;                                        // the carried entry lands
        }
    }
    if (moved) *any = 1;
}

// end of a pass: one that swapped nothing stops the sort (cuthill.cpp:81)
__global__ void k_comb_flag(int *flag)
{
    if (!flag[1] && !flag[0]) flag[1] = 1;
    flag[0] = 0;
}

inline unsigned nblk(long long n, int b = 256) { return (unsigned)((n + b - 1) / b); }

}  // namespace

int sort_elements_device(hipStream_t s, int n, const unsigned *score_dev, int *perm_dev, unsigned long long *key,
                         unsigned long long *tmp, unsigned long long *red, unsigned long long *cin, int *flag,
                         int *passes)
{
    k_sort_keys<<<nblk(n), 256, 0, s>>>(n, score_dev, key);
    XFK_CHECK(hipMemsetAsync(flag, 0, 2 * sizeof(int), s));   // (this pass moved, stopped)
    int gap = n, np = 0;
    do {
        if (gap > 1) {   // cuthill.cpp:63-70
            gap = (gap * 10) / 13;
            if ((gap == 10) || (gap == 9)) gap = 11;
        }
        const long long R = ((long long)n + gap - 1) / gap;
        const long long nb = (R + kRows - 1) / kRows;
        if (nb > 1) {
            k_comb_reduce<<<nblk((nb - 1) * gap), 256, 0, s>>>((nb - 1) * gap, gap, key, red, flag + 1);
            if (nb - 1 <= 64) k_comb_carry_seq<<<nblk(gap), 256, 0, s>>>(gap, nb, red, cin, flag + 1);
            else k_comb_carry_wg<<<gap, 256, 0, s>>>(gap, nb, red, cin, flag + 1);
        }
        k_comb_scan<<<nblk(nb * gap), 256, 0, s>>>(n, gap, nb, key, cin, tmp, flag);
        k_comb_flag<<<1, 1, 0, s>>>(flag);
        std::swap(key, tmp);
        ++np;
    } while (gap > 1);   // (the stop on a pass without swaps is the device flag's)
    k_sort_perm<<<nblk(n), 256, 0, s>>>(n, key, perm_dev);
    XFK_CHECK(hipGetLastError());
    if (passes) *passes = np;
    return XFK_OK;
}

}  // namespace xfk

// xfk_device_init: loads this translation unit's code object onto the device
// (the first use of any of its kernels would otherwise do it inside a solve)
hipError_t xfk::warm_module_sort()
{
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&k_sort_keys));
}
