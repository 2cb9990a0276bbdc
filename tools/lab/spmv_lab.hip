// SpMV variant lab (dev tool, not product): times CSR SpMV kernels on a real
// matrix dumped by tools/lab/spmv_lab.py (rowptr / col / val of the configs[2]
// system) and checks each against the reference kernel bit for bit.
//
//   V0  current product kernel (xfk_spmv.h cg_tile_spmv, 512-row LDS tiles)
//   V1  V0 with 16-bit column offsets (col - row), 10 B / nonzero
//   V2  256-row tiles, 16 products per thread per LDS pass
//   V3  one row per lane, direct gathers (no LDS)
//   V4  V1 with wide (16 B) loads of val / offsets
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

typedef int nt_i4 __attribute__((ext_vector_type(4)));
typedef int nt_i2 __attribute__((ext_vector_type(2)));
typedef double nt_d2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int xcd_tile(int b, int nb)
{
    const int q = nb >> 3, r = nb & 7, x = b & 7, k = b >> 3;
    return x * q + min(x, r) + k;
}

template <int B, int PER>
__global__ void __launch_bounds__(B) k_v0(int N, const int *__restrict__ rowptr, const int *__restrict__ col,
                                          const double *__restrict__ val, const double *__restrict__ x,
                                          double *__restrict__ y)
{
    constexpr int CAP = PER * B;
    __shared__ double lds[CAP];
    const int t = xcd_tile(blockIdx.x, gridDim.x);
    const int r0 = t * B;
    const int r = r0 + threadIdx.x;
    const int rend = min(r0 + B, N);
    const int s = rowptr[r0], e = rowptr[rend];
    const int my_s = (r < N) ? rowptr[r] : 0, my_e = (r < N) ? rowptr[r + 1] : 0;
    double acc = 0.0;
    for (int c0 = s; c0 < e; c0 += CAP) {
        const int c1 = min(e, c0 + CAP);
        int cidx[PER];
        double v[PER];
#pragma unroll
        for (int m = 0; m < PER; ++m) {
            const int k = c0 + threadIdx.x + m * B;
            cidx[m] = (k < c1) ? col[k] : -1;
            v[m] = (k < c1) ? val[k] : 0.0;
        }
#pragma unroll
        for (int m = 0; m < PER; ++m) {
            const int k = c0 + threadIdx.x + m * B;
            if (cidx[m] >= 0) lds[k - c0] = v[m] * x[cidx[m]];
        }
        __syncthreads();
        const int a = max(my_s, c0), z = min(my_e, c1);
        for (int k = a; k < z; ++k) acc += lds[k - c0];
        __syncthreads();
    }
    if (r < N) y[r] = acc;
}

// 16-bit column offsets: the nonzero's row is found from the tile's row
// pointers staged in LDS (binary search), col = row + off
template <int B, int PER>
__global__ void __launch_bounds__(B) k_v1(int N, const int *__restrict__ rowptr, const short *__restrict__ off,
                                          const double *__restrict__ val, const double *__restrict__ x,
                                          double *__restrict__ y)
{
    constexpr int CAP = PER * B;
    __shared__ double lds[CAP];
    __shared__ int srp[B + 1];
    const int t = xcd_tile(blockIdx.x, gridDim.x);
    const int r0 = t * B;
    const int r = r0 + threadIdx.x;
    const int rend = min(r0 + B, N);
    for (int k = threadIdx.x; k <= rend - r0; k += B) srp[k] = rowptr[r0 + k];
    __syncthreads();
    const int nr = rend - r0;
    const int s = srp[0], e = srp[nr];
    const int my_s = (r < N) ? srp[threadIdx.x] : 0, my_e = (r < N) ? srp[threadIdx.x + 1] : 0;
    double acc = 0.0;
    for (int c0 = s; c0 < e; c0 += CAP) {
        const int c1 = min(e, c0 + CAP);
#pragma unroll
        for (int m = 0; m < PER; ++m) {
            const int k = c0 + threadIdx.x + m * B;
            if (k < c1) {
                // row of nonzero k: largest i with srp[i] <= k
                int lo = 0, hi = nr - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (srp[mid] <= k) lo = mid;
                    else hi = mid - 1;
                }
                lds[k - c0] = val[k] * x[r0 + lo + off[k]];
            }
        }
        __syncthreads();
        const int a = max(my_s, c0), z = min(my_e, c1);
        for (int k = a; k < z; ++k) acc += lds[k - c0];
        __syncthreads();
    }
    if (r < N) y[r] = acc;
}

// one row per lane
__global__ void __launch_bounds__(256) k_v3(int N, const int *__restrict__ rowptr, const int *__restrict__ col,
                                            const double *__restrict__ val, const double *__restrict__ x,
                                            double *__restrict__ y)
{
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= N) return;
    double acc = 0.0;
    for (int k = rowptr[r]; k < rowptr[r + 1]; ++k) acc += val[k] * x[col[k]];
    y[r] = acc;
}

// V4: row-per-lane order of products with wide loads: a wave takes 64 rows;
// the tile's (off, val) stream is read 16 B per lane into LDS, then each lane
// sums its row -- same summation order as V0
template <int B>
__global__ void __launch_bounds__(B) k_v4(int N, const int *__restrict__ rowptr, const int *__restrict__ col,
                                          const double *__restrict__ val, const double *__restrict__ x,
                                          double *__restrict__ y)
{
    constexpr int CAP = 8 * B;
    __shared__ double lds[CAP];
    const int t = xcd_tile(blockIdx.x, gridDim.x);
    const int r0 = t * B;
    const int r = r0 + threadIdx.x;
    const int rend = min(r0 + B, N);
    const int s = rowptr[r0], e = rowptr[rend];
    const int my_s = (r < N) ? rowptr[r] : 0, my_e = (r < N) ? rowptr[r + 1] : 0;
    double acc = 0.0;
    const int s2 = s & ~1;   // 16-B aligned start of val pairs
    for (int c0 = s2; c0 < e; c0 += CAP) {
        const int c1 = min(e, c0 + CAP);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int k = c0 + 2 * (threadIdx.x + m * B);   // even
            if (k + 1 < c1 && k >= s) {
                const double2 v = *reinterpret_cast<const double2 *>(val + k);
                const int2 c = *reinterpret_cast<const int2 *>(col + k);
                lds[k - c0] = v.x * x[c.x];
                lds[k + 1 - c0] = v.y * x[c.y];
            } else {
                if (k >= s && k < c1) lds[k - c0] = val[k] * x[col[k]];
                if (k + 1 >= s && k + 1 < c1) lds[k + 1 - c0] = val[k + 1] * x[col[k + 1]];
            }
        }
        __syncthreads();
        const int a = max(my_s, c0), z = min(my_e, c1);
        for (int k = a; k < z; ++k) acc += lds[k - c0];
        __syncthreads();
    }
    if (r < N) y[r] = acc;
}

// V5: 4 entries per lane-slot: one 16-B int4 load of col + two 16-B double2
// loads of val (the tile's stream realigned to 4 entries), PER slots per lane
template <int B, int PER, bool NT>
__global__ void __launch_bounds__(B) k_v5(int N, const int *__restrict__ rowptr, const int *__restrict__ col,
                                          const double *__restrict__ val, const double *__restrict__ x,
                                          double *__restrict__ y)
{
    constexpr int CAP = 4 * PER * B;
    __shared__ double lds[CAP];
    const int t = xcd_tile(blockIdx.x, gridDim.x);
    const int r0 = t * B;
    const int r = r0 + threadIdx.x;
    const int rend = min(r0 + B, N);
    const int s = rowptr[r0], e = rowptr[rend];
    const int my_s = (r < N) ? rowptr[r] : 0, my_e = (r < N) ? rowptr[r + 1] : 0;
    double acc = 0.0;
    const int s4 = s & ~3;
    for (int c0 = s4; c0 < e; c0 += CAP) {
        const int c1 = min(e, c0 + CAP);
#pragma unroll
        for (int m = 0; m < PER; ++m) {
            const int k = c0 + 4 * (threadIdx.x + m * B);
            if (k + 3 < c1 && k >= s) {
                int4 c;
                double2 v0, v1;
                if (NT) {
                    const nt_i4 ci = __builtin_nontemporal_load(reinterpret_cast<const nt_i4 *>(col + k));
                    const nt_d2 a0 = __builtin_nontemporal_load(reinterpret_cast<const nt_d2 *>(val + k));
                    const nt_d2 a1 = __builtin_nontemporal_load(reinterpret_cast<const nt_d2 *>(val + k + 2));
                    c = make_int4(ci.x, ci.y, ci.z, ci.w);
                    v0 = make_double2(a0.x, a0.y);
                    v1 = make_double2(a1.x, a1.y);
                } else {
                    c = *reinterpret_cast<const int4 *>(col + k);
                    v0 = *reinterpret_cast<const double2 *>(val + k);
                    v1 = *reinterpret_cast<const double2 *>(val + k + 2);
                }
                lds[k - c0] = v0.x * x[c.x];
                lds[k + 1 - c0] = v0.y * x[c.y];
                lds[k + 2 - c0] = v1.x * x[c.z];
                lds[k + 3 - c0] = v1.y * x[c.w];
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (k + q >= s && k + q < c1) lds[k + q - c0] = val[k + q] * x[col[k + q]];
            }
        }
        __syncthreads();
        const int a = max(my_s, c0), z = min(my_e, c1);
        for (int k = a; k < z; ++k) acc += lds[k - c0];
        __syncthreads();
    }
    if (r < N) y[r] = acc;
}

// V6: V4 (pairs) with nontemporal matrix loads
template <int B>
__global__ void __launch_bounds__(B) k_v6(int N, const int *__restrict__ rowptr, const int *__restrict__ col,
                                          const double *__restrict__ val, const double *__restrict__ x,
                                          double *__restrict__ y)
{
    constexpr int CAP = 8 * B;
    __shared__ double lds[CAP];
    const int t = xcd_tile(blockIdx.x, gridDim.x);
    const int r0 = t * B;
    const int r = r0 + threadIdx.x;
    const int rend = min(r0 + B, N);
    const int s = rowptr[r0], e = rowptr[rend];
    const int my_s = (r < N) ? rowptr[r] : 0, my_e = (r < N) ? rowptr[r + 1] : 0;
    double acc = 0.0;
    const int s2 = s & ~1;
    for (int c0 = s2; c0 < e; c0 += CAP) {
        const int c1 = min(e, c0 + CAP);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int k = c0 + 2 * (threadIdx.x + m * B);
            if (k + 1 < c1 && k >= s) {
                const nt_d2 v = __builtin_nontemporal_load(reinterpret_cast<const nt_d2 *>(val + k));
                const nt_i2 c = __builtin_nontemporal_load(reinterpret_cast<const nt_i2 *>(col + k));
                lds[k - c0] = v.x * x[c.x];
                lds[k + 1 - c0] = v.y * x[c.y];
            } else {
                if (k >= s && k < c1) lds[k - c0] = val[k] * x[col[k]];
                if (k + 1 >= s && k + 1 < c1) lds[k + 1 - c0] = val[k + 1] * x[col[k + 1]];
            }
        }
        __syncthreads();
        const int a = max(my_s, c0), z = min(my_e, c1);
        for (int k = a; k < z; ++k) acc += lds[k - c0];
        __syncthreads();
    }
    if (r < N) y[r] = acc;
}

int main(int argc, char **argv)
{
    const char *path = argc > 1 ? argv[1] : "/tmp/csr.bin";
    FILE *f = std::fopen(path, "rb");
    if (!f) {
        std::perror(path);
        return 1;
    }
    int n = 0, nnz = 0;
    if (std::fread(&n, 4, 1, f) != 1 || std::fread(&nnz, 4, 1, f) != 1) return 1;
    std::vector<int> rp(n + 1), col(nnz);
    std::vector<double> val(nnz), x(n);
    if (std::fread(rp.data(), 4, n + 1, f) != (size_t)n + 1 || std::fread(col.data(), 4, nnz, f) != (size_t)nnz ||
        std::fread(val.data(), 8, nnz, f) != (size_t)nnz)
        return 1;
    std::fclose(f);
    for (int i = 0; i < n; ++i) x[i] = 1.0 + 1e-3 * (i % 977);
    std::vector<short> off(nnz);
    int bad = 0;
    for (int i = 0; i < n; ++i)
        for (int k = rp[i]; k < rp[i + 1]; ++k) {
            const int d = col[k] - i;
            if (d < -32768 || d > 32767) ++bad;
            off[k] = (short)d;
        }
    std::printf("n %d nnz %d offsets out of int16 range: %d\n", n, nnz, bad);
    int *d_rp, *d_col;
    short *d_off;
    double *d_val, *d_x, *d_y, *d_y0;
    CK(hipMalloc(&d_rp, 4 * (n + 1)));
    CK(hipMalloc(&d_col, 4 * (size_t)nnz));
    CK(hipMalloc(&d_off, 2 * (size_t)nnz));
    CK(hipMalloc(&d_val, 8 * (size_t)nnz));
    CK(hipMalloc(&d_x, 8 * (size_t)n));
    CK(hipMalloc(&d_y, 8 * (size_t)n));
    CK(hipMalloc(&d_y0, 8 * (size_t)n));
    CK(hipMemcpy(d_rp, rp.data(), 4 * (n + 1), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_col, col.data(), 4 * (size_t)nnz, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_off, off.data(), 2 * (size_t)nnz, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_val, val.data(), 8 * (size_t)nnz, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_x, x.data(), 8 * (size_t)n, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> y0(n), y(n);
    auto run = [&](const char *name, double bytes, auto launch) {
        for (int w = 0; w < 5; ++w) launch();
        CK(hipDeviceSynchronize());
        const int it = 200;
        CK(hipEventRecord(e0));
        for (int w = 0; w < it; ++w) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / it;
        CK(hipMemcpy(y.data(), d_y, 8 * (size_t)n, hipMemcpyDeviceToHost));
        const bool same = std::memcmp(y.data(), y0.data(), 8 * (size_t)n) == 0;
        double md = 0;
        for (int i = 0; i < n; ++i) md = std::max(md, std::abs(y[i] - y0[i]));
        std::printf("%-34s %8.2f us  %7.1f GB/s (algorithmic %.1f MB)  bitwise %s  maxdiff %.3g\n", name, us,
                    bytes / (us * 1e-6) / 1e9, bytes / 1e6, same ? "yes" : "NO", md);
    };
    const double by12 = 12.0 * nnz + 4.0 * (n + 1) + 16.0 * n;
    const double by10 = 10.0 * nnz + 4.0 * (n + 1) + 16.0 * n;
    {
        const int g = (n + 511) / 512;
        k_v0<512, 8><<<g, 512>>>(n, d_rp, d_col, d_val, d_x, d_y0);
        CK(hipMemcpy(y0.data(), d_y0, 8 * (size_t)n, hipMemcpyDeviceToHost));
        run("V0 tile512 x8 (product)", by12, [&] { k_v0<512, 8><<<g, 512>>>(n, d_rp, d_col, d_val, d_x, d_y); });
        run("V1 tile512 x8 int16 offsets", by10, [&] { k_v1<512, 8><<<g, 512>>>(n, d_rp, d_off, d_val, d_x, d_y); });
        run("V4 tile512 16-B val/col pairs", by12, [&] { k_v4<512><<<g, 512>>>(n, d_rp, d_col, d_val, d_x, d_y); });
        run("V5 tile512 int4+2xdouble2 x2", by12, [&] { k_v5<512, 2, false><<<g, 512>>>(n, d_rp, d_col, d_val, d_x, d_y); });
        run("V5nt tile512 int4+2xdouble2 x2 NT", by12, [&] { k_v5<512, 2, true><<<g, 512>>>(n, d_rp, d_col, d_val, d_x, d_y); });
        run("V6 tile512 pairs NT", by12, [&] { k_v6<512><<<g, 512>>>(n, d_rp, d_col, d_val, d_x, d_y); });
    }
    {
        const int g = (n + 255) / 256;
        run("V2 tile256 x16", by12, [&] { k_v0<256, 16><<<g, 256>>>(n, d_rp, d_col, d_val, d_x, d_y); });
        run("V2b tile256 x8", by12, [&] { k_v0<256, 8><<<g, 256>>>(n, d_rp, d_col, d_val, d_x, d_y); });
        run("V1b tile256 x16 int16 offsets", by10, [&] { k_v1<256, 16><<<g, 256>>>(n, d_rp, d_off, d_val, d_x, d_y); });
        run("V3 row per lane", by12, [&] { k_v3<<<g, 256>>>(n, d_rp, d_col, d_val, d_x, d_y); });
        run("V4b tile256 pairs", by12, [&] { k_v4<256><<<g, 256>>>(n, d_rp, d_col, d_val, d_x, d_y); });
        run("V5b tile256 int4 x2", by12, [&] { k_v5<256, 2, false><<<g, 256>>>(n, d_rp, d_col, d_val, d_x, d_y); });
    }
    {
        const int g = (n + 1023) / 1024;
        run("V2c tile1024 x8", by12, [&] { k_v0<1024, 8><<<g, 1024>>>(n, d_rp, d_col, d_val, d_x, d_y); });
        run("V1c tile1024 x8 int16", by10, [&] { k_v1<1024, 8><<<g, 1024>>>(n, d_rp, d_off, d_val, d_x, d_y); });
        run("V4c tile1024 pairs", by12, [&] { k_v4<1024><<<g, 1024>>>(n, d_rp, d_col, d_val, d_x, d_y); });
        run("V5c tile1024 int4 x2", by12, [&] { k_v5<1024, 2, false><<<g, 1024>>>(n, d_rp, d_col, d_val, d_x, d_y); });
    }
    return 0;
}
