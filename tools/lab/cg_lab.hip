// Microbenchmark lab for the PCG building blocks on MI355X (not product code).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/lab/cg_lab.hip -o /tmp/cg_lab
// Matrix: 7-point pattern of the 2M-triangle structured mesh (4 axis + 2
// diagonal neighbours + diagonal), N = (n+1)^2 rows, natural ordering.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) {                                                                  \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

// ---------------------------------------------------------------- stream
__global__ void k_read(const double *__restrict__ a, int n, double *out)
{
    double s = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) s += a[i];
    if (s == 12345.678) out[0] = s;
}
__global__ void k_read2(const double2 *__restrict__ a, int n2, double *out)
{
    double s = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += gridDim.x * blockDim.x) {
        double2 v = a[i];
        s += v.x + v.y;
    }
    if (s == 12345.678) out[0] = s;
}
__global__ void k_copy2(const double2 *__restrict__ a, double2 *__restrict__ b, int n2)
{
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += gridDim.x * blockDim.x) b[i] = a[i];
}

// ---------------------------------------------------------------- CSR scalar (thread per row)
template <int UNR>
__global__ void k_csr_scalar(int N, const int *__restrict__ rp, const int *__restrict__ col,
                             const double *__restrict__ val, const double *__restrict__ x, double *__restrict__ y)
{
    int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= N) return;
    int s = rp[r], e = rp[r + 1];
    double acc = 0;
#pragma unroll UNR
    for (int k = s; k < e; ++k) acc += val[k] * x[col[k]];
    y[r] = acc;
}

// ---------------------------------------------------------------- CSR stream (LDS row tiles)
template <int BS, int PER>
__global__ void __launch_bounds__(BS) k_csr_stream(int N, const int *__restrict__ rp, const int *__restrict__ col,
                                                   const double *__restrict__ val, const double *__restrict__ x,
                                                   double *__restrict__ y)
{
    __shared__ double lds[BS * PER];
    const int r0 = blockIdx.x * BS;
    const int r = r0 + threadIdx.x;
    const int rend = min(r0 + BS, N);
    const int s = rp[r0], e = rp[rend];
    const int ms = (r < N) ? rp[r] : 0, me = (r < N) ? rp[r + 1] : 0;
    double acc = 0;
    for (int c0 = s; c0 < e; c0 += BS * PER) {
        const int c1 = min(e, c0 + BS * PER);
        int ci[PER];
        double v[PER];
#pragma unroll
        for (int m = 0; m < PER; ++m) {
            int k = c0 + threadIdx.x + m * BS;
            ci[m] = k < c1 ? col[k] : 0;
            v[m] = k < c1 ? val[k] : 0.0;
        }
#pragma unroll
        for (int m = 0; m < PER; ++m) {
            int k = c0 + threadIdx.x + m * BS;
            if (k < c1) lds[k - c0] = v[m] * x[ci[m]];
        }
        __syncthreads();
        for (int k = max(ms, c0); k < min(me, c1); ++k) acc += lds[k - c0];
        __syncthreads();
    }
    if (r < N) y[r] = acc;
}

// ---------------------------------------------------------------- CSR vector: 8 lanes per row
__global__ void k_csr_vec8(int N, const int *__restrict__ rp, const int *__restrict__ col,
                           const double *__restrict__ val, const double *__restrict__ x, double *__restrict__ y)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int r = t >> 3, l = t & 7;
    double acc = 0;
    if (r < N) {
        int s = rp[r], e = rp[r + 1];
        for (int k = s + l; k < e; k += 8) acc += val[k] * x[col[k]];
    }
    acc += __shfl_xor(acc, 1, 8);
    acc += __shfl_xor(acc, 2, 8);
    acc += __shfl_xor(acc, 4, 8);
    if (r < N && l == 0) y[r] = acc;
}

// ---------------------------------------------------------------- SELL-64 (slice = wave)
// slice s covers rows [64 s, 64 s + 64); width w_s; val/col stored [slice][j][lane]
__global__ void k_sell64(int N, const int *__restrict__ soff, const int *__restrict__ swid,
                         const int *__restrict__ col, const double *__restrict__ val, const double *__restrict__ x,
                         double *__restrict__ y)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    const int sl = r >> 6, lane = r & 63;
    if (sl * 64 >= N) return;
    const int off = soff[sl], w = swid[sl];
    double acc = 0;
    for (int j = 0; j < w; ++j) {
        int k = off + j * 64 + lane;
        acc += val[k] * x[col[k]];
    }
    if (r < N) y[r] = acc;
}

// SELL-64 with 16-bit column offsets relative to the row (banded matrices)
__global__ void k_sell64_s16(int N, const int *__restrict__ soff, const int *__restrict__ swid,
                             const short *__restrict__ dcol, const double *__restrict__ val,
                             const double *__restrict__ x, double *__restrict__ y)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    const int sl = r >> 6, lane = r & 63;
    if (sl * 64 >= N) return;
    const int off = soff[sl], w = swid[sl];
    double acc = 0;
    for (int j = 0; j < w; ++j) {
        int k = off + j * 64 + lane;
        acc += val[k] * x[r + dcol[k]];
    }
    if (r < N) y[r] = acc;
}

// ---------------------------------------------------------------- helpers
struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    void start() { CK(hipEventRecord(a)); }
    float stop() { CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); float m; CK(hipEventElapsedTime(&m, a, b)); return m; }
};

template <class F>
static double bench(F f, int reps = 50)
{
    f();
    CK(hipDeviceSynchronize());
    Timer t;
    std::vector<float> ts;
    for (int i = 0; i < reps; ++i) {
        t.start();
        f();
        ts.push_back(t.stop());
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main(int argc, char **argv)
{
    int n = argc > 1 ? atoi(argv[1]) : 1000;
    int m = n + 1;
    int N = m * m;
    // 7-point pattern: (i,j) ~ (i+-1,j), (i,j+-1), (i+1,j+1), (i-1,j-1)
    std::vector<int> rp(N + 1, 0), col;
    std::vector<double> val;
    col.reserve(7 * N);
    val.reserve(7 * N);
    for (int j = 0; j < m; ++j)
        for (int i = 0; i < m; ++i) {
            int r = j * m + i;
            int nb[7][2] = {{i - 1, j - 1}, {i, j - 1}, {i - 1, j}, {i, j}, {i + 1, j}, {i, j + 1}, {i + 1, j + 1}};
            for (auto &q : nb) {
                if (q[0] < 0 || q[1] < 0 || q[0] >= m || q[1] >= m) continue;
                int c = q[1] * m + q[0];
                col.push_back(c);
                val.push_back(c == r ? 7.0 : -1.0);
            }
            rp[r + 1] = (int)col.size();
        }
    const int nnz = (int)col.size();
    printf("N=%d nnz=%d (%.2f per row)\n", N, nnz, (double)nnz / N);
    // SELL-64
    int nsl = (N + 63) / 64;
    std::vector<int> soff(nsl + 1, 0), swid(nsl);
    for (int s = 0; s < nsl; ++s) {
        int w = 0;
        for (int l = 0; l < 64; ++l) {
            int r = s * 64 + l;
            if (r < N) w = std::max(w, rp[r + 1] - rp[r]);
        }
        swid[s] = w;
        soff[s + 1] = soff[s] + 64 * w;
    }
    std::vector<int> scol(soff[nsl]);
    std::vector<short> sdcol(soff[nsl]);
    std::vector<double> sval(soff[nsl], 0.0);
    for (int s = 0; s < nsl; ++s)
        for (int l = 0; l < 64; ++l) {
            int r = s * 64 + l;
            for (int j = 0; j < swid[s]; ++j) {
                int k = soff[s] + j * 64 + l;
                if (r < N && j < rp[r + 1] - rp[r]) {
                    scol[k] = col[rp[r] + j];
                    sval[k] = val[rp[r] + j];
                } else {
                    scol[k] = (r < N) ? r : 0;
                    sval[k] = 0.0;
                }
                sdcol[k] = (short)(scol[k] - (r < N ? r : 0));
            }
        }
    printf("SELL-64 padded entries %d (%.1f%% padding)\n", soff[nsl], 100.0 * (soff[nsl] - nnz) / nnz);

    int *d_rp, *d_col, *d_soff, *d_swid, *d_scol;
    short *d_sdcol;
    double *d_val, *d_sval, *d_x, *d_y, *d_big, *d_big2, *d_out;
    CK(hipMalloc(&d_rp, 4 * (N + 1)));
    CK(hipMalloc(&d_col, 4 * nnz));
    CK(hipMalloc(&d_val, 8 * nnz));
    CK(hipMalloc(&d_soff, 4 * (nsl + 1)));
    CK(hipMalloc(&d_swid, 4 * nsl));
    CK(hipMalloc(&d_scol, 4 * soff[nsl]));
    CK(hipMalloc(&d_sdcol, 2 * soff[nsl]));
    CK(hipMalloc(&d_sval, 8 * soff[nsl]));
    CK(hipMalloc(&d_x, 8 * N));
    CK(hipMalloc(&d_y, 8 * N));
    CK(hipMalloc(&d_out, 8));
    CK(hipMemcpy(d_rp, rp.data(), 4 * (N + 1), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_col, col.data(), 4 * nnz, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_val, val.data(), 8 * nnz, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_soff, soff.data(), 4 * (nsl + 1), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_swid, swid.data(), 4 * nsl, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_scol, scol.data(), 4 * soff[nsl], hipMemcpyHostToDevice));
    CK(hipMemcpy(d_sdcol, sdcol.data(), 2 * soff[nsl], hipMemcpyHostToDevice));
    CK(hipMemcpy(d_sval, sval.data(), 8 * soff[nsl], hipMemcpyHostToDevice));
    std::vector<double> hx(N);
    for (int i = 0; i < N; ++i) hx[i] = 1.0 + (i % 7) * 0.25;
    CK(hipMemcpy(d_x, hx.data(), 8 * N, hipMemcpyHostToDevice));

    const double csr_bytes = 12.0 * nnz + 4.0 * (N + 1) + 16.0 * N;
    auto rep = [&](const char *name, double ms, double bytes) {
        printf("%-34s %8.2f us  %7.0f GB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    };
    // stream ceilings at several footprints
    for (size_t mb : {64, 176, 512, 2048}) {
        size_t cnt = mb * 1024 * 1024 / 8;
        CK(hipMalloc(&d_big, cnt * 8));
        CK(hipMalloc(&d_big2, cnt * 8));
        CK(hipMemset(d_big, 0, cnt * 8));
        char nm[64];
        for (int grid : {1024, 4096, 16384}) {
            double ms = bench([&] { k_read2<<<grid, 256>>>((const double2 *)d_big, (int)(cnt / 2), d_out); });
            snprintf(nm, sizeof nm, "read %zu MB dwordx4 grid %d", mb, grid);
            rep(nm, ms, cnt * 8.0);
        }
        double ms = bench([&] { k_copy2<<<8192, 256>>>((const double2 *)d_big, (double2 *)d_big2, (int)(cnt / 2)); });
        snprintf(nm, sizeof nm, "copy %zu MB dwordx4", mb);
        rep(nm, ms, cnt * 16.0);
        CK(hipFree(d_big));
        CK(hipFree(d_big2));
    }
    // SpMV variants
    rep("csr scalar (thread/row)", bench([&] { k_csr_scalar<8><<<(N + 255) / 256, 256>>>(N, d_rp, d_col, d_val, d_x, d_y); }), csr_bytes);
    rep("csr vec8 (8 lanes/row)", bench([&] { k_csr_vec8<<<(8 * N + 255) / 256, 256>>>(N, d_rp, d_col, d_val, d_x, d_y); }), csr_bytes);
    rep("csr stream BS256 PER8", bench([&] { k_csr_stream<256, 8><<<(N + 255) / 256, 256>>>(N, d_rp, d_col, d_val, d_x, d_y); }), csr_bytes);
    rep("csr stream BS512 PER8", bench([&] { k_csr_stream<512, 8><<<(N + 511) / 512, 512>>>(N, d_rp, d_col, d_val, d_x, d_y); }), csr_bytes);
    rep("csr stream BS1024 PER8", bench([&] { k_csr_stream<1024, 8><<<(N + 1023) / 1024, 1024>>>(N, d_rp, d_col, d_val, d_x, d_y); }), csr_bytes);
    const double sell_bytes = 12.0 * soff[nsl] + 8.0 * nsl + 16.0 * N;
    rep("sell64 (algorithmic csr bytes)", bench([&] { k_sell64<<<(N + 255) / 256, 256>>>(N, d_soff, d_swid, d_scol, d_sval, d_x, d_y); }), csr_bytes);
    rep("sell64 (own bytes incl pad)", bench([&] { k_sell64<<<(N + 255) / 256, 256>>>(N, d_soff, d_swid, d_scol, d_sval, d_x, d_y); }), sell_bytes);
    rep("sell64 s16 (csr bytes)", bench([&] { k_sell64_s16<<<(N + 255) / 256, 256>>>(N, d_soff, d_swid, d_sdcol, d_sval, d_x, d_y); }), csr_bytes);
    printf("done\n");
    return 0;
}
