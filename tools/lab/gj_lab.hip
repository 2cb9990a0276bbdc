// Dense-coarsest lab: times the pivot-block inverse (bgj_diag_inv) and the
// whole blocked Gauss-Jordan of xfk_amg.hip on synthetic SPD matrices, plus
// variants.  Build (dev container) and run (GPU box):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I xfemm_amd/csrc -I include tools/lab/gj_lab.hip \
//         -o tools/lab/gj_lab -L xfemm_amd/lib -lxfemm_kernels -Wl,-rpath,$PWD/xfemm_amd/lib
//   timeout -k 10 60 tools/lab/gj_lab
#include "../../xfemm_amd/csrc/xfk_amg.hip"

#include <cstdio>
#include <random>
#include <vector>

using namespace xfk;

#define LAB_CHECK(x)                                                              \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

namespace {

// empty-work floor: load the 64 x 64 block and store it back
__global__ void __launch_bounds__(256) k_copy_block(int ld, const double *__restrict__ M, double *__restrict__ D)
{
    const int j = threadIdx.x & 63, w = threadIdx.x >> 6;
    double a[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) a[m] = M[(size_t)(16 * w + m) * ld + j];
#pragma unroll
    for (int m = 0; m < 16; ++m) D[(16 * w + m) * kBj + j] = a[m];
}

// n x n SPD: a 2-D 5-point Laplacian-like operator plus a random symmetric
// perturbation, unit-diagonal scaled (as the coarsest level after k_dense_dscale)
std::vector<double> make_spd(int n, unsigned seed)
{
    std::mt19937 g(seed);
    std::uniform_real_distribution<double> u(0.0, 1.0);
    std::vector<double> A((size_t)n * n, 0.0);
    const int side = (int)std::ceil(std::sqrt((double)n));
    for (int i = 0; i < n; ++i) {
        const int xi = i % side, yi = i / side;
        double d = 1e-3;
        for (int j : {i + 1, i + side}) {
            if (j >= n) continue;
            const int xj = j % side, yj = j / side;
            if (std::abs(xi - xj) + std::abs(yi - yj) != 1) continue;
            const double v = -(0.5 + u(g));
            A[(size_t)i * n + j] += v;
            A[(size_t)j * n + i] += v;
            A[(size_t)i * n + i] -= v;
            A[(size_t)j * n + j] -= v;
        }
        A[(size_t)i * n + i] += d;
    }
    std::vector<double> s(n);
    for (int i = 0; i < n; ++i) s[i] = 1.0 / std::sqrt(A[(size_t)i * n + i]);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) A[(size_t)i * n + j] *= s[i] * s[j];
    return A;
}

double inv_residual(int n, const std::vector<double> &A, const std::vector<double> &X)
{
    double worst = 0;
    for (int i = 0; i < n; i += std::max(1, n / 64))
        for (int j = 0; j < n; ++j) {
            double s = 0;
            for (int k = 0; k < n; ++k) s += A[(size_t)i * n + k] * X[(size_t)k * n + j];
            worst = std::max(worst, std::fabs(s - (i == j ? 1.0 : 0.0)));
        }
    return worst;
}

template <class F>
float time_launches(F &&launch, int reps, hipStream_t s)
{
    hipEvent_t a, b;
    LAB_CHECK(hipEventCreate(&a));
    LAB_CHECK(hipEventCreate(&b));
    launch();
    LAB_CHECK(hipStreamSynchronize(s));
    LAB_CHECK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r) launch();
    LAB_CHECK(hipEventRecord(b, s));
    LAB_CHECK(hipEventSynchronize(b));
    float ms = 0;
    LAB_CHECK(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return 1000.f * ms / reps;
}

// variant: NT threads (RPT = 4096 / NT rows of one column per thread), rank-4
// steps as bgj_diag_inv, optional fast reciprocal (v_rcp_f64 + 2 Newton steps)
template <bool FAST>
__device__ __forceinline__ double recip(double x)
{
    if constexpr (FAST) {
        double r = __builtin_amdgcn_rcp(x);
        r = fma(fma(-x, r, 1.0), r, r);
        r = fma(fma(-x, r, 1.0), r, r);
        return r;
    } else {
        return 1.0 / x;
    }
}

template <int NT, bool FAST, int ABL = 0>
__global__ void __launch_bounds__(NT) k_diag_var(int ld, const double *__restrict__ M, const double *__restrict__ maxd,
                                                 double *__restrict__ D)
{
    constexpr int RPT = 4096 / NT;
    __shared__ __attribute__((aligned(16))) double lds[2 * 4 * kBj + 2 * 4 * kBj];
    const int j = threadIdx.x & 63, w = threadIdx.x >> 6;
    double a[RPT];
#pragma unroll
    for (int m = 0; m < RPT; ++m) a[m] = M[(size_t)(RPT * w + m) * ld + j];
    const double thr = 1e-11 * (*maxd);
    int phase = 0;
    for (int p0 = 0; p0 < kBj; p0 += 4) {
        const int buf = phase & 1;
        const int mb = p0 % RPT, wp = p0 / RPT;
        double *R4 = lds + buf * 4 * kBj, *C4 = lds + 8 * kBj + buf * 4 * kBj;
        if (w == wp)
#pragma unroll
            for (int m = 0; m < RPT; ++m)
                if (m >= mb && m < mb + 4) R4[(m - mb) * kBj + j] = a[m];
        if (j >= p0 && j < p0 + 4)
#pragma unroll
            for (int m = 0; m < RPT; ++m) C4[(RPT * w + m) * 4 + (j - p0)] = a[m];
        if (!(ABL & 4)) __syncthreads();
        ++phase;
        double Dv[4][4];
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
            for (int t = 0; t < 4; ++t) Dv[s2][t] = R4[s2 * kBj + p0 + t];
        bool ok = true;
#pragma unroll
        for (int q = 0; q < 4 * !(ABL & 2); ++q) {
            const double piv = Dv[q][q];
            ok = ok && (fabs(piv) > thr);
            const double ip = recip<FAST>(piv);
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
        (void)ok;   // lab: SPD inputs only
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
        const double4 *cr = reinterpret_cast<const double4 *>(&C4[RPT * w * 4]);
#pragma unroll
        for (int m = 0; m < RPT * !(ABL & 1); ++m) {
            const double4 c = cr[m];
            a[m] -= c.x * r[0] + c.y * r[1] + c.z * r[2] + c.w * r[3];
        }
        if (w == wp)
#pragma unroll
            for (int m = 0; m < RPT; ++m) {
                const int s2 = m - mb;
                a[m] += (s2 == 0 ? r[0] : 0.0) + (s2 == 1 ? r[1] : 0.0) + (s2 == 2 ? r[2] : 0.0) +
                        (s2 == 3 ? r[3] : 0.0);
            }
    }
#pragma unroll
    for (int m = 0; m < RPT; ++m) D[(RPT * w + m) * kBj + j] = a[m];
}

// the MFMA-update inverse (bgj_inv_mfma) with ablations: ABL & 1 no MFMA
// update, & 2 no 4 x 4 inverse, & 4 no barrier, & 8 fast reciprocal
template <int ABL>
__global__ void __launch_bounds__(256) k_inv_mfma_var(int ld, const double *__restrict__ M, const double *__restrict__ maxd,
                                                      double *__restrict__ D)
{
    __shared__ __attribute__((aligned(16))) double lds[kBjInvLds];
    dbl4 c[2][2];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int r = 0; r < 4; ++r) c[ti][tj][r] = M[(size_t)bgj_row(ti, r) * ld + bgj_col(tj)];
    if constexpr (ABL == 0) {
        bgj_inv_mfma(c, 1e-11 * (*maxd), lds);
    } else {
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        const int li = lane & 15, lk = lane >> 4;
        const int R0 = 32 * (w >> 1), C0 = 32 * (w & 1);
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const int p0 = 4 * s;
            const int tp = (p0 >> 4) & 1, rp = (p0 & 15) >> 2;
            double *RS = lds + (s & 1) * 8 * kBj;
            double *CS = RS + 4 * kBj;
            const bool rowhold = (w >> 1) == (p0 >> 5);
            if (rowhold)
#pragma unroll
                for (int tj = 0; tj < 2; ++tj) RS[lk * kBj + C0 + 16 * tj + li] = c[tp][tj][rp];
            if ((w & 1) == (p0 >> 5) && li >= (p0 & 15) && li < (p0 & 15) + 4)
#pragma unroll
                for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                    for (int r = 0; r < 4; ++r) CS[(R0 + 16 * ti + lk + 4 * r) * 4 + li - (p0 & 15)] = c[ti][tp][r];
            if (!(ABL & 4)) __syncthreads();
            double W[4][4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int t = 0; t < 4; ++t) W[q][t] = RS[q * kBj + p0 + t];
            if (!(ABL & 2))
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const double ip = (ABL & 8) ? recip<true>(W[q][q]) : 1.0 / W[q][q];
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
            if (!(ABL & 1))
#pragma unroll
                for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                    for (int tj = 0; tj < 2; ++tj)
                        c[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(aop[ti], bop[tj], c[ti][tj], 0, 0, 0);
            else
                c[0][0][0] += aop[0] + aop[1] + bop[0] + bop[1];
            if (rowhold)
#pragma unroll
                for (int tj = 0; tj < 2; ++tj) c[tp][tj][rp] += bop[tj];
        }
    }
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int r = 0; r < 4; ++r) D[bgj_row(ti, r) * kBj + bgj_col(tj)] = c[ti][tj][r];
}

}  // namespace

int main()
{
    hipStream_t s;
    LAB_CHECK(hipStreamCreate(&s));
    // 1. pivot-block inverse alone
    {
        const int n = 64;
        std::vector<double> A = make_spd(n, 1);
        double *dM, *dD, *dmax;
        LAB_CHECK(hipMalloc(&dM, sizeof(double) * n * n));
        LAB_CHECK(hipMalloc(&dD, sizeof(double) * n * n));
        LAB_CHECK(hipMalloc(&dmax, sizeof(double)));
        LAB_CHECK(hipMemcpy(dM, A.data(), sizeof(double) * n * n, hipMemcpyHostToDevice));
        const double one = 1.0;
        LAB_CHECK(hipMemcpy(dmax, &one, sizeof(double), hipMemcpyHostToDevice));
        const float t_copy = time_launches([&] { k_copy_block<<<1, 256, 0, s>>>(n, dM, dD); }, 200, s);
        const float t_diag = time_launches([&] { k_bgj_diag<<<1, 256, 0, s>>>(0, n, dM, dmax, dD); }, 200, s);
        std::vector<double> X((size_t)n * n);
        LAB_CHECK(hipMemcpy(X.data(), dD, sizeof(double) * n * n, hipMemcpyDeviceToHost));
        std::printf("{\"test\": \"pivot64\", \"us_copy\": %.2f, \"us_diag\": %.2f, \"inv_res\": %.3e}\n", t_copy, t_diag,
                    inv_residual(n, A, X));
        auto run_var = [&](const char *name, auto kern, int nt) {
            LAB_CHECK(hipMemset(dD, 0, sizeof(double) * n * n));
            const float t = time_launches([&] { kern<<<1, nt, 0, s>>>(n, dM, dmax, dD); }, 200, s);
            LAB_CHECK(hipMemcpy(X.data(), dD, sizeof(double) * n * n, hipMemcpyDeviceToHost));
            std::printf("{\"test\": \"pivot64 %s\", \"us\": %.2f, \"inv_res\": %.3e}\n", name, t, inv_residual(n, A, X));
        };
        run_var("256 exact", k_diag_var<256, false>, 256);
        run_var("256 fast", k_diag_var<256, true>, 256);
        run_var("512 exact", k_diag_var<512, false>, 512);
        run_var("512 fast", k_diag_var<512, true>, 512);
        run_var("1024 exact", k_diag_var<1024, false>, 1024);
        run_var("1024 fast", k_diag_var<1024, true>, 1024);
        run_var("256 ablate update", k_diag_var<256, false, 1>, 256);
        run_var("256 ablate 4x4 inverse", k_diag_var<256, false, 2>, 256);
        run_var("256 ablate barrier", k_diag_var<256, false, 4>, 256);
        run_var("256 ablate update+inverse", k_diag_var<256, false, 3>, 256);
        run_var("256 ablate all", k_diag_var<256, false, 7>, 256);
        run_var("64 (1 wave) exact", k_diag_var<64, false>, 64);
        run_var("mfma", k_inv_mfma_var<0>, 256);
        run_var("mfma (lab copy)", k_inv_mfma_var<16>, 256);
        run_var("mfma fast recip", k_inv_mfma_var<8>, 256);
        run_var("mfma ablate update", k_inv_mfma_var<1>, 256);
        run_var("mfma ablate 4x4 inverse", k_inv_mfma_var<2>, 256);
        run_var("mfma ablate barrier", k_inv_mfma_var<4>, 256);
        run_var("mfma ablate all", k_inv_mfma_var<7>, 256);
        (void)hipFree(dM);
        (void)hipFree(dD);
        (void)hipFree(dmax);
    }
    // 2. the whole blocked Gauss-Jordan at the configs[2] coarsest size
    for (int inv_mode = 0; inv_mode < 2; ++inv_mode)
    for (int n : {64, 128, 1024, 1600}) {
        const int nbk = (n + kBj - 1) / kBj, ld = nbk * kBj;
        const size_t T2 = (size_t)kBj * kBj;
        std::vector<double> A = make_spd(ld, 2);
        double *dA, *dM, *tmp;
        LAB_CHECK(hipMalloc(&dA, sizeof(double) * ld * ld));
        LAB_CHECK(hipMalloc(&dM, sizeof(double) * ld * ld));
        LAB_CHECK(hipMalloc(&tmp, sizeof(double) * (4 * (size_t)nbk * T2 + 2 * T2 + 1)));
        LAB_CHECK(hipMemcpy(dA, A.data(), sizeof(double) * ld * ld, hipMemcpyHostToDevice));
        double *Dbuf = tmp + 4 * (size_t)nbk * T2;
        double *maxd = Dbuf + 2 * T2;
        const double one = 1.0;
        LAB_CHECK(hipMemcpy(maxd, &one, sizeof(double), hipMemcpyHostToDevice));
        auto reset = [&] { LAB_CHECK(hipMemcpyAsync(dM, dA, sizeof(double) * ld * ld, hipMemcpyDeviceToDevice, s)); };
        double *Rs[2] = {tmp, tmp + (size_t)nbk * T2}, *Cs[2] = {tmp + 2 * (size_t)nbk * T2, tmp + 3 * (size_t)nbk * T2};
        auto new_gj = [&] {
            reset();
            k_bgj_snap<<<2 * nbk, 256, 0, s>>>(0, nbk, ld, dM, Rs[0], Cs[0]);
            k_bgj_diag<<<1, 256, 0, s>>>(0, ld, dM, maxd, Dbuf);
            for (int k = 0; k < nbk; ++k) {
                const int p = k & 1, q = (k + 1) & 1;
                k_bgj_step<<<nbk * nbk, 256, 0, s>>>(k, nbk, ld, dM, Dbuf + p * T2, Rs[p], Cs[p], Dbuf + q * T2, Rs[q],
                                                     Cs[q], maxd, inv_mode);
            }
        };
        std::vector<double> X((size_t)ld * ld);
        const float t_reset = time_launches(reset, 10, s);
        const float t_new = time_launches(new_gj, 10, s);
        LAB_CHECK(hipMemcpy(X.data(), dM, sizeof(double) * ld * ld, hipMemcpyDeviceToHost));
        const double res_new = inv_residual(ld, A, X);
        const int k = nbk / 2;
        const float t_step = time_launches(
            [&] {
                k_bgj_step<<<nbk * nbk, 256, 0, s>>>(k, nbk, ld, dM, Dbuf, Rs[0], Cs[0], Dbuf + T2, Rs[1], Cs[1], maxd,
                                                     inv_mode);
            },
            50, s);
        const float t_step_last = time_launches(
            [&] {
                k_bgj_step<<<nbk * nbk, 256, 0, s>>>(nbk - 1, nbk, ld, dM, Dbuf, Rs[0], Cs[0], Dbuf + T2, Rs[1], Cs[1],
                                                     maxd, inv_mode);
            },
            50, s);
        std::printf("{\"test\": \"bgj n=%d inv_mode %d\", \"nbk\": %d, \"us_new\": %.1f, "
                    "\"res_new\": %.3e, \"us_step\": %.2f, \"us_step_no_pivot\": %.2f}\n",
                    n, inv_mode, nbk, t_new - t_reset, res_new, t_step, t_step_last);
        (void)hipFree(dA);
        (void)hipFree(dM);
        (void)hipFree(tmp);
    }
    std::fflush(stdout);
    LAB_CHECK(hipStreamDestroy(s));
    return 0;
}
