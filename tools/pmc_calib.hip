// PMC calibration: known-byte streaming kernels at the access widths the
// fsolver kernels use (4-B int / 8-B double / 16-B double2 per lane), so that
// rocprofv3's FETCH_SIZE / WRITE_SIZE can be converted to bytes per width
// (MI355X_MICROARCH.md calibrates only 16-B reads: FETCH_SIZE = 1/2 of them).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o xfemm_amd/bin/pmc_calib tools/pmc_calib.hip
// Run:   rocprofv3 --pmc FETCH_SIZE -T -f csv -d DIR -o run -- xfemm_amd/bin/pmc_calib
//        (and a second pass with WRITE_SIZE); tools/pmc_summary.py --calib DIR_FETCH DIR_WRITE
// Each kernel streams a 512 MiB buffer (twice the 256 MiB Infinity Cache)
// once; the host prints the bytes each launch moves.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

template <class T>
__device__ __forceinline__ double as_d(T v) { return (double)v; }
template <>
__device__ __forceinline__ double as_d<double2>(double2 v) { return v.x + v.y; }

// grid-stride read of n elements of T; one partial per block (written, so the
// loads are not dead)
template <class T>
__global__ void __launch_bounds__(256) k_calib_read(const T *__restrict__ a, long long n, double *__restrict__ out)
{
    double s = 0.0;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) s += as_d(a[i]);
    if (s == 12345.678) out[blockIdx.x] = s;   // never true for the zero-filled buffers: no stores
}

template <class T>
__global__ void __launch_bounds__(256) k_calib_write(T *__restrict__ a, long long n, T v)
{
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) a[i] = v;
}

int main()
{
    const size_t bytes = 512ull << 20;
    void *buf = nullptr;
    double *out = nullptr;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 65536 * sizeof(double)));
    CK(hipMemset(buf, 0, bytes));
    const int grid = 8192;
    for (int rep = 0; rep < 3; ++rep) {
        k_calib_read<int><<<grid, 256>>>((const int *)buf, (long long)(bytes / 4), out);
        k_calib_read<double><<<grid, 256>>>((const double *)buf, (long long)(bytes / 8), out);
        k_calib_read<double2><<<grid, 256>>>((const double2 *)buf, (long long)(bytes / 16), out);
        k_calib_write<int><<<grid, 256>>>((int *)buf, (long long)(bytes / 4), 0);
        k_calib_write<double><<<grid, 256>>>((double *)buf, (long long)(bytes / 8), 0.0);
        k_calib_write<double2><<<grid, 256>>>((double2 *)buf, (long long)(bytes / 16), make_double2(0.0, 0.0));
    }
    CK(hipDeviceSynchronize());
    std::printf("{\"bytes_per_launch\": %zu}\n", bytes);
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
