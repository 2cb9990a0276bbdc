// Lab probe: where a fresh process's HIP bring-up goes (round 6, cold
// bin/fsolver).  Built three ways by tools/lab/r06_init.sh: plain HIP, linked
// against librccl (as libxfemm_kernels.so is), and linked against
// libxfemm_kernels.so; prints the wall time of each bring-up step.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#ifdef WITH_XFK
extern "C" int xfk_device_init(int device);
#endif

static double ms_since(std::chrono::steady_clock::time_point t)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main()
{
    auto t = std::chrono::steady_clock::now();
    int n = 0;
    (void)hipGetDeviceCount(&n);
    printf("hipGetDeviceCount %.1f ms (%d devices)\n", ms_since(t), n);
    t = std::chrono::steady_clock::now();
    (void)hipSetDevice(0);
    (void)hipFree(nullptr);
    printf("hipSetDevice + hipFree(0) %.1f ms\n", ms_since(t));
    t = std::chrono::steady_clock::now();
    hipStream_t s;
    (void)hipStreamCreate(&s);
    printf("hipStreamCreate %.1f ms\n", ms_since(t));
#ifdef WITH_XFK
    t = std::chrono::steady_clock::now();
    int rc = xfk_device_init(0);
    printf("xfk_device_init %.1f ms (rc %d)\n", ms_since(t), rc);
#endif
    return 0;
}
