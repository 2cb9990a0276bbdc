// Lab (round 6): the host round trip of one dependent step -- enqueue a tiny
// kernel and a 64-byte device-to-host copy, wait, enqueue the next -- with
// the waits the fsolver could use: hipStreamSynchronize (what the PCG polls
// and the setup's host checks do), a hipStreamQuery busy loop, an event
// (hipEventSynchronize), and each of those after
// hipSetDeviceFlags(hipDeviceScheduleSpin / hipDeviceScheduleYield).
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/lab/sync_probe tools/lab/sync_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

__global__ void k_tick(int *p) { if (threadIdx.x == 0) p[0] += 1; }

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv)
{
    const char *mode = argc > 1 ? argv[1] : "auto";
    if (!std::strcmp(mode, "spin")) hipSetDeviceFlags(hipDeviceScheduleSpin);
    else if (!std::strcmp(mode, "yield")) hipSetDeviceFlags(hipDeviceScheduleYield);
    else if (!std::strcmp(mode, "blocking")) hipSetDeviceFlags(hipDeviceScheduleBlockingSync);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    int *d, *h;
    hipMalloc(&d, 64);
    hipHostMalloc(&h, 64, 0);
    hipMemset(d, 0, 64);
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    const int N = 2000;
    for (int way = 0; way < 3; ++way) {
        // warm
        for (int i = 0; i < 50; ++i) {
            k_tick<<<1, 64, 0, s>>>(d);
            hipMemcpyAsync(h, d, 64, hipMemcpyDeviceToHost, s);
            hipStreamSynchronize(s);
        }
        const double t0 = now_us();
        for (int i = 0; i < N; ++i) {
            k_tick<<<1, 64, 0, s>>>(d);
            hipMemcpyAsync(h, d, 64, hipMemcpyDeviceToHost, s);
            if (way == 0) hipStreamSynchronize(s);
            else if (way == 1) {
                while (hipStreamQuery(s) == hipErrorNotReady) {
                }
            } else {
                hipEventRecord(ev, s);
                hipEventSynchronize(ev);
            }
        }
        const double t1 = now_us();
        static const char *names[] = {"hipStreamSynchronize", "hipStreamQuery loop", "hipEventSynchronize"};
        std::printf("flags=%-8s %-22s %.2f us per kernel + copy + wait (last value %d)\n", mode, names[way],
                    (t1 - t0) / N, h[0]);
    }
    return 0;
}
