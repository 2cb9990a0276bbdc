// Host I/O and page-fault costs on the GPU box's file system (round-5 lab):
// writing 128 MiB by one fwrite, by pwrite from 16 threads, through a shared
// mapping from 16 threads; first-touch of a fresh 128 MiB allocation by 1 /
// 16 threads, with and without MADV_HUGEPAGE.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <string>
#include <sys/mman.h>
#include <thread>
#include <unistd.h>
#include <vector>

static double now() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
template <class F> static void par(int T, F f) { std::vector<std::thread> th; for (int t = 1; t < T; ++t) th.emplace_back(f, t); f(0); for (auto &x : th) x.join(); }

int main(int argc, char **argv)
{
    const char *dir = argc > 1 ? argv[1] : "/tmp";
    const size_t N = 128ull << 20;
    const int T = 16;
    std::vector<char> src(N, 'x');
    std::string path = std::string(dir) + "/io_probe.bin";
    for (int rep = 0; rep < 2; ++rep) {
        double t = now();
        FILE *fp = fopen(path.c_str(), "w");
        fwrite(src.data(), 1, N, fp);
        fclose(fp);
        printf("fwrite 1 thread      %7.1f ms\n", now() - t);
        unlink(path.c_str());
        t = now();
        int fd = open(path.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
        par(T, [&](int k) { size_t a = N * k / T, b = N * (k + 1) / T; if (pwrite(fd, src.data() + a, b - a, a) < 0) perror("pwrite"); });
        close(fd);
        printf("pwrite %d threads    %7.1f ms\n", T, now() - t);
        unlink(path.c_str());
        t = now();
        fd = open(path.c_str(), O_CREAT | O_TRUNC | O_RDWR, 0644);
        if (ftruncate(fd, N) != 0) perror("ftruncate");
        char *m = (char *)mmap(nullptr, N, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        par(T, [&](int k) { size_t a = N * k / T, b = N * (k + 1) / T; memcpy(m + a, src.data() + a, b - a); });
        munmap(m, N);
        close(fd);
        printf("mmap %d threads      %7.1f ms\n", T, now() - t);
        t = now();
        fd = open(path.c_str(), O_RDONLY);
        std::vector<char> dst(N);
        printf("  (vector value-init %7.1f ms)\n", now() - t);
        t = now();
        par(T, [&](int k) { size_t a = N * k / T, b = N * (k + 1) / T; if (pread(fd, dst.data() + a, b - a, a) < 0) perror("pread"); });
        printf("pread %d threads     %7.1f ms (touched)\n", T, now() - t);
        close(fd);
        unlink(path.c_str());
        for (int hp = 0; hp < 2; ++hp)
            for (int th : {1, 16}) {
                t = now();
                char *p = (char *)aligned_alloc(2 << 20, N);
                if (hp) madvise(p, N, MADV_HUGEPAGE);
                par(th, [&](int k) { size_t a = N * k / th, b = N * (k + 1) / th; memset(p + a, 0, b - a); });
                printf("first touch %2d thr hugepage %d %7.1f ms\n", th, hp, now() - t);
                t = now();
                par(th, [&](int k) { size_t a = N * k / th, b = N * (k + 1) / th; memset(p + a, 1, b - a); });
                printf("  second touch           %7.1f ms\n", now() - t);
                free(p);
            }
    }
    FILE *f = fopen("/sys/kernel/mm/transparent_hugepage/enabled", "r");
    char b[256] = {0};
    if (f) { if (fgets(b, sizeof b, f)) printf("THP: %s", b); fclose(f); }
    return 0;
}
