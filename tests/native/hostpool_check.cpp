// Checks xfemm::HostPool (xfemm_amd/csrc/fsolver/hostpool.h): every index of a
// loop runs exactly once; a job that throws on a worker or on the caller has
// its first exception rethrown by run() on the calling thread after every
// claimed chunk finished, and the pool stays usable afterwards.
// Prints "hostpool ok" on success, the first failure otherwise.
#include <atomic>
#include <cstdio>
#include <stdexcept>
#include <vector>

#include "../../xfemm_amd/csrc/fsolver/hostpool.h"

int main()
{
    xfemm::HostPool &pool = xfemm::HostPool::get();
    for (int round = 0; round < 200; ++round) {
        const int n = 1 + round % 97;
        std::vector<std::atomic<int>> hit(n);
        for (auto &h : hit) h = 0;
        pool.run(n, [&](int t) { hit[t]++; });
        for (int t = 0; t < n; ++t)
            if (hit[t] != 1) {
                std::printf("index %d of %d ran %d times\n", t, n, (int)hit[t]);
                return 1;
            }
    }
    for (int round = 0; round < 100; ++round) {
        const int n = 64, bad = round % n;
        std::atomic<int> done{0};
        bool caught = false;
        try {
            pool.run(n, [&](int t) {
                if (t == bad) throw std::runtime_error("chunk failed");
                done++;
            });
        } catch (const std::runtime_error &e) {
            caught = true;
        }
        if (!caught) {
            std::printf("exception of chunk %d not rethrown\n", bad);
            return 1;
        }
        // pooled: every other chunk still ran, and had finished when run()
        // returned; one thread: a plain loop, which stops at the throw
        if (pool.size() > 1 ? done != n - 1 : done != bad) {
            std::printf("round %d: %d of %d chunks finished\n", round, (int)done, n - 1);
            return 1;
        }
    }
    std::atomic<long long> sum{0};
    pool.run(1000, [&](int t) { sum += t; });
    if (sum != 999LL * 1000 / 2) {
        std::printf("pool unusable after exceptions\n");
        return 1;
    }
    std::printf("hostpool ok (%d threads)\n", pool.size());
    return 0;
}
