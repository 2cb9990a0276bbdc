// A persistent pool of host threads for the product path's parallel loops.
//
// The host stages of FSolver (mesh parsing, renumbering, the comb sort's ~70
// passes, the .ans formatting) dispatch a parallel loop a few hundred times
// per analysis; creating and joining 15 threads per dispatch costs ~0.5 ms on
// the GPU box's host, i.e. tens of ms per analysis.  The pool's workers live
// for the process and take loop chunks through an atomic counter; a dispatch
// costs a wake-up.  A loop started from inside a pool job, or while another
// thread's loop holds the pool, runs on the calling thread alone.  A job that
// throws on any thread has its first exception rethrown by run() on the
// calling thread, after every claimed chunk has finished.
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace xfemm {

class HostPool {
  public:
    static HostPool &get()
    {
        static HostPool *p = new HostPool();   // (never destroyed: workers outlive static destructors)
        return *p;
    }
    // threads a loop may use (workers + the caller), at most 16
    int size() const { return (int)workers_.size() + 1; }

    // f(t) for t in [0, n), spread over the pool and the calling thread
    template <class F>
    void run(int n, F &&f)
    {
        if (n <= 0) return;
        std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
        if (n == 1 || workers_.empty() || in_job_ || !busy.owns_lock()) {
            for (int t = 0; t < n; ++t) f(t);
            return;
        }
        std::function<void(int)> job(std::ref(f));
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = &job;
            n_ = n;
            ++gen_;
            left_.store(n, std::memory_order_relaxed);
            ticket_.store((gen_ & 0xffffffffULL) << 32, std::memory_order_release);
        }
        cv_.notify_all();
        work();
        // the caller helped; wait for the chunks still running elsewhere
        for (int spin = 0; left_.load(std::memory_order_acquire) > 0; ++spin) {
            if (spin < 20000) {
                std::this_thread::yield();
                continue;
            }
            std::unique_lock<std::mutex> lk(mu_);
            done_cv_.wait(lk, [&] { return left_.load(std::memory_order_acquire) == 0; });
        }
        std::exception_ptr err;
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = nullptr;
            std::swap(err, err_);
        }
        if (err) std::rethrow_exception(err);
    }

  private:
    HostPool()
    {
        // XFEMM_HOST_THREADS overrides the thread count (1..64; tests)
        unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        hw = std::min(hw, 16u);
        if (const char *e = std::getenv("XFEMM_HOST_THREADS")) {
            const int v = std::atoi(e);
            if (v >= 1 && v <= 64) hw = (unsigned)v;
        }
        const int nw = (int)hw - 1;
        for (int i = 0; i < nw; ++i) workers_.emplace_back([this] { loop(); });
        for (auto &w : workers_) w.detach();
    }
    // chunks are claimed from a ticket (generation : 32 | next index : 32),
    // so a thread that read an older job's function can never claim -- and
    // so never call -- a chunk of a newer job; and the caller waits until
    // every claimed chunk of its job has finished, so a claimed chunk's
    // function is alive
    void work()
    {
        std::function<void(int)> *j;
        int n;
        unsigned long long g;
        {
            std::lock_guard<std::mutex> lk(mu_);
            j = job_;
            n = n_;
            g = gen_ & 0xffffffffULL;
        }
        if (!j) return;
        const bool was = in_job_;
        in_job_ = true;
        for (;;) {
            unsigned long long v = ticket_.load(std::memory_order_acquire);
            int t = -1;
            while ((v >> 32) == g && (int)(v & 0xffffffffULL) < n) {
                if (ticket_.compare_exchange_weak(v, v + 1, std::memory_order_acq_rel)) {
                    t = (int)(v & 0xffffffffULL);
                    break;
                }
            }
            if (t < 0) break;
            try {
                (*j)(t);
            } catch (...) {   // (kept for run(); the chunk still counts as done)
                std::lock_guard<std::mutex> lk(mu_);
                if (!err_) err_ = std::current_exception();
            }
            if (left_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                std::lock_guard<std::mutex> lk(mu_);
                done_cv_.notify_all();
            }
        }
        in_job_ = was;
    }
    void loop()
    {
        unsigned long long seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_ != seen && job_ != nullptr; });
                seen = gen_;
            }
            work();
        }
    }

    std::vector<std::thread> workers_;
    std::mutex run_mu_;   // one loop at a time
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::function<void(int)> *job_ = nullptr;
    std::exception_ptr err_;   // first exception of the running job (under mu_)
    int n_ = 0;
    unsigned long long gen_ = 0;
    std::atomic<unsigned long long> ticket_{0};
    std::atomic<int> left_{0};
    static inline thread_local bool in_job_ = false;
};

}  // namespace xfemm
