// Communicators of the sharded solve (xfk_comm.h): RCCL and the in-process
// local group, plus their C-ABI constructors (include/xfemm_kernels.h).
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "xfk_comm.h"
#include "xfk_internal.h"

namespace xfk {

#define XFK_NCCL(call)                                                                        \
    do {                                                                                      \
        ncclResult_t _r = (call);                                                             \
        if (_r != ncclSuccess) {                                                              \
            ::xfk::set_error(std::string(#call) + ": " + ncclGetErrorString(_r));             \
            return XFK_ERR_HIP;                                                               \
        }                                                                                     \
    } while (0)

// ---------------------------------------------------------------- RCCL
struct RcclComm final : xfk_comm {
    ncclComm_t comm = nullptr;
    ~RcclComm() override
    {
        if (comm) (void)ncclCommDestroy(comm);
    }
    int allreduce_sum(const double *send, double *recv, size_t n, hipStream_t s) override
    {
        XFK_NCCL(ncclAllReduce(send, recv, n, ncclDouble, ncclSum, comm, s));
        return XFK_OK;
    }
    int exchange(const HaloPlan &h, double *vec, hipStream_t s) override
    {
        if (h.send.empty() && h.recv.empty()) return XFK_OK;
        XFK_NCCL(ncclGroupStart());
        for (const HaloRange &r : h.recv) XFK_NCCL(ncclRecv(vec + r.off, r.len, ncclDouble, r.peer, comm, s));
        for (const HaloRange &t : h.send) XFK_NCCL(ncclSend(vec + t.off, t.len, ncclDouble, t.peer, comm, s));
        XFK_NCCL(ncclGroupEnd());
        return XFK_OK;
    }
    int allgather(const double *send, double *recv, size_t n, hipStream_t s) override
    {
        XFK_NCCL(ncclAllGather(send, recv, n, ncclDouble, comm, s));
        return XFK_OK;
    }
    int allgather_bytes(const void *send, void *recv, size_t bytes, hipStream_t s) override
    {
        XFK_NCCL(ncclAllGather(send, recv, bytes, ncclChar, comm, s));
        return XFK_OK;
    }
    const char *kind() const override { return "rccl"; }
};

// ---------------------------------------------------------------- local group
constexpr int kMaxLocalRanks = 16;

struct SumPtrs {
    const double *p[kMaxLocalRanks];
    int n;
};

// recv[i] = sum_q p_q[i], in rank order (same bits on every rank)
__global__ void k_sum_ptrs(double *__restrict__ recv, SumPtrs P, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        double s = 0.0;
        for (int q = 0; q < P.n; ++q) s += P.p[q][i];
        recv[i] = s;
    }
}

struct LocalHub {
    int size;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    long long generation = 0;
    bool broken = false;
    std::vector<const double *> src;     // per rank: buffer published for this collective
    std::vector<const HaloPlan *> plan;
    std::vector<hipEvent_t> ready, done;
    explicit LocalHub(int n) : size(n), src(n), plan(n), ready(n, nullptr), done(n, nullptr) {}
    ~LocalHub()
    {
        for (auto e : ready)
            if (e) (void)hipEventDestroy(e);
        for (auto e : done)
            if (e) (void)hipEventDestroy(e);
    }
    // generation barrier with a timeout: a rank that failed never arrives
    bool barrier()
    {
        std::unique_lock<std::mutex> lk(mu);
        if (broken) return false;
        const long long gen = generation;
        if (++arrived == size) {
            arrived = 0;
            ++generation;
            cv.notify_all();
            return true;
        }
        if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return generation != gen || broken; }) || broken) {
            broken = true;
            cv.notify_all();
            return false;
        }
        return true;
    }
};

struct LocalComm final : xfk_comm {
    std::shared_ptr<LocalHub> hub;

    int ensure_events()
    {
        if (!hub->ready[rank]) {
            XFK_CHECK(hipEventCreateWithFlags(&hub->ready[rank], hipEventDisableTiming));
            XFK_CHECK(hipEventCreateWithFlags(&hub->done[rank], hipEventDisableTiming));
        }
        return XFK_OK;
    }
    int sync_point(const char *what)
    {
        if (!hub->barrier()) {
            set_error(std::string("local communicator: a rank did not arrive at ") + what);
            return XFK_ERR_HIP;
        }
        return XFK_OK;
    }
    // publish `src`, wait until every rank's data is ready, run `body`, then make
    // this rank's later work wait until every rank has finished reading
    template <class F>
    int collective(const double *src, const HaloPlan *plan, hipStream_t s, const char *what, F body)
    {
        int rc = ensure_events();
        if (rc != XFK_OK) return rc;
        hub->src[rank] = src;
        hub->plan[rank] = plan;
        XFK_CHECK(hipEventRecord(hub->ready[rank], s));
        if ((rc = sync_point(what)) != XFK_OK) return rc;
        for (int q = 0; q < size; ++q) XFK_CHECK(hipStreamWaitEvent(s, hub->ready[q], 0));
        rc = body();
        if (rc != XFK_OK) return rc;
        XFK_CHECK(hipEventRecord(hub->done[rank], s));
        if ((rc = sync_point(what)) != XFK_OK) return rc;
        for (int q = 0; q < size; ++q) XFK_CHECK(hipStreamWaitEvent(s, hub->done[q], 0));
        // No third barrier: a rank re-records `ready` only after the second
        // barrier (every wait on it is enqueued by then) and `done` only after
        // the next collective's first barrier (every wait on it likewise).
        return XFK_OK;
    }
    int allreduce_sum(const double *send, double *recv, size_t n, hipStream_t s) override
    {
        return collective(send, nullptr, s, "allreduce", [&]() -> int {
            SumPtrs P{};
            P.n = size;
            for (int q = 0; q < size; ++q) P.p[q] = hub->src[q];
            const int grid = (int)std::min<size_t>((n + 255) / 256, 1024);
            if (n) k_sum_ptrs<<<grid, 256, 0, s>>>(recv, P, n);
            XFK_CHECK(hipGetLastError());
            return XFK_OK;
        });
    }
    int exchange(const HaloPlan &h, double *vec, hipStream_t s) override
    {
        return collective(vec, &h, s, "halo exchange", [&]() -> int {
            for (const HaloRange &r : h.recv) {
                const HaloPlan *peer = hub->plan[r.peer];
                const HaloRange *t = nullptr;
                for (const HaloRange &c : peer->send)   // (a peer may send several ranges: match by start)
                    if (c.peer == rank && c.g0 == r.g0) t = &c;
                if (!t || t->len != r.len || t->g0 != r.g0) {
                    set_error("local communicator: halo ranges of two ranks disagree");
                    return XFK_ERR_ARG;
                }
                XFK_CHECK(hipMemcpyAsync(vec + r.off, hub->src[r.peer] + t->off, sizeof(double) * r.len,
                                         hipMemcpyDeviceToDevice, s));
            }
            return XFK_OK;
        });
    }
    int allgather(const double *send, double *recv, size_t n, hipStream_t s) override
    {
        return collective(send, nullptr, s, "allgather", [&]() -> int {
            for (int q = 0; q < size; ++q)
                XFK_CHECK(hipMemcpyAsync(recv + (size_t)q * n, hub->src[q], sizeof(double) * n,
                                         hipMemcpyDeviceToDevice, s));
            return XFK_OK;
        });
    }
    int allgather_bytes(const void *send, void *recv, size_t bytes, hipStream_t s) override
    {
        return collective(static_cast<const double *>(send), nullptr, s, "allgather", [&]() -> int {
            for (int q = 0; q < size; ++q)
                XFK_CHECK(hipMemcpyAsync(static_cast<char *>(recv) + (size_t)q * bytes, hub->src[q], bytes,
                                         hipMemcpyDeviceToDevice, s));
            return XFK_OK;
        });
    }
    const char *kind() const override { return "local"; }
};

}  // namespace xfk

using namespace xfk;

extern "C" {

int xfk_comm_unique_id(void *out, int bytes)
{
    XFK_REQUIRE(out && bytes >= NCCL_UNIQUE_ID_BYTES, XFK_ERR_ARG, "unique id buffer too small (128 bytes)");
    ncclUniqueId id;
    XFK_NCCL(ncclGetUniqueId(&id));
    std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return XFK_OK;
}

int xfk_comm_create_rccl(const void *unique_id, int bytes, int rank, int nranks, int device, xfk_comm **out)
{
    XFK_REQUIRE(unique_id && out && bytes >= NCCL_UNIQUE_ID_BYTES, XFK_ERR_ARG, "bad unique id");
    XFK_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, XFK_ERR_ARG, "bad rank / size");
    *out = nullptr;
    XFK_CHECK(hipSetDevice(device));
    ncclUniqueId id;
    std::memcpy(id.internal, unique_id, NCCL_UNIQUE_ID_BYTES);
    auto *c = new RcclComm();
    c->rank = rank;
    c->size = nranks;
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
    if (r != ncclSuccess) {
        set_error(std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
        c->comm = nullptr;
        delete c;
        return XFK_ERR_HIP;
    }
    *out = c;
    return XFK_OK;
}

int xfk_comm_create_local(int nranks, xfk_comm **out)
{
    XFK_REQUIRE(out && nranks >= 1 && nranks <= kMaxLocalRanks, XFK_ERR_ARG, "local group: 1..16 ranks");
    auto hub = std::make_shared<LocalHub>(nranks);
    for (int q = 0; q < nranks; ++q) {
        auto *c = new LocalComm();
        c->rank = q;
        c->size = nranks;
        c->hub = hub;
        out[q] = c;
    }
    return XFK_OK;
}

void xfk_comm_destroy(xfk_comm *c) { delete c; }

int xfk_comm_rank(const xfk_comm *c) { return c ? c->rank : -1; }
int xfk_comm_size(const xfk_comm *c) { return c ? c->size : -1; }

}  // extern "C"
