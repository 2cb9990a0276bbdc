// Communicators of the sharded solve (xfk_comm.h): the issue-ordered,
// optionally recorded collectives of the base class, RCCL, the in-process
// local group and the replay of a recording, plus their C-ABI constructors
// (include/xfemm_kernels.h).
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
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

// ---------------------------------------------------------------- recording
// One rank's log of collectives and (mode 2) the bytes it received, in
// device chunks, in call order: per call, its received blocks (all-reduce:
// recv; all-gather: recv; exchange: each receive range in plan order).
struct CommRecording {
    int mode = 0;
    int device = 0;
    std::vector<xfk_comm_op> ops;
    struct Block {
        size_t chunk, off;
        long long bytes;
    };
    struct Call {
        int op;
        long long bytes;          // all-reduce / all-gather payload; exchange: receive ranges
        size_t first, n;          // blocks
    };
    std::vector<Call> calls;
    std::vector<size_t> segments;  // first call of each solve (xfk_comm::solve_boundary)
    std::vector<Block> blocks;
    std::vector<std::unique_ptr<DBuf<char>>> chunks;
    size_t used = 0;              // bytes used in the last chunk
    static constexpr size_t kChunk = size_t(64) << 20;

    // device copy of `bytes` at `src` into the arena, ordered on s
    int keep(const void *src, long long bytes, hipStream_t s)
    {
        const size_t b = (size_t)bytes, a = (b + 255) & ~size_t(255);
        if (chunks.empty() || used + a > chunks.back()->n) {
            chunks.emplace_back(new DBuf<char>());
            ArenaScope own(nullptr);   // (the recording outlives the problem whose solve it records)
            XFK_CHECK(chunks.back()->alloc(std::max(kChunk, a)));
            used = 0;
        }
        blocks.push_back({chunks.size() - 1, used, bytes});
        if (b) XFK_CHECK(hipMemcpyAsync(chunks.back()->p + used, src, b, hipMemcpyDeviceToDevice, s));
        used += a;
        return XFK_OK;
    }
    const char *at(const Block &k) const { return chunks[k.chunk]->p + k.off; }
};

static const char *op_name(int op)
{
    switch (op) {
    case XFK_COMM_ALLREDUCE: return "all-reduce";
    case XFK_COMM_EXCHANGE: return "halo exchange";
    case XFK_COMM_ALLGATHER: return "all-gather";
    default: return "?";
    }
}

}  // namespace xfk

using namespace xfk;

xfk_comm::~xfk_comm()
{
    if (order_ev) (void)hipEventDestroy(order_ev);
    for (const Timed &t : timed) {
        (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
    }
    for (hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
}

int xfk_comm::pooled_event(hipEvent_t *e)
{
    if (!ev_pool.empty()) {
        *e = ev_pool.back();
        ev_pool.pop_back();
        return XFK_OK;
    }
    XFK_CHECK(hipEventCreate(e));
    return XFK_OK;
}

int xfk_comm::take_timing(long long calls[3], double us_total[3], double us_max[3])
{
    for (int k = 0; k < 3; ++k) {
        calls[k] = 0;
        us_total[k] = 0.0;
        us_max[k] = 0.0;
    }
    int rc = XFK_OK;
    for (const Timed &t : timed) {
        float ms = 0.f;
        if (rc == XFK_OK && (hipEventSynchronize(t.b) != hipSuccess || hipEventElapsedTime(&ms, t.a, t.b) != hipSuccess))
            rc = XFK_ERR_HIP;
        calls[t.slot] += 1;
        us_total[t.slot] += 1e3 * ms;
        us_max[t.slot] = std::max(us_max[t.slot], 1e3 * (double)ms);
        ev_pool.push_back(t.a);
        ev_pool.push_back(t.b);
    }
    timed.clear();
    if (rc != XFK_OK) set_error("xfk_comm_timing: a collective's events could not be read");
    return rc;
}

// every collective runs after the previous one of this communicator: a new
// stream first waits for the event recorded after the previous collective
int xfk_comm::begin(int op, hipStream_t s, int &idx, int &waited)
{
    if (!order_ev) XFK_CHECK(hipEventCreateWithFlags(&order_ev, hipEventDisableTiming));
    waited = 0;
    if (order_s && order_s != s) {
        XFK_CHECK(hipStreamWaitEvent(s, order_ev, 0));
        waited = 1;
    }
    idx = -1;
    for (size_t k = 0; k < streams.size(); ++k)
        if (streams[k] == s) idx = (int)k;
    if (idx < 0) {
        idx = (int)streams.size();
        streams.push_back(s);
    }
    if (op_slot >= 0) ev_pool.push_back(op_start);   // (a collective that failed before end(): its start event back)
    op_slot = -1;
    if (timing) {   // the start event follows the order wait: the interval is the collective itself
        op_slot = op == XFK_COMM_ALLREDUCE ? 0 : op == XFK_COMM_EXCHANGE ? 1 : 2;
        if (pooled_event(&op_start) != XFK_OK) return XFK_ERR_HIP;
        XFK_CHECK(hipEventRecord(op_start, s));
    }
    return XFK_OK;
}

int xfk_comm::solve_boundary()
{
    if (rec && rec->mode > 0) rec->segments.push_back(rec->calls.size());
    return XFK_OK;
}

int xfk_comm::end(hipStream_t s)
{
    if (op_slot >= 0) {
        hipEvent_t stop;
        if (pooled_event(&stop) != XFK_OK) return XFK_ERR_HIP;
        XFK_CHECK(hipEventRecord(stop, s));
        timed.push_back({op_slot, op_start, stop});
        op_slot = -1;
    }
    XFK_CHECK(hipEventRecord(order_ev, s));
    order_s = s;
    ++n_collectives;
    return XFK_OK;
}

namespace {
xfk_comm_op make_op(long long seq, int op, int stream, int waited, int peer, long long bytes, long long g0)
{
    xfk_comm_op o;
    o.seq = seq;
    o.op = op;
    o.stream = stream;
    o.waited = waited;
    o.peer = peer;
    o.bytes = bytes;
    o.g0 = g0;
    return o;
}
}  // namespace

int xfk_comm::allreduce_sum(const double *send, double *recv, size_t n, hipStream_t s)
{
    int idx, waited, rc;
    if ((rc = begin(XFK_COMM_ALLREDUCE, s, idx, waited)) != XFK_OK) return rc;
    if ((rc = do_allreduce_sum(send, recv, n, s)) != XFK_OK) return rc;
    if (rec && rec->mode > 0) {
        const long long seq = (long long)rec->calls.size();
        const long long b = (long long)(n * sizeof(double));
        rec->ops.push_back(make_op(seq, XFK_COMM_ALLREDUCE, idx, waited, -1, b, 0));
        rec->calls.push_back({XFK_COMM_ALLREDUCE, b, rec->blocks.size(), rec->mode == 2 ? 1u : 0u});
        if (rec->mode == 2 && (rc = rec->keep(recv, b, s)) != XFK_OK) return rc;
    }
    return end(s);
}

int xfk_comm::exchange(const HaloPlan &h, double *vec, hipStream_t s)
{
    int idx, waited, rc;
    if ((rc = begin(XFK_COMM_EXCHANGE, s, idx, waited)) != XFK_OK) return rc;
    if ((rc = do_exchange(h, vec, s)) != XFK_OK) return rc;
    if (rec && rec->mode > 0) {
        const long long seq = (long long)rec->calls.size();
        rec->ops.push_back(
            make_op(seq, XFK_COMM_EXCHANGE, idx, waited, -1, 0, (long long)(h.send.size() + h.recv.size())));
        for (const HaloRange &t : h.send)
            rec->ops.push_back(make_op(seq, XFK_COMM_SEND, idx, waited, t.peer, 8LL * t.len, t.g0));
        for (const HaloRange &r : h.recv)
            rec->ops.push_back(make_op(seq, XFK_COMM_RECV, idx, waited, r.peer, 8LL * r.len, r.g0));
        rec->calls.push_back({XFK_COMM_EXCHANGE, (long long)h.recv.size(), rec->blocks.size(),
                              rec->mode == 2 ? h.recv.size() : 0u});
        if (rec->mode == 2)
            for (const HaloRange &r : h.recv)
                if ((rc = rec->keep(vec + r.off, 8LL * r.len, s)) != XFK_OK) return rc;
    }
    return end(s);
}

int xfk_comm::allgather_bytes(const void *send, void *recv, size_t bytes, hipStream_t s)
{
    int idx, waited, rc;
    if ((rc = begin(XFK_COMM_ALLGATHER, s, idx, waited)) != XFK_OK) return rc;
    if ((rc = do_allgather_bytes(send, recv, bytes, s)) != XFK_OK) return rc;
    if (rec && rec->mode > 0) {
        const long long seq = (long long)rec->calls.size();
        rec->ops.push_back(make_op(seq, XFK_COMM_ALLGATHER, idx, waited, -1, (long long)bytes, 0));
        rec->calls.push_back({XFK_COMM_ALLGATHER, (long long)bytes, rec->blocks.size(), rec->mode == 2 ? 1u : 0u});
        if (rec->mode == 2 && (rc = rec->keep(recv, (long long)bytes * size, s)) != XFK_OK) return rc;
    }
    return end(s);
}

int xfk_comm::allgather(const double *send, double *recv, size_t n, hipStream_t s)
{
    int idx, waited, rc;
    if ((rc = begin(XFK_COMM_ALLGATHER, s, idx, waited)) != XFK_OK) return rc;
    if ((rc = do_allgather(send, recv, n, s)) != XFK_OK) return rc;
    if (rec && rec->mode > 0) {
        const long long seq = (long long)rec->calls.size();
        const long long b = (long long)(n * sizeof(double));
        rec->ops.push_back(make_op(seq, XFK_COMM_ALLGATHER, idx, waited, -1, b, 0));
        rec->calls.push_back({XFK_COMM_ALLGATHER, b, rec->blocks.size(), rec->mode == 2 ? 1u : 0u});
        if (rec->mode == 2 && (rc = rec->keep(recv, b * size, s)) != XFK_OK) return rc;
    }
    return end(s);
}

namespace xfk {

// ---------------------------------------------------------------- replay
struct ReplayComm final : xfk_comm {
    std::shared_ptr<const CommRecording> src;
    size_t cursor = 0;
    int seg = -1;          // segment (recorded solve) being served

    size_t seg_begin(int k) const { return src->segments.empty() ? 0 : src->segments[k]; }
    size_t seg_end(int k) const
    {
        return (size_t)k + 1 < src->segments.size() ? src->segments[k + 1] : src->calls.size();
    }
    int solve_boundary() override
    {
        const int nseg = std::max<int>(1, (int)src->segments.size());
        if (seg >= 0 && cursor != seg_end(seg)) {
            set_error("replay: the last solve issued " + std::to_string((long long)cursor - (long long)seg_begin(seg)) +
                      " collectives, the recorded solve " + std::to_string(seg_end(seg) - seg_begin(seg)));
            return XFK_ERR_ARG;
        }
        seg = std::min(seg + 1, nseg - 1);
        cursor = seg_begin(seg);
        return XFK_OK;
    }

    int next(int op, long long bytes, const CommRecording::Call *&c)
    {
        XFK_REQUIRE(!src->calls.empty(), XFK_ERR_ARG, "replay: empty recording");
        if (seg < 0) seg = 0;   // (collectives before the first solve: the first segment)
        XFK_REQUIRE(cursor < seg_end(seg), XFK_ERR_ARG,
                    "replay: more collectives than the recorded solve issued (" + std::to_string(cursor) + ")");
        c = &src->calls[cursor];
        if (c->op != op || c->bytes != bytes) {
            set_error(std::string("replay: collective ") + std::to_string(cursor) + " is a " + op_name(op) + " of " +
                      std::to_string(bytes) + ", the recording has a " + op_name(c->op) + " of " +
                      std::to_string(c->bytes));
            return XFK_ERR_ARG;
        }
        ++cursor;
        return XFK_OK;
    }
    int copy(const CommRecording::Call &c, size_t k, void *dst, long long bytes, hipStream_t s)
    {
        XFK_REQUIRE(k < c.n && src->blocks[c.first + k].bytes == bytes, XFK_ERR_ARG,
                    "replay: received block size differs from the recording");
        if (bytes) XFK_CHECK(hipMemcpyAsync(dst, src->at(src->blocks[c.first + k]), (size_t)bytes,
                                            hipMemcpyDeviceToDevice, s));
        return XFK_OK;
    }
    int do_allreduce_sum(const double *, double *recv, size_t n, hipStream_t s) override
    {
        const CommRecording::Call *c;
        const long long b = (long long)(n * sizeof(double));
        int rc = next(XFK_COMM_ALLREDUCE, b, c);
        return rc != XFK_OK ? rc : copy(*c, 0, recv, b, s);
    }
    int do_exchange(const HaloPlan &h, double *vec, hipStream_t s) override
    {
        const CommRecording::Call *c;
        int rc = next(XFK_COMM_EXCHANGE, (long long)h.recv.size(), c);
        for (size_t k = 0; rc == XFK_OK && k < h.recv.size(); ++k)
            rc = copy(*c, k, vec + h.recv[k].off, 8LL * h.recv[k].len, s);
        return rc;
    }
    int do_allgather(const double *, double *recv, size_t n, hipStream_t s) override
    {
        const CommRecording::Call *c;
        const long long b = (long long)(n * sizeof(double));
        int rc = next(XFK_COMM_ALLGATHER, b, c);
        return rc != XFK_OK ? rc : copy(*c, 0, recv, b * size, s);
    }
    int do_allgather_bytes(const void *, void *recv, size_t bytes, hipStream_t s) override
    {
        const CommRecording::Call *c;
        int rc = next(XFK_COMM_ALLGATHER, (long long)bytes, c);
        return rc != XFK_OK ? rc : copy(*c, 0, recv, (long long)bytes * size, s);
    }
    const char *kind() const override { return "replay"; }
};

// ---------------------------------------------------------------- RCCL
struct RcclComm final : xfk_comm {
    ncclComm_t comm = nullptr;
    ~RcclComm() override
    {
        if (comm) (void)ncclCommDestroy(comm);
    }
    int do_allreduce_sum(const double *send, double *recv, size_t n, hipStream_t s) override
    {
        XFK_NCCL(ncclAllReduce(send, recv, n, ncclDouble, ncclSum, comm, s));
        return XFK_OK;
    }
    int do_exchange(const HaloPlan &h, double *vec, hipStream_t s) override
    {
        if (h.send.empty() && h.recv.empty()) return XFK_OK;
        XFK_NCCL(ncclGroupStart());
        for (const HaloRange &r : h.recv) XFK_NCCL(ncclRecv(vec + r.off, r.len, ncclDouble, r.peer, comm, s));
        for (const HaloRange &t : h.send) XFK_NCCL(ncclSend(vec + t.off, t.len, ncclDouble, t.peer, comm, s));
        XFK_NCCL(ncclGroupEnd());
        return XFK_OK;
    }
    int do_allgather(const double *send, double *recv, size_t n, hipStream_t s) override
    {
        XFK_NCCL(ncclAllGather(send, recv, n, ncclDouble, comm, s));
        return XFK_OK;
    }
    int do_allgather_bytes(const void *send, void *recv, size_t bytes, hipStream_t s) override
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
    int do_allreduce_sum(const double *send, double *recv, size_t n, hipStream_t s) override
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
    int do_exchange(const HaloPlan &h, double *vec, hipStream_t s) override
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
    int do_allgather(const double *send, double *recv, size_t n, hipStream_t s) override
    {
        return collective(send, nullptr, s, "allgather", [&]() -> int {
            for (int q = 0; q < size; ++q)
                XFK_CHECK(hipMemcpyAsync(recv + (size_t)q * n, hub->src[q], sizeof(double) * n,
                                         hipMemcpyDeviceToDevice, s));
            return XFK_OK;
        });
    }
    int do_allgather_bytes(const void *send, void *recv, size_t bytes, hipStream_t s) override
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

int xfk_comm_record(xfk_comm *c, int mode)
{
    XFK_REQUIRE(c && mode >= 0 && mode <= 2, XFK_ERR_ARG, "xfk_comm_record: null communicator or mode not 0..2");
    if (mode == 0) {
        if (c->rec) c->rec->mode = -c->rec->mode;   // stopped: no new records, the log stays readable
        return XFK_OK;
    }
    auto r = std::make_shared<CommRecording>();
    r->mode = mode;
    (void)hipGetDevice(&r->device);
    c->rec = r;
    return XFK_OK;
}

int xfk_comm_time(xfk_comm *c, int on)
{
    XFK_REQUIRE(c, XFK_ERR_ARG, "xfk_comm_time: null communicator");
    c->timing = on != 0;
    return XFK_OK;
}

int xfk_comm_timing(xfk_comm *c, long long calls[3], double us_total[3], double us_max[3])
{
    XFK_REQUIRE(c && calls && us_total && us_max, XFK_ERR_ARG, "xfk_comm_timing: null argument");
    return c->take_timing(calls, us_total, us_max);
}

int xfk_comm_log(const xfk_comm *c, xfk_comm_op *out, int cap, int *count)
{
    XFK_REQUIRE(c && count, XFK_ERR_ARG, "null argument");
    const int n = c->rec ? (int)c->rec->ops.size() : 0;
    *count = n;
    if (out)
        for (int k = 0; k < n && k < cap; ++k) out[k] = c->rec->ops[k];
    return XFK_OK;
}

int xfk_comm_create_replay(const xfk_comm *recorded, xfk_comm **out)
{
    XFK_REQUIRE(recorded && out, XFK_ERR_ARG, "null argument");
    XFK_REQUIRE(recorded->rec && std::abs(recorded->rec->mode) == 2 && !recorded->rec->calls.empty(), XFK_ERR_ARG,
                "replay: the communicator holds no data recording (xfk_comm_record mode 2)");
    auto *c = new ReplayComm();
    c->rank = recorded->rank;
    c->size = recorded->size;
    c->src = recorded->rec;
    *out = c;
    return XFK_OK;
}

}  // extern "C"

// xfk_device_init: loads this translation unit's code object onto the device
// (the first use of any of its kernels would otherwise do it inside a solve)
hipError_t xfk::warm_module_comm()
{
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&k_sum_ptrs));
}
