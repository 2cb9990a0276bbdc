// Communicator of the sharded solve: the collectives the distributed PCG /
// Newton loop / AMG setup need, stream-ordered on the caller's HIP stream.
//
//   RCCL (production): one process per GPU, ncclAllReduce / grouped
//     ncclSend+ncclRecv / ncclAllGather over xGMI.  Created from a unique id
//     the caller distributes (e.g. torch.distributed broadcast).
//   Local group: N ranks inside ONE process, one host thread per rank, on one
//     or several devices.  Exchanges are device copies and a sum kernel,
//     ordered by HIP events and a host barrier.  It exists so that the sharded
//     GPU path runs end to end on a single-GPU machine (RCCL refuses two ranks
//     on one device) -- it is the test transport, not the production one.
//   Replay: one rank of a recorded run served from its recording (every
//     collective's received bytes, device resident): the rank's own kernels
//     run alone on its GPU, bit-identical to the recorded run, with no peer --
//     the per-rank compute-only measurement of the sharded path.
//
// Issue order.  RCCL matches collectives by their order on the communicator,
// not by stream, and its kernels block until the peers' matching kernels run.
// The sharded path issues halo exchanges on a side stream (overlapped with
// interior tiles) and the all-reduces / all-gathers on the main stream, so
// two collectives of one communicator on different streams must never be
// able to run out of issue order.  The base class makes that true by
// construction: every collective first waits (hipStreamWaitEvent) for the
// event recorded after the previous collective whenever the stream changes,
// then records that event itself.  Every rank therefore executes its
// collectives in issue order, and the recording (xfk_comm_record) proves the
// issue order is the same on every rank.
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <vector>

#include "xfk_partition.h"

namespace xfk {
struct CommRecording;
}

struct xfk_comm {
    int rank = 0, size = 1;
    virtual ~xfk_comm();
    // recv[i] = sum over ranks of send[i] (identical bits on every rank); send != recv
    int allreduce_sum(const double *send, double *recv, size_t n, hipStream_t s);
    // fill the halo part of vec: every recv range from its peer's matching send range
    int exchange(const xfk::HaloPlan &h, double *vec, hipStream_t s);
    // recv[q * n + i] = send_q[i]
    int allgather(const double *send, double *recv, size_t n, hipStream_t s);
    // the same for raw bytes (integer arrays): recv[q * bytes + i] = send_q[i]
    int allgather_bytes(const void *send, void *recv, size_t bytes, hipStream_t s);
    virtual const char *kind() const = 0;
    // a solve begins (xfk_static2d): a recording starts a new segment; the
    // replay checks that the last solve issued exactly its segment's calls and
    // moves to the next segment (the last one repeats)
    virtual int solve_boundary();

    // issue-order bookkeeping (see above) and the optional recording
    hipEvent_t order_ev = nullptr;
    hipStream_t order_s = nullptr;
    std::vector<hipStream_t> streams;            // first-use order: the stream index of a record
    std::shared_ptr<xfk::CommRecording> rec;     // non-null while recording
    long long n_collectives = 0;
    // xfk_comm_time: (op slot, start, stop) per timed collective, and a pool
    // of events to reuse once read
    bool timing = false;
    struct Timed {
        int slot;
        hipEvent_t a, b;
    };
    std::vector<Timed> timed;
    std::vector<hipEvent_t> ev_pool;
    int take_timing(long long calls[3], double us_total[3], double us_max[3]);

   protected:
    virtual int do_allreduce_sum(const double *send, double *recv, size_t n, hipStream_t s) = 0;
    virtual int do_exchange(const xfk::HaloPlan &h, double *vec, hipStream_t s) = 0;
    virtual int do_allgather_bytes(const void *send, void *recv, size_t bytes, hipStream_t s) = 0;
    virtual int do_allgather(const double *send, double *recv, size_t n, hipStream_t s)
    {
        return do_allgather_bytes(send, recv, n * sizeof(double), s);
    }

   private:
    int begin(int op, hipStream_t s, int &stream_idx, int &waited);
    int end(hipStream_t s);
    int op_slot = -1;   // (the timed collective in flight between begin and end)
    hipEvent_t op_start = nullptr;
    int pooled_event(hipEvent_t *e);
};
