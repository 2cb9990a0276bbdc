// Communicator of the sharded solve: the three collectives the distributed
// PCG / Newton loop needs, stream-ordered on the caller's HIP stream.
//
//   RCCL (production): one process per GPU, ncclAllReduce / grouped
//     ncclSend+ncclRecv / ncclAllGather over xGMI.  Created from a unique id
//     the caller distributes (e.g. torch.distributed broadcast).
//   Local group: N ranks inside ONE process, one host thread per rank, on one
//     or several devices.  Exchanges are device copies and a sum kernel,
//     ordered by HIP events and a host barrier.  It exists so that the sharded
//     GPU path runs end to end on a single-GPU machine (RCCL refuses two ranks
//     on one device) -- it is the test transport, not the production one.
#pragma once

#include <hip/hip_runtime.h>

#include "xfk_partition.h"

struct xfk_comm {
    int rank = 0, size = 1;
    virtual ~xfk_comm() {}
    // recv[i] = sum over ranks of send[i] (identical bits on every rank); send != recv
    virtual int allreduce_sum(const double *send, double *recv, size_t n, hipStream_t s) = 0;
    // fill the halo part of vec: every recv range from its peer's matching send range
    virtual int exchange(const xfk::HaloPlan &h, double *vec, hipStream_t s) = 0;
    // recv[q * n + i] = send_q[i]
    virtual int allgather(const double *send, double *recv, size_t n, hipStream_t s) = 0;
    // the same for raw bytes (integer arrays): recv[q * bytes + i] = send_q[i]
    virtual int allgather_bytes(const void *send, void *recv, size_t bytes, hipStream_t s) = 0;
    virtual const char *kind() const = 0;
};
