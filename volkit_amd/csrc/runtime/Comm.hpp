// Comm.hpp -- internal: the RCCL binding and the plane transport shared by the Z-slab
// exchange (Comm.cpp) and the Z-slab Range calls (Slab.cpp).
#pragma once

#include "Runtime.hpp"
#include "volkit_hip.h"

#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

// A communicator and its round watcher.  Every RCCL round returns once enqueued; with a
// deadline (timeoutMs > 0) the round's start / end events go to the watcher thread, which times
// the round from the moment its start event completes (work queued ahead of it is not the
// round's), polls ncclCommGetAsyncError, and on a timeout or an asynchronous error aborts the
// communicator: its kernels exit, and every later call on it -- and vktHipCommSynchronize --
// returns vktInvalidValue naming the failure.
struct vktHipComm_impl
{
    struct Round
    {
        hipEvent_t start = nullptr, end = nullptr;
        int64_t timeoutMs = 0;
        std::string what;
    };

    std::atomic<ncclComm_t> comm{nullptr};   // nullptr once aborted
    int32_t rank = 0, nranks = 0;
    int device = 0;
    int64_t timeoutMs = 0;            // vktHipCommSetTimeout, VKT_COMM_TIMEOUT_MS; 0: no deadline
    hipStream_t stream = nullptr;     // the communicator's own stream (overlapped rounds), lazily
    // em: one enqueue (ncclGroupStart .. ncclGroupEnd + the round's bookkeeping) at a time, so
    // rounds are issued and judged in order.  The watcher never blocks on it: a blocking
    // ncclGroupEnd may wait for a peer that died, and the abort is what releases it -- the
    // watcher aborts under em when the enqueue in flight lets go within kEnqueueGraceMs, and
    // without it otherwise (comm.cpp watch()).
    std::timed_mutex em;
    std::mutex m;                     // rounds, failure, timeoutMs (never held across an RCCL call)
    std::condition_variable cv;
    std::deque<Round> rounds;         // enqueued, not yet judged (front: being judged)
    std::thread watcher;
    bool stop = false;
    std::atomic<bool> aborted{false}; // a round failed or timed out: the communicator was aborted
    std::string failure;              // why (the first failure)
};

namespace vkt
{
namespace comm
{
    // planes [z0, z1) of a ceil partition of n planes over `world` ranks (slab.py:slab_bounds)
    void slabBounds(int32_t n, int32_t world, int32_t rank, int32_t& z0, int32_t& z1);

    // Bytes of one plane of a view (dimX * dimY * bpv); 0 for an invalid format.
    size_t planeBytes(vktHipVolumeView_t const& v);

    // Global planes [g0, g1) of a buffer that holds global planes [z0, z0 + v.dimZ): the device
    // pointer of plane g0 and the byte count, or an error when the buffer does not hold them.
    vktError planeSpan(vktHipVolumeView_t const& v, int32_t z0, int32_t g0, int32_t g1, char const* what,
                       uint8_t*& ptr, size_t& bytes);

    // One point-to-point move of a byte range: `send` to / receive from `peer`.
    struct Xfer
    {
        int32_t peer;
        int32_t send;
        uint8_t* ptr;
        size_t bytes;
    };

    // The moves as ONE ncclGroupStart .. ncclGroupEnd round of ncclSend / ncclRecv on `stream`
    // (pairs of ranks match their moves in issue order); returns once enqueued.  With
    // comm->timeoutMs > 0 the watcher judges the round under that deadline (see above): a peer
    // that never joins, or an asynchronous RCCL error, aborts the communicator instead of leaving
    // every later call on the stream hanging (SURVEY §5 failure detection).  A call on an
    // aborted communicator fails at once.
    vktError rcclRound(vktHipComm_t comm, std::vector<Xfer> const& xs, hipStream_t stream, char const* what);

    // rt::finishLaunch, then -- with async execution off -- vktHipCommSynchronize: a call that
    // enqueued a round returns that round's failure (timeout, asynchronous RCCL error).
    vktError finishRound(vktHipComm_t comm, char const* name);

    // A device-to-device copy on `stream` (the in-process transport: every slab of a
    // partition held by this process on the library's device).
    vktError localMove(uint8_t* dst, uint8_t const* src, size_t bytes, hipStream_t stream, char const* what);
} // namespace comm
} // namespace vkt
