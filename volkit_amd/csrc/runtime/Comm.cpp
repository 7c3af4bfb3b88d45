// Comm.cpp -- in-library Z-slab halo exchange over RCCL (xGMI) for C and C++ callers.
//
// The reference is single-device and has no communication layer (its CudaContext is
// declaration-only: include/c/vkt/CudaContext.h:17-65).  SURVEY.md §8(e) asks for Z-slab
// partitions with the Resample halo moved by ncclSend / ncclRecv inside one group; the
// Python layer does the same through torch.distributed (volkit_amd/slab.py).  This file is
// the native path: the plan (which global source planes every rank owns, holds and moves --
// the same ceil partition and exact z index table as slab.py, checked against it by
// tests/test_comm.py) and one grouped RCCL send/receive round on the library's compute
// stream, so a Resample enqueued next on that stream reads the halo.

#include "Comm.hpp"
#include "volkit_codec.hpp"

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

namespace vkt
{
namespace
{
    static_assert(sizeof(vktHipCommId_t) == sizeof(ncclUniqueId), "vktHipCommId_t mirrors ncclUniqueId");

    // RCCL is bound at first use, not linked: a process that already holds an RCCL (PyTorch
    // ships its own librccl.so.1) keeps that one -- linking /opt/rocm's made the loader pick
    // whichever came first for both users, and two ROCm builds' RCCL/HIP in one process
    // aborted at exit (free(): invalid pointer).
    struct Rccl
    {
        decltype(&::ncclGetUniqueId) getUniqueId = nullptr;
        decltype(&::ncclCommInitRank) commInitRank = nullptr;
        decltype(&::ncclCommDestroy) commDestroy = nullptr;
        decltype(&::ncclGroupStart) groupStart = nullptr;
        decltype(&::ncclGroupEnd) groupEnd = nullptr;
        decltype(&::ncclSend) send = nullptr;
        decltype(&::ncclRecv) recv = nullptr;
        decltype(&::ncclGetErrorString) errorString = nullptr;
        decltype(&::ncclCommGetAsyncError) getAsyncError = nullptr;   // optional (deadline only without it)
        decltype(&::ncclCommAbort) abort = nullptr;
        bool ok = false;
    };

    Rccl const& rccl()
    {
        static Rccl r;
        static std::once_flag once;
        std::call_once(once, [] {
            void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
            if (h == nullptr)
                h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
            if (h == nullptr)
                h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
            if (h == nullptr)
                return;
            auto sym = [&](auto& f, char const* name) {
                f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
                return f != nullptr;
            };
            r.ok = sym(r.getUniqueId, "ncclGetUniqueId") && sym(r.commInitRank, "ncclCommInitRank") &&
                   sym(r.commDestroy, "ncclCommDestroy") && sym(r.groupStart, "ncclGroupStart") &&
                   sym(r.groupEnd, "ncclGroupEnd") && sym(r.send, "ncclSend") && sym(r.recv, "ncclRecv") &&
                   sym(r.errorString, "ncclGetErrorString") && sym(r.abort, "ncclCommAbort");
            sym(r.getAsyncError, "ncclCommGetAsyncError");
        });
        return r;
    }

    vktError ncclFail(char const* what, ncclResult_t r)
    {
        return rt::fail((std::string(what) + ": " + rccl().errorString(r)).c_str());
    }

    vktError noRccl(char const* what)
    {
        return rt::fail((std::string(what) + ": librccl.so.1 not found").c_str());
    }

    using comm::slabBounds;

    // global source planes rank r's dst slab reads (empty slab: [0, 0))
    vktError needOf(int32_t dstG, int32_t srcG, int32_t world, int32_t r, vktFilterMode fm, int32_t chain,
                    int32_t& s0, int32_t& s1)
    {
        int32_t d0, d1;
        slabBounds(dstG, world, r, d0, d1);
        s0 = s1 = 0;
        if (d1 <= d0)
            return vktNoError;
        return vktHipResampleSlabSourceRange(dstG, d0, d1, srcG, fm, chain, &s0, &s1);
    }

    // slab.py:plan_resample -- every rank computes the same global plan; sends are the
    // peers' needs this rank owns, receives its own needs the peers own
    vktError plan(int32_t dstG, int32_t srcG, int32_t world, int32_t rank, vktFilterMode fm, int32_t chain,
                  int32_t& lo, int32_t& hi, std::vector<vktHipSlabTransfer_t>& xs)
    {
        if (world <= 0 || rank < 0 || rank >= world || dstG <= 0 || srcG <= 0)
            return rt::fail("vktHipSlabResamplePlan: invalid rank / world / depths");
        std::vector<int32_t> n0(world), n1(world);
        for (int32_t r = 0; r < world; ++r)
        {
            vktError const e = needOf(dstG, srcG, world, r, fm, chain, n0[r], n1[r]);
            if (e != vktNoError)
                return e;
        }
        int32_t o0, o1;
        slabBounds(srcG, world, rank, o0, o1);
        bool const needs = n1[rank] > n0[rank];
        lo = needs ? std::min(o0, n0[rank]) : o0;
        hi = needs ? std::max(o1, n1[rank]) : o1;
        xs.clear();
        for (int32_t peer = 0; peer < world; ++peer)
        {
            if (peer == rank)
                continue;
            int32_t p0, p1;
            slabBounds(srcG, world, peer, p0, p1);
            if (needs)
            {
                int32_t const a = std::max(n0[rank], p0), b = std::min(n1[rank], p1);
                if (b > a)
                    xs.push_back(vktHipSlabTransfer_t{peer, a, b, 0});
            }
            if (n1[peer] > n0[peer])
            {
                int32_t const a = std::max(n0[peer], o0), b = std::min(n1[peer], o1);
                if (b > a)
                    xs.push_back(vktHipSlabTransfer_t{peer, a, b, 1});
            }
        }
        return vktNoError;
    }
} // namespace

namespace comm
{
    void slabBounds(int32_t n, int32_t world, int32_t rank, int32_t& z0, int32_t& z1)
    {
        int64_t const size = (static_cast<int64_t>(n) + world - 1) / world;
        z0 = static_cast<int32_t>(std::min<int64_t>(static_cast<int64_t>(rank) * size, n));
        z1 = static_cast<int32_t>(std::min<int64_t>(z0 + size, n));
    }

    size_t planeBytes(vktHipVolumeView_t const& v)
    {
        uint32_t const bpv = codec::bytesPerVoxel(v.dataFormat);
        if (bpv == 255u || v.dimX < 0 || v.dimY < 0)
            return 0;
        return static_cast<size_t>(v.dimX) * static_cast<size_t>(v.dimY) * bpv;
    }

    vktError planeSpan(vktHipVolumeView_t const& v, int32_t z0, int32_t g0, int32_t g1, char const* what,
                       uint8_t*& ptr, size_t& bytes)
    {
        size_t const plane = planeBytes(v);
        if (v.data == nullptr || plane == 0 || v.dimZ < 0)
            return rt::fail((std::string(what) + ": invalid slab view").c_str());
        if (g0 < z0 || g1 > z0 + v.dimZ || g1 < g0)
            return rt::fail((std::string(what) + ": the slab buffer does not hold the planes the plan moves").c_str());
        ptr = v.data + static_cast<size_t>(g0 - z0) * plane;
        bytes = static_cast<size_t>(g1 - g0) * plane;
        return vktNoError;
    }

    // Aborts the communicator after a failed round enqueue (its kernels exit; every later call
    // on it fails fast) and returns the failure.  c->em held by the caller (the enqueue), c->m not.
    vktError abortAfterEnqueue(vktHipComm_t c, std::string const& why)
    {
        std::string msg;
        {
            std::lock_guard<std::mutex> g(c->m);
            if (c->failure.empty())
                c->failure = why + " (communicator aborted)";
            c->aborted.store(true);
            msg = c->failure;
        }
        if (ncclComm_t const dead = c->comm.exchange(nullptr))
            (void)rccl().abort(dead);
        return rt::fail(msg.c_str());
    }

    // A round enqueue that does not let go of c->em within this long is taken to be stuck in
    // RCCL (a blocking ncclGroupEnd waiting for a dead peer): the watcher aborts without it.
    constexpr int64_t kEnqueueGraceMs = 2000;

    // The two events of a round with a deadline; destroyed on every early return of the enqueue
    // (the watcher destroys them once the round is handed over: release()).
    struct RoundEvents
    {
        hipEvent_t start = nullptr, end = nullptr;
        ~RoundEvents()
        {
            if (start != nullptr)
                (void)hipEventDestroy(start);
            if (end != nullptr)
                (void)hipEventDestroy(end);
        }
        void release() { start = end = nullptr; }
    };

    // A kernel that keeps one wave busy for `ms` milliseconds of wall clock (knob
    // comm.test_stall_ms: a round that outlives its deadline, for the watcher's test); every
    // wave leaves once the time is up.
    __global__ void stallKernel(uint64_t ticks)
    {
        uint64_t const t0 = wall_clock64();
        while (wall_clock64() - t0 < ticks)
            __builtin_amdgcn_s_sleep(64);
    }

    vktError stall(hipStream_t stream, int64_t ms)
    {
        int khz = 0;
        VKT_HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, rt::device()));
        hipLaunchKernelGGL(stallKernel, dim3(1), dim3(64), 0, stream, static_cast<uint64_t>(ms) * static_cast<uint64_t>(khz));
        return rt::check(hipGetLastError(), "stallKernel");
    }

    // Polls an event until it completes; false (and *err set) on an error of the event, an
    // asynchronous RCCL error or, with a deadline (ms > 0, counted from the call), a timeout.
    bool pollEvent(vktHipComm_t c, hipEvent_t ev, int64_t ms, std::string& err)
    {
        auto const t0 = std::chrono::steady_clock::now();
        for (uint32_t polls = 0;; ++polls)
        {
            hipError_t const q = hipEventQuery(ev);
            if (q == hipSuccess)
                return true;
            if (q != hipErrorNotReady)
            {
                err = std::string("hipEventQuery: ") + hipGetErrorString(q);
                return false;
            }
            // (no lock: the comm pointer is atomic, and an enqueue may be blocked inside RCCL)
            ncclComm_t const nc = c->comm.load();
            ncclResult_t as = ncclSuccess;
            if (nc != nullptr && rccl().getAsyncError != nullptr && rccl().getAsyncError(nc, &as) == ncclSuccess &&
                as != ncclSuccess && as != ncclInProgress)
            {
                err = std::string("RCCL asynchronous error: ") + rccl().errorString(as);
                return false;
            }
            if (ms > 0 && std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0)
                                  .count() >= ms)
            {
                err = "a peer did not complete its side of the round within " + std::to_string(ms) + " ms";
                return false;
            }
            // spin briefly (a halo round on xGMI takes tens of microseconds), then back off
            if (polls > 256)
                std::this_thread::sleep_for(std::chrono::microseconds(polls > 4096 ? 1000 : 50));
        }
    }

    // The watcher thread of a communicator: judges its rounds in order (comm/Comm.hpp).
    void watch(vktHipComm_t c)
    {
        (void)hipSetDevice(c->device);
        for (;;)
        {
            vktHipComm_impl::Round r;
            {
                std::unique_lock<std::mutex> g(c->m);
                c->cv.wait(g, [&] { return c->stop || !c->rounds.empty(); });
                if (c->rounds.empty())
                    return;
                r = c->rounds.front();
            }
            std::string err;
            // the round starts when the work queued ahead of it has finished: that wait has no
            // deadline of the round's (it is not the round's time) ...
            bool ok = pollEvent(c, r.start, 0, err);
            // ... its transfers have one, counted from their start
            ok = ok && pollEvent(c, r.end, r.timeoutMs, err);
            {
                // the failure is known now: record it, refuse later rounds and release the
                // waiters (vktHipCommSynchronize) before the abort, which returns only once the
                // communicator's queued work has left the GPU (its kernels exit on the abort flag)
                std::lock_guard<std::mutex> g(c->m);
                if (!ok)
                {
                    if (c->failure.empty())
                        c->failure = r.what + ": " + err + " (communicator aborted)";
                    c->aborted.store(true);
                    VKT_LOG(rt::LogLevel::Error) << c->failure;
                }
                c->rounds.pop_front();
            }
            c->cv.notify_all();
            if (!ok)
            {
                // An enqueue in flight finishes its RCCL calls on the comm before it goes (no
                // use after the abort frees it) -- unless it is stuck in RCCL, when only the
                // abort releases it.
                bool const quiet = c->em.try_lock_for(std::chrono::milliseconds(kEnqueueGraceMs));
                if (ncclComm_t const dead = c->comm.exchange(nullptr))
                    (void)rccl().abort(dead);
                if (quiet)
                    c->em.unlock();
            }
            (void)hipEventDestroy(r.start);
            (void)hipEventDestroy(r.end);
        }
    }

    vktError rcclRound(vktHipComm_t c, std::vector<Xfer> const& xs, hipStream_t stream, char const* what)
    {
        if (xs.empty())
            return vktNoError;
        if (!rccl().ok)
            return noRccl(what);
        std::lock_guard<std::timed_mutex> enqueue(c->em);
        auto refused = [&]() {
            std::lock_guard<std::mutex> g(c->m);
            return rt::fail((std::string(what) + ": the communicator was aborted after an earlier failure: " + c->failure)
                                .c_str());
        };
        int64_t deadline = 0;
        {
            std::lock_guard<std::mutex> g(c->m);
            deadline = c->timeoutMs;
        }
        ncclComm_t const nc = c->comm.load();
        if (c->aborted.load() || nc == nullptr)
            return refused();
        RoundEvents ev;
        if (deadline > 0)
        {
            if (rt::check(hipEventCreateWithFlags(&ev.start, hipEventDisableTiming), "hipEventCreate") != vktNoError ||
                rt::check(hipEventCreateWithFlags(&ev.end, hipEventDisableTiming), "hipEventCreate") != vktNoError ||
                rt::check(hipEventRecord(ev.start, stream), "hipEventRecord(round start)") != vktNoError)
                return vktInvalidValue;
        }
        ncclResult_t res = rccl().groupStart();
        if (res != ncclSuccess)
            return ncclFail((std::string(what) + ": ncclGroupStart").c_str(), res);
        for (Xfer const& x : xs)
        {
            res = x.send ? rccl().send(x.ptr, x.bytes, ncclUint8, x.peer, nc, stream)
                         : rccl().recv(x.ptr, x.bytes, ncclUint8, x.peer, nc, stream);
            if (res != ncclSuccess)
            {
                (void)rccl().groupEnd();
                return ncclFail((std::string(what) + ": ncclSend/ncclRecv").c_str(), res);
            }
        }
        res = rccl().groupEnd();
        if (c->aborted.load())   // the watcher aborted the communicator meanwhile (an earlier round)
            return refused();
        if (res != ncclSuccess)
            return abortAfterEnqueue(c, std::string(what) + ": ncclGroupEnd: " + rccl().errorString(res));
        if (deadline <= 0)
            return vktNoError;
        // (test knob comm.test_stall_ms: the round outlives its deadline after its transfers)
        int64_t const stallMs = rt::knob(rt::Knob::CommTestStallMs);
        if (stallMs > 0)
            (void)stall(stream, stallMs);
        if (rt::check(hipEventRecord(ev.end, stream), "hipEventRecord(round end)") != vktNoError)
            return vktInvalidValue;
        vktHipComm_impl::Round r;
        r.start = ev.start;
        r.end = ev.end;
        r.timeoutMs = deadline;
        r.what = what;
        {
            std::lock_guard<std::mutex> g(c->m);
            c->rounds.push_back(r);
            ev.release();   // the watcher destroys them
            if (!c->watcher.joinable())
                c->watcher = std::thread(watch, c);
        }
        c->cv.notify_all();
        return vktNoError;
    }

    // Entry points that enqueue a round return after finishLaunch; with async execution off
    // that is the compute stream drained, and the rounds are judged too (vktHipCommSynchronize),
    // so a round that timed out or failed asynchronously fails the call that issued it, as the
    // synchronous mode promises -- not a later comm call.
    vktError finishRound(vktHipComm_t c, char const* name)
    {
        vktError const e = rt::finishLaunch(name);
        if (e != vktNoError || rt::asyncExecution())
            return e;
        return vktHipCommSynchronize(c);
    }

    // Planes [a, b) of a view holding global planes [z0, z0 + v.dimZ).
    vktHipVolumeView_t planesOf(vktHipVolumeView_t v, int32_t z0, int32_t a, int32_t b)
    {
        v.data += static_cast<size_t>(a - z0) * planeBytes(v);
        v.dimZ = b - a;
        return v;
    }

    // The halo exchange of one rank overlapped with its interior (slab.py:resample_slab_overlapped):
    // `transport(side)` enqueues the rank's moves on the side stream after the work queued so far
    // on the compute stream; the dst planes that read only owned source planes resample on the
    // compute stream meanwhile (a source sub-view of exactly those planes, so nothing reads the
    // planes in flight); the compute stream then waits for the moves and resamples the rest.
    // Every part is a slab resample of its own (the same exact index tables): the result equals
    // exchange + vktHipResampleSlab.
    template <class Transport>
    vktError overlappedResample(vktHipVolumeView_t dst, vktHipVolumeView_t src, int32_t localZ0, int32_t rank,
                                int32_t world, int32_t dstG, int32_t srcG, vktFilterMode fm, int32_t chain,
                                bool receives, hipStream_t side, Transport&& transport, char const* what)
    {
        int32_t d0, d1, o0, o1;
        slabBounds(dstG, world, rank, d0, d1);
        slabBounds(srcG, world, rank, o0, o1);
        if (dst.dimZ != d1 - d0)
            return rt::fail((std::string(what) + ": dst must hold exactly the rank's dst slab").c_str());
        // dk: [d0, dk) reads only owned planes (binary search, slab.py:interior_split)
        int32_t dk = d1;
        if (receives && d1 > d0)
        {
            int32_t lo = d0, hi = d1;
            while (lo < hi)
            {
                int32_t const mid = lo + (hi - lo + 1) / 2;
                int32_t b = 0, en = 0;
                vktError const err = vktHipResampleSlabSourceRange(dstG, d0, mid, srcG, fm, chain, &b, &en);
                if (err != vktNoError)
                    return err;
                if (b >= o0 && en <= o1)
                    lo = mid;
                else
                    hi = mid - 1;
            }
            dk = lo;
        }
        hipStream_t const cs = rt::computeStream();
        hipEvent_t ready = nullptr, moved = nullptr;
        VKT_HIP_TRY(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
        vktError e = rt::check(hipEventCreateWithFlags(&moved, hipEventDisableTiming), "hipEventCreate");
        if (e == vktNoError)
            e = rt::check(hipEventRecord(ready, cs), "hipEventRecord(compute)");
        if (e == vktNoError)
            e = rt::check(hipStreamWaitEvent(side, ready, 0), "hipStreamWaitEvent(side)");
        if (e == vktNoError)
            e = transport(side);
        if (e == vktNoError)
            e = rt::check(hipEventRecord(moved, side), "hipEventRecord(side)");
        for (int part = 0; part < 2 && e == vktNoError; ++part)
        {
            int32_t const a = part == 0 ? d0 : dk, b = part == 0 ? dk : d1;
            if (part == 1)
                e = rt::check(hipStreamWaitEvent(cs, moved, 0), "hipStreamWaitEvent(compute)");
            if (e != vktNoError || b <= a)
                continue;
            int32_t s0 = 0, s1 = 0;
            e = vktHipResampleSlabSourceRange(dstG, a, b, srcG, fm, chain, &s0, &s1);
            if (e == vktNoError && (s0 < localZ0 || s1 > localZ0 + src.dimZ))
                e = rt::fail((std::string(what) + ": the source slab does not hold the planes the dst slab reads").c_str());
            if (e == vktNoError)
                e = vktHipResampleSlab(planesOf(dst, d0, a, b), planesOf(src, localZ0, s0, s1), fm, dstG, a, srcG, s0);
        }
        (void)hipEventDestroy(ready);
        (void)hipEventDestroy(moved);
        return e;
    }

    vktError localMove(uint8_t* dst, uint8_t const* src, size_t bytes, hipStream_t stream, char const* what)
    {
        if (bytes == 0 || dst == src)
            return vktNoError;
        return rt::check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, stream), what);
    }
} // namespace comm
} // namespace vkt

using namespace vkt;

extern "C" {

vktError vktHipSlabResamplePlan(int32_t dstGlobalDimZ, int32_t srcGlobalDimZ, int32_t nranks, int32_t rank,
                                vktFilterMode fm, int32_t needsNeighbours, int32_t* localZ0, int32_t* localZ1,
                                vktHipSlabTransfer_t* transfers, int32_t capacity, int32_t* count)
{
    if (localZ0 == nullptr || localZ1 == nullptr || count == nullptr)
        return rt::fail("vktHipSlabResamplePlan: null pointer");
    std::vector<vktHipSlabTransfer_t> xs;
    vktError const e = plan(dstGlobalDimZ, srcGlobalDimZ, nranks, rank, fm, needsNeighbours, *localZ0, *localZ1, xs);
    if (e != vktNoError)
        return e;
    *count = static_cast<int32_t>(xs.size());
    if (transfers != nullptr)
    {
        if (capacity < *count)
            return rt::fail("vktHipSlabResamplePlan: transfer array too small");
        std::copy(xs.begin(), xs.end(), transfers);
    }
    return vktNoError;
}

vktError vktHipCommGetUniqueId(vktHipCommId_t* id)
{
    if (id == nullptr)
        return rt::fail("vktHipCommGetUniqueId: null pointer");
    ncclUniqueId u;
    if (!rccl().ok)
        return noRccl("vktHipCommGetUniqueId");
    ncclResult_t const r = rccl().getUniqueId(&u);
    if (r != ncclSuccess)
        return ncclFail("vktHipCommGetUniqueId", r);
    std::memcpy(id->internal, u.internal, sizeof(u.internal));
    return vktNoError;
}

vktError vktHipCommInitRank(vktHipComm_t* comm, int32_t nranks, vktHipCommId_t id, int32_t rank)
{
    if (comm == nullptr)
        return rt::fail("vktHipCommInitRank: null pointer");
    *comm = nullptr;
    if (nranks <= 0 || rank < 0 || rank >= nranks)
        return rt::fail("vktHipCommInitRank: invalid rank / nranks");
    if (!rccl().ok)
        return noRccl("vktHipCommInitRank");
    VKT_HIP_TRY(hipSetDevice(rt::device()));   // the communicator lives on the library's device
    ncclUniqueId u;
    std::memcpy(u.internal, id.internal, sizeof(u.internal));
    ncclComm_t nc = nullptr;
    ncclResult_t const r = rccl().commInitRank(&nc, nranks, u, rank);
    if (r != ncclSuccess)
        return ncclFail("vktHipCommInitRank", r);
    auto* c = new vktHipComm_impl;
    c->comm.store(nc);
    c->rank = rank;
    c->nranks = nranks;
    c->device = rt::device();
    // default round deadline: VKT_COMM_TIMEOUT_MS (0 = no deadline), else 300 s
    char const* env = std::getenv("VKT_COMM_TIMEOUT_MS");
    c->timeoutMs = env != nullptr ? std::max<int64_t>(0, std::strtoll(env, nullptr, 10)) : 300000;
    *comm = c;
    return vktNoError;
}

vktError vktHipCommSetTimeout(vktHipComm_t comm, int64_t milliseconds)
{
    if (comm == nullptr || milliseconds < 0)
        return rt::fail("vktHipCommSetTimeout: null communicator or negative timeout");
    std::lock_guard<std::mutex> g(comm->m);
    comm->timeoutMs = milliseconds;
    return vktNoError;
}

vktError vktHipCommSynchronize(vktHipComm_t comm)
{
    if (comm == nullptr)
        return rt::fail("vktHipCommSynchronize: null communicator");
    std::unique_lock<std::mutex> g(comm->m);
    comm->cv.wait(g, [&] { return comm->rounds.empty(); });
    if (comm->aborted.load())
        return rt::fail(comm->failure.c_str());
    return vktNoError;
}

vktError vktHipCommDestroy(vktHipComm_t comm)
{
    if (comm == nullptr)
        return vktNoError;
    {
        std::lock_guard<std::mutex> g(comm->m);
        comm->stop = true;   // the watcher judges the rounds still queued, then leaves
    }
    comm->cv.notify_all();
    if (comm->watcher.joinable())
        comm->watcher.join();
    ncclComm_t const nc = comm->comm.exchange(nullptr);
    ncclResult_t const r = comm->aborted.load() || nc == nullptr ? ncclSuccess : rccl().commDestroy(nc);
    if (comm->stream != nullptr)
        (void)hipStreamDestroy(comm->stream);
    delete comm;
    return r == ncclSuccess ? vktNoError : ncclFail("vktHipCommDestroy", r);
}

vktError vktHipSlabExchangeHalo(vktHipComm_t comm, vktHipVolumeView_t localSrc, int32_t localZ0,
                                int32_t dstGlobalDimZ, int32_t srcGlobalDimZ, vktFilterMode fm,
                                int32_t needsNeighbours)
{
    if (comm == nullptr)
        return rt::fail("vktHipSlabExchangeHalo: null communicator");
    int32_t lo, hi;
    std::vector<vktHipSlabTransfer_t> xs;
    vktError e = plan(dstGlobalDimZ, srcGlobalDimZ, comm->nranks, comm->rank, fm, needsNeighbours, lo, hi, xs);
    if (e != vktNoError || xs.empty())
        return e;
    // every plane moved must lie in the local buffer (global planes [localZ0, localZ0 + dimZ))
    std::vector<comm::Xfer> moves;
    for (vktHipSlabTransfer_t const& x : xs)
    {
        comm::Xfer m{x.peer, x.send, nullptr, 0};
        e = comm::planeSpan(localSrc, localZ0, x.z0, x.z1, "vktHipSlabExchangeHalo", m.ptr, m.bytes);
        if (e != vktNoError)
            return e;
        moves.push_back(m);
    }
    e = comm::rcclRound(comm, moves, rt::computeStream(), "vktHipSlabExchangeHalo");
    return e != vktNoError ? e : comm::finishRound(comm, "SlabExchangeHalo_hip");
}

vktError vktHipSlabExchangeHaloLocal(int32_t numSlabs, vktHipVolumeView_t const* localSrc, int32_t const* localZ0,
                                     int32_t dstGlobalDimZ, int32_t srcGlobalDimZ, vktFilterMode fm,
                                     int32_t needsNeighbours)
{
    if (numSlabs <= 0 || localSrc == nullptr || localZ0 == nullptr)
        return rt::fail("vktHipSlabExchangeHaloLocal: invalid slab arrays");
    // the same plan as the RCCL exchange, every rank's receives executed as device copies from
    // the owning slab's buffer (the sends are the other side of the same moves)
    hipStream_t const s = rt::computeStream();
    for (int32_t r = 0; r < numSlabs; ++r)
    {
        int32_t lo, hi;
        std::vector<vktHipSlabTransfer_t> xs;
        vktError e = plan(dstGlobalDimZ, srcGlobalDimZ, numSlabs, r, fm, needsNeighbours, lo, hi, xs);
        if (e != vktNoError)
            return e;
        for (vktHipSlabTransfer_t const& x : xs)
        {
            if (x.send)
                continue;
            uint8_t *to, *from;
            size_t n, m;
            e = comm::planeSpan(localSrc[r], localZ0[r], x.z0, x.z1, "vktHipSlabExchangeHaloLocal", to, n);
            if (e == vktNoError)
                e = comm::planeSpan(localSrc[x.peer], localZ0[x.peer], x.z0, x.z1, "vktHipSlabExchangeHaloLocal",
                                    from, m);
            if (e == vktNoError && n != m)
                e = rt::fail("vktHipSlabExchangeHaloLocal: slabs of different plane sizes");
            if (e == vktNoError)
                e = comm::localMove(to, from, n, s, "vktHipSlabExchangeHaloLocal: hipMemcpyAsync");
            if (e != vktNoError)
                return e;
        }
    }
    return rt::finishLaunch("SlabExchangeHaloLocal_hip");
}

vktError vktHipSlabExchangeHaloPeer(int32_t numSlabs, vktHipVolumeView_t const* localSrc, int32_t const* localZ0,
                                    int32_t const* devices, int32_t dstGlobalDimZ, int32_t srcGlobalDimZ,
                                    vktFilterMode fm, int32_t needsNeighbours)
{
    if (numSlabs <= 0 || localSrc == nullptr || localZ0 == nullptr || devices == nullptr)
        return rt::fail("vktHipSlabExchangeHaloPeer: invalid slab arrays");
    int32_t nDev = 0;
    VKT_HIP_TRY(hipGetDeviceCount(&nDev));
    for (int32_t r = 0; r < numSlabs; ++r)
        if (devices[r] < 0 || devices[r] >= nDev)
            return rt::fail("vktHipSlabExchangeHaloPeer: device id out of range");
    // every receive of the plan as a peer copy into the receiving slab's device, on a stream of
    // that device (the library's compute stream for its own device); each device's copies are
    // ordered after the work already queued on the library's compute stream (for the library's
    // device) and the call returns once every plane has landed
    int const libDev = rt::device();
    int cur = 0;
    VKT_HIP_TRY(hipGetDevice(&cur));
    std::vector<hipStream_t> streams(static_cast<size_t>(nDev), nullptr);
    std::vector<char> owned(static_cast<size_t>(nDev), 0);
    // the copies into other devices run on streams of their own: each first waits for the work
    // already queued on the library's compute stream (a kernel that is still writing a source
    // slab of the library's device)
    hipEvent_t queued = nullptr;
    VKT_HIP_TRY(hipEventCreateWithFlags(&queued, hipEventDisableTiming));
    vktError e = rt::check(hipEventRecord(queued, rt::computeStream()), "hipEventRecord(compute)");
    auto streamOf = [&](int dev) -> hipStream_t {
        if (dev == libDev)
            return rt::computeStream();
        if (!streams[static_cast<size_t>(dev)])
        {
            // cached only once it waits for the compute stream: a stream that could not be
            // ordered after the kernels writing the source slabs is destroyed, never reused
            hipStream_t st = nullptr;
            if (rt::check(hipSetDevice(dev), "hipSetDevice") == vktNoError &&
                rt::check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate") == vktNoError)
            {
                if (rt::check(hipStreamWaitEvent(st, queued, 0), "hipStreamWaitEvent(peer copy)") == vktNoError)
                {
                    streams[static_cast<size_t>(dev)] = st;
                    owned[static_cast<size_t>(dev)] = 1;
                }
                else
                {
                    (void)hipStreamDestroy(st);
                    st = nullptr;
                }
            }
            (void)hipSetDevice(cur);
            return st;
        }
        return streams[static_cast<size_t>(dev)];
    };
    for (int32_t r = 0; r < numSlabs && e == vktNoError; ++r)
    {
        int32_t lo, hi;
        std::vector<vktHipSlabTransfer_t> xs;
        e = plan(dstGlobalDimZ, srcGlobalDimZ, numSlabs, r, fm, needsNeighbours, lo, hi, xs);
        for (size_t k = 0; k < xs.size() && e == vktNoError; ++k)
        {
            vktHipSlabTransfer_t const& x = xs[k];
            if (x.send)
                continue;
            uint8_t *to, *from;
            size_t n, m;
            e = comm::planeSpan(localSrc[r], localZ0[r], x.z0, x.z1, "vktHipSlabExchangeHaloPeer", to, n);
            if (e == vktNoError)
                e = comm::planeSpan(localSrc[x.peer], localZ0[x.peer], x.z0, x.z1, "vktHipSlabExchangeHaloPeer", from, m);
            if (e == vktNoError && n != m)
                e = rt::fail("vktHipSlabExchangeHaloPeer: slabs of different plane sizes");
            if (e != vktNoError)
                break;
            int const dd = devices[r], sd = devices[x.peer];
            hipStream_t const st = streamOf(dd);
            if (!st)
            {
                e = rt::fail("vktHipSlabExchangeHaloPeer: no stream on the receiving device");
                break;
            }
            if (dd != sd)
            {
                int can = 0;
                if (hipDeviceCanAccessPeer(&can, dd, sd) == hipSuccess && can)
                {
                    (void)hipSetDevice(dd);
                    hipError_t const pe = hipDeviceEnablePeerAccess(sd, 0);
                    if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled)
                        (void)hipGetLastError();
                    else if (pe == hipErrorPeerAccessAlreadyEnabled)
                        (void)hipGetLastError();
                    (void)hipSetDevice(cur);
                }
            }
            e = rt::check(hipMemcpyPeerAsync(to, dd, from, sd, n, st), "vktHipSlabExchangeHaloPeer: hipMemcpyPeerAsync");
        }
    }
    // every plane landed before the call returns (the slabs' owners may read them on any stream)
    for (int d = 0; d < nDev; ++d)
        if (streams[static_cast<size_t>(d)])
        {
            if (e == vktNoError)
                e = rt::check(hipStreamSynchronize(streams[static_cast<size_t>(d)]), "hipStreamSynchronize");
            if (owned[static_cast<size_t>(d)])
            {
                (void)hipSetDevice(d);
                (void)hipStreamDestroy(streams[static_cast<size_t>(d)]);
            }
        }
    (void)hipSetDevice(cur);
    if (e == vktNoError)
        e = rt::check(hipStreamSynchronize(rt::computeStream()), "hipStreamSynchronize");
    (void)hipEventDestroy(queued);
    return e != vktNoError ? e : rt::finishLaunch("SlabExchangeHaloPeer_hip");
}

vktError vktHipCommExchange(vktHipComm_t comm, int32_t peer, void const* sendBuf, void* recvBuf, size_t bytes)
{
    if (comm == nullptr || peer < 0 || peer >= comm->nranks || (bytes > 0 && (sendBuf == nullptr || recvBuf == nullptr)))
        return rt::fail("vktHipCommExchange: null communicator / buffer or peer out of range");
    std::vector<comm::Xfer> xs;
    if (bytes > 0)
    {
        xs.push_back(comm::Xfer{peer, 1, static_cast<uint8_t*>(const_cast<void*>(sendBuf)), bytes});
        xs.push_back(comm::Xfer{peer, 0, static_cast<uint8_t*>(recvBuf), bytes});
    }
    vktError const e = comm::rcclRound(comm, xs, rt::computeStream(), "vktHipCommExchange");
    return e != vktNoError ? e : comm::finishRound(comm, "CommExchange_hip");
}

vktError vktHipResampleSlabOverlapped(vktHipComm_t comm, vktHipVolumeView_t dst, vktHipVolumeView_t localSrc,
                                      int32_t localZ0, int32_t dstGlobalDimZ, int32_t srcGlobalDimZ, vktFilterMode fm,
                                      int32_t needsNeighbours)
{
    char const* const what = "vktHipResampleSlabOverlapped";
    if (comm == nullptr)
        return rt::fail("vktHipResampleSlabOverlapped: null communicator");
    int32_t lo, hi;
    std::vector<vktHipSlabTransfer_t> xs;
    vktError e = plan(dstGlobalDimZ, srcGlobalDimZ, comm->nranks, comm->rank, fm, needsNeighbours, lo, hi, xs);
    if (e != vktNoError)
        return e;
    std::vector<comm::Xfer> moves;
    bool receives = false;
    for (vktHipSlabTransfer_t const& x : xs)
    {
        comm::Xfer m{x.peer, x.send, nullptr, 0};
        e = comm::planeSpan(localSrc, localZ0, x.z0, x.z1, what, m.ptr, m.bytes);
        if (e != vktNoError)
            return e;
        receives = receives || !x.send;
        moves.push_back(m);
    }
    {
        std::lock_guard<std::mutex> g(comm->m);
        if (comm->stream == nullptr &&
            rt::check(hipStreamCreateWithFlags(&comm->stream, hipStreamNonBlocking), "hipStreamCreate(comm)") != vktNoError)
            return vktInvalidValue;
    }
    e = comm::overlappedResample(dst, localSrc, localZ0, comm->rank, comm->nranks, dstGlobalDimZ, srcGlobalDimZ, fm,
                                 needsNeighbours, receives, comm->stream,
                                 [&](hipStream_t side) { return comm::rcclRound(comm, moves, side, what); }, what);
    return e != vktNoError ? e : comm::finishRound(comm, "ResampleSlabOverlapped_hip");
}

vktError vktHipResampleSlabsOverlappedLocal(int32_t numSlabs, vktHipVolumeView_t const* dst,
                                            vktHipVolumeView_t const* localSrc, int32_t const* localZ0,
                                            int32_t dstGlobalDimZ, int32_t srcGlobalDimZ, vktFilterMode fm,
                                            int32_t needsNeighbours)
{
    char const* const what = "vktHipResampleSlabsOverlappedLocal";
    if (numSlabs <= 0 || dst == nullptr || localSrc == nullptr || localZ0 == nullptr)
        return rt::fail("vktHipResampleSlabsOverlappedLocal: invalid slab arrays");
    for (int32_t r = 0; r < numSlabs; ++r)
    {
        int32_t lo, hi;
        std::vector<vktHipSlabTransfer_t> xs;
        vktError e = plan(dstGlobalDimZ, srcGlobalDimZ, numSlabs, r, fm, needsNeighbours, lo, hi, xs);
        if (e != vktNoError)
            return e;
        // the receives of slab r: device copies from the owning slabs' buffers (the sends are
        // the other side of the same moves)
        std::vector<std::pair<uint8_t*, uint8_t const*>> to;
        std::vector<size_t> bytes;
        for (vktHipSlabTransfer_t const& x : xs)
        {
            if (x.send)
                continue;
            uint8_t *t, *f;
            size_t n, m;
            e = comm::planeSpan(localSrc[r], localZ0[r], x.z0, x.z1, what, t, n);
            if (e == vktNoError)
                e = comm::planeSpan(localSrc[x.peer], localZ0[x.peer], x.z0, x.z1, what, f, m);
            if (e == vktNoError && n != m)
                e = rt::fail("vktHipResampleSlabsOverlappedLocal: slabs of different plane sizes");
            if (e != vktNoError)
                return e;
            to.emplace_back(t, f);
            bytes.push_back(n);
        }
        auto copies = [&](hipStream_t side) {
            for (size_t k = 0; k < to.size(); ++k)
                if (vktError const ce = comm::localMove(to[k].first, to[k].second, bytes[k], side, what); ce != vktNoError)
                    return ce;
            return vktNoError;
        };
        e = comm::overlappedResample(dst[r], localSrc[r], localZ0[r], r, numSlabs, dstGlobalDimZ, srcGlobalDimZ, fm,
                                     needsNeighbours, !to.empty(), rt::copyStream(), copies, what);
        if (e != vktNoError)
            return e;
    }
    return rt::finishLaunch("ResampleSlabsOverlappedLocal_hip");
}

} // extern "C"
