// Memory.cpp -- allocation, copies and deferred migration on HIP.
//
// Reference: Allocate/Free/Memcpy/MemsetRange dispatch on the thread policy
// (src/vkt/Memory.cpp:30-80) to malloc/free/memcpy or cudaMalloc/cudaFree/synchronous
// cudaMemcpy (src/vkt/Memory_cuda.hpp:16-24), and ManagedBuffer::migrate
// (include/cpp/vkt/ManagedBuffer.hpp:168-198) allocates on the new device, copies, and frees
// under the old policy.
//
// MI355X design: host<->device traffic goes through a side copy stream.  The copy stream
// first waits (event) for everything already queued on the compute stream, so a D2H
// migration after GPU kernels sees their results; an H2D copy is followed by an event the
// compute stream waits on.  Host-facing copies return only when the bytes have landed (the
// reference's cudaMemcpy contract: the caller may free or read host memory right after).
// Device-to-device copies stay on the compute stream, ordered with the kernels.

#include "Runtime.hpp"
#include "volkit_hip.h"

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <map>
#include <mutex>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace vkt
{
namespace hipk
{
    // Pattern fill kernel launcher (kernels/Memset.hip).
    vktError memsetRange(void* dst, void const* pattern, std::size_t dstSize, std::size_t patternSize);
}

namespace
{
    bool onGpu(ExecutionPolicy const& p) { return p.device == ExecutionPolicy::Device::GPU; }

    // Optional pinned (page-locked) host allocations for CPU-policy buffers: migrations then
    // DMA straight from/to the user's buffer instead of through HIP's pageable staging.
    std::atomic<int> gPinnedHost{0};
    std::mutex gPinnedMutex;
    std::unordered_set<void*>& pinnedSet()
    {
        static auto* s = new std::unordered_set<void*>;
        return *s;
    }

    // Small device allocations (<= kPoolMax bytes: bricks, lookup tables, small volumes) come from
    // 64-MiB hipMalloc chunks in 256-B size classes instead of one hipMalloc each: a
    // BrickDecomposeResize of a 1024^3 volume into 16^3 bricks makes 262 144 allocations.  Freed
    // blocks wait on a pending list; the first allocation that would reuse one synchronises the
    // device once for the whole batch (the guarantee hipFree gave: no kernel or copy still uses
    // the block), then serves them.  Chunks are kept for the process (like a caching allocator);
    // knob memory.pool = 0 allocates every buffer with hipMalloc.
    constexpr std::size_t kPoolMax = 4u << 20;
    constexpr std::size_t kPoolChunk = 64u << 20;
    constexpr std::size_t kPoolAlign = 256;

    struct DevicePool
    {
        std::unordered_map<std::size_t, std::vector<void*>> freeBlocks;   // by class
        std::unordered_map<std::size_t, std::vector<void*>> pending;      // by class: freed, not yet synchronised
        char* bump = nullptr;
        std::size_t left = 0;
    };

    struct Pools
    {
        std::mutex m;
        std::unordered_map<int, DevicePool> byDevice;
        std::unordered_map<void*, std::pair<int, std::size_t>> owner;   // block -> (device, class)
    };

    Pools& pools()
    {
        static auto* p = new Pools;   // (never destroyed: frees may run during static destruction)
        return *p;
    }

    void* poolAllocate(std::size_t bytes)
    {
        std::size_t const cls = (bytes + kPoolAlign - 1) / kPoolAlign * kPoolAlign;
        int const dev = rt::device();
        Pools& P = pools();
        std::lock_guard<std::mutex> lock(P.m);
        DevicePool& d = P.byDevice[dev];
        auto reuse = [&]() -> void* {
            auto it = d.freeBlocks.find(cls);
            if (it == d.freeBlocks.end() || it->second.empty())
                return nullptr;
            void* b = it->second.back();
            it->second.pop_back();
            return b;
        };
        void* b = reuse();
        auto mine = d.pending.find(cls);
        if (!b && mine != d.pending.end() && !mine->second.empty() &&
            rt::check(hipDeviceSynchronize(), "hipDeviceSynchronize(pool)") == vktNoError)
        {
            for (auto& q : d.pending)   // every class: the one synchronisation covers them all
            {
                auto& f = d.freeBlocks[q.first];
                f.insert(f.end(), q.second.begin(), q.second.end());
                q.second.clear();
            }
            b = reuse();
        }
        if (!b)
        {
            if (d.left < cls)
            {
                void* c = nullptr;
                if (rt::check(hipMalloc(&c, kPoolChunk), "hipMalloc(pool chunk)") != vktNoError)
                    return nullptr;
                d.bump = static_cast<char*>(c);
                d.left = kPoolChunk;
            }
            b = d.bump;
            d.bump += cls;
            d.left -= cls;
        }
        P.owner[b] = {dev, cls};
        return b;
    }

    // true when p is a pool block (then it is queued for reuse)
    bool poolFree(void* p)
    {
        Pools& P = pools();
        std::lock_guard<std::mutex> lock(P.m);
        auto it = P.owner.find(p);
        if (it == P.owner.end())
            return false;
        P.byDevice[it->second.first].pending[it->second.second].push_back(p);
        P.owner.erase(it);
        return true;
    }

    // Large device buffers (> kPoolMax) are carved first-fit from arena chunks of at least
    // kArenaChunk bytes, 2-MiB aligned, instead of one hipMalloc each: a 1024^3 UInt16 SumRange
    // over three separately allocated volumes ran in one of two placement states (0.98-1.00 ms or
    // 1.04-1.07 ms, ~40 % of allocations), over three volumes carved from one block at 0.99-1.01 ms
    // every time (tools/alloc_probe.py).  Freed blocks wait on a pending list; an
    // allocation that finds no room synchronises the device once, returns them (coalescing) and
    // releases chunks left empty (hipFree), then retries; a chunk that cannot be allocated falls
    // back to a plain hipMalloc of the request.  Knob memory.arena = 0: one hipMalloc per buffer.
    constexpr std::size_t kArenaChunk = std::size_t(16) << 30;
    constexpr std::size_t kArenaAlign = std::size_t(2) << 20;

    struct ArenaChunk
    {
        char* base = nullptr;
        std::size_t size = 0, used = 0;
        std::map<std::size_t, std::size_t> holes;   // offset -> length, coalesced
    };

    struct ArenaBlock
    {
        ArenaChunk* chunk;
        std::size_t off, len;
    };

    struct Arenas
    {
        std::mutex m;
        std::unordered_map<int, std::vector<ArenaChunk*>> chunks;
        std::unordered_map<int, std::vector<ArenaBlock>> pending;
        std::unordered_map<void*, std::pair<int, ArenaBlock>> owner;
    };

    Arenas& arenas()
    {
        static auto* a = new Arenas;   // (never destroyed: frees may run during static destruction)
        return *a;
    }

    void arenaRelease(ArenaBlock const& b)
    {
        ArenaChunk& c = *b.chunk;
        c.used -= b.len;
        auto next = c.holes.lower_bound(b.off);
        std::size_t off = b.off, len = b.len;
        if (next != c.holes.begin())
        {
            auto prev = std::prev(next);
            if (prev->first + prev->second == off)
            {
                off = prev->first;
                len += prev->second;
                c.holes.erase(prev);
            }
        }
        if (next != c.holes.end() && off + len == next->first)
        {
            len += next->second;
            c.holes.erase(next);
        }
        c.holes[off] = len;
    }

    void* arenaCarve(std::vector<ArenaChunk*>& list, std::size_t len, int dev, Arenas& A)
    {
        for (ArenaChunk* c : list)
            for (auto it = c->holes.begin(); it != c->holes.end(); ++it)
                if (it->second >= len)
                {
                    std::size_t const off = it->first, rest = it->second - len;
                    c->holes.erase(it);
                    if (rest > 0)
                        c->holes[off + len] = rest;
                    c->used += len;
                    void* p = c->base + off;
                    A.owner[p] = {dev, ArenaBlock{c, off, len}};
                    return p;
                }
        return nullptr;
    }

    // nullptr: the caller allocates the buffer with its own hipMalloc
    void* arenaAllocate(std::size_t bytes)
    {
        std::size_t const len = (bytes + kArenaAlign - 1) / kArenaAlign * kArenaAlign;
        int const dev = rt::device();
        Arenas& A = arenas();
        std::lock_guard<std::mutex> lock(A.m);
        std::vector<ArenaChunk*>& list = A.chunks[dev];
        if (void* p = arenaCarve(list, len, dev, A))
            return p;
        std::vector<ArenaBlock>& pend = A.pending[dev];
        if (!pend.empty() && hipDeviceSynchronize() == hipSuccess)
        {
            for (ArenaBlock const& b : pend)
                arenaRelease(b);
            pend.clear();
            for (auto it = list.begin(); it != list.end();)
                if ((*it)->used == 0)
                {
                    (void)hipFree((*it)->base);
                    delete *it;
                    it = list.erase(it);
                }
                else
                    ++it;
            if (void* p = arenaCarve(list, len, dev, A))
                return p;
        }
        std::size_t const size = len > kArenaChunk ? len : kArenaChunk;
        void* base = nullptr;
        if (hipMalloc(&base, size) != hipSuccess)
        {
            (void)hipGetLastError();   // (the request alone may still fit: plain hipMalloc)
            return nullptr;
        }
        auto* c = new ArenaChunk;
        c->base = static_cast<char*>(base);
        c->size = size;
        c->holes[0] = size;
        list.push_back(c);
        return arenaCarve(list, len, dev, A);
    }

    bool arenaFree(void* p)
    {
        Arenas& A = arenas();
        std::lock_guard<std::mutex> lock(A.m);
        auto it = A.owner.find(p);
        if (it == A.owner.end())
            return false;
        A.pending[it->second.first].push_back(it->second.second);
        A.owner.erase(it);
        return true;
    }

} // namespace

namespace detail
{
    vktError memcpyHip(void* dst, void const* src, std::size_t size, CopyKind ck)
    {
        if (size == 0)
            return vktNoError;
        switch (ck)
        {
        case CopyKind::HostToHost:
            std::memcpy(dst, src, size);
            return vktNoError;
        case CopyKind::DeviceToDevice:
            VKT_HIP_TRY(hipMemcpyAsync(dst, src, size, hipMemcpyDeviceToDevice, rt::computeStream()));
            return rt::finishLaunch("Memcpy(DeviceToDevice)");
        case CopyKind::HostToDevice:
        case CopyKind::DeviceToHost:
        {
            hipMemcpyKind kind = ck == CopyKind::HostToDevice ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost;
            vktError e = rt::copyStreamAfterCompute();
            if (e != vktNoError)
                return e;
            VKT_HIP_TRY(hipMemcpyAsync(dst, src, size, kind, rt::copyStream()));
            if (ck == CopyKind::HostToDevice)
            {
                e = rt::computeStreamAfterCopy();
                if (e != vktNoError)
                    return e;
            }
            VKT_HIP_TRY(hipStreamSynchronize(rt::copyStream()));
            return vktNoError;
        }
        }
        return rt::fail("Memcpy: unknown CopyKind");
    }

    void* AllocateOn(std::size_t bytes, ExecutionPolicy const& owner)
    {
        if (bytes == 0)
            return nullptr;
        if (onGpu(owner))
        {
            (void)rt::device();   // bind the context's device before allocating
            if (bytes <= kPoolMax && rt::knob(rt::Knob::MemoryPool) != 0)
                return poolAllocate(bytes);
            if (bytes > kPoolMax && rt::knob(rt::Knob::MemoryArena) != 0)
                if (void* a = arenaAllocate(bytes))
                    return a;
            void* p = nullptr;
            if (rt::check(hipMalloc(&p, bytes), "hipMalloc") != vktNoError)
                return nullptr;
            return p;
        }
        if (gPinnedHost.load())
        {
            void* p = nullptr;
            if (rt::check(hipHostMalloc(&p, bytes, hipHostMallocDefault), "hipHostMalloc") == vktNoError)
            {
                std::lock_guard<std::mutex> lock(gPinnedMutex);
                pinnedSet().insert(p);
                return p;
            }
        }
        void* p = std::malloc(bytes);
        if (p == nullptr)
            rt::fail("Allocate: host malloc failed");
        return p;
    }

    void FreeOn(void* data, ExecutionPolicy const& owner)
    {
        if (data == nullptr)
            return;
        if (onGpu(owner))
        {
            if (!poolFree(data) && !arenaFree(data))
                (void)rt::check(hipFree(data), "hipFree");
            return;
        }
        {
            std::lock_guard<std::mutex> lock(gPinnedMutex);
            auto it = pinnedSet().find(data);
            if (it != pinnedSet().end())
            {
                pinnedSet().erase(it);
                (void)rt::check(hipHostFree(data), "hipHostFree");
                return;
            }
        }
        std::free(data);
    }

    void CopyOn(void* dst, void const* src, std::size_t bytes, ExecutionPolicy const& owner)
    {
        (void)memcpyHip(dst, src, bytes, onGpu(owner) ? CopyKind::DeviceToDevice : CopyKind::HostToHost);
    }

    void* MigrateBuffer(void* data, std::size_t bytes, ExecutionPolicy& last)
    {
        ExecutionPolicy ep = GetThreadExecutionPolicy();
        if (ep.device == last.device)
            return data;
        void* fresh = AllocateOn(bytes, ep);
        if (bytes > 0 && data != nullptr && fresh != nullptr)
            (void)memcpyHip(fresh, data, bytes,
                            onGpu(ep) ? CopyKind::HostToDevice : CopyKind::DeviceToHost);
        FreeOn(data, last);
        last = ep;
        return fresh;
    }
} // detail

void Allocate(void** ptr, std::size_t size)
{
    if (ptr != nullptr)
        *ptr = detail::AllocateOn(size, GetThreadExecutionPolicy());
}

void Free(void* ptr) { detail::FreeOn(ptr, GetThreadExecutionPolicy()); }

void Memcpy(void* dst, void const* src, std::size_t size, CopyKind ck) { (void)detail::memcpyHip(dst, src, size, ck); }

void MemsetRange(void* dst, void const* src, std::size_t dstSize, std::size_t srcSize)
{
    if (onGpu(GetThreadExecutionPolicy()))
    {
        (void)hipk::memsetRange(dst, src, dstSize, srcSize);
        return;
    }
    // Host-resident buffers (CPU policy): a plain pattern copy, as MemsetRange_serial
    // (reference src/vkt/Memory_serial.hpp:24-37).  This is buffer housekeeping of
    // ManagedBuffer::fill, not one of the StructuredVolume algorithms.
    if (srcSize == 0)
        return;
    std::size_t n = dstSize / srcSize;
    for (std::size_t i = 0; i < n; ++i)
        std::memcpy(static_cast<char*>(dst) + i * srcSize, src, srcSize);
}

} // vkt

namespace vkt
{
namespace rt
{
    // Copy stream waits for the compute stream's current tail.
    vktError copyStreamAfterCompute()
    {
        hipEvent_t ev;
        VKT_HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        vktError e = check(hipEventRecord(ev, computeStream()), "hipEventRecord(compute)");
        if (e == vktNoError)
            e = check(hipStreamWaitEvent(copyStream(), ev, 0), "hipStreamWaitEvent(copy)");
        (void)hipEventDestroy(ev);
        return e;
    }

    // Compute stream waits for the copy stream's current tail.
    vktError computeStreamAfterCopy()
    {
        hipEvent_t ev;
        VKT_HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        vktError e = check(hipEventRecord(ev, copyStream()), "hipEventRecord(copy)");
        if (e == vktNoError)
            e = check(hipStreamWaitEvent(computeStream(), ev, 0), "hipStreamWaitEvent(compute)");
        (void)hipEventDestroy(ev);
        return e;
    }
} // rt
} // vkt

extern "C" {

void vktAllocate(void** ptr, size_t size) { vkt::Allocate(ptr, size); }

void vktFree(void* ptr) { vkt::Free(ptr); }

void vktMemcpy(void* dst, void const* src, size_t size, vktCopyKind ck)
{
    vkt::Memcpy(dst, src, size, static_cast<vkt::CopyKind>(ck));
}

vktError vktHipAllocate(void** ptr, size_t size)
{
    if (ptr == nullptr)
        return vkt::rt::fail("vktHipAllocate: null pointer");
    vkt::ExecutionPolicy gpu;
    gpu.device = vkt::ExecutionPolicy::Device::GPU;
    *ptr = vkt::detail::AllocateOn(size, gpu);
    return (*ptr != nullptr || size == 0) ? vktNoError : vktInvalidValue;
}

vktError vktHipFree(void* ptr)
{
    if (ptr == nullptr)
        return vktNoError;
    if (vkt::poolFree(ptr) || vkt::arenaFree(ptr))
        return vktNoError;
    return vkt::rt::check(hipFree(ptr), "hipFree");
}

vktError vktHipMemcpy(void* dst, void const* src, size_t size, vktCopyKind ck)
{
    return vkt::detail::memcpyHip(dst, src, size, static_cast<vkt::CopyKind>(ck));
}

vktError vktHipSetPinnedHostAllocation(int32_t enable)
{
    vkt::gPinnedHost.store(enable != 0);
    return vktNoError;
}

vktError vktHipMemsetRange(void* dst, void const* pattern, size_t dstSize, size_t patternSize)
{
    return vkt::hipk::memsetRange(dst, pattern, dstSize, patternSize);
}

} // extern "C"
