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

#include "HostPool.hpp"
#include "Runtime.hpp"
#include "volkit_hip.h"

#include <sys/mman.h>
#include <unistd.h>
#include <thread>

#include <algorithm>
#include <atomic>
#include <condition_variable>
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

    // ---- host side of a migration (ManagedBuffer::migrate -> MigrateBuffer) ------------------
    // Measured on the MI355X box for a 2 GiB volume (profiles/r04/migrate_breakdown.txt): the
    // PCIe copy itself runs at 55-57 GB/s from pageable (pages written) or pinned memory, but a
    // migrate ran at 9.5-13 GB/s -- the rest was host memory management around it: a D2H copy into
    // a FRESH pageable buffer faults its pages in during the DMA (10 GB/s), freeing the 2 GiB host
    // buffer after an H2D copy (munmap) costs more than the copy, and hipHostMalloc / hipHostFree of
    // 2 GiB pinned take 138 / 78 ms.  So, for large buffers (>= kBigHost):
    //  * a fresh pageable destination is faulted in by the host pool's threads before the copy
    //    (transparent huge pages requested: 2-MiB faults);
    //  * the old pageable buffer is freed on a background thread (the copy has completed: the
    //    migrate's memcpy is synchronous);
    //  * freed pinned buffers are kept for reuse by an allocation of the same size (at most
    //    pinnedCacheCap() in all), returned by vktHipReleaseCachedMemory or when hipHostMalloc fails.
    constexpr std::size_t kBigHost = std::size_t(64) << 20;
    std::size_t physicalBytes()
    {
        long const pages = sysconf(_SC_PHYS_PAGES), page = sysconf(_SC_PAGESIZE);
        return pages > 0 && page > 0 ? static_cast<std::size_t>(pages) * static_cast<std::size_t>(page) : 0;
    }

    // page-locked memory kept for reuse: at most min(16 GiB, physical memory / 16)
    std::size_t pinnedCacheCap()
    {
        static std::size_t const cap = std::min(std::size_t(16) << 30, physicalBytes() / 16);
        return cap;
    }
    std::vector<std::pair<void*, std::size_t>>& pinnedCache()
    {
        static auto* c = new std::vector<std::pair<void*, std::size_t>>;
        return *c;
    }
    std::size_t gPinnedCached = 0;   // under gPinnedMutex
    std::unordered_map<void*, std::size_t>& pinnedSizes()
    {
        static auto* m = new std::unordered_map<void*, std::size_t>;
        return *m;
    }

    std::size_t releasePinnedCache()
    {
        std::vector<std::pair<void*, std::size_t>> drop;
        {
            std::lock_guard<std::mutex> lock(gPinnedMutex);
            drop.swap(pinnedCache());
            gPinnedCached = 0;
        }
        std::size_t n = 0;
        for (auto& e : drop)
        {
            (void)rt::check(hipHostFree(e.first), "hipHostFree");
            n += e.second;
        }
        return n;
    }

    // Large pageable host buffers freed by a migration to the GPU, kept (pages resident) for the
    // next migration back of the same size: a D2H copy into resident pages runs at the PCIe rate
    // (56 GB/s), into fresh ones at 10-15 GB/s even with the pages faulted in beforehand.  At most
    // min(8 GiB, physical memory / 8) in all; returned by vktHipReleaseCachedMemory.
    std::vector<std::pair<void*, std::size_t>>& hostCache()
    {
        static auto* c = new std::vector<std::pair<void*, std::size_t>>;
        return *c;
    }
    std::size_t gHostCached = 0;   // under gPinnedMutex

    std::size_t hostCacheCap()
    {
        static std::size_t const cap = std::min(std::size_t(8) << 30, physicalBytes() / 8);
        return cap;
    }

    void* takeHostCached(std::size_t bytes)
    {
        std::lock_guard<std::mutex> lock(gPinnedMutex);
        auto& c = hostCache();
        for (auto it = c.begin(); it != c.end(); ++it)
            if (it->second == bytes)
            {
                void* const p = it->first;
                gHostCached -= bytes;
                c.erase(it);
                return p;
            }
        return nullptr;
    }

    bool keepHostCached(void* p, std::size_t bytes)
    {
        std::lock_guard<std::mutex> lock(gPinnedMutex);
        if (gHostCached + bytes > hostCacheCap())
            return false;
        hostCache().emplace_back(p, bytes);
        gHostCached += bytes;
        return true;
    }

    std::size_t releaseHostCache()
    {
        std::vector<std::pair<void*, std::size_t>> drop;
        {
            std::lock_guard<std::mutex> lock(gPinnedMutex);
            drop.swap(hostCache());
            gHostCached = 0;
        }
        std::size_t n = 0;
        for (auto& e : drop)
        {
            std::free(e.first);
            n += e.second;
        }
        return n;
    }

    void prefaultHost(void* p, std::size_t bytes)
    {
        uintptr_t const a = reinterpret_cast<uintptr_t>(p);
        uintptr_t const h0 = (a + (std::size_t(2) << 20) - 1) & ~((std::size_t(2) << 20) - 1);
        uintptr_t const h1 = (a + bytes) & ~((std::size_t(2) << 20) - 1);
        if (h1 > h0)
            (void)madvise(reinterpret_cast<void*>(h0), h1 - h0, MADV_HUGEPAGE);
        constexpr std::size_t kPage = 4096;
        std::size_t const pages = (bytes + kPage - 1) / kPage;
        volatile uint8_t* const b = static_cast<volatile uint8_t*>(p);
        rt::parallelFor(pages, 2048, [&](std::size_t i0, std::size_t i1) {
            for (std::size_t i = i0; i < i1; ++i)
                b[std::min(i * kPage, bytes - 1)] = 0;
        });
    }

    // ---- device heap: the library's caching allocator for GPU buffers ----------------------
    // Small buffers (<= kPoolMax bytes: bricks, lookup tables, small volumes) come from 64-MiB
    // pool chunks in 256-B size classes instead of one hipMalloc each: a BrickDecomposeResize of a
    // 1024^3 volume into 16^3 bricks makes 262 144 allocations.  Larger buffers are carved
    // first-fit, 2-MiB aligned, from arena chunks: a 1024^3 UInt16 SumRange over three separately
    // allocated volumes ran in one of two placement states (0.98-1.00 ms or 1.04-1.07 ms, ~40 % of
    // allocations), over three volumes carved from one block at 0.99-1.01 ms every time
    // (tools/alloc_probe.py).  An arena chunk is sized for a group of like buffers
    // (kArenaGroup times the request: the src / dst / operand volumes of one pipeline land in one
    // chunk), at least kArenaMin, growing geometrically (twice the newest chunk while it is
    // allocated, up to kArenaGrowCap) for runs of like-sized smaller buffers, and never more than 1/4 of the device's free
    // memory beyond the request -- a 5 MiB buffer reserves 64 MiB, not a 16-GiB chunk.
    // Freed blocks are not reusable at once (a queued kernel or copy may still use them): they
    // wait on a pending list until a drain records one event on each of the library's streams
    // (compute, copy) and waits for the two -- the guarantee hipFree gave, without stalling
    // torch's or RCCL's streams as a hipDeviceSynchronize did.  A pool allocation drains when a
    // pending block of its class exists; an arena allocation when nothing fits; a free that
    // leaves an arena chunk without live blocks drains and returns the chunk to HIP.  Pool chunks
    // are cached; vktHipReleaseCachedMemory (and any allocation that fails) drains and releases
    // every empty chunk.  Knobs: memory.pool / memory.arena = 0 give those buffers their own
    // hipMalloc; memory.arena_chunk_mib (tests) fixes the arena chunk size.
    constexpr std::size_t kPoolMax = 4u << 20;
    constexpr std::size_t kPoolChunk = 64u << 20;
    constexpr std::size_t kPoolAlign = 256;
    constexpr std::size_t kArenaAlign = std::size_t(2) << 20;
    constexpr std::size_t kArenaMin = std::size_t(64) << 20;
    constexpr std::size_t kArenaGroup = 4;
    constexpr std::size_t kArenaGrowCap = std::size_t(1) << 30;

    struct PoolChunk
    {
        char* base = nullptr;
        std::size_t bump = 0;   // bytes handed out from the start (never given back but by release)
        std::size_t live = 0;   // blocks currently allocated (not freed)
    };

    struct ArenaChunk
    {
        char* base = nullptr;
        std::size_t size = 0, used = 0;             // used: carved bytes (live + pending)
        std::size_t live = 0;                        // live bytes (not freed)
        std::map<std::size_t, std::size_t> holes;   // offset -> length, coalesced
    };

    struct HeapBlock
    {
        int dev;
        bool arena;
        std::size_t len;   // pool: class; arena: carved length
        PoolChunk* pc;
        ArenaChunk* ac;
        std::size_t off;
    };

    struct DeviceHeap
    {
        std::vector<PoolChunk*> poolChunks;
        std::unordered_map<std::size_t, std::vector<std::pair<void*, PoolChunk*>>> poolFree;   // by class
        std::unordered_map<std::size_t, std::size_t> pendingByClass;    // pool classes on the pending list
        std::vector<ArenaChunk*> arenaChunks;
        ArenaChunk* lastChunk = nullptr;   // the newest arena chunk while it exists, and its request
        std::size_t lastReq = 0;
        std::vector<void*> pending;   // freed, not yet known idle
        bool pendingForeign = false;  // a pending block was freed through the public free entry points
        hipEvent_t evCompute = nullptr, evCopy = nullptr;
    };

    struct Heaps
    {
        std::mutex m;
        std::unordered_map<int, DeviceHeap> byDevice;
        std::unordered_map<void*, HeapBlock> owner;   // live and pending blocks
    };

    Heaps& heaps()
    {
        static auto* h = new Heaps;   // (never destroyed: frees may run during static destruction)
        return *h;
    }

    void arenaRelease(ArenaChunk& c, std::size_t off, std::size_t len)
    {
        c.used -= len;
        auto next = c.holes.lower_bound(off);
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

    // Waits until no queued work of the library's streams can use a pending block, then makes
    // them reusable (H.m held).  Blocks of another device than the context's: a device
    // synchronisation of that device (rare).
    void drain(DeviceHeap& d, int dev, Heaps& H)
    {
        if (d.pending.empty())
            return;
        bool idle = false;
        if (dev == rt::device() && !d.pendingForeign)
        {
            if (!d.evCompute && (hipEventCreateWithFlags(&d.evCompute, hipEventDisableTiming) != hipSuccess ||
                                 hipEventCreateWithFlags(&d.evCopy, hipEventDisableTiming) != hipSuccess))
                (void)hipGetLastError();
            idle = d.evCopy && hipEventRecord(d.evCompute, rt::computeStream()) == hipSuccess &&
                   hipEventRecord(d.evCopy, rt::copyStream()) == hipSuccess &&
                   hipEventSynchronize(d.evCompute) == hipSuccess && hipEventSynchronize(d.evCopy) == hipSuccess;
        }
        if (!idle)
        {
            int cur = 0;
            idle = hipGetDevice(&cur) == hipSuccess && hipSetDevice(dev) == hipSuccess &&
                   hipDeviceSynchronize() == hipSuccess;
            (void)hipSetDevice(cur);
        }
        if (!idle)
        {
            (void)hipGetLastError();
            return;   // keep them pending: never hand out a block that may still be in use
        }
        for (void* p : d.pending)
        {
            auto it = H.owner.find(p);
            HeapBlock const b = it->second;
            H.owner.erase(it);
            if (b.arena)
                arenaRelease(*b.ac, b.off, b.len);
            else
                d.poolFree[b.len].push_back({p, b.pc});
        }
        d.pending.clear();
        d.pendingByClass.clear();
        d.pendingForeign = false;
    }

    // Returns arena chunks without carved blocks to HIP; with `pools`, also pool chunks without
    // live blocks (their free blocks leave the class lists).  Bytes released.
    std::size_t releaseEmpty(DeviceHeap& d, bool pools)
    {
        std::size_t freed = 0;
        for (auto it = d.arenaChunks.begin(); it != d.arenaChunks.end();)
            if ((*it)->used == 0)
            {
                (void)hipFree((*it)->base);
                freed += (*it)->size;
                if (*it == d.lastChunk)
                    d.lastChunk = nullptr;   // (a later burst starts small again)
                delete *it;
                it = d.arenaChunks.erase(it);
            }
            else
                ++it;
        if (!pools)
            return freed;
        std::vector<PoolChunk*> keep, gone;
        for (PoolChunk* c : d.poolChunks)
            (c->live == 0 && d.pendingByClass.empty() ? gone : keep).push_back(c);
        if (gone.empty())
            return freed;
        auto inGone = [&](std::pair<void*, PoolChunk*> const& f) {
            return std::find(gone.begin(), gone.end(), f.second) != gone.end();
        };
        for (auto& f : d.poolFree)
            f.second.erase(std::remove_if(f.second.begin(), f.second.end(), inGone), f.second.end());
        for (PoolChunk* c : gone)
        {
            (void)hipFree(c->base);
            freed += kPoolChunk;
            delete c;
        }
        d.poolChunks = keep;
        return freed;
    }

    // hipMalloc; on failure drain + release every empty chunk of the device, then once more
    void* deviceMalloc(std::size_t bytes, DeviceHeap& d, int dev, Heaps& H, bool quiet)
    {
        void* p = nullptr;
        if (hipMalloc(&p, bytes) == hipSuccess)
            return p;
        (void)hipGetLastError();
        drain(d, dev, H);
        releaseEmpty(d, true);
        if (hipMalloc(&p, bytes) == hipSuccess)
            return p;
        if (quiet)
            (void)hipGetLastError();
        else
            (void)rt::check(hipErrorOutOfMemory, "hipMalloc");
        return nullptr;
    }

    void* poolAllocate(std::size_t bytes, DeviceHeap& d, int dev, Heaps& H)
    {
        std::size_t const cls = (bytes + kPoolAlign - 1) / kPoolAlign * kPoolAlign;
        PoolChunk* pc = nullptr;
        auto reuse = [&]() -> void* {
            auto it = d.poolFree.find(cls);
            if (it == d.poolFree.end() || it->second.empty())
                return nullptr;
            auto const f = it->second.back();
            it->second.pop_back();
            pc = f.second;
            return f.first;
        };
        void* b = reuse();
        if (!b && d.pendingByClass.count(cls))
        {
            drain(d, dev, H);   // one wait covers every pending block of every class
            b = reuse();
        }
        if (!b)
        {
            pc = d.poolChunks.empty() ? nullptr : d.poolChunks.back();
            if (!pc || kPoolChunk - pc->bump < cls)
            {
                void* base = deviceMalloc(kPoolChunk, d, dev, H, false);
                if (!base)
                    return nullptr;
                pc = new PoolChunk;
                pc->base = static_cast<char*>(base);
                d.poolChunks.push_back(pc);
            }
            b = pc->base + pc->bump;
            pc->bump += cls;
        }
        pc->live += 1;
        H.owner[b] = HeapBlock{dev, false, cls, pc, nullptr, 0};
        return b;
    }

    void* arenaCarve(DeviceHeap& d, std::size_t len, int dev, Heaps& H)
    {
        for (ArenaChunk* c : d.arenaChunks)
            for (auto it = c->holes.begin(); it != c->holes.end(); ++it)
                if (it->second >= len)
                {
                    std::size_t const off = it->first, rest = it->second - len;
                    c->holes.erase(it);
                    if (rest > 0)
                        c->holes[off + len] = rest;
                    c->used += len;
                    c->live += len;
                    void* p = c->base + off;
                    H.owner[p] = HeapBlock{dev, true, len, nullptr, c, off};
                    return p;
                }
        return nullptr;
    }

    // size of a new arena chunk for a request of len bytes (see above)
    std::size_t arenaChunkSize(DeviceHeap const& d, std::size_t len)
    {
        int64_t const fixed = rt::knob(rt::Knob::MemoryArenaChunkMiB);
        if (fixed > 0)
            return std::max(len, static_cast<std::size_t>(fixed) << 20);
        std::size_t want = std::max(kArenaMin, kArenaGroup * len);
        // a run of like buffers that outgrew the newest chunk (still allocated): twice its size
        if (d.lastChunk && d.lastReq <= 2 * len && 2 * d.lastReq >= len)
            want = std::max(want, std::min(2 * d.lastChunk->size, kArenaGrowCap));
        std::size_t freeB = 0, totalB = 0;
        // the group's extra room is a cache other allocators in the process (torch, RCCL) cannot
        // reclaim: at most a quarter of the device's free memory beyond the request
        if (want > len && hipMemGetInfo(&freeB, &totalB) == hipSuccess && freeB > len)
            want = std::min(want, len + (freeB - len) / 4);
        else
            (void)hipGetLastError();
        return (std::max(want, len) + kArenaAlign - 1) / kArenaAlign * kArenaAlign;
    }

    // nullptr: the caller allocates the buffer with its own hipMalloc
    void* arenaAllocate(std::size_t bytes, DeviceHeap& d, int dev, Heaps& H)
    {
        std::size_t const len = (bytes + kArenaAlign - 1) / kArenaAlign * kArenaAlign;
        if (void* p = arenaCarve(d, len, dev, H))
            return p;
        if (!d.pending.empty())
        {
            drain(d, dev, H);
            releaseEmpty(d, false);
            if (void* p = arenaCarve(d, len, dev, H))
                return p;
        }
        std::size_t size = arenaChunkSize(d, len);
        void* base = nullptr;
        if (hipMalloc(&base, size) != hipSuccess)
        {
            (void)hipGetLastError();
            size = len;   // the group does not fit: a chunk of the request alone
            if (!(base = deviceMalloc(size, d, dev, H, true)))
                return nullptr;
        }
        auto* c = new ArenaChunk;
        c->base = static_cast<char*>(base);
        c->size = size;
        c->holes[0] = size;
        d.arenaChunks.push_back(c);
        d.lastChunk = c;
        d.lastReq = len;
        return arenaCarve(d, len, dev, H);
    }

    void* heapAllocate(std::size_t bytes)
    {
        if (rt::takeKnobCount(rt::Knob::MemoryFailNextAlloc))
        {
            (void)rt::check(hipErrorOutOfMemory, "hipMalloc (memory.fail_next_alloc)");
            return nullptr;
        }
        int const dev = rt::device();
        Heaps& H = heaps();
        std::lock_guard<std::mutex> lock(H.m);
        DeviceHeap& d = H.byDevice[dev];
        if (bytes <= kPoolMax && rt::knob(rt::Knob::MemoryPool) != 0)
            return poolAllocate(bytes, d, dev, H);
        if (bytes > kPoolMax && rt::knob(rt::Knob::MemoryArena) != 0)
            if (void* p = arenaAllocate(bytes, d, dev, H))
                return p;
        return deviceMalloc(bytes, d, dev, H, false);   // a plain buffer (freed with hipFree)
    }

    // true when p is a heap block (then it is queued for reuse).  foreign: freed through the
    // public vktHipFree / vktFree / Free, whose caller may have used the buffer on streams of its
    // own -- its reuse then waits for a device synchronisation (hipFree's guarantee), not only
    // for the library's streams.
    bool heapFree(void* p, bool foreign)
    {
        Heaps& H = heaps();
        std::lock_guard<std::mutex> lock(H.m);
        auto it = H.owner.find(p);
        if (it == H.owner.end())
            return false;
        HeapBlock const& b = it->second;
        DeviceHeap& d = H.byDevice[b.dev];
        d.pending.push_back(p);
        d.pendingForeign = d.pendingForeign || foreign;
        if (b.arena)
        {
            b.ac->live -= b.len;
            if (b.ac->live == 0)
            {
                // the chunk's last live block: drain now and give the chunk back to HIP
                int const dev = b.dev;
                drain(d, dev, H);
                releaseEmpty(d, false);
            }
        }
        else
        {
            b.pc->live -= 1;
            d.pendingByClass[b.len] += 1;
        }
        return true;
    }

    std::size_t heapReleaseCached()
    {
        Heaps& H = heaps();
        std::lock_guard<std::mutex> lock(H.m);
        std::size_t freed = 0;
        for (auto& kv : H.byDevice)
        {
            drain(kv.second, kv.first, H);
            freed += releaseEmpty(kv.second, true);
        }
        return freed;
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

    // The public copies (vktHipMemcpy, vkt::Memcpy / vktMemcpy) take caller pointers: the device
    // side of each copy kind must be memory the device can address.  memcpyHip itself trusts its
    // (library-allocated) pointers.  A pointer the HIP runtime does not track is refused here
    // rather than handed to hipMemcpyAsync, which treats an untracked address as host memory
    // and reads or writes it on the CPU (the r5a SIGSEGV).
    vktError memcpyChecked(void* dst, void const* src, std::size_t size, CopyKind ck)
    {
        if (size == 0)
            return vktNoError;
        if (dst == nullptr || src == nullptr)
            return rt::fail("Memcpy: null pointer");
        bool const devDst = ck == CopyKind::HostToDevice || ck == CopyKind::DeviceToDevice;
        bool const devSrc = ck == CopyKind::DeviceToHost || ck == CopyKind::DeviceToDevice;
        if (devDst)
        {
            vktError const e = rt::requireDevicePointer(dst, size, "Memcpy: destination is not device memory");
            if (e != vktNoError)
                return e;
        }
        if (devSrc)
        {
            vktError const e = rt::requireDevicePointer(src, size, "Memcpy: source is not device memory");
            if (e != vktNoError)
                return e;
        }
        return memcpyHip(dst, src, size, ck);
    }

    void* AllocateOn(std::size_t bytes, ExecutionPolicy const& owner)
    {
        if (bytes == 0)
            return nullptr;
        if (onGpu(owner))
        {
            (void)rt::device();   // bind the context's device before allocating
            return heapAllocate(bytes);
        }
        if (gPinnedHost.load())
        {
            {
                std::lock_guard<std::mutex> lock(gPinnedMutex);
                auto& c = pinnedCache();
                for (auto it = c.begin(); it != c.end(); ++it)
                    if (it->second == bytes)
                    {
                        void* const p = it->first;
                        gPinnedCached -= it->second;
                        c.erase(it);
                        pinnedSet().insert(p);
                        pinnedSizes()[p] = bytes;
                        return p;
                    }
            }
            void* p = nullptr;
            hipError_t err = hipHostMalloc(&p, bytes, hipHostMallocDefault);
            if (err != hipSuccess && releasePinnedCache() > 0)
            {
                (void)hipGetLastError();
                err = hipHostMalloc(&p, bytes, hipHostMallocDefault);
            }
            if (rt::check(err, "hipHostMalloc") == vktNoError)
            {
                std::lock_guard<std::mutex> lock(gPinnedMutex);
                pinnedSet().insert(p);
                pinnedSizes()[p] = bytes;
                return p;
            }
        }
        void* p = std::malloc(bytes);
        if (p == nullptr)
            rt::fail("Allocate: host malloc failed");
        return p;
    }

    void freeOn(void* data, ExecutionPolicy const& owner, bool foreign)
    {
        if (data == nullptr)
            return;
        if (onGpu(owner))
        {
            if (!heapFree(data, foreign))
                (void)rt::check(hipFree(data), "hipFree");
            return;
        }
        {
            std::lock_guard<std::mutex> lock(gPinnedMutex);
            auto it = pinnedSet().find(data);
            if (it != pinnedSet().end())
            {
                pinnedSet().erase(it);
                std::size_t const bytes = pinnedSizes()[data];
                pinnedSizes().erase(data);
                if (bytes >= kBigHost && gPinnedCached + bytes <= pinnedCacheCap())
                {
                    pinnedCache().emplace_back(data, bytes);   // for the next migration of this size
                    gPinnedCached += bytes;
                    return;
                }
                (void)rt::check(hipHostFree(data), "hipHostFree");
                return;
            }
        }
        std::free(data);
    }

    void FreeOn(void* data, ExecutionPolicy const& owner) { freeOn(data, owner, false); }

}   // detail

namespace
{
    // Frees large pageable host buffers off the calling thread (munmap of 2 GiB costs more than
    // its PCIe copy) on ONE worker thread, started on first use.  At most kReaperQueue buffers
    // wait; beyond that the caller frees synchronously (back-pressure instead of unbounded
    // threads or memory).  At process exit (static destruction) shutdown() frees what is queued
    // and joins the worker; the reaper itself is never destroyed, so a free after that is
    // well-defined and runs on the caller.
    class HostReaper
    {
    public:
        static constexpr std::size_t kReaperQueue = 4;

        void shutdown()
        {
            {
                std::lock_guard<std::mutex> g(m_);
                stopped_ = true;
            }
            cv_.notify_all();
            if (worker_.joinable())
                worker_.join();
            std::lock_guard<std::mutex> g(m_);
            for (void* p : queue_)
                std::free(p);
            queue_.clear();
        }

        void release(void* data)
        {
            {
                std::lock_guard<std::mutex> g(m_);
                if (!stopped_ && queue_.size() < kReaperQueue)
                {
                    queue_.push_back(data);
                    if (!worker_.joinable())
                        worker_ = std::thread([this] { loop(); });
                    cv_.notify_one();
                    return;
                }
            }
            std::free(data);
        }

    private:
        void loop()
        {
            std::unique_lock<std::mutex> g(m_);
            for (;;)
            {
                cv_.wait(g, [&] { return stopped_ || !queue_.empty(); });
                if (queue_.empty())
                    return;   // stopped
                void* const p = queue_.front();
                queue_.erase(queue_.begin());
                g.unlock();
                std::free(p);
                g.lock();
            }
        }

        std::mutex m_;
        std::condition_variable cv_;
        std::vector<void*> queue_;
        std::thread worker_;
        bool stopped_ = false;
    };

    HostReaper& reaper()
    {
        static auto* r = new HostReaper;   // (never destroyed, see above)
        return *r;
    }

    struct ReaperShutdown
    {
        ~ReaperShutdown() { reaper().shutdown(); }
    } gReaperShutdown;
} // namespace

namespace detail
{
    void freeHostLater(void* data) { reaper().release(data); }

    void CopyOn(void* dst, void const* src, std::size_t bytes, ExecutionPolicy const& owner)
    {
        (void)memcpyHip(dst, src, bytes, onGpu(owner) ? CopyKind::DeviceToDevice : CopyKind::HostToHost);
    }

    // The reference allocates, copies and frees the source unconditionally
    // (include/cpp/vkt/ManagedBuffer.hpp:168-198, errors dropped by src/vkt/Memory.cpp:70), so a
    // failed allocation or copy loses the only copy of the data.  Here the source is released
    // only once the copy has completed: on failure the buffer stays where it was (`last` and
    // the returned pointer unchanged), the error is recorded (rt::noteMigrationFailure, the
    // thread's last error), and the algorithm that asked for the bytes fails with InvalidValue
    // (rt::deviceData).
    void CopyBetween(void* dst, ExecutionPolicy const& dstOwner, void const* src, ExecutionPolicy const& srcOwner,
                     std::size_t bytes)
    {
        if (dst == nullptr || src == nullptr)
            return;
        CopyKind const ck = onGpu(dstOwner) ? (onGpu(srcOwner) ? CopyKind::DeviceToDevice : CopyKind::HostToDevice)
                                            : (onGpu(srcOwner) ? CopyKind::DeviceToHost : CopyKind::HostToHost);
        (void)memcpyHip(dst, src, bytes, ck);
    }

    void* MigrateBuffer(void* data, std::size_t bytes, ExecutionPolicy& last)
    {
        ExecutionPolicy ep = GetThreadExecutionPolicy();
        if (ep.device == last.device)
            return data;
        char const* const dir = onGpu(ep) ? "host -> device" : "device -> host";
        // a pageable destination on the host: a cached buffer of this size first (resident pages)
        void* fresh = !onGpu(ep) && bytes >= kBigHost && !gPinnedHost.load() ? takeHostCached(bytes) : nullptr;
        bool const reused = fresh != nullptr;
        if (!reused)
            fresh = AllocateOn(bytes, ep);
        if (fresh == nullptr && bytes > 0)
        {
            rt::noteMigrationFailure(std::string("migrate (") + dir + ", " + std::to_string(bytes) +
                                     " bytes): allocation failed; the data stays where it was");
            return data;
        }
        bool pinnedFresh = false, pinnedOld = false;
        if (bytes >= kBigHost)
        {
            std::lock_guard<std::mutex> lock(gPinnedMutex);
            pinnedFresh = fresh != nullptr && pinnedSet().count(fresh) != 0;
            pinnedOld = data != nullptr && pinnedSet().count(data) != 0;
        }
        if (bytes >= kBigHost && !onGpu(ep) && fresh != nullptr && !pinnedFresh && !reused && data != nullptr)
            prefaultHost(fresh, bytes);   // (the copy below then writes resident pages)
        if (bytes > 0 && data != nullptr)
        {
            vktError const e = memcpyHip(fresh, data, bytes, onGpu(ep) ? CopyKind::HostToDevice : CopyKind::DeviceToHost);
            if (e != vktNoError)
            {
                // the destination never received the bytes: give it back, keep the source
                if (reused)
                {
                    if (!keepHostCached(fresh, bytes))
                        std::free(fresh);
                }
                else
                    FreeOn(fresh, ep);
                rt::noteMigrationFailure(std::string("migrate (") + dir + ", " + std::to_string(bytes) +
                                         " bytes): copy failed (" + vktHipGetLastErrorString() +
                                         "); the data stays where it was");
                return data;
            }
        }
        if (bytes >= kBigHost && !onGpu(last) && !pinnedOld && data != nullptr)
        {
            if (!keepHostCached(data, bytes))   // the copy is complete (memcpyHip synchronises)
                freeHostLater(data);
        }
        else
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

void Free(void* ptr) { detail::freeOn(ptr, GetThreadExecutionPolicy(), true); }

void Memcpy(void* dst, void const* src, std::size_t size, CopyKind ck) { (void)detail::memcpyChecked(dst, src, size, ck); }

namespace
{
    // Host-resident buffers: a plain pattern copy, as MemsetRange_serial (reference
    // src/vkt/Memory_serial.hpp:24-37).  This is buffer housekeeping of ManagedBuffer::fill,
    // not one of the StructuredVolume algorithms.
    void hostMemsetRange(void* dst, void const* src, std::size_t dstSize, std::size_t srcSize)
    {
        if (srcSize == 0 || dst == nullptr || src == nullptr)
            return;
        std::size_t n = dstSize / srcSize;
        for (std::size_t i = 0; i < n; ++i)
            std::memcpy(static_cast<char*>(dst) + i * srcSize, src, srcSize);
    }
} // namespace

// The reference dispatches on the thread policy (src/vkt/Memory.cpp:77-80).  Under the GPU
// policy the pattern kernel refuses a pointer the device cannot address (hipk::memsetRange ->
// rt::requireDevicePointer) instead of faulting on it.
void MemsetRange(void* dst, void const* src, std::size_t dstSize, std::size_t srcSize)
{
    if (onGpu(GetThreadExecutionPolicy()))
    {
        (void)hipk::memsetRange(dst, src, dstSize, srcSize);
        return;
    }
    hostMemsetRange(dst, src, dstSize, srcSize);
}

namespace detail
{
    // ManagedBuffer<T>::fill (reference include/cpp/vkt/ManagedBuffer.hpp:252-258): the bytes
    // are filled where they live.  After a failed migration (MigrateBuffer keeps the buffer in
    // host memory under the GPU policy) that is the host pattern loop, not the pattern kernel.
    void MemsetRangeOn(void* dst, void const* src, std::size_t dstSize, std::size_t srcSize,
                       ExecutionPolicy const& owner)
    {
        if (onGpu(owner))
            (void)hipk::memsetRange(dst, src, dstSize, srcSize);
        else
            hostMemsetRange(dst, src, dstSize, srcSize);
    }
} // detail

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

    vktError requireDevicePointer(void const* p, std::size_t bytes, char const* what)
    {
        hipPointerAttribute_t a{};
        hipError_t const err = hipPointerGetAttributes(&a, p);
        if (err != hipSuccess)
            (void)hipGetLastError();   // (untracked pointers: an error, not a sticky one)
        bool const ok = err == hipSuccess &&
                        (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged ||
                         a.type == hipMemoryTypeUnified ||
                         (a.type == hipMemoryTypeHost && a.devicePointer == p));
        if (!ok)
            return fail(what);
        if (bytes > 0 && a.type == hipMemoryTypeDevice)
        {
            hipDeviceptr_t base = nullptr;
            std::size_t size = 0;
            if (hipMemGetAddressRange(&base, &size, const_cast<void*>(p)) == hipSuccess && base != nullptr)
            {
                auto const b = reinterpret_cast<uintptr_t>(base), q = reinterpret_cast<uintptr_t>(p);
                if (q - b > size || bytes > size - (q - b))
                    return fail(what);
            }
            else
                (void)hipGetLastError();   // (VMM mappings: no range to check against)
        }
        return vktNoError;
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
    if (vkt::heapFree(ptr, true))
        return vktNoError;
    return vkt::rt::check(hipFree(ptr), "hipFree");
}

vktError vktHipReleaseCachedMemory(size_t* releasedBytes)
{
    std::size_t const n = vkt::heapReleaseCached() + vkt::releasePinnedCache() + vkt::releaseHostCache();
    if (releasedBytes != nullptr)
        *releasedBytes = n;
    return vktNoError;
}

vktError vktHipMemcpy(void* dst, void const* src, size_t size, vktCopyKind ck)
{
    return vkt::detail::memcpyChecked(dst, src, size, static_cast<vkt::CopyKind>(ck));
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
