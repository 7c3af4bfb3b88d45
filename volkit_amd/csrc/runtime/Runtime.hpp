// Runtime.hpp -- internal runtime services of libvolkit (not installed).
//
// One HIP context per process (one process per GPU is the multi-GPU model): the device
// chosen by vktHipSetDevice (default: the current HIP device at first use), a blocking
// compute stream (ordered with the legacy NULL stream, like the reference's default-stream
// launches), a side copy stream for migrate(), and error/timing bookkeeping.
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>
#include <sstream>
#include <string>

#include "volkit_c.h"
#include "volkit.hpp"

namespace vkt
{
namespace rt
{
    enum class LogLevel { Error = 0, Warning = 1, Info = 2 };

    // VKT_LOG equivalent (reference src/vkt/Logging.hpp:41): message is emitted when the
    // temporary is destroyed; VKT_LOG_LEVEL=0/1/2 filters (default 2 = everything).
    class LogStream
    {
    public:
        explicit LogStream(LogLevel level) : level_(level) {}
        ~LogStream();
        std::ostream& stream() { return stream_; }

    private:
        std::ostringstream stream_;
        LogLevel level_;
    };

    // Context accessors (created lazily, thread-safe).
    hipStream_t computeStream();
    hipStream_t copyStream();
    bool asyncExecution();
    int device();

    // Error handling: record the message as the thread's last error, log it, return
    // vktInvalidValue; vktNoError for hipSuccess.
    vktError check(hipError_t err, char const* what);
    vktError fail(char const* what);          // non-HIP failure (bad arguments)
    void setLastError(std::string const& msg);

    // A migration that could not move a buffer (allocation or copy failure) leaves the bytes
    // where they were (detail::MigrateBuffer keeps the only copy) and records why here, per
    // thread; takeMigrationFailure() returns and clears it (empty: none since the last take).
    void noteMigrationFailure(std::string const& msg);
    std::string takeMigrationFailure();
    // e unchanged; when e is an error and a migration failed since the last take, the thread's
    // last error names that failure (the backend's own message would only say "invalid view").
    vktError explainFailure(vktError e, char const* name);

    // Bytes of a buffer (StructuredVolume, LookupTable, Histogram...) for a backend call on
    // the thread's device: getData() migrates them there first.  A buffer whose migration
    // failed is still resident elsewhere and yields nullptr, which every backend rejects
    // (validView) before it launches anything.
    template <class Buffer>
    auto deviceData(Buffer& b) -> decltype(b.getData())
    {
        auto* p = b.getData();
        return b.residentOn(GetThreadExecutionPolicy()) ? p : nullptr;
    }

    // Called by every backend entry point right after its launches: picks up launch
    // errors and, if async execution is off, waits for the compute stream.
    vktError finishLaunch(char const* what);

    // printPerformance / vktHipGetLastKernelMs support: brackets a backend call with
    // events on the compute stream.
    class ScopedKernelTimer
    {
    public:
        ScopedKernelTimer(char const* name, bool log);
        ~ScopedKernelTimer();

    private:
        char const* name_;
        bool active_;
        bool log_;
        hipEvent_t start_ = nullptr;
        hipEvent_t stop_ = nullptr;
    };

    bool kernelTimingEnabled();

    // Tuning knobs (vktHipSetTuningKnob): defaults are the measured best settings; tests and
    // tools/bench_configs.py change them to reach rare code paths (multi-launch splits) and to
    // A/B a choice inside one process on the same allocations.
    enum class Knob : int
    {
        PointwisePaddedRows = 0,       // 1: multi-row boxes use padded row items (no scalar edges)
        PointwiseMaxQuanta,            // launch split, in quanta of the default unroll (2^20)
        PointwiseGeneral,              // 0: boxes the aligned path cannot take use the scalar kernel
        PointwiseMergeSectors,         // 0: no 64-B sector completion at row ends
        PointwiseGeneral32,            // 0: the general path uses 64-bit addressing everywhere (tests)
        HistogramPacked16,             // 2 (default): packed 16-bit counters, in tiles beyond one launch; 1: one launch only (beyond: PAIR / 32-bit tiles); 0: one pass per 32-bit tile
        HistogramMulShift,             // 0: UInt16 bins other than code >> s keep the float formula
        HistogramP16Step,              // 0: P16 threshold tests after each item, not each wave-step
        PointwiseU8Pairs,              // 0: UInt8 multi-row boxes keep the 8-voxel per-item loop
        RenderBricks,                  // 0: multi-scattering samples the dense volume, not an 8^3-brick copy
        DecomposeAlignedLds,           // cut words: 0 per-voxel, 1 aligned LDS pieces, 2 every word so, 3 branch-free (dump bytes), 4 row-end voxel loop, 5 (default) 4 for UInt8 else 0
        DecomposeStageWords,           // source words per thread in flight in the staged copy (5, 6, 8)
        PointwiseU8Wide,               // 0: UInt8 general-path boxes keep 8-voxel items
        PointwiseF32Halves,            // 0: padded 4-byte rows keep the per-item loop
        PointwiseF32Wide,              // 4-byte general-path boxes with 16-B items: 1 every op, 2 one-source ops
        AggregatesCodes,               // bit 0 UInt8, bit 1 UInt16: ComputeAggregates from one pass of code counts
        ReduceU8Rows16,                // UInt8 code counts over range rows with 16-voxel items (codeCountsU8RowsKernel)
        DecomposeGrid,                 // 0: uniform brick grids keep the per-brick descriptor table
        MemoryPool,                    // 0: every device buffer from its own hipMalloc (no small-block pool)
        MemoryArena,                   // 0: buffers > 4 MiB from their own hipMalloc (no arena chunks)
        AggregatesMoments,             // ComputeAggregates in one pass of moments: bit 0 UInt16 unit mapping (integer), bit 1 UInt16 other mappings / Float32 (float), bit 2 (with bit 1) Int16 / UInt32 (float)
        MemoryArenaChunkMiB,           // > 0: arena chunks of exactly max(request, this many MiB) (tests)
        DecomposeBlock,                // threads per BrickDecompose workgroup over one 16-KiB chunk: 256 or 128
        PointwiseDwordShift,           // 0: 4-byte general-path windows keep the byte-align stage (whole-dword offsets)
        AggregatesMomentsPipe,         // integer moments: 0 one buffer x 4 items, 1 (default) / 2 / 4 two buffers x 4 / 8 / 2 items, 3 one buffer x 8
        DecomposeBatch,                // 1: BrickDecompose plans / copies in up to 8 batches of brick planes (measured slower: off)
        DecomposeGather,               // 1: uniform brick grids stage source rows and gather items (measured no faster: off)
        DecomposePipe,                 // 1: uniform brick grids on a resident, double-buffered walk (measured slower: off)
        DecomposePair,                 // 1: two x-neighbour bricks of <= 16 KiB per workgroup (uniform grids)
        MemoryFailNextAlloc,           // n > 0: the next n device allocations fail (tests of the failure paths)
        CommTestStallMs,               // > 0: every RCCL round with a deadline also stalls its stream this long (watcher test)
        PointwiseRowKernel,            // one-row (whole-volume) copies / arithmetic on the MODE-0 kernel: bit 0 UInt8, bit 1 UInt16
        PointwiseRowLds,               // bytes of dynamic LDS per UInt16 row-kernel workgroup (occupancy cap; 0 = none)
        PointwiseU8Unroll,             // items per lane of the UInt8 row kernel (2, 4, 8)
        PointwiseU16Unroll,            // items per lane of the UInt16 row kernel (1, 2)
        PointwiseRowLdsU8,             // the same occupancy cap for the UInt8 row kernel
        PointwiseRowSwizzle,           // > 0: the row kernel gives each XCD runs of this many consecutive quanta
        PointwiseRowsKernel,           // multi-row boxes (32-bit rows, no scalar edges) on the MODE-1 kernel: bit 0 UInt8, bit 1 UInt16
        TransformShape,                // device-functor Transform vector kernels: 0 256x4, 1 64x2, 2 64x1 (read via vktHipGetTuningKnob)
        DecomposeDirect,               // halo-free aligned brick grids: 1 direct copy (small bricks P per workgroup), 2 one brick per workgroup, 0 LDS-staged
        ResamplePrefetch,              // LDS gather loads the next task's row during the current one: 1 2-byte destinations, 2 all, 0 (default) off
        ResampleAnyRows,               // 1: the LDS gather also stages source rows that are not 16-B multiples (rowChunk)
        HistogramPairTiles,            // histograms of 2..4 tiles side by side in one launch (PAIR): 1 where P16 does not apply, 2 always, 0 never
        ResampleLdsPad,                // LDS gathers: 16 B of padding per 256 B of a staged row (bank spread): 1 UInt8 sources, 2 all, 0 none
        DecomposeRowImage,             // uniform grids of <= 16-KiB bricks through per-row LDS images (brickRowImageKernel): 2 UInt8, 1 all, 0 off
        ResampleDstRows,               // LDS gathers over destination-row tasks (resampleGatherDstRowKernel): 0 off, 1 UInt8 rows not 16-B multiples, >= 2 all (grid cap in 1024s of workgroups)
        HistogramU16Codes,             // 16-bit float-formula bins through code counts + fold: 2 (default) beyond the replicated counters, 1 beyond one LDS tile, 0 off (Int16: always unless 0)
        HistogramPartials,             // tiled histogram launches store per-workgroup counter words summed by one kernel: 1 (default) packed-16 launches, 2 every tiled launch, 0 global atomics per counter
        Count
    };
    int64_t knob(Knob k);
    // A counting knob: true (and the knob decremented) when it was > 0.
    bool takeKnobCount(Knob k);

    // Stream ordering between the compute stream and the side copy stream (event based):
    // the copy stream waits for everything queued on the compute stream so far / the compute
    // stream waits for everything queued on the copy stream so far.
    vktError copyStreamAfterCompute();
    vktError computeStreamAfterCopy();

    // vktNoError when the device can address [p, p + bytes): HBM (hipMalloc, VMM, managed) or
    // pinned host memory mapped at the same address.  Anything else -- pageable host memory, or
    // an address the runtime does not track -- records `what` as the thread's last error and
    // returns vktInvalidValue, before any kernel or copy is queued on it (no XNACK on this pool:
    // a kernel on a pageable pointer is a memory-access fault).  A device range that runs past
    // its allocation is refused the same way.
    vktError requireDevicePointer(void const* p, std::size_t bytes, char const* what);

    // Device scratch for one backend call site, reused across calls (no per-call hipMalloc,
    // and no stream-ordered pool: hipMallocAsync blocks filled by an H2D copy were
    // intermittently seen stale by the next kernel on gfx950/ROCm 7.2 -- DESIGN.md §4.6).
    // acquire(stream) hands the buffer out again right away when the previous user released
    // it on the same stream (stream order protects it); after a stream switch it first waits
    // (host) for the previous user's work.
    class StreamScratch
    {
    public:
        // Returns nullptr (and records the error) on allocation failure.  Holds the lock
        // until release().
        void* acquire(std::size_t bytes, hipStream_t stream);
        // Records completion of the work that uses the buffer on `stream`, unlocks.
        void release(hipStream_t stream);

    private:
        std::mutex m_;
        void* p_ = nullptr;
        std::size_t cap_ = 0;
        hipEvent_t done_ = nullptr;
        hipStream_t last_ = nullptr;
        bool pending_ = false;
    };

} // rt

namespace detail
{
    // Copy with the stream ordering described in runtime/Memory.cpp.
    vktError memcpyHip(void* dst, void const* src, std::size_t size, CopyKind ck);
    // memcpyHip after checking that the device side(s) of `ck` are device-addressable
    // (rt::requireDevicePointer): the public copy entry points, which take caller pointers.
    vktError memcpyChecked(void* dst, void const* src, std::size_t size, CopyKind ck);
}
} // vkt

#define VKT_LOG(LEVEL) ::vkt::rt::LogStream(LEVEL).stream()
#define VKT_HIP_TRY(EXPR)                                                            \
    do {                                                                             \
        vktError vkt_err_ = ::vkt::rt::check((EXPR), #EXPR);                         \
        if (vkt_err_ != vktNoError)                                                  \
            return vkt_err_;                                                         \
    } while (0)
