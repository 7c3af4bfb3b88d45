/*
 * volkit_hip.h -- the HIP/gfx950 backend seam, as a plain C ABI.
 *
 * The reference plugs its GPU backend in by name pasting: VKT_LEGACY_CALL__(FUNC, ...)
 * calls FUNC##_cuda(...) when the thread policy says Device::GPU
 * (reference src/vkt/Callable.hpp:82-113).  Each vktHip* entry point below replaces
 * one of those _cuda functions; it takes a plain voxel-array view (pointer + dims +
 * format + mapping, the fields of the reference's kernel argument
 * StructuredVolumeView, src/vkt/StructuredVolumeView.hpp:221-225) instead of C++
 * objects, so it can be bound from C, ctypes, cgo or JNI without C++ types.
 *
 * All pointers in a view are DEVICE pointers (hipMalloc'ed, or any pointer valid on
 * the current HIP device).  Work is enqueued on the backend's compute stream
 * (vktHipGetComputeStream) and is NOT waited for unless async execution is switched
 * off (vktHipSetAsyncExecution(0)); errors are returned, never ignored (the reference
 * drops them, src/vkt/macros.hpp:10).  Out-of-bounds ranges are rejected with
 * vktInvalidValue before any launch (in the reference they are undefined behaviour).
 */
#ifndef VOLKIT_HIP_H
#define VOLKIT_HIP_H

#include "volkit_c.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Kernel-argument view of one structured volume (reference StructuredVolumeView). */
typedef struct {
    uint8_t* data;       /* device pointer to dense x-fastest voxels */
    int32_t dimX, dimY, dimZ;
    int32_t dataFormat;  /* vktDataFormat value */
    float mappingLo, mappingHi;
} vktHipVolumeView_t;

/* Arithmetic operator codes: order of reference src/vkt/Arithmetic_serial.hpp:47-258. */
typedef enum {
    vktHipOpSum, vktHipOpDiff, vktHipOpProd, vktHipOpQuot, vktHipOpAbsDiff,
    vktHipOpSafeSum, vktHipOpSafeDiff, vktHipOpSafeProd, vktHipOpSafeQuot, vktHipOpSafeAbsDiff,
    vktHipOpCount
} vktHipArithmeticOp;

/* ---- runtime / context (design intent of reference include/c/vkt/CudaContext.h:17-65,
 *      which is declared there but never defined) ----------------------------------- */
VKTAPI vktError vktHipSetDevice(int32_t device);        /* before first GPU use */
VKTAPI vktError vktHipGetDevice(int32_t* device);
VKTAPI vktError vktHipSetAsyncExecution(int32_t async);  /* 0: every call synchronises */
VKTAPI vktError vktHipGetAsyncExecution(int32_t* async);
/* Replace the compute stream (e.g. with torch.cuda.current_stream().cuda_stream);
 * NULL restores the backend's own blocking stream. */
VKTAPI vktError vktHipSetComputeStream(void* hipStream);
VKTAPI vktError vktHipGetComputeStream(void** hipStream);
/* Replace the side copy stream of migrate() / streams (NULL restores the backend's own). */
VKTAPI vktError vktHipSetCopyStream(void* hipStream);
VKTAPI vktError vktHipGetCopyStream(void** hipStream);
VKTAPI vktError vktHipSynchronize(void);
/* Context handles -- the reference's vktCudaContext API (include/c/vkt/CudaContext.h:17-65,
 * declared there, defined nowhere) for HIP: a context holds numStreams streams (created
 * blocking and owned by it, or the caller's via SetStream), a compute and a copy stream id and
 * the async flag.  vktHipContextMakeCurrent(ctx) binds it to the backend (one HIP context per
 * process): algorithms then run on streams[computeId], migrations on streams[copyId]; setters
 * on the current context take effect at once.  MakeCurrent(NULL) and destroying the current
 * context restore the backend's own streams.  A new context has 2 streams, compute 0, copy 1. */
typedef struct vktHipContext_impl* vktHipContext;
VKTAPI vktError vktHipContextCreate(vktHipContext* context);
VKTAPI vktError vktHipContextDestroy(vktHipContext context);
VKTAPI vktError vktHipContextMakeCurrent(vktHipContext context);
VKTAPI vktError vktHipContextSetAsyncExecution(vktHipContext context, int32_t async);
VKTAPI vktError vktHipContextGetAsyncExecution(vktHipContext context, int32_t* async);
VKTAPI vktError vktHipContextSetNumStreams(vktHipContext context, int32_t numStreams);
VKTAPI vktError vktHipContextGetNumStreams(vktHipContext context, int32_t* numStreams);
VKTAPI vktError vktHipContextSetStream(vktHipContext context, int32_t streamId, void* hipStream);
VKTAPI vktError vktHipContextGetStream(vktHipContext context, int32_t streamId, void** hipStream);
VKTAPI vktError vktHipContextSetComputeStreamId(vktHipContext context, int32_t streamId);
VKTAPI vktError vktHipContextGetComputeStreamId(vktHipContext context, int32_t* streamId);
VKTAPI vktError vktHipContextSetCopyStreamId(vktHipContext context, int32_t streamId);
VKTAPI vktError vktHipContextGetCopyStreamId(vktHipContext context, int32_t* streamId);
/* Last HIP error string seen by the backend (thread-local), "" if none. */
VKTAPI const char* vktHipGetLastErrorString(void);
/* Milliseconds of the most recent kernel launched by the calling thread, measured with
 * hipEvents on the compute stream when timing is enabled (vktHipSetKernelTiming(1));
 * this is how printPerformance is implemented. */
VKTAPI vktError vktHipSetKernelTiming(int32_t enable);
VKTAPI vktError vktHipGetLastKernelMs(float* ms);

/* Scope for a kernel launched by the CALLER on the compute stream (used by the
 * device-functor Transform templates of volkit_transform.hpp): Begin checks the thread
 * policy (GPU, else vktInvalidValue), opens the roctx range and the printPerformance timer
 * and returns the compute stream; End picks up launch errors, waits when async execution
 * is off, and closes the scope. */
typedef struct vktHipKernelScope_impl* vktHipKernelScope;
VKTAPI vktError vktHipKernelScopeBegin(const char* name, vktHipKernelScope* scope, void** hipStream);
VKTAPI vktError vktHipKernelScopeEnd(vktHipKernelScope scope);
/* Tuning knobs (process-wide; a negative value restores the default): "pointwise.padded_rows"
 * (1), "pointwise.max_quanta_per_launch" (2^20), "pointwise.general" (1; 0 sends boxes the
 * aligned vector path cannot take to the per-voxel kernel), "pointwise.merge_sectors" (1; 0 stops
 * the pointwise kernels from completing the 64-B sectors at the row ends of a box by rewriting the
 * destination's own bytes around it; 2 extends it to the aligned path's 2-byte 3-stream ops),
 * "pointwise.general_32bit" (1; 0 makes the general path use
 * its 64-bit addressing, otherwise taken only for operands beyond 4 GiB from their 16-B aligned base), "pointwise.u8_pairs"
 * (1; 0 keeps UInt8 multi-row boxes on the 8-voxel per-item loop instead of 16-B accesses on a
 * 16-voxel row grid), "histogram.packed16" (2; histograms with more bins than one LDS tile of
 * 32-bit counters count in packed 16-bit counters, one pass per tile of twice as many bins; 1 only
 * when one such tile holds every bin; 0 one pass per tile of 32-bit counters), "histogram.mulshift" (1; 0 makes UInt16 histograms whose bins are (code * numBins)
 * >> 16 keep the float bin formula), "histogram.p16_step" (1; 0 runs the packed-16 counters'
 * threshold tests after every item instead of once per wave-step), "render.bricks" (1; 0 makes
 * MultiScattering sample the dense volume instead of its 8^3-brick copy), "decompose.aligned_lds"
 * (0; 1 / 2 write the row-end / every staged word to LDS as aligned pieces), "decompose.stage_words"
 * (6; 5 or 8 source words in flight per thread), "pointwise.u8_wide" (1; 0 keeps UInt8 boxes of the
 * general path on 8-voxel items), "pointwise.f32_halves" (1; 0 keeps 4-byte padded multi-row boxes
 * on the per-item loop), "pointwise.f32_wide" (2; 4-byte general-path boxes with 16-B items: 1 for
 * every op, 2 for the ops of at most one source (copies), 0 for none),
 * "aggregates.codes" (3; bit 0 UInt8, bit 1 UInt16: ComputeAggregates from one pass of code counts
 * instead of the two float passes), "reduce.u8_rows16" (1; UInt8 code counts over range rows on 16-voxel
 * items, row-end bytes subtracted inside the main loop; 2 subtracts them in a row walk after it;
 * 0 keeps the 8-voxel item walk), "decompose.grid" (1; 0 makes uniform brick grids load a
 * per-brick descriptor instead of deriving it from the brick index), "memory.pool" (1; 0 gives every
 * device buffer of <= 4 MiB its own hipMalloc instead of a 256-B class of a 64-MiB pooled chunk), "memory.arena" (1; 0 gives every larger buffer its
 * own hipMalloc instead of a 2-MiB aligned block of an arena chunk), "memory.arena_chunk_mib" (0; > 0 makes
 * new arena chunks exactly max(request, value MiB): tests), "decompose.block" (256; 128 copies each
 * 16-KiB BrickDecompose chunk with 128 threads), "pointwise.dword_shift" (1; 0 keeps the byte-align
 * stage of the general path's window shift for 4-byte voxels at 4-B aligned addresses), "aggregates.moments" (7; bit 0: UInt16
 * ComputeAggregates under the unit mapping from one pass of exact integer moments, bit 1: UInt16
 * under other mappings and Float32 from one pass of floating-point moments, bit 2 (with bit 1):
 * Int16 and UInt32 the same -- all instead of
 * "aggregates.codes" / the two float passes), "aggregates.moments_pipe" (1; integer-moments kernel
 * variant: 0 one register buffer of 4 items per lane and wave-step, 1 two buffers of 4 (the next
 * step's loads in flight during this step's arithmetic), 2 two of 8, 3 one of 8, 4 two of 2, 5 as 1
 * bound to 7 waves per SIMD),
 * "decompose.batch" (0; 1 plans and copies BrickDecompose in up to 8 batches of brick planes),
 * "decompose.gather" (0; 1 makes uniform brick grids stage source rows in LDS and gather each
 * output item from them instead of scattering source words into the brick layout),
 * "decompose.pipe" (0; 1 runs uniform brick grids on a resident grid that loads chunk k + 1 while
 * it stores chunk k instead of one workgroup per 16-KiB chunk), "decompose.pair" (0; 1 copies
 * two x-neighbour bricks of at most 16 KiB per workgroup from one staging of their rows' union),
 * "resample.prefetch" (0; 1 / 2: the LDS gather loads the next task's source row during the current
 * one for 2-byte / every destination), "resample.any_rows" (1; 0 sends source rows that are not
 * 16-B multiples to the per-voxel gather), "resample.lds_pad" (1; staged LDS rows get 16 B of
 * padding per 256 B -- LDS bank spread -- for UInt8 sources; 2 for every format, 0 none),
 * "resample.dst_rows" (1; the gather over destination-row tasks for UInt8 source rows that are not
 * 16-B multiples; 0 off; >= 2 for every eligible 1- / 2-byte gather, grid cap in 1024s of workgroups),
 * "histogram.u16_codes" (2; UInt16 histograms whose bins are not integer functions of the code and
 * exceed the replicated LDS counters, and every Int16 histogram, count the 65 536 codes in one pass
 * and fold the counts into the bins; 1 only UInt16 bins beyond one LDS tile; 0 the per-voxel
 * kernels), "histogram.partials" (1; packed-16 histogram workgroups store their counter words and
 * one kernel sums them instead of a 64-bit atomic per counter; 2 every tiled launch; 0 atomics).
 * The full list with defaults: volkit_amd/csrc/runtime/HipContext.cpp (kKnobs).
 * For tests and in-process A/B measurements; unknown names return
 * vktInvalidValue.
 *
 * Writes outside a range box: FillRange / CopyRange / ArithmeticRange / convert and device-functor
 * TransformRange may rewrite, with the destination's own unchanged bytes, up to one 64-B sector around each row
 * of the box (64-B sector completion; off with "pointwise.merge_sectors" = 0 for
 * the pointwise ops).  Every call runs on the one compute stream, so the library's own calls
 * never race; a caller that writes bytes within 64 B of a box row from another stream or the
 * host while such a call runs must order the two itself. */
VKTAPI vktError vktHipSetTuningKnob(const char* name, int64_t value);
/* The current value of a tuning knob (read by the header-only Transform templates of
 * volkit_transform.hpp, e.g. "transform.shape"); vktInvalidValue for an unknown name. */
VKTAPI vktError vktHipGetTuningKnob(const char* name, int64_t* value);
/* Record `message` as the calling thread's last error, log it; returns vktInvalidValue. */
VKTAPI vktError vktHipReportError(const char* message);

/* ---- memory: replaces Allocate_cuda/Free_cuda/MemsetRange_cuda
 *      (reference src/vkt/Memory_cuda.hpp:16-31) and the cudaMemcpy of src/vkt/Memory.cpp:40-75
 * Device buffers are blocks of pooled / arena chunks (knobs "memory.pool", "memory.arena"): release every pointer
 * from vktHipAllocate / vktAllocate with vktHipFree / vktFree, never with hipFree.
 * Ordering of a free: a block freed through vktHipFree / vktFree / vkt::Free is handed out again
 * only after a device synchronisation (hipFree's guarantee: work the caller queued on streams
 * of its own is finished).  Buffers the library frees itself (volumes, bricks, lookup tables,
 * scratch) wait only for the library's compute and copy streams, which are blocking streams
 * (ordered with the legacy NULL stream): a caller that used a volume's getData() pointer on a
 * non-blocking stream of its own synchronises that stream before destroying the volume. */
VKTAPI vktError vktHipAllocate(void** ptr, size_t size);
VKTAPI vktError vktHipFree(void* ptr);
/* The library caches device memory (pool chunks of small buffers; arena chunks of large ones,
 * sized for a group of like buffers -- four times the request, at least 64 MiB -- and returned to
 * HIP as soon as their last buffer is freed).  This call waits for the library's streams, then
 * returns every chunk that holds no live buffer to HIP; *releasedBytes (may be NULL) receives the
 * bytes released.  A device allocation that fails does the same and retries once.  It also frees
 * the host buffers the migrations keep: pinned buffers of >= 64 MiB freed by the caller (at most
 * 16 GiB, reused by a pinned allocation of the same size) and pageable buffers of >= 64 MiB a
 * migration to the GPU released (at most min(8 GiB, physical memory / 8), the destination of the
 * next migration back of the same size: its pages already resident). */
VKTAPI vktError vktHipReleaseCachedMemory(size_t* releasedBytes);
VKTAPI vktError vktHipMemcpy(void* dst, void const* src, size_t size, vktCopyKind ck);
/* Host buffers allocated under the CPU policy from now on are page-locked (hipHostMalloc),
 * so migrate() DMAs directly to/from them (default 0: malloc, as the reference). */
VKTAPI vktError vktHipSetPinnedHostAllocation(int32_t enable);
/* Repeat the `patternSize`-byte host pattern over `dstSize` device bytes (no device
 * allocation per call, 64-bit grid; reference truncates at 2^32 elements, Memory_cuda.cu:40). */
VKTAPI vktError vktHipMemsetRange(void* dst, void const* pattern, size_t dstSize, size_t patternSize);

/* ---- algorithms (first/last/dstOffset are voxel coordinates, ranges half-open) ---- */

/* replaces FillRange_cuda (reference src/vkt/Fill_cuda.hpp:13, Fill_cuda.cu:22-55);
 * semantics of FillRange_serial (src/vkt/Fill_serial.hpp:20-26). */
VKTAPI vktError vktHipFillRange(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last, float value);

/* replaces CopyRange_cuda (reference src/vkt/Copy_cuda.hpp:11-17); semantics of
 * CopyRange_serial (src/vkt/Copy_serial.hpp:13-82): source index clamped to the
 * source dims, dst index = x - first + dstOffset, bytewise iff format and mapping match. */
VKTAPI vktError vktHipCopyRange(vktHipVolumeView_t dst, vktHipVolumeView_t src,
                                vktVec3i_t first, vktVec3i_t last, vktVec3i_t dstOffset);

/* replaces {Sum,...,SafeAbsDiff}Range_cuda (reference src/vkt/Arithmetic_cuda.hpp:10-98);
 * semantics of ArithmeticOp (src/vkt/Arithmetic_serial.hpp:15-45): sources read at the
 * absolute x, dest written at x + dstOffset, Safe* clamps to the dest mapping. */
VKTAPI vktError vktHipArithmeticRange(vktHipArithmeticOp op, vktHipVolumeView_t dest,
                                      vktHipVolumeView_t source1, vktHipVolumeView_t source2,
                                      vktVec3i_t first, vktVec3i_t last, vktVec3i_t dstOffset);

/* replaces Resample_cuda (reference src/vkt/Resample_cuda.hpp:12-17); semantics of
 * Resample_serial (src/vkt/Resample_serial.hpp:26-71), including the same-dims
 * conversion branch that the CUDA path lacks. */
VKTAPI vktError vktHipResample(vktHipVolumeView_t dst, vktHipVolumeView_t src, vktFilterMode fm);

/* Z-slab Resample for multi-GPU partitions (no reference counterpart):
 * `dst` holds global dst planes [dstZ0, dstZ0 + dst.dimZ) of a volume whose global depth
 * is dstGlobalDimZ; `src` holds global source planes [srcZ0, srcZ0 + src.dimZ) of a
 * volume of global depth srcGlobalDimZ.  X/Y dims are global.  The planes the exact
 * index table asks for (vktHipResampleSlabSourceRange) must be inside `src`. */
VKTAPI vktError vktHipResampleSlab(vktHipVolumeView_t dst, vktHipVolumeView_t src, vktFilterMode fm,
                                   int32_t dstGlobalDimZ, int32_t dstZ0,
                                   int32_t srcGlobalDimZ, int32_t srcZ0);
/* Source planes [*srcZBegin, *srcZEnd) that dst planes [dstZ0, dstZ1) read, for the
 * given filter and formats (Linear with a non-integer-exact source reads the clamped
 * z+1 neighbour plane too). */
VKTAPI vktError vktHipResampleSlabSourceRange(int32_t dstGlobalDimZ, int32_t dstZ0, int32_t dstZ1,
                                              int32_t srcGlobalDimZ, vktFilterMode fm,
                                              int32_t needsNeighbours,
                                              int32_t* srcZBegin, int32_t* srcZEnd);

/* Z-slab plan for Resample over `nranks` ranks (no reference counterpart): the
 * global source planes [*localZ0, *localZ1) rank `rank` holds (its ceil-partition slab plus
 * the halo its dst slab reads) and the plane ranges it sends to / receives from each peer.
 * *count receives the number of transfers; `transfers` (may be NULL to query the count) must
 * hold `capacity` >= *count entries.  Same plan as volkit_amd/slab.py:plan_resample. */
typedef struct vktHipSlabTransfer
{
    int32_t peer;
    int32_t z0, z1;   /* global source planes [z0, z1) */
    int32_t send;     /* 1: this rank sends them to peer, 0: receives them from peer */
} vktHipSlabTransfer_t;
VKTAPI vktError vktHipSlabResamplePlan(int32_t dstGlobalDimZ, int32_t srcGlobalDimZ, int32_t nranks, int32_t rank,
                                       vktFilterMode fm, int32_t needsNeighbours, int32_t* localZ0,
                                       int32_t* localZ1, vktHipSlabTransfer_t* transfers, int32_t capacity,
                                       int32_t* count);

/* In-library halo exchange over RCCL (xGMI): one communicator per process / GPU.  Rank 0
 * creates the id, the caller distributes it (MPI, a file, torch.distributed ...), every rank
 * calls vktHipCommInitRank with it on the device the library uses (vktHipSetDevice). */
typedef struct
{
    char internal[128];   /* ncclUniqueId */
} vktHipCommId_t;
typedef struct vktHipComm_impl* vktHipComm_t;
VKTAPI vktError vktHipCommGetUniqueId(vktHipCommId_t* id);
VKTAPI vktError vktHipCommInitRank(vktHipComm_t* comm, int32_t nranks, vktHipCommId_t id, int32_t rank);
VKTAPI vktError vktHipCommDestroy(vktHipComm_t comm);
/* Failure detection: every RCCL round the library issues on `comm` (halo
 * exchange, overlapped slab resample, slab Range moves) returns once enqueued -- the host is
 * never blocked.  A watcher thread of the communicator times each round from the moment the
 * work queued ahead of it on its stream has finished, up to `milliseconds`, polling
 * ncclCommGetAsyncError; a peer that never joins, or an asynchronous RCCL error, aborts the
 * communicator (its kernels exit instead of hanging every rank) and every later call on it,
 * and vktHipCommSynchronize, return vktInvalidValue naming the failure.  0: no deadline.
 * Default 300 000 ms, or the environment variable VKT_COMM_TIMEOUT_MS at vktHipCommInitRank. */
VKTAPI vktError vktHipCommSetTimeout(vktHipComm_t comm, int64_t milliseconds);
/* Waits until the watcher has judged every round enqueued so far (complete, or the
 * communicator aborted); vktInvalidValue if the communicator was aborted. */
VKTAPI vktError vktHipCommSynchronize(vktHipComm_t comm);
/* One round on the compute stream: `bytes` of sendBuf to `peer` and as many from `peer` into
 * recvBuf (device buffers; peer may be this rank).  Returns once enqueued, judged like every
 * round (vktHipCommSetTimeout). */
VKTAPI vktError vktHipCommExchange(vktHipComm_t comm, int32_t peer, void const* sendBuf, void* recvBuf, size_t bytes);
/* `localSrc` holds global source planes [localZ0, localZ0 + localSrc.dimZ) (X/Y dims global).
 * Sends the owned planes the peers' dst slabs read and receives this rank's halo planes into
 * the buffer: one ncclGroupStart .. ncclGroupEnd round of ncclSend / ncclRecv on the compute
 * stream, so a vktHipResampleSlab enqueued next reads the halo.  Returns once enqueued. */
VKTAPI vktError vktHipSlabExchangeHalo(vktHipComm_t comm, vktHipVolumeView_t localSrc, int32_t localZ0,
                                       int32_t dstGlobalDimZ, int32_t srcGlobalDimZ, vktFilterMode fm,
                                       int32_t needsNeighbours);
/* Halo exchange overlapped with the interior (the compute / copy stream split of the reference's
 * CudaContext, include/c/vkt/CudaContext.h:41-65; volkit_amd/slab.py:resample_slab_overlapped):
 * the RCCL round runs on the communicator's own stream after the work queued so far on the
 * compute stream; meanwhile the dst planes that read only owned source planes resample on the
 * compute stream; the compute stream then waits for the round and resamples the remaining
 * planes.  `dst` holds exactly this rank's dst slab (ceil partition of dstGlobalDimZ);
 * `localSrc` as for vktHipSlabExchangeHalo.  Equal to vktHipSlabExchangeHalo +
 * vktHipResampleSlab; returns once enqueued. */
VKTAPI vktError vktHipResampleSlabOverlapped(vktHipComm_t comm, vktHipVolumeView_t dst, vktHipVolumeView_t localSrc,
                                             int32_t localZ0, int32_t dstGlobalDimZ, int32_t srcGlobalDimZ,
                                             vktFilterMode fm, int32_t needsNeighbours);
/* The same for `numSlabs` slabs in this process on the library's device (slab r = rank r):
 * each slab's receives are device copies on the copy stream, overlapped with its interior. */
VKTAPI vktError vktHipResampleSlabsOverlappedLocal(int32_t numSlabs, vktHipVolumeView_t const* dst,
                                                   vktHipVolumeView_t const* localSrc, int32_t const* localZ0,
                                                   int32_t dstGlobalDimZ, int32_t srcGlobalDimZ, vktFilterMode fm,
                                                   int32_t needsNeighbours);
/* The same exchange for a partition whose `numSlabs` slabs all live in this process on the
 * library's device (slab r = rank r of numSlabs; localSrc[r] holds global source planes
 * [localZ0[r], localZ0[r] + localSrc[r].dimZ)): every receive of the plan is a device-to-device
 * hipMemcpyAsync from the owning slab's buffer on the compute stream. */
VKTAPI vktError vktHipSlabExchangeHaloLocal(int32_t numSlabs, vktHipVolumeView_t const* localSrc,
                                            int32_t const* localZ0, int32_t dstGlobalDimZ, int32_t srcGlobalDimZ,
                                            vktFilterMode fm, int32_t needsNeighbours);
/* The same for slabs on SEVERAL devices of this process (slab r on HIP device devices[r]; the
 * multi-device single-process model of the reference's CudaContext, include/c/vkt/CudaContext.h:
 * 41-65): every receive is a hipMemcpyPeerAsync into the receiving slab's device (peer access
 * enabled where the devices support it), ordered after the library's compute stream for its own
 * device; returns once every plane has landed. */
VKTAPI vktError vktHipSlabExchangeHaloPeer(int32_t numSlabs, vktHipVolumeView_t const* localSrc,
                                           int32_t const* localZ0, int32_t const* devices, int32_t dstGlobalDimZ,
                                           int32_t srcGlobalDimZ, vktFilterMode fm, int32_t needsNeighbours);

/* ---- Range calls over Z-slab partitioned volumes (no reference counterpart)
 * A volume of global depth globalDimZ is split over nranks ranks by the ceil partition: rank r
 * OWNS global planes [r*ceil(D/n), min((r+1)*ceil(D/n), D)).  A slab is one rank's part: `view`
 * (X/Y dims global) holds global planes [z0, z0 + view.dimZ), which must include the owned ones
 * (it may hold halo planes too).  first / last / dstOffset are GLOBAL coordinates with the
 * reference's semantics (FillRange: dst[x] for x in [first, last); CopyRange:
 * dst[x - first + dstOffset] = src[clamp(x)], Copy_serial.hpp:38-47; arithmetic:
 * dst[x + dstOffset] = f(s1[x], s2[x]) at absolute x, Arithmetic_serial.hpp:25-41).  Each rank
 * writes only the dst planes it owns.  The source planes its dst planes read that other ranks
 * own -- the planes a dstOffset.z (or a clamped halo) moves across slab boundaries -- are sent
 * by their owners into a gather buffer; then the rank runs the local op piece by piece.  Global
 * arguments (ranges, depths) are checked before anything moves, identically on every rank. */
typedef struct vktHipSlab
{
    vktHipVolumeView_t view;
    int32_t z0;           /* global plane of view plane 0 */
    int32_t globalDimZ;   /* depth of the whole volume */
} vktHipSlab_t;

/* One local piece of a rank's part of a Range call: loop planes [zBegin, zEnd) of the
 * reference's z loop (global), writing global dst planes from dstZ on; per source k, the global
 * source planes [srcZ[k], srcZ[k] + srcPlanes[k]) it reads (after the CopyRange clamp) and where
 * from: bufPlane[k] = -1 the own slab, else that plane of the rank's gather buffer for source k. */
typedef struct vktHipSlabPiece
{
    int32_t zBegin, zEnd;
    int32_t dstZ;
    int32_t srcZ[2];
    int32_t srcPlanes[2];
    int32_t bufPlane[2];
} vktHipSlabPiece_t;
/* One move of source planes between two ranks: global planes [z0, z1) of source `source`
 * (0: src / source1, 1: source2) go from their owner to the receiver's gather buffer at plane
 * bufPlane.  send = 1: this rank is the owner (peer receives); 0: this rank receives. */
typedef struct vktHipSlabMove
{
    int32_t peer;
    int32_t send;
    int32_t source;
    int32_t z0, z1;
    int32_t bufPlane;
} vktHipSlabMove_t;
typedef enum { vktHipSlabFill = 0, vktHipSlabCopy = 1, vktHipSlabArithmetic = 2 } vktHipSlabOpKind;
/* The plan of rank `rank` (pieces in z order; moves in the global order every rank issues them,
 * so two ranks' moves pair up in order); bufPlanes[k] = planes of its gather buffer for source
 * k.  src2GlobalDimZ is ignored unless kind is vktHipSlabArithmetic; source globals unused for
 * Fill.  Arrays may be NULL to query the counts; capacities must cover them otherwise. */
VKTAPI vktError vktHipSlabRangePlan(vktHipSlabOpKind kind, int32_t nranks, int32_t rank, int32_t dstGlobalDimZ,
                                    int32_t src1GlobalDimZ, int32_t src2GlobalDimZ, vktVec3i_t first,
                                    vktVec3i_t last, vktVec3i_t dstOffset, vktHipSlabPiece_t* pieces,
                                    int32_t pieceCapacity, int32_t* numPieces, vktHipSlabMove_t* moves,
                                    int32_t moveCapacity, int32_t* numMoves, int32_t* bufPlanes);
/* The Range calls.  comm != NULL: one slab per process (numSlabs = 1, this rank's slab; rank
 * and world from the communicator), moves over RCCL in one group on the compute stream.
 * comm == NULL: the process holds every slab on the library's device (numSlabs ranks; slab i
 * is rank i), moves are device copies on the compute stream.  Returns once enqueued. */
VKTAPI vktError vktHipSlabFillRange(vktHipComm_t comm, int32_t numSlabs, vktHipSlab_t const* dst,
                                    vktVec3i_t first, vktVec3i_t last, float value);
VKTAPI vktError vktHipSlabCopyRange(vktHipComm_t comm, int32_t numSlabs, vktHipSlab_t const* dst,
                                    vktHipSlab_t const* src, vktVec3i_t first, vktVec3i_t last,
                                    vktVec3i_t dstOffset);
VKTAPI vktError vktHipSlabArithmeticRange(vktHipComm_t comm, vktHipArithmeticOp op, int32_t numSlabs,
                                          vktHipSlab_t const* dest, vktHipSlab_t const* source1,
                                          vktHipSlab_t const* source2, vktVec3i_t first, vktVec3i_t last,
                                          vktVec3i_t dstOffset);
/* TransformRange with a host callback over a Z-slab partitioned volume (Transform shards with
 * no exchange): rank `rank` of nranks transforms the planes it owns of the GLOBAL
 * range [first, last) of its slab; the callback sees global coordinates, in the serial order
 * within the rank (ranks 0..n-1 called in turn reproduce the whole serial loop).  Device
 * functors: vkt::TransformRangeSlab (include/volkit_transform.hpp). */
VKTAPI vktError vktHipSlabTransformRange1(int32_t nranks, int32_t rank, vktHipSlab_t slab, vktVec3i_t first,
                                          vktVec3i_t last, vktTransformUnaryOp unaryOp);
/* The local half of a Range call whose moves the CALLER carried out (volkit_amd/slab.py moves
 * them over torch.distributed): runs rank `rank`'s pieces, reading remote source planes from
 * gather1 / gather2 (device buffers holding bufPlanes[0] / bufPlanes[1] planes of source 1 / 2
 * in plan order; NULL when the plan reads none).  op is ignored unless kind is arithmetic. */
VKTAPI vktError vktHipSlabRangePieces(vktHipSlabOpKind kind, vktHipArithmeticOp op, int32_t nranks, int32_t rank,
                                      vktHipSlab_t dst, vktHipSlab_t const* source1, vktHipSlab_t const* source2,
                                      vktVec3i_t first, vktVec3i_t last, vktVec3i_t dstOffset, float value,
                                      void* gather1, void* gather2);

/* replaces TransformRange_cuda (reference src/vkt/Transform_cuda.hpp:12-30, an empty
 * stub there): host callbacks cannot run on the GPU, so the range is staged to host,
 * transformed in the serial order, and written back. */
VKTAPI vktError vktHipTransformRange1(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last,
                                      vktTransformUnaryOp unaryOp);
VKTAPI vktError vktHipTransformRange2(vktHipVolumeView_t volume1, vktHipVolumeView_t volume2,
                                      vktVec3i_t first, vktVec3i_t last, vktVec3i_t volume2Offset,
                                      vktTransformBinaryOp binaryOp);

/* One brick of a decomposition: CopyRange(brick, source, first, last, {0,0,0}). */
typedef struct {
    vktHipVolumeView_t brick;
    vktVec3i_t first;   /* may be negative / past the source (halo): source reads clamp */
    vktVec3i_t last;
} vktHipBrickRange_t;

/* replaces BrickDecompose_cuda (reference src/vkt/Decompose_cuda.cu:8-26, an empty stub);
 * semantics of BrickDecompose_serial (src/vkt/Decompose_serial.hpp:15-46), i.e. one
 * CopyRange per brick.  All bricks whose format and mapping equal the source's are copied
 * by ONE batched kernel launch; the others go through the CopyRange conversion path.
 * Every range is validated against its brick before anything is launched. */
VKTAPI vktError vktHipBrickDecompose(vktHipVolumeView_t source, vktHipBrickRange_t const* bricks,
                                     int32_t numBricks);

/* A uniform brick grid: numBricks = ceil(source dims / brickSize) per axis (reference
 * Decompose.cpp:103-121); brick (ix, iy, iz), linear index ix + nbx * (iy + nby * iz), holds the
 * source box [c - haloNeg, c + size + haloPos), c = (ix, iy, iz) * brickSize, size = brickSize
 * except the last brick of an axis (the remainder). */
typedef struct vktHipBrickGrid_t
{
    vktVec3i_t numBricks;
    vktVec3i_t brickSize;
    vktVec3i_t haloNeg;
    vktVec3i_t haloPos;
} vktHipBrickGrid_t;

/* BrickDecompose of a uniform grid whose bricks are allocated exactly at their box size in the
 * source's data format and voxel mapping (what BrickDecomposeResize builds), brick i's voxels
 * at brickData[i] on the device.  The CALLER guarantees those dims / formats / mappings (the
 * C / C++ front-ends check them per brick and otherwise call vktHipBrickDecompose); this checks
 * the grid against the source, the pointers (non-null, none inside the source) and copies from
 * the brick index alone -- no per-brick range list, no descriptor table: one pass over the
 * bricks on the host instead of two (same bytes as vktHipBrickDecompose on the equivalent
 * ranges; grids the index-derived kernel cannot take go through that path internally).
 * brickData is read before the call returns. */
VKTAPI vktError vktHipBrickDecomposeGrid(vktHipVolumeView_t source, vktHipBrickGrid_t grid, uint8_t* const* brickData);

/* ---- reductions --------------------------------------------------
 * replaces ComputeAggregatesRange_cuda (declared by reference src/vkt/Aggregates_cuda.hpp,
 * never implemented); semantics of ComputeAggregatesRange_serial
 * (src/vkt/Aggregates_serial.hpp:20-83): min/max/argmin/argmax bit-exact (first occurrence
 * in z,y,x order), sum/prod/var accumulated in double from the reference's per-voxel float
 * terms (within the serial path's own rounding error), mean and var divided by the voxel
 * count of the WHOLE volume like the reference. */
VKTAPI vktError vktHipAggregatesRange(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last,
                                      vktAggregates_t* aggregates);

/* Partial aggregates, for combining Z-slabs of one volume across ranks (multi-GPU): pass 1
 * fills min/max (with GLOBAL linear voxel indices: z + zGlobalOffset), sum, prod, count;
 * pass 2 fills sumSq = sum of (v - mean)^2 with the reference's float difference and square.
 * Combine partials of all slabs (vktHipAggregatePartialCombine, associative), derive the
 * float mean of the whole volume (vktHipAggregatesMean), run pass 2, combine, then
 * vktHipAggregatesFinish. */
typedef struct {
    double sum, prod, sumSq;
    float minValue, maxValue;
    uint64_t minIndex, maxIndex;   /* global linear index z*dimY*dimX + y*dimX + x; ~0 = none */
    uint64_t count;
} vktHipAggregatePartial_t;
VKTAPI vktError vktHipAggregatePartialInit(vktHipAggregatePartial_t* partial);
VKTAPI vktError vktHipAggregatePartialCombine(vktHipAggregatePartial_t* acc, vktHipAggregatePartial_t const* other);
VKTAPI float vktHipAggregatesMean(vktHipAggregatePartial_t const* pass1, uint64_t numElems);
VKTAPI vktError vktHipAggregatesPass(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last,
                                     int32_t zGlobalOffset, int32_t pass, float mean,
                                     vktHipAggregatePartial_t* partial);
VKTAPI vktError vktHipAggregatesFinish(vktHipAggregatePartial_t const* pass1, vktHipAggregatePartial_t const* pass2,
                                       uint64_t numElems, int32_t dimX, int32_t dimY, vktAggregates_t* aggregates);
/* UInt8 / UInt16 slabs in ONE pass (the code-count form of vktHipAggregatesRange, DESIGN.md
 * §4.8): every rank counts the codes of its range (vktHipAggregateCodeCounts: a DEVICE array of
 * 256 / 65 536 uint64 counters, overwritten); the counts are summed over the ranks (one
 * all-reduce); vktHipAggregatesFromCodes turns the global counts into pass 1 (sum, prod, count,
 * min / max values; indices ~0) and pass 2 (sumSq) and names the code holding each extreme
 * (codes[0] min, codes[1] max; -1 when the counts cannot tell which voxel comes first: a mapping
 * that rounds two present codes onto an extreme or a non-finite value -- then use the two
 * passes); each rank searches its range for the first voxels with those codes
 * (vktHipAggregateFirstCodes, global indices as vktHipAggregatesPass, ~0 = none), the minimum
 * over ranks fills pass1.minIndex / maxIndex, and vktHipAggregatesFinish completes.
 * vktHipAggregateCodesSupported: 1 when the range takes the code-count walk (a 16-B aligned
 * volume with dimX % 8 == 0; empty ranges too), else 0. */
VKTAPI int32_t vktHipAggregateCodesSupported(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last);
VKTAPI vktError vktHipAggregateCodeCounts(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last,
                                          uint64_t* counts);
VKTAPI vktError vktHipAggregatesFromCodes(uint64_t const* counts, int32_t dataFormat, float mappingLo, float mappingHi,
                                          uint64_t numElems, vktHipAggregatePartial_t* pass1,
                                          vktHipAggregatePartial_t* pass2, int32_t* codes);
VKTAPI vktError vktHipAggregateFirstCodes(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last,
                                          int32_t zGlobalOffset, int32_t minCode, int32_t maxCode,
                                          uint64_t* indices);
/* Slabs in ONE pass of moments (the moments forms of vktHipAggregatesRange, DESIGN.md §4.8:
 * UInt16 -- exact integer moments under the unit mapping, float moments otherwise -- and
 * Float32): every rank reduces its range to one vktHipMomentPartial_t (vktHipAggregateMoments;
 * global indices as vktHipAggregatesPass; an empty range gives count 0), the partials are
 * exchanged (e.g. one all-gather of sizeof(vktHipMomentPartial_t) bytes per rank) and
 * vktHipAggregatesFromMoments combines them IN THE ORDER GIVEN (rank order: deterministic) and
 * finishes the aggregates of the whole volume.  *complete = 0 when the float form's terms may
 * leave the normal float range (non-finite / huge / tiny values: use the two passes, as
 * vktHipAggregatesRange does); every rank gets the same answer from the same partials.
 * vktHipAggregateMoments returns vktInvalidValue for a format / range that takes no moments
 * form (vktHipAggregateMomentsSupported: 1 when it does, empty ranges included). */
typedef struct {
    uint64_t count;
    uint64_t codeSum, codeSumSqLo, codeSumSqHi;   /* form 1: sum of the codes, 128-bit sum of their squares */
    double mean, m2;                             /* form 2: mean, sum of squared deviations of the values */
    double sum, prod;                            /* form 2: sum; both forms: product of the values */
    float minValue, maxValue;
    uint64_t minIndex, maxIndex;                 /* global linear indices, ~0 = none */
    int32_t form;                                /* 1 integer (UInt16, unit mapping), 2 float */
    uint32_t flags;                              /* form 2: bit 0 non-finite value, bit 1 tiny value */
} vktHipMomentPartial_t;
VKTAPI int32_t vktHipAggregateMomentsSupported(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last);
VKTAPI vktError vktHipAggregateMoments(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last,
                                       int32_t zGlobalOffset, vktHipMomentPartial_t* partial);
VKTAPI vktError vktHipAggregatesFromMoments(vktHipMomentPartial_t const* partials, int32_t numPartials,
                                            uint64_t numElems, int32_t dimX, int32_t dimY,
                                            vktAggregates_t* aggregates, int32_t* complete);

/* replaces ComputeHistogramRange_cuda (reference src/vkt/Histogram_cuda.cu:45-76, which
 * ignores `first`); semantics of ComputeHistogramRange_serial (src/vkt/Histogram_serial.hpp:
 * 20-50): bins[(size_t)((v - lo) * ((float)numBins / (hi - lo)))]++ over the range.  `bins`
 * is a DEVICE array of numBins uint64 counters; zeroed first unless `accumulate` (slab
 * partial histograms summed in place / all-reduced).  Indices the reference would write out
 * of bounds (v outside [lo, hi], NaN) are not counted. */
VKTAPI vktError vktHipHistogramRange(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last, uint64_t* bins,
                                     uint64_t numBins, int32_t accumulate);

/* ---- rendering (reference src/vkt/Render_kernel.hpp) -----------------
 * One frame = one sample per pixel of the reference's RayMarching / ImplicitIso /
 * MultiScattering kernels, accumulated as accum = (1 - 1/f)*accum + (1/f)*sample
 * (AccumulationKernel::accum).  Camera basis precomputed on the host: the primary ray of
 * pixel (x, y) (y = 0 is the bottom row) with jitter (jx, jy) has direction
 * normalize(W + sx*U + sy*V), sx = 2(x+jx)/width - 1, sy = 2(y+jy)/height - 1; a thin lens of
 * radius lensRadius refocuses it at focalDistance along W.  Volume texture: nearest, clamp
 * (Render.cpp:446-447), unorm values (code / 255 or / 65535; Float32 normalised by its
 * mapping); transfer function: RGBA32F nearest / clamp, or none. */
typedef struct {
    int32_t algo;                 /* vktRenderAlgo: 0 RayMarching, 1 ImplicitIso, 2 MultiScattering */
    int32_t width, height;
    uint32_t frameBegin;          /* frames frameBegin+1 .. frameBegin+numFrames; 0 = clear */
    float eye[3], U[3], V[3], W[3], right[3], up[3];
    float lensRadius, focalDistance;
    float bbox[3];                /* object box [0, bbox] = dims * dist */
    float dtRayMarching, dtImplicitIso, majorant;
    int32_t numIsoSurfaces;
    float isoSurfaces[10];
    int32_t sRGB;
    float const* lut;             /* device RGBA32F table, or NULL */
    int32_t lutSize;
} vktHipRenderParams_t;
/* accum / color: device arrays of width*height RGBA floats (row-major, row 0 = bottom);
 * color = sRGB(accum) when params->sRGB. */
VKTAPI vktError vktHipRender(vktHipVolumeView_t volume, vktHipRenderParams_t const* params, float* accum,
                             float* color, int32_t numFrames);
/* The parameter block vkt::Render / vktRenderSV build from a render state (camera from
 * initialCamera or view_all of the box; lut left NULL). */
VKTAPI vktError vktHipRenderParamsFromState(vktRenderState_t const* renderState, vktVec3f_t bbox,
                                            vktHipRenderParams_t* params);

/* Synthetic benchmark/test input: byte i of the volume = byte (i % 8) of
 * splitmix64(seed + (i / 8)) -- counter-based, so the oracle reproduces it exactly
 * (oracle/vkt_oracle.c: vkt_oracle_synth). */
VKTAPI vktError vktHipSynthesize(vktHipVolumeView_t volume, uint64_t seed);

#ifdef __cplusplus
}
#endif

#endif /* VOLKIT_HIP_H */
