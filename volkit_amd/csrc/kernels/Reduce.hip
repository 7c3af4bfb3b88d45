// Reduce.hip -- ComputeAggregates / ComputeHistogram on gfx950.
//
// Reference semantics (the serial path; the CUDA Aggregates is a missing stub and the CUDA
// Histogram ignores `first`, src/vkt/Histogram_cuda.cu:27-40):
//  * ComputeAggregatesRange_serial (src/vkt/Aggregates_serial.hpp:20-83): min/max updated on
//    a strict `<` / `>` in z->y->x order starting from +FLT_MAX / -FLT_MAX (so NaN and values
//    at or beyond +-FLT_MAX never become min/max; argmin/argmax = first occurrence, {0,0,0}
//    if none); mean and sum = float accumulation of the values; prod = float product;
//    mean /= N and var = sum((v - mean)^2) / N where N is the voxel count of the WHOLE volume
//    (not the range; :61-63, :80); stddev = sqrtf(var).
//  * ComputeHistogramRange_serial (src/vkt/Histogram_serial.hpp:20-50): bins zeroed, then
//    bins[(size_t)((v - lo) * (numBins / (hi - lo)))]++ with float arithmetic.
//
// Exactness: min/max/argmin/argmax and every histogram count are bit-exact.  The float sums
// of the reference are order-dependent; here sum, prod and sum((v-mean)^2) accumulate the same
// per-voxel float terms in double precision with a deterministic tree (run-to-run identical)
// and round once -- equal to the serial result within the serial path's own rounding error
// (tests state the bound).  Histogram indices outside [0, numBins) and NaN, which the
// reference writes out of bounds (UB), are not counted.
//
// MI355X design: one wave per range row (x across lanes, coalesced), grid-stride over rows
// with ~8 workgroups per CU; per-wave shuffle reductions, LDS across waves, one partial per
// workgroup, a single-workgroup tree for the final result (no float atomics: deterministic).
// Histogram: per-workgroup LDS bins (u32) when they fit, flushed with 64-bit global atomics;
// a wave whose 64 voxels fall into one bin adds them with one atomic.

#include "KernelCommon.hpp"
#include "../runtime/Runtime.hpp"
#include "volkit_hip.h"

#include <cfloat>
#include <cmath>
#include <algorithm>
#include <cstring>
#include <mutex>
#include <unordered_map>

namespace vkt
{
namespace hipk
{
    bool validView(vktHipVolumeView_t const& v);

    struct BoxArgs
    {
        uint8_t const* data;
        int32_t dimX, dimY;         // volume pitch
        int32_t fx, fy, fz;         // range origin (voxel coordinates of the local buffer)
        int32_t nx;
        uint32_t rows;              // ny * nz
        FastDiv fdNy;
        int32_t fmt;
        float lo, hi;
        int64_t zGlobal;            // added to z for global linear indices (Z-slab offset)
    };

    // Visits every voxel of the range: one wave per row, grid-stride over rows.  VEC (rows
    // start on an 8-voxel boundary, row length a multiple of 8, 16-B aligned base): lane l
    // loads voxels [8l + 512k, +8) with one 8/16/32-byte load, two chunks in flight per lane.
    // visit(value, x-offset in the row, row base index of the local buffer, z, y).
    template <int BPV, bool VEC, class Visit>
    __device__ __forceinline__ void forEachVoxel(BoxArgs const& a, Visit&& visit)
    {
        int const lane = threadIdx.x & 63;
        uint32_t const wavesPerBlock = blockDim.x >> 6;
        uint32_t const totalWaves = gridDim.x * wavesPerBlock;
        for (uint32_t r = blockIdx.x * wavesPerBlock + (threadIdx.x >> 6); r < a.rows; r += totalWaves)
        {
            uint32_t const zr = fdiv(r, a.fdNy);
            uint32_t const yr = r - zr * a.fdNy.d;
            int64_t const z = a.fz + static_cast<int64_t>(zr), y = a.fy + static_cast<int64_t>(yr);
            uint64_t const rowBase = (static_cast<uint64_t>(z) * static_cast<uint64_t>(a.dimY) + static_cast<uint64_t>(y)) *
                                         static_cast<uint64_t>(a.dimX) +
                                     static_cast<uint64_t>(a.fx);
            if constexpr (VEC)
            {
                for (int32_t x0 = 8 * lane; x0 < a.nx; x0 += 2 * 512)
                {
                    uint32_t c0[8], c1[8];
                    int32_t const x1 = x0 + 512;
                    bool const has1 = x1 < a.nx;
                    load8<BPV>(a.data, rowBase + static_cast<uint64_t>(x0), c0);
                    load8<BPV>(a.data, rowBase + static_cast<uint64_t>(has1 ? x1 : x0), c1);
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        visit(codec::decode(c0[i], a.fmt, a.lo, a.hi), x0 + i, z, y);
                    if (has1)
                    {
#pragma unroll
                        for (int i = 0; i < 8; ++i)
                            visit(codec::decode(c1[i], a.fmt, a.lo, a.hi), x1 + i, z, y);
                    }
                }
            }
            else
            {
                for (int32_t x = lane; x < a.nx; x += 64)
                    visit(codec::decode(loadCode<BPV>(a.data, rowBase + static_cast<uint64_t>(x)), a.fmt, a.lo, a.hi), x,
                          z, y);
            }
        }
    }

    // ---- Aggregates ---------------------------------------------------------------------
    constexpr uint64_t kNoIndex = ~0ull;

    __device__ __forceinline__ void minCombine(float& v, uint64_t& i, float v2, uint64_t i2)
    {
        if (v2 < v || (v2 == v && i2 < i))
        {
            v = v2;
            i = i2;
        }
    }

    __device__ __forceinline__ void maxCombine(float& v, uint64_t& i, float v2, uint64_t i2)
    {
        if (v2 > v || (v2 == v && i2 < i))
        {
            v = v2;
            i = i2;
        }
    }

    __device__ __forceinline__ double shflXorD(double v, int m)
    {
        return __shfl_xor(v, m);
    }

    __device__ __forceinline__ uint64_t shflXorU(uint64_t v, int m)
    {
        uint32_t lo = __shfl_xor(static_cast<uint32_t>(v), m);
        uint32_t hi = __shfl_xor(static_cast<uint32_t>(v >> 32), m);
        return (static_cast<uint64_t>(hi) << 32) | lo;
    }

    // Whole-wave / workgroup reduction of a partial (lane 0 of the block ends with it); WAVES =
    // the workgroup's waves.
    template <int WAVES = kBlock / 64>
    __device__ void blockReduce(vktHipAggregatePartial_t& p)
    {
        for (int m = 32; m >= 1; m >>= 1)
        {
            float mv = __shfl_xor(p.minValue, m), xv = __shfl_xor(p.maxValue, m);
            uint64_t mi = shflXorU(p.minIndex, m), xi = shflXorU(p.maxIndex, m);
            double s = shflXorD(p.sum, m), q = shflXorD(p.prod, m), s2 = shflXorD(p.sumSq, m);
            uint64_t c = shflXorU(p.count, m);
            minCombine(p.minValue, p.minIndex, mv, mi);
            maxCombine(p.maxValue, p.maxIndex, xv, xi);
            p.sum += s;
            p.prod *= q;
            p.sumSq += s2;
            p.count += c;
        }
        __shared__ vktHipAggregatePartial_t lds[WAVES];
        int const wave = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0)
            lds[wave] = p;
        __syncthreads();
        if (threadIdx.x == 0)
        {
            for (int w = 1; w < static_cast<int>(blockDim.x >> 6); ++w)
            {
                vktHipAggregatePartial_t const& o = lds[w];
                minCombine(p.minValue, p.minIndex, o.minValue, o.minIndex);
                maxCombine(p.maxValue, p.maxIndex, o.maxValue, o.maxIndex);
                p.sum += o.sum;
                p.prod *= o.prod;
                p.sumSq += o.sumSq;
                p.count += o.count;
            }
        }
    }

    __device__ __forceinline__ vktHipAggregatePartial_t emptyPartial()
    {
        vktHipAggregatePartial_t p;
        p.sum = 0.0;
        p.prod = 1.0;
        p.sumSq = 0.0;
        p.minValue = FLT_MAX;
        p.maxValue = -FLT_MAX;
        p.minIndex = kNoIndex;
        p.maxIndex = kNoIndex;
        p.count = 0;
        return p;
    }

    // PASS 1: min/argmin/max/argmax/sum/prod/count.  PASS 2: sumSq of (v - mean)^2 with the
    // float difference and square of the reference, mean read from `meanPtr` (device) when
    // non-null, else `meanValue`.
    template <int PASS, int BPV, bool VEC>
    __global__ __launch_bounds__(kBlock) void aggregatesKernel(BoxArgs a, float const* meanPtr, float meanValue,
                                                              vktHipAggregatePartial_t* partials)
    {
        float const mean = PASS == 2 ? (meanPtr ? *meanPtr : meanValue) : 0.f;
        vktHipAggregatePartial_t p = emptyPartial();
        uint64_t const px = static_cast<uint64_t>(a.dimX), py = static_cast<uint64_t>(a.dimY);
        forEachVoxel<BPV, VEC>(a, [&](float v, int32_t x, int64_t z, int64_t y) {
            if constexpr (PASS == 1)
            {
                if (v < p.minValue || v > p.maxValue)   // rare after the first voxels: index math only then
                {
                    uint64_t const gi = (static_cast<uint64_t>(z + a.zGlobal) * py + static_cast<uint64_t>(y)) * px +
                                        static_cast<uint64_t>(a.fx + x);
                    if (v < p.minValue)   // v < FLT_MAX implied by the FLT_MAX start
                    {
                        p.minValue = v;
                        p.minIndex = gi;
                    }
                    if (v > p.maxValue)
                    {
                        p.maxValue = v;
                        p.maxIndex = gi;
                    }
                }
                p.sum += static_cast<double>(v);
                p.prod *= static_cast<double>(v);
                p.count += 1;
            }
            else
            {
                float const d = v - mean;
                float const d2 = d * d;
                p.sumSq += static_cast<double>(d2);
            }
        });
        blockReduce(p);
        if (threadIdx.x == 0)
            partials[blockIdx.x] = p;
    }

    // One workgroup reduces n partials into out[0]; optionally derives the reference's float
    // mean for pass 2: mean = (float)((double)(float)sum / numElems).
    __global__ __launch_bounds__(kBlock) void aggregatesFinalKernel(vktHipAggregatePartial_t const* partials,
                                                                   uint32_t n, vktHipAggregatePartial_t* out,
                                                                   float* meanOut, double numElems)
    {
        vktHipAggregatePartial_t p = emptyPartial();
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
        {
            vktHipAggregatePartial_t const& o = partials[i];
            minCombine(p.minValue, p.minIndex, o.minValue, o.minIndex);
            maxCombine(p.maxValue, p.maxIndex, o.maxValue, o.maxIndex);
            p.sum += o.sum;
            p.prod *= o.prod;
            p.sumSq += o.sumSq;
            p.count += o.count;
        }
        blockReduce(p);
        if (threadIdx.x == 0)
        {
            *out = p;
            if (meanOut)
                *meanOut = static_cast<float>(static_cast<double>(static_cast<float>(p.sum)) / numElems);
        }
    }

    // ---- Histogram ----------------------------------------------------------------------
    struct HistArgs
    {
        unsigned long long* bins;
        uint64_t numBins;
        float scale;                // (float)numBins / (hi - lo), as the reference computes it
        int32_t useLds;
        uint64_t tileBase;          // LDS path: this launch counts bins [tileBase, tileBase + tileBins)
        uint32_t tileBins;
    };

    // bin of one value, or ~0 when the reference would index out of bounds / NaN
    __device__ __forceinline__ uint64_t binOf(float v, float lo, float scale, uint64_t numBins)
    {
        float const f = (v - lo) * scale;
        // (size_t)f on x86-64: truncation toward zero; (-1, 0) -> 0; NaN / negative -> OOB
        if (!(f > -1.0f) || !(f < 9.2233720e18f))
            return ~0ull;
        uint64_t const b = static_cast<uint64_t>(static_cast<int64_t>(f));
        return b < numBins ? b : ~0ull;
    }

    // u32 counters a workgroup may hold in LDS (device limit per workgroup, 64 KiB at least)
    uint32_t ldsBinCapacity()
    {
        static uint32_t const cap = [] {
            int bytes = 0;
            if (hipDeviceGetAttribute(&bytes, hipDeviceAttributeMaxSharedMemoryPerBlock, rt::device()) != hipSuccess ||
                bytes < 65536)
                bytes = 65536;
            return static_cast<uint32_t>(bytes / sizeof(uint32_t));
        }();
        return cap;
    }

    // Each lane run-length-combines consecutive voxels of the same bin before it touches the
    // counters (constant or smooth regions: one atomic per run instead of per voxel).
    template <int BPV, bool VEC>
    __global__ __launch_bounds__(kBlock) void histogramKernel(BoxArgs a, HistArgs h)
    {
        extern __shared__ uint32_t ldsBins[];
        uint32_t const nb = h.tileBins;
        if (h.useLds)
        {
            for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x)
                ldsBins[i] = 0;
            __syncthreads();
        }
        uint64_t runBin = ~0ull;
        uint32_t runCount = 0;
        auto flush = [&]() {
            if (runCount)
            {
                if (h.useLds)
                {
                    uint64_t const t = runBin - h.tileBase;   // wraps high for bins below the tile
                    if (t < nb)
                        atomicAdd(&ldsBins[static_cast<uint32_t>(t)], runCount);
                }
                else
                    atomicAdd(&h.bins[runBin], static_cast<unsigned long long>(runCount));
            }
        };
        forEachVoxel<BPV, VEC>(a, [&](float v, int32_t, int64_t, int64_t) {
            uint64_t const b = binOf(v, a.lo, h.scale, h.numBins);
            if (b == runBin)
            {
                runCount += b != ~0ull ? 1u : 0u;   // uncounted voxels never accumulate
                return;
            }
            flush();
            runBin = b;
            runCount = b != ~0ull ? 1u : 0u;
        });
        flush();
        if (h.useLds)
        {
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x)
            {
                uint32_t const c = ldsBins[i];
                if (c)
                    atomicAdd(&h.bins[h.tileBase + i], static_cast<unsigned long long>(c));
            }
        }
    }

    // ---- Histogram, streaming path (UInt8 / UInt16 / Float32, <= kFastMaxBins bins) --------
    // The per-voxel work of histogramKernel (runtime-format decode, 64-bit bin math, run
    // tracking) made it VALU-bound at ~2 TB/s; here the format is a template parameter, the bin
    // index is 32-bit and the counters live in LDS:
    //  * up to kReplicatedMaxBins bins (!TILED, 256-thread workgroups, 4 per CU): R = 2^rShift
    //    copies of each counter, interleaved so lane l adds to copy l mod R: with R = 32 the 32
    //    lanes of each LDS lane group hit 32 different banks (MI355X_MICROARCH.md §LDS:
    //    ds_write_b32/ds_add_u32 bank = (addr/4) mod 32).  Out-of-range / NaN voxels add to a
    //    trash row (bin nb) instead of branching.
    //  * more bins (TILED, one 1024-thread workgroup per CU holding up to ~40 K counters): one
    //    pass over the range per tile of bins, adds outside the tile masked off.
    // UInt8 looks the counter offset up in a 256-entry LDS table (its decode has a true IEEE
    // division); UInt16 / Float32 evaluate decode and the bin in packed f32 pairs
    // (v_pk_mul/add_f32, the same roundings as the scalar form: no contraction).
    // Items: 8 consecutive voxels of one range row; a wave takes 4 x 64 items per step (all
    // loads in flight before the first atomic), grid-stride; CONTIG ranges are one span.
    constexpr uint32_t kReplicatedMaxBins = 10240;
    constexpr uint32_t kP16Flush = 0x4000u;   // packed 16-bit counters: moved to HBM at 2^14
    constexpr uint32_t kFastMaxTiles = 8;
    constexpr uint32_t kPairMaxTiles = 4;   // PAIR: tiles side by side in one launch
    constexpr int kTileBlock = 1024;

    struct FastHistArgs
    {
        uint8_t const* data;        // CONTIG: first voxel of the span; else the volume base
        uint64_t items;             // 8-voxel items in the range
        FastDiv fdIpr, fdNy;        // non-CONTIG: items per row, rows per plane of the range
        int32_t dimX, dimY, fx, fy, fz;
        float lo, hi, scale, nbf;
        uint32_t nb, rShift;
        uint32_t binShift;          // SHIFT: bin = (code * binMul) >> binShift
        uint32_t binMul;            // 1 for the power-of-two bins; numBins for UInt16 mul-shift bins
        uint32_t p16Step;           // P16: threshold tests once per wave-step (knob histogram.p16_step)
        uint32_t tileBase, tileBins;   // TILED: this launch counts bins [tileBase, +tileBins)
        unsigned long long* bins;
        uint64_t giBase;            // aggregates, CONTIG: global linear index of the span start
        int64_t zGlobal;            // aggregates: Z-slab offset added to z for global indices
        // padded rows (range rows starting or ending off the 8-voxel grid): items cover each row
        // from px0 = fx & ~7 to the 8-aligned end; voxels outside [rx0, rx1) are not visited
        int32_t px0, rx0, rx1;
        uint32_t padded;
        uint32_t rows;              // codeCountsU8RowsKernel: range rows (ny * nz)
        uint32_t pairTiles;         // PAIR: tiles counted side by side in one launch (tileBins each)
        uint32_t* partials;         // TILED, not PAIR: per-workgroup counts [blockIdx.x][tileBins] (no atomics)
    };

    typedef float f32x2 __attribute__((ext_vector_type(2)));

    __device__ __forceinline__ uint32_t fastBin(float f, float nbf, uint32_t nb)
    {
        // == binOf for numBins <= 2^24: -1 < f < numBins <=> 0 <= (size_t)f < numBins
        return (f > -1.0f && f < nbf) ? static_cast<uint32_t>(static_cast<int32_t>(f)) : nb;
    }

    // first voxel of 8-voxel item `item` (offset into h.data); non-CONTIG items < 2^32
    template <bool CONTIG>
    __device__ __forceinline__ uint64_t spanVoxel(FastHistArgs const& h, uint64_t item)
    {
        if constexpr (CONTIG)
            return item * 8;
        else
        {
            uint32_t const i = static_cast<uint32_t>(item);
            uint32_t const r = fdiv(i, h.fdIpr);
            uint32_t const xi = i - r * h.fdIpr.d;
            uint32_t const zr = fdiv(r, h.fdNy);
            uint32_t const yr = r - zr * h.fdNy.d;
            return ((static_cast<uint64_t>(h.fz + zr) * static_cast<uint64_t>(h.dimY) + (h.fy + yr)) *
                        static_cast<uint64_t>(h.dimX) +
                    static_cast<uint64_t>(h.px0)) +
                   8ull * xi;
        }
    }

    // Valid voxels of item `item` (bit j = voxel j): all of them except in padded rows' end items.
    template <bool CONTIG>
    __device__ __forceinline__ uint32_t itemMask(FastHistArgs const& h, uint64_t item)
    {
        if (CONTIG || !h.padded)
            return 0xFFu;
        uint32_t const i = static_cast<uint32_t>(item);
        uint32_t const xi = i - fdiv(i, h.fdIpr) * h.fdIpr.d;
        int32_t const x0 = h.px0 + 8 * static_cast<int32_t>(xi);
        if (x0 >= h.rx0 && x0 + 8 <= h.rx1)
            return 0xFFu;
        uint32_t m = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            m |= (x0 + j >= h.rx0 && x0 + j < h.rx1) ? 1u << j : 0u;
        return m;
    }

    // spanVoxel and itemMask of one item from ONE row division (the two computed apart divided the
    // item index twice per item on the non-CONTIG walks)
    template <bool CONTIG>
    __device__ __forceinline__ uint64_t spanVoxelMask(FastHistArgs const& h, uint64_t item, uint32_t& mask)
    {
        if constexpr (CONTIG)
        {
            mask = 0xFFu;
            return item * 8;
        }
        else
        {
            uint32_t const i = static_cast<uint32_t>(item);
            uint32_t const r = fdiv(i, h.fdIpr);
            uint32_t const xi = i - r * h.fdIpr.d;
            uint32_t const zr = fdiv(r, h.fdNy);
            uint32_t const yr = r - zr * h.fdNy.d;
            int32_t const x0 = h.px0 + 8 * static_cast<int32_t>(xi);
            uint32_t m = 0xFFu;
            if (h.padded && !(x0 >= h.rx0 && x0 + 8 <= h.rx1))
            {
                m = 0;
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    m |= (x0 + j >= h.rx0 && x0 + j < h.rx1) ? 1u << j : 0u;
            }
            mask = m;
            return ((static_cast<uint64_t>(h.fz + zr) * static_cast<uint64_t>(h.dimY) + (h.fy + yr)) *
                        static_cast<uint64_t>(h.dimX) +
                    static_cast<uint64_t>(h.px0)) +
                   8ull * xi;
        }
    }

    // SHIFT: the bin of every code is code >> binShift, so one shift replaces the decode, the
    // range test and the conversion (UInt16) or the LDS table read (UInt8).  UInt16: taken
    // for the unit mapping (+0, 1) and numBins = 2^k, k <= 16, where decode(c) = c * 2^-16
    // exactly (codec::decodeUnit), scale = numBins / 1 = 2^k, and f = c * 2^(k-16) is exact and
    // in [0, numBins), so the reference's (size_t)((v - lo) * scale) is c >> (16 - k).
    // UInt8: taken when the host evaluation of all 256 bins (hostBinU8) is such a shift.
    // Mul-shift (UInt16, any other bin count <= 2^16): bin = (code * numBins) >> 16 whenever the
    // host evaluation of the kernel's float formula over all 65 536 codes (hostBinU16) gives
    // exactly that -- e.g. the unit mapping with numBins = o * 2^j, o <= 256 (c * numBins * 2^-16
    // is then exact in f32), or mapping [0, 2] with 1000 bins.  One v_mul_u32_u24 and a shift
    // instead of the decode, the range test and the conversion (10 240 bins: 0.48 -> see DESIGN).
    //
    // P16 (TILED, UInt16 / Float32, more bins than one tile of 32-bit counters -- a UInt16
    // histogram with one bin per code): two 16-bit counters per LDS word, so up to ~80 K bins
    // take ONE pass instead of one pass per tile.  A half must never reach 2^16 (its carry
    // would corrupt the neighbour, and a wrap could not be told from the neighbour's carry):
    // a lane whose add returned a half >= kP16Flush moves kP16Flush from that half to the bin
    // in HBM with a compare-and-swap that succeeds only while the half still holds that much.
    // Every move is exact whatever the order of the racing adds and movers (and whatever an
    // LDS atomic returns to same-address lanes of one instruction), a half never goes below
    // 0, and it stays < 2^16 unless 49 152 adds to that one counter land while every lane
    // that saw it above the threshold is still on its way to the CAS.  Adds here are 1 per
    // lane (wave-uniform items go to the run registers below), and same-address lanes of an
    // LDS atomic serialise (measured: ~2 cycles per lane), so that needs the movers stalled
    // for ~100 000 cycles while the other waves of the workgroup keep issuing; a context save
    // stops the whole workgroup.  (A first version flushed on exactly kP16Flush - 1 returned:
    // 60 moves went missing on 64 Mi voxels alternating between the two halves of one word.)
    //
    // PAIR (TILED, not P16; knob histogram.pair_tiles): the T = h.pairTiles tiles of 32-bit
    // counters in ONE launch instead of one launch per tile.  Workgroups b and b + 8 run on the
    // same XCD (workgroups are dealt to the 8 XCDs round robin), so the T workgroups of a group
    // -- same XCD, one tile each -- walk the same items side by side: the first read of an item
    // comes from HBM, the others from that XCD's L2.  Each voxel is decoded T times but added
    // once, with non-returning LDS adds (no 16-bit halves to watch).
    template <int FMT, bool CONTIG, bool TILED, int BLOCK, bool SHIFT = false, bool P16 = false, bool PAIR = false>
    __global__ __launch_bounds__(BLOCK) void histogramFastKernel(FastHistArgs hArg)
    {
        static_assert(!PAIR || (TILED && !P16), "PAIR: tiles of 32-bit counters");
        FastHistArgs h = hArg;
        uint32_t group = blockIdx.x, groups = gridDim.x;
        if constexpr (PAIR)
        {
            uint32_t const T = h.pairTiles;
            uint32_t const tile = (blockIdx.x >> 3) % T;
            group = (blockIdx.x / (8u * T)) * 8u + (blockIdx.x & 7u);
            groups = gridDim.x / T;
            h.tileBase = tile * h.tileBins;
            h.tileBins = min(h.tileBins, h.nb - h.tileBase);
        }
        constexpr int BPV = FMT == codec::FmtUInt8 ? 1 : FMT == codec::FmtUInt16 ? 2 : 4;
        constexpr int U = 4;
        constexpr uint32_t kOff = ~0u;   // UInt8 table: code outside the tile
        extern __shared__ uint32_t cnt[];
        __shared__ uint32_t lut[FMT == codec::FmtUInt8 ? 256 : 1];
        uint32_t const rowShift = h.rShift + 2;   // byte offset of a counter row
        static_assert(!P16 || (TILED && FMT != codec::FmtUInt8), "P16: tiled UInt16 / Float32");
        uint32_t const total = TILED ? (P16 ? (h.tileBins + 1) / 2 : h.tileBins) : (h.nb + 1) << h.rShift;
        for (uint32_t i = threadIdx.x; i < total; i += BLOCK)
            cnt[i] = 0;
        if constexpr (FMT == codec::FmtUInt8 && !SHIFT)
        {
            for (uint32_t c = threadIdx.x; c < 256; c += BLOCK)
            {
                float const v = codec::decode(c, codec::FmtUInt8, h.lo, h.hi);
                uint32_t const b = fastBin((v - h.lo) * h.scale, h.nbf, h.nb);
                if constexpr (TILED)
                    lut[c] = b - h.tileBase < h.tileBins ? (b - h.tileBase) << 2 : kOff;
                else
                    lut[c] = b << rowShift;
            }
        }
        __syncthreads();
        uint32_t const lane = threadIdx.x & 63;
        // this lane's copy of counter row 0; row b is at + (b << rowShift) (one v_lshl_add)
        char* const cLane = reinterpret_cast<char*>(cnt) + (TILED ? 0u : (lane & ((1u << h.rShift) - 1u)) << 2);

        uint32_t runBin = ~0u, runCount = 0u;   // TILED: the wave's run of uniform voxels
        auto add = [&](uint32_t b) {
            if constexpr (TILED)
            {
                uint32_t const t = b - h.tileBase;
                if (t < h.tileBins)
                    atomicAdd(&cnt[t], 1u);
            }
            else
                atomicAdd(reinterpret_cast<uint32_t*>(cLane + (b << rowShift)), 1u);
        };
        // The 8 bins of an item.  TILED (no counter replicas): an item whose 8 voxels are on one
        // bin in every active lane of the wave (constant regions -- empty space) never touches
        // LDS: the wave counts it in a run register (runBin, runCount; identical in every lane, lane 0
        // always active) that goes to HBM with one 64-bit atomic when the wave's uniform bin
        // changes and at the end.  64 lanes adding to one LDS word serialise: a constant 1024^3
        // volume took 3.5 ms against 0.33 ms streaming.  Other items add 1 per voxel.
        auto flushRun = [&] {
            if (runCount != 0u && lane == 0u)
                atomicAdd(&h.bins[h.tileBase + runBin], static_cast<unsigned long long>(runCount));
        };
        // TILED: an item whose 8 voxels are on one bin in every active lane goes to the run
        // register; true when it was taken.  One check per item -- first the wave-wide test of
        // voxel 0 (fails at once on varied data, one compare + ballot), the other 7 voxels only
        // when it holds.
        auto takeUniform = [&](uint32_t const (&b)[8]) -> bool {
            uint32_t const t0 = __builtin_amdgcn_readfirstlane(b[0] - h.tileBase);
            bool uniform = __all(b[0] - h.tileBase == t0);
            if (uniform)
            {
                bool same = true;
#pragma unroll
                for (int j = 1; j < 8; ++j)
                    same = same && b[j] == b[0];
                uniform = __all(same);
            }
            if (uniform && t0 < h.tileBins)
            {
                if (t0 != runBin)
                {
                    flushRun();
                    runBin = t0;
                    runCount = 0u;
                }
                runCount += 8u * static_cast<uint32_t>(__popcll(__activemask()));
            }
            return uniform;
        };
        // P16: the 8 returning adds of an item; returns the OR of the returned words
        auto p16Adds = [&](uint32_t const (&b)[8], uint32_t (&old)[8]) -> uint32_t {
            uint32_t any = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j)
            {
                uint32_t const t = b[j] - h.tileBase;
                old[j] = t < h.tileBins ? atomicAdd(&cnt[t >> 1], 1u << ((t & 1u) << 4)) : 0u;
                any |= old[j];
            }
            return any;
        };
        // P16: a lane whose add returned a half >= kP16Flush moves kP16Flush to HBM.  The tests
        // run only when the OR of the returned words has bit 14 or 15 of either half set (a
        // superset of "some half >= 2^14", almost never true on varied data).
        static_assert(kP16Flush == 0x4000u, "threshold bits");
        constexpr uint32_t kP16Bits = 0xC000C000u;
        auto p16Moves = [&](uint32_t const (&b)[8], uint32_t const (&old)[8]) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
            {
                uint32_t const t = b[j] - h.tileBase;
                uint32_t const sh = (t & 1u) << 4;
                if (t < h.tileBins && ((old[j] >> sh) & 0xFFFFu) >= kP16Flush)
                {
                    // move kP16Flush to HBM if the half still holds that much: a CAS, so
                    // racing movers never take more than is there
                    uint32_t cur = atomicAdd(&cnt[t >> 1], 0u);
                    while (((cur >> sh) & 0xFFFFu) >= kP16Flush)
                    {
                        uint32_t const prev = atomicCAS(&cnt[t >> 1], cur, cur - (kP16Flush << sh));
                        if (prev == cur)
                        {
                            atomicAdd(&h.bins[h.tileBase + t], static_cast<unsigned long long>(kP16Flush));
                            break;
                        }
                        cur = prev;
                    }
                }
            }
        };
        auto add8 = [&](uint32_t const (&b)[8]) {
            if constexpr (TILED)
            {
                if (takeUniform(b))
                    return;
                if constexpr (P16)
                {
                    uint32_t old[8];
                    if (p16Adds(b, old) & kP16Bits)
                        p16Moves(b, old);
                }
                else
                {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                    {
                        uint32_t const t = b[j] - h.tileBase;
                        if (t < h.tileBins)
                            atomicAdd(&cnt[t], 1u);
                    }
                }
            }
            else
            {
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    add(b[j]);
            }
        };
        // m: valid voxels of the item (padded rows); the others go to the trash row / no tile.
        // bins8: the 8 bins of an item (UInt16 / Float32; UInt8 counts through its LDS table)
        auto bins8 = [&](uint32_t const (&c)[8], uint32_t m, uint32_t (&b)[8]) {
            if constexpr (SHIFT)
            {
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    // (HIP's __umul24 returns int: codes >= 2^15 times 65 536 bins are negative)
                    b[j] = (m >> j) & 1u ? static_cast<uint32_t>(__umul24(c[j], h.binMul)) >> h.binShift : h.nb;
            }
            else
            {
#pragma unroll
                for (int j = 0; j < 8; j += 2)
                {
                    f32x2 v;
                    if constexpr (FMT == codec::FmtUInt16)
                    {
                        // decode: lerp(lo, hi, code / 65535.999f), 65535.999f == 2^16 (exact)
                        f32x2 const t = f32x2{static_cast<float>(c[j]), static_cast<float>(c[j + 1])} *
                                        (1.0f / 65536.0f);
                        f32x2 const s = 1.0f - t;
                        f32x2 const p = s * h.lo;
                        f32x2 const q = t * h.hi;
                        v = p + q;
                    }
                    else
                        v = f32x2{codec::bitsToFloat(c[j]), codec::bitsToFloat(c[j + 1])};
                    f32x2 const f = (v - h.lo) * h.scale;
                    b[j] = (m >> j) & 1u ? fastBin(f.x, h.nbf, h.nb) : h.nb;
                    b[j + 1] = (m >> (j + 1)) & 1u ? fastBin(f.y, h.nbf, h.nb) : h.nb;
                }
            }
        };
        auto count8 = [&](uint32_t const (&c)[8], uint32_t m) {
            if constexpr (FMT == codec::FmtUInt8 && !SHIFT)
            {
#pragma unroll
                for (int j = 0; j < 8; ++j)
                {
                    uint32_t const o = (m >> j) & 1u ? lut[c[j]] : (TILED ? kOff : h.nb << rowShift);
                    if (!TILED || o != kOff)
                        atomicAdd(reinterpret_cast<uint32_t*>(cLane + o), 1u);
                }
            }
            else
            {
                uint32_t b[8];
                bins8(c, m, b);
                add8(b);
            }
        };
        // P16, one wave-step of U items: every item's returning adds are in flight before the
        // (rare) threshold tests, which wait for the returns only once per step
        auto countStepP16 = [&](uint32_t const (&c)[U][8], uint32_t const (&msk)[U]) {
            uint32_t b[U][8], old[U][8];
            bool uni[U];
            uint32_t any = 0;
#pragma unroll
            for (int k = 0; k < U; ++k)
            {
                bins8(c[k], msk[k], b[k]);
                uni[k] = takeUniform(b[k]);
                if (!uni[k])
                    any |= p16Adds(b[k], old[k]);
            }
            if (any & kP16Bits)
            {
#pragma unroll
                for (int k = 0; k < U; ++k)
                    if (!uni[k])
                        p16Moves(b[k], old[k]);
            }
        };

        uint64_t const wave = static_cast<uint64_t>(group) * (BLOCK / 64) + (threadIdx.x >> 6);
        uint64_t const waves = static_cast<uint64_t>(groups) * (BLOCK / 64);
        uint64_t const steps = h.items / (64 * U);
        // Float32 spans: lane l's "item" of a 64-item block is the 4-voxel halves at 4l and
        // 256 + 4l, so each 16-B load instruction of the wave reads one contiguous KiB (a
        // histogram does not care which lane counts which voxel; two 16-B halves of a 32-B item
        // per lane had each instruction touch every other 16 B of 2 KiB)
        bool const halves = CONTIG && BPV == 4 && (reinterpret_cast<uintptr_t>(h.data) & 15u) == 0;
        for (uint64_t st = wave; st < steps; st += waves)
        {
            uint32_t c[U][8];
            if (halves)
            {
#pragma unroll
                for (int k = 0; k < U; ++k)
                {
                    uint8_t const* p = h.data + ((st * (64 * U) + k * 64) * 8 + 4 * lane) * 4;
                    u32x4 const x = loadVec<u32x4, true>(p), y = loadVec<u32x4, true>(p + 1024);
                    c[k][0] = x.x; c[k][1] = x.y; c[k][2] = x.z; c[k][3] = x.w;
                    c[k][4] = y.x; c[k][5] = y.y; c[k][6] = y.z; c[k][7] = y.w;
                }
            }
            uint32_t msk[U];
#pragma unroll
            for (int k = 0; k < U; ++k)
                msk[k] = 0xFFu;
            if (!halves)
            {
#pragma unroll
                for (int k = 0; k < U; ++k)
                    load8<BPV, true>(h.data, spanVoxelMask<CONTIG>(h, st * (64 * U) + k * 64 + lane, msk[k]), c[k]);
            }
            if (P16 && h.p16Step)
                countStepP16(c, msk);
            else
            {
#pragma unroll
                for (int k = 0; k < U; ++k)
                    count8(c[k], msk[k]);
            }
        }
        for (uint64_t it = steps * (64 * U) + wave * 64 + lane; it < h.items; it += waves * 64)
        {
            uint32_t c[8], m;
            load8<BPV, true>(h.data, spanVoxelMask<CONTIG>(h, it, m), c);
            count8(c, m);
        }
        if constexpr (TILED)
            flushRun();   // (every lane reconverged; lane 0 holds the run)
        __syncthreads();
        if constexpr (TILED)
        {
            if (!PAIR && h.partials != nullptr)
            {
                // this workgroup's counter words as they are (P16: two 16-bit counts per word),
                // every one written; histogramPartialsKernel sums them
                uint32_t const words = P16 ? (h.tileBins + 1) / 2 : h.tileBins;
                uint32_t* const out = h.partials + static_cast<uint64_t>(blockIdx.x) * words;
                for (uint32_t t = threadIdx.x; t < words; t += BLOCK)
                    __builtin_nontemporal_store(cnt[t], out + t);
            }
            else
            {
                for (uint32_t t = threadIdx.x; t < h.tileBins; t += BLOCK)
                {
                    uint32_t const c = P16 ? (cnt[t >> 1] >> ((t & 1u) << 4)) & 0xFFFFu : cnt[t];
                    if (c)
                        atomicAdd(&h.bins[h.tileBase + t], static_cast<unsigned long long>(c));
                }
            }
        }
        else
        {
            // sum the R copies of each bin (rotated start: the lanes of a group read different banks)
            uint32_t const R = 1u << h.rShift;
            for (uint32_t b = threadIdx.x; b < h.nb; b += BLOCK)
            {
                uint32_t sum = 0;
                for (uint32_t r = 0; r < R; ++r)
                    sum += cnt[(b << h.rShift) + ((r + b) & (R - 1))];
                if (sum)
                    atomicAdd(&h.bins[b], static_cast<unsigned long long>(sum));
            }
        }
    }

    // ---- Aggregates, streaming path (UInt8 / UInt16 / Float32, 8-voxel-aligned rows) -----
    // Same item walk as histogramFastKernel (4 x 64 items per wave-step, all loads in flight
    // first; CONTIG ranges one span) with a compile-time decode.  A lane visits its voxels in
    // increasing index order, so the strict </> updates keep the first occurrence within the
    // lane and minCombine/maxCombine (index tie-break) keep it across lanes: arg indices are
    // exact whatever the schedule.  Sums accumulate per lane in double, then the fixed
    // shuffle / LDS / partials tree (deterministic for a given grid).
    // UNIT: the mapping is the unit mapping (+0, 1), decode without the lerp (codec::decodeUnit).
    // CODES (UInt8, pass 1): no decode, no float terms and no compares -- every voxel of a UInt8
    // volume has one of 256 values, so the kernel only counts CODES (LDS counters, 2^rShift
    // copies, flushed to the 256 u64 bins h.bins; no partials).  The sums, the product, the second
    // pass's sum of squares and the extreme values follow from the 256 counts
    // (aggregatesCodesFinalKernel); the first occurrence of each extreme's code is searched from
    // the start of the range (aggregatesFindHeadKernel, which stops early): one pass over the
    // data instead of two.
    template <int PASS, int FMT, bool CONTIG, bool UNIT = false, bool CODES = false>
    __global__ __launch_bounds__(kBlock) void aggregatesFastKernel(FastHistArgs h, float const* meanPtr,
                                                                  float meanValue, vktHipAggregatePartial_t* partials)
    {
        constexpr int BPV = FMT == codec::FmtUInt8 ? 1 : FMT == codec::FmtUInt16 ? 2 : 4;
        constexpr int U = 4;
        static_assert(!CODES || (PASS == 1 && FMT == codec::FmtUInt8), "code counts: UInt8 pass 1");
        float const mean = PASS == 2 ? (meanPtr ? *meanPtr : meanValue) : 0.f;
        vktHipAggregatePartial_t p = emptyPartial();
        uint32_t const lane = threadIdx.x & 63;
        extern __shared__ uint32_t codeCnt[];
        uint32_t const rowShift = h.rShift + 2;
        char* const cLane = reinterpret_cast<char*>(codeCnt) + ((lane & ((1u << h.rShift) - 1u)) << 2);
        if constexpr (CODES)
        {
            for (uint32_t i = threadIdx.x; i < (256u << h.rShift); i += kBlock)
                codeCnt[i] = 0;
            __syncthreads();
        }
        uint64_t const px = static_cast<uint64_t>(h.dimX), py = static_cast<uint64_t>(h.dimY);
        // global linear index of voxel j of item `item`
        auto globalIndex = [&](uint64_t item, int j) -> uint64_t {
            if constexpr (CONTIG)
                return h.giBase + item * 8 + static_cast<uint64_t>(j);
            else
            {
                uint32_t const i = static_cast<uint32_t>(item);
                uint32_t const r = fdiv(i, h.fdIpr);
                uint32_t const xi = i - r * h.fdIpr.d;
                uint32_t const zr = fdiv(r, h.fdNy);
                uint32_t const yr = r - zr * h.fdNy.d;
                return (static_cast<uint64_t>(h.fz + zr + h.zGlobal) * py + static_cast<uint64_t>(h.fy + yr)) * px +
                       static_cast<uint64_t>(h.px0) + 8ull * xi + static_cast<uint64_t>(j);
            }
        };
        // hb (Float32 spans, `halves`): c holds the halves at 4l and 256 + 4l of the 64-item block
        // starting at item hb -- still in increasing index order per lane, which the first-
        // occurrence tie-break of argmin / argmax relies on
        auto visit8 = [&](uint32_t const (&c)[8], uint64_t item, uint64_t hb = ~0ull, uint32_t mIn = 0x100u) {
            uint32_t const m = mIn != 0x100u ? mIn : itemMask<CONTIG>(h, item);
            auto gIndex = [&](int j) -> uint64_t {
                if (CONTIG && hb != ~0ull)
                    return h.giBase + hb * 8 + 4 * lane + (j < 4 ? static_cast<uint64_t>(j) : 252ull + j);
                return globalIndex(item, j);
            };
            if constexpr (CODES)
            {
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if ((m >> j) & 1u)
                        atomicAdd(reinterpret_cast<uint32_t*>(cLane + (c[j] << rowShift)), 1u);
                return;
            }
            // pass 1 over spans: one test per item (its min / max against the lane's) instead of
            // one branch per voxel; the voxel-by-voxel strict updates run in order only when it
            // holds.  1024^3 UInt8 pass 1 272 -> 248 us; padded rows (non-CONTIG) lost 300 ->
            // 350 us with it (UInt16) and keep the per-voxel test.
            bool update = true;
            if constexpr (PASS == 1 && CONTIG)
            {
                float lo = FLT_MAX, hi = -FLT_MAX;
#pragma unroll
                for (int j = 0; j < 8; ++j)
                {
                    float const v = (m >> j) & 1u ? (UNIT ? codec::decodeUnit(c[j], FMT)
                                                          : codec::decode(c[j], FMT, h.lo, h.hi))
                                                  : p.minValue;
                    lo = fminf(lo, v);   // (NaN never qualifies: minNum / maxNum skip it)
                    hi = fmaxf(hi, v);
                }
                update = lo < p.minValue || hi > p.maxValue;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j)
            {
                if (!((m >> j) & 1u))
                    continue;   // padded rows: outside the range
                float const v = UNIT ? codec::decodeUnit(c[j], FMT) : codec::decode(c[j], FMT, h.lo, h.hi);
                if constexpr (PASS == 1)
                {
                    if (update && (v < p.minValue || v > p.maxValue))   // rare after the first voxels
                    {
                        uint64_t const gi = gIndex(j);
                        if (v < p.minValue)
                        {
                            p.minValue = v;
                            p.minIndex = gi;
                        }
                        if (v > p.maxValue)
                        {
                            p.maxValue = v;
                            p.maxIndex = gi;
                        }
                    }
                    p.sum += static_cast<double>(v);
                    p.prod *= static_cast<double>(v);
                }
                else
                {
                    float const d = v - mean;
                    float const d2 = d * d;
                    p.sumSq += static_cast<double>(d2);
                }
            }
            if constexpr (PASS == 1)
                p.count += __builtin_popcount(m);
        };
        uint64_t const wave = static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
        uint64_t const waves = static_cast<uint64_t>(gridDim.x) * (kBlock / 64);
        uint64_t const steps = h.items / (64 * U);
        bool const halves = CONTIG && BPV == 4 && (reinterpret_cast<uintptr_t>(h.data) & 15u) == 0;
        // UInt8 spans: lane l takes items 2l, 2l + 1 of each 128-item pair of blocks with one
        // 16-B load (8-B loads per lane otherwise); still increasing order per lane
        bool const pairs = CONTIG && BPV == 1 && U % 2 == 0 && (reinterpret_cast<uintptr_t>(h.data) & 15u) == 0;
        for (uint64_t st = wave; st < steps; st += waves)
        {
            uint32_t c[U][8];
            if (pairs)
            {
#pragma unroll
                for (int k = 0; k < U; k += 2)
                {
                    uint64_t const item = st * (64 * U) + static_cast<uint64_t>(k) * 64 + 2 * lane;
                    u32x4 const x = loadVec<u32x4, true>(h.data + item * 8);
                    uint32_t const w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                    {
                        c[k][i] = (w[i / 4] >> (8 * (i % 4))) & 0xFFu;
                        c[k + 1][i] = (w[2 + i / 4] >> (8 * (i % 4))) & 0xFFu;
                    }
                }
#pragma unroll
                for (int k = 0; k < U; k += 2)
                {
                    uint64_t const item = st * (64 * U) + static_cast<uint64_t>(k) * 64 + 2 * lane;
                    visit8(c[k], item);
                    visit8(c[k + 1], item + 1);
                }
            }
            else if (halves)   // contiguous 16-B lanes, as in histogramFastKernel
            {
#pragma unroll
                for (int k = 0; k < U; ++k)
                {
                    uint8_t const* p = h.data + ((st * (64 * U) + k * 64) * 8 + 4 * lane) * 4;
                    u32x4 const x = loadVec<u32x4, true>(p), y = loadVec<u32x4, true>(p + 1024);
                    c[k][0] = x.x; c[k][1] = x.y; c[k][2] = x.z; c[k][3] = x.w;
                    c[k][4] = y.x; c[k][5] = y.y; c[k][6] = y.z; c[k][7] = y.w;
                }
#pragma unroll
                for (int k = 0; k < U; ++k)
                    visit8(c[k], st * (64 * U) + k * 64 + lane, st * (64 * U) + k * 64);
            }
            else
            {
                uint32_t msk[U];
#pragma unroll
                for (int k = 0; k < U; ++k)
                    load8<BPV, true>(h.data, spanVoxelMask<CONTIG>(h, st * (64 * U) + k * 64 + lane, msk[k]), c[k]);
#pragma unroll
                for (int k = 0; k < U; ++k)
                    visit8(c[k], st * (64 * U) + k * 64 + lane, ~0ull, msk[k]);
            }
        }
        for (uint64_t it = steps * (64 * U) + wave * 64 + lane; it < h.items; it += waves * 64)
        {
            uint32_t c[8], m;
            load8<BPV, true>(h.data, spanVoxelMask<CONTIG>(h, it, m), c);
            visit8(c, it, ~0ull, m);
        }
        if constexpr (CODES)
        {
            __syncthreads();
            uint32_t const R = 1u << h.rShift;
            for (uint32_t b = threadIdx.x; b < 256u; b += kBlock)
            {
                uint32_t sum = 0;
                for (uint32_t r = 0; r < R; ++r)
                    sum += codeCnt[(b << h.rShift) + ((r + b) & (R - 1))];
                if (sum)
                    atomicAdd(&h.bins[b], static_cast<unsigned long long>(sum));
            }
            return;
        }
        blockReduce(p);
        if (threadIdx.x == 0)
            partials[blockIdx.x] = p;
    }

    // UInt8 code counts over range ROWS (the non-CONTIG form of aggregatesFastKernel<CODES>):
    // 16-voxel items, one aligned 16-B load per lane, covering each row from h.px0 = fx & ~15 to
    // the 16-aligned end (h.fdIpr = items per row; dimX % 16 == 0, 16-B aligned volume).  Counts
    // need no order and no mask: every loaded byte is counted, then the bytes of each row outside
    // [rx0, rx1) (at most 15 + 15, at the same offsets in every row) are subtracted again.  The
    // 8-voxel walk spent 3 fast divisions, a mask and 8 branches per 8 bytes, with 8-B loads:
    // an 800^3 sub-box of 1024^3 took longer than the whole 1024^3 volume.
    // INLOOP (rows of >= 9 items): each wave-step also subtracts the end bytes of the rows whose
    // first / last item lies in its 256 items -- lane l re-reads the first (l < 32) or last item
    // of row rA + l % 32, lines the step has just fetched; else a row walk after the main loop
    // (its end items are separate sectors fetched again from HBM: 800^3 sub-box at x0 = 100,
    // 139 us against 103 us for the same box at x0 = 0).
    // Counters: 32 copies (h.rShift = 5) as in aggregatesFastKernel; a workgroup's net count of a
    // code may be negative (its subtracted rows are not its counted items): the copies are summed
    // mod 2^32 and flushed sign-extended.
    template <bool INLOOP>
    __global__ __launch_bounds__(kBlock) void codeCountsU8RowsKernel(FastHistArgs h)
    {
        constexpr int U = 4;
        constexpr uint32_t kRowShift = 7;   // byte offset of a code's 32 counter copies
        extern __shared__ uint32_t codeCnt[];
        uint32_t const lane = threadIdx.x & 63;
        char* const cLane = reinterpret_cast<char*>(codeCnt) + ((lane & 31u) << 2);
        for (uint32_t i = threadIdx.x; i < (256u << 5); i += kBlock)
            codeCnt[i] = 0;
        __syncthreads();
        auto rowStart = [&](uint32_t r) -> uint8_t const* {
            uint32_t const zr = fdiv(r, h.fdNy);
            uint32_t const yr = r - zr * h.fdNy.d;
            return h.data + ((static_cast<uint64_t>(h.fz + zr) * static_cast<uint64_t>(h.dimY) + (h.fy + yr)) *
                                 static_cast<uint64_t>(h.dimX) +
                             static_cast<uint64_t>(h.px0));
        };
        auto itemPtr = [&](uint32_t i) -> uint8_t const* {
            uint32_t const r = fdiv(i, h.fdIpr);
            return rowStart(r) + 16u * (i - r * h.fdIpr.d);
        };
        auto addByte = [&](uint32_t c, uint32_t v) {
            atomicAdd(reinterpret_cast<uint32_t*>(cLane + (c << kRowShift)), v);
        };
        auto count16 = [&](u32x4 const& x) {
            uint32_t const w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    addByte(__builtin_amdgcn_ubfe(w[q], 8 * b, 8), 1u);
        };
        uint32_t const items = static_cast<uint32_t>(h.items);
        uint32_t const wave = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
        uint32_t const waves = gridDim.x * (kBlock / 64);
        int32_t const head = h.rx0 - h.px0;   // bytes [0, head) of a row's first item are outside
        int32_t const tail = h.rx1 - h.px0 - 16 * static_cast<int32_t>(h.fdIpr.d - 1);   // [tail, 16) of its last
        uint32_t const lastItem = 16u * (h.fdIpr.d - 1);
        if constexpr (INLOOP)
        {
            // every step whole-wave: the last one's items past the range are not counted
            uint32_t const steps = (items + 64 * U - 1) / (64 * U);
            bool const tailSide = lane >= 32;
            for (uint32_t st = wave; st < steps; st += waves)
            {
                uint32_t const s0 = st * (64 * U), s1 = min(s0 + 64 * U, items);
                u32x4 x[U];
#pragma unroll
                for (int k = 0; k < U; ++k)
                    x[k] = loadVec<u32x4, true>(itemPtr(min(s0 + k * 64 + lane, items - 1)));
                // the end items of this step's rows (first / last item inside [s0, s1))
                uint32_t const rA = fdiv(s0, h.fdIpr), rB = fdiv(s1 - 1, h.fdIpr);
                uint32_t const row = rA + (lane & 31u);
                uint32_t const ie = row * h.fdIpr.d + (tailSide ? h.fdIpr.d - 1 : 0u);
                bool const edge = row <= rB && ie >= s0 && ie < s1 && (tailSide ? tail < 16 : head > 0);
                u32x4 ex = {0u, 0u, 0u, 0u};
                if (edge)
                    ex = loadVec<u32x4, false>(rowStart(row) + (tailSide ? lastItem : 0u));
#pragma unroll
                for (int k = 0; k < U; ++k)
                    if (s0 + k * 64 + lane < s1)
                        count16(x[k]);
                uint32_t const w[4] = {ex.x, ex.y, ex.z, ex.w};
#pragma unroll
                for (int b = 0; b < 16; ++b)
                {
                    bool const out = tailSide ? b >= tail : b < head;
                    if (edge && out)
                        addByte(__builtin_amdgcn_ubfe(w[b / 4], 8 * (b % 4), 8), ~0u);
                }
            }
        }
        else
        {
            uint32_t const steps = items / (64 * U);
            for (uint32_t st = wave; st < steps; st += waves)
            {
                u32x4 x[U];
#pragma unroll
                for (int k = 0; k < U; ++k)
                    x[k] = loadVec<u32x4, true>(itemPtr(st * (64 * U) + k * 64 + lane));
#pragma unroll
                for (int k = 0; k < U; ++k)
                    count16(x[k]);
            }
            for (uint32_t it = steps * (64 * U) + wave * 64 + lane; it < items; it += waves * 64)
                count16(loadVec<u32x4, true>(itemPtr(it)));
        }
        if (!INLOOP && h.padded)
        {
            // subtract each row's bytes outside the range: bytes [0, head) of its first item and
            // [tail, 16) of its last -- the same offsets in every row (uniform branches); the two
            // items of RU rows are loaded before the first subtraction
            constexpr int RU = 4;
            uint32_t const rows = h.rows, stride = gridDim.x * kBlock;
            auto sub16 = [&](u32x4 const& x, int32_t b0, int32_t b1) {   // bytes [b0, b1) of x
                uint32_t const w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                for (int b = 0; b < 16; ++b)
                    if (b >= b0 && b < b1)
                        addByte(__builtin_amdgcn_ubfe(w[b / 4], 8 * (b % 4), 8), ~0u);
            };
            for (uint32_t r0 = blockIdx.x * kBlock + threadIdx.x; r0 < rows; r0 += RU * stride)
            {
                u32x4 hx[RU], tx[RU];
                bool live[RU];
#pragma unroll
                for (int u = 0; u < RU; ++u)
                {
                    uint32_t const r = r0 + u * stride;
                    live[u] = r < rows;
                    uint8_t const* const p = rowStart(live[u] ? r : r0);
                    hx[u] = loadVec<u32x4, true>(p);
                    tx[u] = loadVec<u32x4, true>(p + lastItem);
                }
#pragma unroll
                for (int u = 0; u < RU; ++u)
                    if (live[u])
                    {
                        sub16(hx[u], 0, head);
                        sub16(tx[u], tail, 16);
                    }
            }
        }
        __syncthreads();
        for (uint32_t c = threadIdx.x; c < 256u; c += kBlock)
        {
            uint32_t sum = 0;
            for (uint32_t r = 0; r < 32u; ++r)
                sum += codeCnt[(c << 5) + ((r + c) & 31u)];
            if (sum)
                atomicAdd(&h.bins[c], static_cast<unsigned long long>(static_cast<int64_t>(static_cast<int32_t>(sum))));
        }
    }

    // UInt8 aggregates from the code counts of aggregatesFastKernel<CODES>: one workgroup, thread
    // c = code c.  Each present code contributes count * its value to the sum, value^count to the
    // product and count * (float)((value - mean)^2) to the sum of squares -- the per-voxel float
    // terms of Aggregates_serial.hpp:37-80, summed in double in another order (the same parity
    // bound as the streaming passes).  min / max are the extreme VALUES among the present codes;
    // targets[0] / [1] the code holding each, whose first occurrence aggregatesFindHead/TailKernel
    // then write to res[0].minIndex / maxIndex.  res[1].count = 1 when the counts determine the
    // result: every present value finite and below FLT_MAX in magnitude and each extreme held by
    // ONE code (a mapping that rounds two present codes onto an extreme makes the caller rerun
    // the two float passes); 0 otherwise (targets -1).
    // PHASE 0: one workgroup runs both loops (UInt8: 256 threads, one code each).  UInt16 (65 536
    // codes) splits them over kCodeFinalBlocks workgroups of 1024 threads, one code each, in two
    // launches: PHASE 1 the first loop, PHASE 2 the second (it needs the mean and the value
    // extremes of all codes); in each, every workgroup publishes a partial and the LAST one to
    // finish (work->ticket) combines them in block order (deterministic).  One 1024-thread
    // workgroup running both loops over 65 536 codes (pow() per present code) took 139 us, the
    // multi-workgroup first loop with the second in the last workgroup 44 us.  work->ticket /
    // work->bad must be 0 at the PHASE 1 launch (PHASE 2's last workgroup leaves them 0).
    constexpr uint32_t kCodeFinalBlocks = 64;
    struct CodeFinalWork
    {
        uint32_t ticket, bad;
        float vmin, vmax, mean, pad[3];
        vktHipAggregatePartial_t parts[kCodeFinalBlocks];
        struct Second
        {
            double sumSq;
            int32_t nmin, nmax, cmin, cmax;
        } parts2[kCodeFinalBlocks];
    };

    // thread 0 of the last workgroup to arrive (after every workgroup's thread 0 published)
    __device__ __forceinline__ bool lastBlock(uint32_t* ticket, int32_t* sLast)
    {
        if (threadIdx.x == 0)
        {
            __threadfence();
            *sLast = atomicAdd(ticket, 1u) == gridDim.x - 1 ? 1 : 0;
        }
        __syncthreads();
        if (!*sLast)
            return false;
        __threadfence();
        return true;
    }

    template <int FMT, int PHASE>
    __global__ __launch_bounds__(FMT == codec::FmtUInt8 ? 256 : 1024) void aggregatesCodesFinalKernel(
        unsigned long long const* counts, float lo, float hi, double numElems, vktHipAggregatePartial_t* res,
        int32_t* targets, CodeFinalWork* work)
    {
        constexpr uint32_t kCodes = FMT == codec::FmtUInt8 ? 256u : 65536u;
        constexpr uint32_t kThreads = FMT == codec::FmtUInt8 ? 256u : 1024u;
        constexpr int kWaves = static_cast<int>(kThreads / 64);
        static_assert(PHASE == 0 || FMT == codec::FmtUInt16, "UInt16 splits the loops");
        __shared__ float sVmin, sVmax, sMean;
        __shared__ int32_t sNmin, sNmax, sCmin, sCmax, sBad, sLast;
        if (threadIdx.x == 0)
        {
            sNmin = sNmax = sBad = 0;
            sCmin = sCmax = -1;
        }
        __syncthreads();
        uint32_t const c0 = blockIdx.x * kThreads + threadIdx.x, cStride = gridDim.x * kThreads;
        vktHipAggregatePartial_t q = emptyPartial();
        if constexpr (PHASE != 2)
        {
            for (uint32_t c = c0; c < kCodes; c += cStride)
            {
                unsigned long long const cnt = counts[c];
                if (cnt == 0ull)
                    continue;
                float const v = codec::decode(c, FMT, lo, hi);
                if (!(fabsf(v) < FLT_MAX))
                    atomicOr(&sBad, 1);
                minCombine(q.minValue, q.minIndex, v, c);
                maxCombine(q.maxValue, q.maxIndex, v, c);
                double const dv = static_cast<double>(v), dn = static_cast<double>(cnt);
                q.sum += dn * dv;
                q.prod *= cnt == 1ull ? dv : pow(dv, dn);
                q.count += cnt;
            }
            if constexpr (PHASE == 1)
            {
                blockReduce<kWaves>(q);
                if (threadIdx.x == 0)
                {
                    work->parts[blockIdx.x] = q;
                    if (sBad)
                        atomicOr(&work->bad, 1u);
                }
                if (!lastBlock(&work->ticket, &sLast))
                    return;
                q = emptyPartial();
                if (threadIdx.x < gridDim.x)
                {
                    // (other workgroups' stores: read past this CU's L1)
                    vktHipAggregatePartial_t const volatile& o = work->parts[threadIdx.x];
                    q.sum = o.sum;
                    q.prod = o.prod;
                    q.count = o.count;
                    q.minValue = o.minValue;
                    q.maxValue = o.maxValue;
                    q.minIndex = o.minIndex;
                    q.maxIndex = o.maxIndex;
                }
            }
            blockReduce<kWaves>(q);
            __syncthreads();
            if (threadIdx.x == 0)
            {
                sVmin = q.minValue;
                sVmax = q.maxValue;
                sMean = static_cast<float>(static_cast<double>(static_cast<float>(q.sum)) / numElems);
                vktHipAggregatePartial_t out = q;   // thread 0: sum / prod / count / value extremes
                out.sumSq = 0.0;
                out.minIndex = kNoIndex;   // set by aggregatesFindHead/TailKernel
                out.maxIndex = kNoIndex;
                res[0] = out;
                if constexpr (PHASE == 1)
                {
                    work->vmin = sVmin;
                    work->vmax = sVmax;
                    work->mean = sMean;
                    work->ticket = 0u;
                }
            }
            if constexpr (PHASE == 1)
                return;
        }
        else if (threadIdx.x == 0)
        {
            sVmin = work->vmin;   // (PHASE 1's stores: a kernel boundary lies between)
            sVmax = work->vmax;
            sMean = work->mean;
        }
        __syncthreads();
        vktHipAggregatePartial_t t = emptyPartial();
        for (uint32_t c = PHASE == 2 ? c0 : threadIdx.x; c < kCodes; c += PHASE == 2 ? cStride : kThreads)
        {
            unsigned long long const cnt = counts[c];
            if (cnt == 0ull)
                continue;
            float const v = codec::decode(c, FMT, lo, hi);
            if (v == sVmin)
            {
                atomicAdd(&sNmin, 1);
                sCmin = static_cast<int32_t>(c);
            }
            if (v == sVmax)
            {
                atomicAdd(&sNmax, 1);
                sCmax = static_cast<int32_t>(c);
            }
            float const d = v - sMean;
            float const d2 = d * d;
            t.sumSq += static_cast<double>(cnt) * static_cast<double>(d2);
        }
        blockReduce<kWaves>(t);
        __syncthreads();
        if constexpr (PHASE == 2)
        {
            if (threadIdx.x == 0)
                work->parts2[blockIdx.x] = CodeFinalWork::Second{t.sumSq, sNmin, sNmax, sCmin, sCmax};
            if (!lastBlock(&work->ticket, &sLast))
                return;
            // every partial loaded at once (one volatile load after another from thread 0 cost a
            // memory latency each: 47 us), then summed in block order by thread 0
            __shared__ CodeFinalWork::Second sParts[kCodeFinalBlocks];
            if (threadIdx.x < gridDim.x)
            {
                CodeFinalWork::Second const volatile& o = work->parts2[threadIdx.x];
                sParts[threadIdx.x] = CodeFinalWork::Second{o.sumSq, o.nmin, o.nmax, o.cmin, o.cmax};
            }
            __syncthreads();
            if (threadIdx.x == 0)
            {
                t.sumSq = 0.0;
                sNmin = sNmax = 0;
                sCmin = sCmax = -1;
                for (uint32_t b = 0; b < gridDim.x; ++b)
                {
                    CodeFinalWork::Second const& o = sParts[b];
                    t.sumSq += o.sumSq;
                    sNmin += o.nmin;
                    sNmax += o.nmax;
                    sCmin = o.cmin >= 0 ? o.cmin : sCmin;
                    sCmax = o.cmax >= 0 ? o.cmax : sCmax;
                }
                sBad = static_cast<int32_t>(*static_cast<uint32_t volatile*>(&work->bad));
                work->ticket = 0u;
                work->bad = 0u;
            }
        }
        if (threadIdx.x == 0)
        {
            bool const ok = sBad == 0 && sNmin == 1 && sNmax == 1;
            vktHipAggregatePartial_t two = emptyPartial();
            two.sumSq = t.sumSq;
            two.count = ok ? 1u : 0u;
            res[1] = two;
            targets[0] = ok ? sCmin : -1;
            targets[1] = ok ? sCmax : -1;
        }
    }

    // global linear index of voxel j of 8-voxel item `item` of a span walk (FastHistArgs)
    template <bool CONTIG>
    __device__ __forceinline__ uint64_t spanGlobalIndex(FastHistArgs const& h, uint64_t item, int j)
    {
        if constexpr (CONTIG)
            return h.giBase + item * 8 + static_cast<uint64_t>(j);
        else
        {
            uint32_t const i = static_cast<uint32_t>(item);
            uint32_t const r = fdiv(i, h.fdIpr);
            uint32_t const xi = i - r * h.fdIpr.d;
            uint32_t const zr = fdiv(r, h.fdNy);
            uint32_t const yr = r - zr * h.fdNy.d;
            return (static_cast<uint64_t>(h.fz + zr + h.zGlobal) * static_cast<uint64_t>(h.dimY) +
                    static_cast<uint64_t>(h.fy + yr)) *
                       static_cast<uint64_t>(h.dimX) +
                   static_cast<uint64_t>(h.px0) + 8ull * xi + static_cast<uint64_t>(j);
        }
    }

    // ---- Aggregates in ONE pass of exact integer moments (UInt16, unit mapping) ----------------
    // Under the unit mapping (+0, 1) a UInt16 voxel's value is v = c * 2^-16 exactly
    // (codec::decodeUnit), so everything Aggregates_serial.hpp:37-80 derives from the values
    // follows from integer sums over the codes, exactly: sum = Sc * 2^-16, and the second pass's
    // sum of squares about the float mean m is
    //     S = 2^-32 * sum (c - mu)^2 = 2^-32 * ((n Sc2 - Sc^2) + (Sc - n mu)^2) / n,   mu = m * 2^16,
    // with Sc = sum c (u64) and Sc2 = sum c^2 (128-bit), so the data is read once.  min / max /
    // argmin / argmax follow the codes (v is strictly increasing in c), first occurrence exact as in
    // aggregatesFastKernel (a lane visits its voxels in increasing index order, the combines
    // tie-break on the index).  prod multiplies the values in double as the other paths do.
    // Per lane and 16-B item (8 codes in 4 dwords w):
    //  * Sc: v_dot2_u32_u16(w, {1, 1}) -- 1 instruction per 2 codes;
    //  * Sc2: c^2 = 2^16 h^2 + r with h = c >> 8, r = 512 h l + l^2 < 2^25: per dword
    //    H += dot2(hb, hb) (hb = the two high bytes) and Q += dot2(w, w) mod 2^32; per wave-step
    //    (32 codes) R = Q - 2^16 H mod 2^32 is the exact sum of the r (< 2^30), so
    //    Sc2 += 2^16 H + R -- 3 instructions per 2 codes, exact;
    //  * extremes: v_pk_min/max_u16 over the 4 dwords, the in-order per-voxel update only when the
    //    item can improve the lane's (rare after the first items);
    //  * prod: (c0 c1) exact in v_mul_u32_u24, four pair products in double scaled by 2^-128 --
    //    skipped once every lane's product is +0 (it stays 0: the values are finite).
    // Voxels outside the range in padded rows' end items (mask m != 0xFF) are masked in the
    // packed words (0 for the sums, 0xFFFF for the min bound, code 2^16 = value 1 for prod).
    // The float paths needed a decode, two double adds / multiplies and float min/max per voxel,
    // plus either a second pass over the data or a 65 536-code LDS count.
    struct MomentPartialU16
    {
        uint64_t count, sumC, sumSqLo, sumSqHi;
        double prod;
        uint32_t cmin;     // 0x10000: none
        int32_t cmax;      // -1: none
        uint64_t minIndex, maxIndex;
    };

    typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));

    __device__ __forceinline__ u16x2 asU16x2(uint32_t w) { return __builtin_bit_cast(u16x2, w); }

    __device__ __forceinline__ void momentCombine(MomentPartialU16& p, MomentPartialU16 const& o)
    {
        uint64_t const lo = p.sumSqLo + o.sumSqLo;
        p.sumSqHi += o.sumSqHi + (lo < p.sumSqLo ? 1u : 0u);
        p.sumSqLo = lo;
        p.count += o.count;
        p.sumC += o.sumC;
        p.prod *= o.prod;
        if (o.cmin < p.cmin || (o.cmin == p.cmin && o.minIndex < p.minIndex))
        {
            p.cmin = o.cmin;
            p.minIndex = o.minIndex;
        }
        if (o.cmax > p.cmax || (o.cmax == p.cmax && o.maxIndex < p.maxIndex))
        {
            p.cmax = o.cmax;
            p.maxIndex = o.maxIndex;
        }
    }

    __device__ __forceinline__ MomentPartialU16 shflXorMoment(MomentPartialU16 const& p, int m)
    {
        MomentPartialU16 o;
        o.count = shflXorU(p.count, m);
        o.sumC = shflXorU(p.sumC, m);
        o.sumSqLo = shflXorU(p.sumSqLo, m);
        o.sumSqHi = shflXorU(p.sumSqHi, m);
        o.prod = shflXorD(p.prod, m);
        o.cmin = __shfl_xor(p.cmin, m);
        o.cmax = __shfl_xor(p.cmax, m);
        o.minIndex = shflXorU(p.minIndex, m);
        o.maxIndex = shflXorU(p.maxIndex, m);
        return o;
    }

    // wave butterfly, then the workgroup's waves in order through LDS (thread 0 ends with it)
    template <int WAVES>
    __device__ void momentBlockReduce(MomentPartialU16& p)
    {
        for (int m = 32; m >= 1; m >>= 1)
            momentCombine(p, shflXorMoment(p, m));
        __shared__ MomentPartialU16 lds[WAVES];
        if ((threadIdx.x & 63) == 0)
            lds[threadIdx.x >> 6] = p;
        __syncthreads();
        if (threadIdx.x == 0)
            for (int w = 1; w < WAVES; ++w)
                momentCombine(p, lds[w]);
    }

    // U items per lane and wave-step; PIPE: the next step's loads are issued before this step's
    // arithmetic (two register buffers), so a wave keeps 16 U bytes per lane in flight while it
    // computes -- without it the loads of a step wait behind the previous step's ALU work.
    // waves per SIMD each variant is built for (without a bound the one-buffer 4-item span kernel
    // took 76 VGPRs: 6 waves; bound to 8 it fits 56 with no spill; the row form spills at 8)
    constexpr int momentWaves(bool contig, int u, bool pipe)
    {
        return pipe ? 4 : u <= 4 ? (contig ? 8 : 6) : (contig ? 6 : 4);
    }

    // WAVES: the launch bound's waves per SIMD (0: momentWaves).  The two-buffer 4-item span kernel
    // takes 76 VGPRs unbounded (6 waves); bound to 7 it fits 72 with 12 B spilled outside the walk
    // (bound to 8, 64 VGPRs, the spills land inside it).
    template <bool CONTIG, int U, bool PIPE, int WAVES = 0>
    __global__ __launch_bounds__(kBlock, WAVES ? WAVES : momentWaves(CONTIG, U, PIPE)) void aggregatesMomentsU16Kernel(FastHistArgs h, MomentPartialU16* partials)
    {
        uint32_t const lane = threadIdx.x & 63;
        MomentPartialU16 p;
        p.count = p.sumC = p.sumSqLo = p.sumSqHi = 0;
        p.prod = 1.0;
        p.cmin = 0x10000u;
        p.cmax = -1;
        p.minIndex = p.maxIndex = kNoIndex;
        uint32_t sc = 0, hq = 0, q = 0, cnt = 0;   // this step's Sc, H, Q and count (see above)
        auto addSq = [&](uint64_t x) {
            uint64_t const lo = p.sumSqLo + x;
            p.sumSqHi += lo < x ? 1u : 0u;
            p.sumSqLo = lo;
        };
        auto flushStep = [&] {
            uint32_t const r = q - (hq << 16);   // exact: the r of <= 8 U codes sum to < 2^30
            addSq((static_cast<uint64_t>(hq) << 16) + r);
            p.sumC += sc;
            p.count += cnt;
            sc = hq = q = cnt = 0;
        };
        // in-order strict updates of the lane's extremes over the valid voxels of one item
        auto extremes = [&](uint32_t const (&w)[4], uint32_t m, uint64_t item) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
            {
                uint32_t const c = (w[j / 2] >> (16 * (j % 2))) & 0xFFFFu;
                if (((m >> j) & 1u) && (c < p.cmin || static_cast<int32_t>(c) > p.cmax))
                {
                    uint64_t const gi = spanGlobalIndex<CONTIG>(h, item, j);
                    if (c < p.cmin)
                    {
                        p.cmin = c;
                        p.minIndex = gi;
                    }
                    if (static_cast<int32_t>(c) > p.cmax)
                    {
                        p.cmax = static_cast<int32_t>(c);
                        p.maxIndex = gi;
                    }
                }
            }
        };
        // one item's sums; mn / mx collect the step's packed extremes bounds.  Voxels outside the
        // range (padded row ends, mask m != 0xFF) enter the sums as 0, the min bound as 0xFFFF
        // and the product as 1 (code 2^16): the same packed instructions for every item.
        auto item8 = [&](uint32_t const (&w)[4], uint32_t m, bool prodLive, u16x2& mn, u16x2& mx) {
            u16x2 const one = {1, 1};
            uint32_t xs[4], xm[4];
            double pf = 1.0;
            if (m == 0xFFu)
            {
#pragma unroll
                for (int d = 0; d < 4; ++d)
                    xs[d] = xm[d] = w[d];
                if (prodLive)
                {
                    double pr[4];
#pragma unroll
                    for (int d = 0; d < 4; ++d)
                        pr[d] = static_cast<double>(static_cast<uint32_t>(__umul24(w[d] & 0xFFFFu, w[d] >> 16)));
                    pf = ((pr[0] * pr[1]) * (pr[2] * pr[3])) * 0x1p-128;
                }
            }
            else
            {
                double pr[4];
#pragma unroll
                for (int d = 0; d < 4; ++d)
                {
                    bool const kl = (m >> (2 * d)) & 1u, kh = (m >> (2 * d + 1)) & 1u;
                    uint32_t const keep = (kl ? 0xFFFFu : 0u) | (kh ? 0xFFFF0000u : 0u);
                    xs[d] = w[d] & keep;
                    xm[d] = w[d] | ~keep;
                    uint32_t const lo = kl ? (w[d] & 0xFFFFu) : 0x10000u, hi = kh ? (w[d] >> 16) : 0x10000u;
                    pr[d] = static_cast<double>(lo) * static_cast<double>(hi);   // exact (< 2^33)
                }
                if (prodLive)
                    pf = ((pr[0] * pr[1]) * (pr[2] * pr[3])) * 0x1p-128;
            }
#pragma unroll
            for (int d = 0; d < 4; ++d)
            {
                u16x2 const x = asU16x2(xs[d]);
                mn = __builtin_elementwise_min(mn, asU16x2(xm[d]));
                mx = __builtin_elementwise_max(mx, x);
                sc = __builtin_amdgcn_udot2(x, one, sc, false);
                // the two high bytes as u16 (v_perm_b32: bytes 1, 3 of the dword, zeros above)
                u16x2 const hb = asU16x2(__builtin_amdgcn_perm(0u, xs[d], 0x0C030C01u));
                hq = __builtin_amdgcn_udot2(hb, hb, hq, false);
                q = __builtin_amdgcn_udot2(x, x, q, false);
            }
            if (prodLive)
                p.prod *= pf;
            cnt += CONTIG ? 8u : static_cast<uint32_t>(__popc(m));
        };
        // a wave-step of U items: sums, then -- only when the step's packed bounds can improve
        // the lane's extremes (rare after the first steps) -- the in-order per-voxel updates
        // The lane's extremes per wave-step, branch-free: a step that holds a new strict minimum
        // (maximum) records its code and the step's base item; the first voxel of that code in
        // that step -- the lane's first occurrence, every earlier step held only larger (smaller)
        // codes -- is looked up once after the walk (resolveStep).  Every item holds a voxel of the
        // range, so the masked packed bounds are the step's true extremes.  (Per-voxel updates
        // inside the step cost ~3x the step's sums: with 64 lanes some lane improves in most
        // of a wave's few dozen steps, and the whole wave runs the divergent branch.)
        uint32_t minStep = ~0u, maxStep = ~0u;   // (steps < 2^32: 2^32 steps would be >= 16 TiB of codes)
        auto doStep = [&](uint32_t const (&w)[U][4], uint32_t const (&msk)[U], uint32_t st, bool prodLive) {
            u16x2 mn = {0xFFFFu, 0xFFFFu}, mx = {0, 0};
#pragma unroll
            for (int k = 0; k < U; ++k)
                item8(w[k], msk[k], prodLive, mn, mx);
            uint32_t const imin = mn.x < mn.y ? mn.x : mn.y, imax = mx.x > mx.y ? mx.x : mx.y;
            bool const lower = imin < p.cmin, higher = static_cast<int32_t>(imax) > p.cmax;
            p.cmin = lower ? imin : p.cmin;
            minStep = lower ? st : minStep;
            p.cmax = higher ? static_cast<int32_t>(imax) : p.cmax;
            maxStep = higher ? st : maxStep;
            flushStep();
        };
        // index of the first voxel with code c in step st (its items reloaded)
        auto resolveStep = [&](uint32_t st, uint32_t c) -> uint64_t {
            uint64_t const base = static_cast<uint64_t>(st) * (64 * U);
            uint64_t at = kNoIndex;
            for (int k = U - 1; k >= 0; --k)
            {
                uint32_t m;
                uint64_t const item = base + static_cast<uint64_t>(k) * 64 + lane;
                u32x4 const x = loadVec<u32x4, false>(h.data + 2 * spanVoxelMask<CONTIG>(h, item, m));
                uint32_t const w[4] = {x.x, x.y, x.z, x.w};
                for (int j = 7; j >= 0; --j)
                    if (((m >> j) & 1u) && ((w[j / 2] >> (16 * (j % 2))) & 0xFFFFu) == c)
                        at = spanGlobalIndex<CONTIG>(h, item, j);
            }
            return at;
        };
        auto loadStep = [&](uint64_t base, uint32_t (&w)[U][4], uint32_t (&msk)[U]) {
#pragma unroll
            for (int k = 0; k < U; ++k)
            {
                u32x4 const x = loadVec<u32x4, true>(h.data + 2 * spanVoxelMask<CONTIG>(h, base + k * 64 + lane, msk[k]));
                w[k][0] = x.x; w[k][1] = x.y; w[k][2] = x.z; w[k][3] = x.w;
            }
        };
        uint64_t const wave = static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
        uint64_t const waves = static_cast<uint64_t>(gridDim.x) * (kBlock / 64);
        uint64_t const steps = h.items / (64 * U);
        if constexpr (PIPE)
        {
            uint32_t wa[U][4], ma[U], wb[U][4], mb[U];
            uint64_t st = wave;
            if (st < steps)
                loadStep(st * (64 * U), wa, ma);
            while (st < steps)   // wave-uniform
            {
                uint64_t const s1 = st + waves;
                if (s1 < steps)
                    loadStep(s1 * (64 * U), wb, mb);
                doStep(wa, ma, static_cast<uint32_t>(st), __any(p.prod != 0.0));
                if (s1 >= steps)
                    break;
                uint64_t const s2 = s1 + waves;
                if (s2 < steps)
                    loadStep(s2 * (64 * U), wa, ma);
                doStep(wb, mb, static_cast<uint32_t>(s1), __any(p.prod != 0.0));
                st = s2;
            }
        }
        else
        {
            for (uint64_t st = wave; st < steps; st += waves)
            {
                uint32_t w[U][4], msk[U];
                loadStep(st * (64 * U), w, msk);
                doStep(w, msk, static_cast<uint32_t>(st), __any(p.prod != 0.0));
            }
        }
        if (minStep != ~0u)
            p.minIndex = resolveStep(minStep, p.cmin);
        if (maxStep != ~0u)
            p.maxIndex = resolveStep(maxStep, static_cast<uint32_t>(p.cmax));
        for (uint64_t it = steps * (64 * U) + wave * 64 + lane; it < h.items; it += waves * 64)
        {
            uint32_t w[1][4], m[1];
            u32x4 const x = loadVec<u32x4, true>(h.data + 2 * spanVoxelMask<CONTIG>(h, it, m[0]));
            w[0][0] = x.x; w[0][1] = x.y; w[0][2] = x.z; w[0][3] = x.w;
            u16x2 mn = {0xFFFFu, 0xFFFFu}, mx = {0, 0};
            item8(w[0], m[0], true, mn, mx);
            extremes(w[0], m[0], it);
            flushStep();
        }
        momentBlockReduce<kBlock / 64>(p);
        if (threadIdx.x == 0)
            partials[blockIdx.x] = p;
    }

    // One workgroup: the n partials of aggregatesMomentsU16Kernel (thread t combines t, t + 256,
    // ... in order, then the fixed tree) -> res[0] (pass-1 fields) and res[1].sumSq = S with
    // res[1].count = 1 (the result is complete: no fallback).  numElems: voxels of the WHOLE
    // volume (the reference divides by it, Aggregates_serial.hpp:61-63).
    __global__ __launch_bounds__(kBlock) void aggregatesMomentsU16FinalKernel(MomentPartialU16 const* partials,
                                                                             uint32_t n, double numElems,
                                                                             vktHipAggregatePartial_t* res)
    {
        MomentPartialU16 p;
        p.count = p.sumC = p.sumSqLo = p.sumSqHi = 0;
        p.prod = 1.0;
        p.cmin = 0x10000u;
        p.cmax = -1;
        p.minIndex = p.maxIndex = kNoIndex;
        for (uint32_t i = threadIdx.x; i < n; i += kBlock)
            momentCombine(p, partials[i]);
        momentBlockReduce<kBlock / 64>(p);
        if (threadIdx.x != 0)
            return;
        vktHipAggregatePartial_t one = emptyPartial();
        one.count = p.count;
        one.sum = static_cast<double>(p.sumC) * 0x1p-16;   // exact (Sc < 2^53)
        one.prod = p.prod;
        if (p.cmin <= 0xFFFFu)
        {
            one.minValue = static_cast<float>(p.cmin) * 0x1p-16f;
            one.minIndex = p.minIndex;
        }
        if (p.cmax >= 0)
        {
            one.maxValue = static_cast<float>(p.cmax) * 0x1p-16f;
            one.maxIndex = p.maxIndex;
        }
        // the reference's float mean (Aggregates_serial.hpp:61-63, as vktHipAggregatesFinish)
        float const m = static_cast<float>(static_cast<double>(static_cast<float>(one.sum)) / numElems);
        double const mu = static_cast<double>(m) * 65536.0;
        unsigned __int128 const sc2 = (static_cast<unsigned __int128>(p.sumSqHi) << 64) | p.sumSqLo;
        unsigned __int128 const t = static_cast<unsigned __int128>(p.count) * sc2 -
                                    static_cast<unsigned __int128>(p.sumC) * p.sumC;   // n Sc2 - Sc^2 >= 0
        double const td = static_cast<double>(static_cast<uint64_t>(t >> 64)) * 0x1p64 +
                          static_cast<double>(static_cast<uint64_t>(t));
        double const dn = static_cast<double>(p.count);
        double const r = fma(-dn, mu, static_cast<double>(p.sumC));   // Sc - n mu, one rounding
        vktHipAggregatePartial_t two = emptyPartial();
        two.sumSq = p.count ? (td + r * r) / dn * 0x1p-32 : 0.0;
        two.count = 1u;
        res[0] = one;
        res[1] = two;
    }

    // ---- Aggregates in ONE pass of floating-point moments (UInt16 other mappings, Float32) ----
    // The values are not integers here, so the sum of squares about the float mean m comes from
    // per-lane moments about a pivot K (the lane's first value): S1 = sum (v - K), S2 = sum
    // (v - K)^2 in double (v - K is exact in double for floats), per lane mean = K + S1/n and
    // M2 = S2 - S1^2/n, combined across lanes / waves / workgroups with the pairwise update
    // (Chan et al.): M2 = M2a + M2b + delta^2 na nb / n -- no cancellation beyond one lane's
    // values.  Then S = M2 + n (mean - m)^2: the EXACT sum (v - m)^2 to ~2^-50, where the
    // reference's float terms fl(fl(v - m)^2) each lie within 3 * 2^-24 of (v - m)^2 (the bound
    // tests/test_reduce.py states).  The float terms can differ by more than that only when a term
    // leaves the normal float range: (v - m)^2 above FLT_MAX (|v - m| >= 2^62 checked from the
    // extremes) or subnormal (a nonzero |v| or |m| below 2^-40: flagged per voxel for Float32,
    // per code on the host for UInt16); and NaN / +-Inf make every sum non-finite.  In those cases
    // res[1].count = 0 and the caller runs the two float passes.  min / max / arg, the extremes
    // filter, prod and the in-order first occurrence as aggregatesFastKernel.
    struct MomentPartialF
    {
        uint64_t count;
        double mean, m2, sum, prod;
        float minValue, maxValue;
        uint64_t minIndex, maxIndex;
        uint32_t flags;   // bit 0: a non-finite value; bit 1: a nonzero |v| < 2^-40
        uint32_t pad;
    };

    constexpr float kTinyValue = 0x1p-40f;

    __device__ __forceinline__ void momentCombineF(MomentPartialF& p, MomentPartialF const& o)
    {
        if (o.count != 0)
        {
            if (p.count == 0)
            {
                p.mean = o.mean;
                p.m2 = o.m2;
            }
            else
            {
                double const na = static_cast<double>(p.count), nb = static_cast<double>(o.count);
                double const n = na + nb, delta = o.mean - p.mean;
                p.mean += delta * (nb / n);
                p.m2 += o.m2 + delta * delta * (na * nb / n);
            }
        }
        p.count += o.count;
        p.sum += o.sum;
        p.prod *= o.prod;
        p.flags |= o.flags;
        minCombine(p.minValue, p.minIndex, o.minValue, o.minIndex);
        maxCombine(p.maxValue, p.maxIndex, o.maxValue, o.maxIndex);
    }

    __device__ __forceinline__ MomentPartialF shflXorMomentF(MomentPartialF const& p, int m)
    {
        MomentPartialF o;
        o.count = shflXorU(p.count, m);
        o.mean = shflXorD(p.mean, m);
        o.m2 = shflXorD(p.m2, m);
        o.sum = shflXorD(p.sum, m);
        o.prod = shflXorD(p.prod, m);
        o.minValue = __shfl_xor(p.minValue, m);
        o.maxValue = __shfl_xor(p.maxValue, m);
        o.minIndex = shflXorU(p.minIndex, m);
        o.maxIndex = shflXorU(p.maxIndex, m);
        o.flags = __shfl_xor(p.flags, m);
        o.pad = 0;
        return o;
    }

    template <int WAVES>
    __device__ void momentBlockReduceF(MomentPartialF& p)
    {
        for (int m = 32; m >= 1; m >>= 1)
            momentCombineF(p, shflXorMomentF(p, m));
        __shared__ MomentPartialF lds[WAVES];
        if ((threadIdx.x & 63) == 0)
            lds[threadIdx.x >> 6] = p;
        __syncthreads();
        if (threadIdx.x == 0)
            for (int w = 1; w < WAVES; ++w)
                momentCombineF(p, lds[w]);
    }

    __device__ __forceinline__ MomentPartialF emptyMomentF()
    {
        MomentPartialF p;
        p.count = 0;
        p.mean = p.m2 = p.sum = 0.0;
        p.prod = 1.0;
        p.minValue = FLT_MAX;
        p.maxValue = -FLT_MAX;
        p.minIndex = p.maxIndex = kNoIndex;
        p.flags = 0;
        p.pad = 0;
        return p;
    }

    // FMT UInt16 (any mapping but the unit one, which takes the integer kernel), Float32, and
    // (round 6) Int16 / UInt32 under any mapping.
    template <int FMT, bool CONTIG>
    __global__ __launch_bounds__(kBlock) void aggregatesMomentsFKernel(FastHistArgs h, MomentPartialF* partials)
    {
        constexpr int BPV = FMT == codec::FmtUInt16 || FMT == codec::FmtInt16 ? 2 : 4;
        constexpr int U = 4;
        uint32_t const lane = threadIdx.x & 63;
        MomentPartialF p = emptyMomentF();
        double K = 0.0, s1 = 0.0, s2 = 0.0;
        uint32_t n = 0;   // this lane's voxels (< 2^32: a lane visits far fewer)
        bool bad = false, tiny = false;
        auto decodeV = [&](uint32_t c) -> float {
            if constexpr (FMT == codec::FmtFloat32)
                return codec::bitsToFloat(c);
            else
                return codec::decode(c, FMT, h.lo, h.hi);
        };
        auto gIndexOf = [&](uint64_t item, uint64_t hb, int j) -> uint64_t {
            if (CONTIG && hb != ~0ull)
                return h.giBase + hb * 8 + 4 * lane + (j < 4 ? static_cast<uint64_t>(j) : 252ull + j);
            return spanGlobalIndex<CONTIG>(h, item, j);
        };
        // STEP: the extremes are the wave-step's (slo / shi, resolved after the walk as in
        // aggregatesMomentsU16Kernel); otherwise (tail items) the in-order per-voxel updates
        auto visit8 = [&](uint32_t const (&c)[8], uint64_t item, uint64_t hb, uint32_t m, bool prodLive, bool step,
                          float& slo, float& shi) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                v[j] = decodeV(c[j]);
            auto gIndex = [&](int j) -> uint64_t { return gIndexOf(item, hb, j); };
            // the lane's pivot: its first valid value (0 when that is not finite: the result then
            // falls back anyway)
            if (n == 0)
            {
                float k0 = 0.f;
#pragma unroll
                for (int j = 7; j >= 0; --j)
                    k0 = (m >> j) & 1u ? v[j] : k0;
                K = fabsf(k0) <= FLT_MAX ? static_cast<double>(k0) : 0.0;
            }
            float lo = FLT_MAX, hi = -FLT_MAX;
#pragma unroll
            for (int j = 0; j < 8; ++j)
            {
                bool const in = (m >> j) & 1u;   // voxels outside the range never qualify
                lo = fminf(lo, in ? v[j] : FLT_MAX);   // (NaN never qualifies: minNum / maxNum skip it)
                hi = fmaxf(hi, in ? v[j] : -FLT_MAX);
            }
            if (step)
            {
                slo = fminf(slo, lo);
                shi = fmaxf(shi, hi);
            }
            else if (lo < p.minValue || hi > p.maxValue)
            {
#pragma unroll
                for (int j = 0; j < 8; ++j)
                {
                    if (!((m >> j) & 1u))
                        continue;
                    if (v[j] < p.minValue)
                    {
                        p.minValue = v[j];
                        p.minIndex = gIndex(j);
                    }
                    if (v[j] > p.maxValue)
                    {
                        p.maxValue = v[j];
                        p.maxIndex = gIndex(j);
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < 8; ++j)
            {
                if (!((m >> j) & 1u))
                    continue;
                double const x = static_cast<double>(v[j]);
                double const d = x - K;
                s1 += d;
                s2 = fma(d, d, s2);
                if (prodLive)
                    p.prod *= x;
                float const a = fabsf(v[j]);
                bad = bad || !(a <= FLT_MAX);
                if constexpr (FMT == codec::FmtFloat32 || FMT == codec::FmtUInt32)   // (per voxel: 2^32 codes)
                    tiny = tiny || (a < kTinyValue && a != 0.f);
            }
            n += static_cast<uint32_t>(__builtin_popcount(m));
        };
        uint64_t const wave = static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
        uint64_t const waves = static_cast<uint64_t>(gridDim.x) * (kBlock / 64);
        uint64_t const steps = h.items / (64 * U);
        bool const halves = CONTIG && BPV == 4 && (reinterpret_cast<uintptr_t>(h.data) & 15u) == 0;
        uint32_t minStep = ~0u, maxStep = ~0u;   // the steps of the lane's extremes (as the integer kernel)
        for (uint64_t st = wave; st < steps; st += waves)
        {
            uint32_t c[U][8], msk[U];
            if (halves)   // contiguous 16-B lanes (as aggregatesFastKernel)
            {
#pragma unroll
                for (int k = 0; k < U; ++k)
                {
                    uint8_t const* q = h.data + ((st * (64 * U) + k * 64) * 8 + 4 * lane) * 4;
                    u32x4 const x = loadVec<u32x4, true>(q), y = loadVec<u32x4, true>(q + 1024);
                    c[k][0] = x.x; c[k][1] = x.y; c[k][2] = x.z; c[k][3] = x.w;
                    c[k][4] = y.x; c[k][5] = y.y; c[k][6] = y.z; c[k][7] = y.w;
                    msk[k] = 0xFFu;
                }
            }
            else
            {
#pragma unroll
                for (int k = 0; k < U; ++k)
                    load8<BPV, true>(h.data, spanVoxelMask<CONTIG>(h, st * (64 * U) + k * 64 + lane, msk[k]), c[k]);
            }
            bool const prodLive = __any(p.prod != 0.0);   // wave-uniform: 0 stays 0 (finite values)
            float slo = FLT_MAX, shi = -FLT_MAX;
#pragma unroll
            for (int k = 0; k < U; ++k)
                visit8(c[k], st * (64 * U) + k * 64 + lane, halves ? st * (64 * U) + k * 64 : ~0ull, msk[k], prodLive,
                       true, slo, shi);
            // strict: a later step reaching the same value keeps the earlier one (first occurrence)
            bool const lower = slo < p.minValue, higher = shi > p.maxValue;
            p.minValue = lower ? slo : p.minValue;
            minStep = lower ? static_cast<uint32_t>(st) : minStep;
            p.maxValue = higher ? shi : p.maxValue;
            maxStep = higher ? static_cast<uint32_t>(st) : maxStep;
        }
        // the first voxel of the lane's extreme value in its step (reloaded); the value is taken
        // from that voxel (of +0 / -0, the first one's sign, as the strict in-order updates)
        auto resolveStep = [&](uint32_t st, float value, uint64_t& index, float& out) {
            uint64_t const base = static_cast<uint64_t>(st) * (64 * U);
            for (int k = U - 1; k >= 0; --k)
            {
                uint32_t cc[8], m = 0xFFu;
                uint64_t const item = base + static_cast<uint64_t>(k) * 64 + lane;
                uint64_t const hb = halves ? base + static_cast<uint64_t>(k) * 64 : ~0ull;
                if (halves)
                {
                    uint8_t const* q = h.data + ((base + k * 64) * 8 + 4 * lane) * 4;
                    u32x4 const x = loadVec<u32x4, false>(q), y = loadVec<u32x4, false>(q + 1024);
                    cc[0] = x.x; cc[1] = x.y; cc[2] = x.z; cc[3] = x.w;
                    cc[4] = y.x; cc[5] = y.y; cc[6] = y.z; cc[7] = y.w;
                }
                else
                    load8<BPV, false>(h.data, spanVoxelMask<CONTIG>(h, item, m), cc);
                for (int j = 7; j >= 0; --j)
                {
                    float const v = decodeV(cc[j]);
                    if (((m >> j) & 1u) && v == value)
                    {
                        index = gIndexOf(item, hb, j);
                        out = v;
                    }
                }
            }
        };
        if (minStep != ~0u)
            resolveStep(minStep, p.minValue, p.minIndex, p.minValue);
        if (maxStep != ~0u)
            resolveStep(maxStep, p.maxValue, p.maxIndex, p.maxValue);
        for (uint64_t it = steps * (64 * U) + wave * 64 + lane; it < h.items; it += waves * 64)
        {
            uint32_t c[8], m;
            load8<BPV, true>(h.data, spanVoxelMask<CONTIG>(h, it, m), c);
            float slo = FLT_MAX, shi = -FLT_MAX;
            visit8(c, it, ~0ull, m, true, false, slo, shi);
        }
        if (n != 0)
        {
            double const dn = static_cast<double>(n);
            p.count = n;
            p.mean = K + s1 / dn;
            p.m2 = fmax(s2 - s1 * (s1 / dn), 0.0);
            p.sum = fma(dn, K, s1);
        }
        p.flags = (bad ? 1u : 0u) | (tiny ? 2u : 0u);
        momentBlockReduceF<kBlock / 64>(p);
        if (threadIdx.x == 0)
            partials[blockIdx.x] = p;
    }

    // One workgroup: the n partials of aggregatesMomentsFKernel -> res[0] (pass-1 fields) and
    // res[1].sumSq = S with res[1].count = 1, or res[1].count = 0 when the float terms may differ
    // from the exact form (see above; the caller runs the two passes).  tinyCodes: the host found a
    // code of the volume's format whose value is a nonzero |v| < 2^-40 (UInt16).
    __global__ __launch_bounds__(kBlock) void aggregatesMomentsFFinalKernel(MomentPartialF const* partials, uint32_t n,
                                                                           double numElems, uint32_t tinyCodes,
                                                                           vktHipAggregatePartial_t* res)
    {
        MomentPartialF p = emptyMomentF();
        for (uint32_t i = threadIdx.x; i < n; i += kBlock)
            momentCombineF(p, partials[i]);
        momentBlockReduceF<kBlock / 64>(p);
        if (threadIdx.x != 0)
            return;
        vktHipAggregatePartial_t one = emptyPartial();
        one.count = p.count;
        one.sum = p.sum;
        one.prod = p.prod;
        one.minValue = p.minValue;
        one.minIndex = p.minIndex;
        one.maxValue = p.maxValue;
        one.maxIndex = p.maxIndex;
        float const m = static_cast<float>(static_cast<double>(static_cast<float>(p.sum)) / numElems);
        double const dm = static_cast<double>(m);
        bool ok = (p.flags & 1u) == 0 && fabs(p.sum) <= DBL_MAX && p.m2 <= DBL_MAX;
        ok = ok && (p.flags & 2u) == 0 && tinyCodes == 0 && (m == 0.f || fabsf(m) >= kTinyValue);
        if (p.count != 0)
            ok = ok && fabs(static_cast<double>(p.maxValue) - dm) < 0x1p62 &&
                 fabs(static_cast<double>(p.minValue) - dm) < 0x1p62;
        double const dd = p.mean - dm;
        vktHipAggregatePartial_t two = emptyPartial();
        two.sumSq = p.count ? p.m2 + static_cast<double>(p.count) * dd * dd : 0.0;
        two.count = ok ? 1u : 0u;
        res[0] = one;
        res[1] = two;
    }

    // One workgroup: the n partials of a moments kernel combined (same order and tree as the
    // final kernels) into out[0], not finished -- one rank's part of a Z-slab volume
    // (vktHipAggregateMoments).
    __global__ __launch_bounds__(kBlock) void momentsCombineU16Kernel(MomentPartialU16 const* partials, uint32_t n,
                                                                     MomentPartialU16* out)
    {
        MomentPartialU16 p;
        p.count = p.sumC = p.sumSqLo = p.sumSqHi = 0;
        p.prod = 1.0;
        p.cmin = 0x10000u;
        p.cmax = -1;
        p.minIndex = p.maxIndex = kNoIndex;
        for (uint32_t i = threadIdx.x; i < n; i += kBlock)
            momentCombine(p, partials[i]);
        momentBlockReduce<kBlock / 64>(p);
        if (threadIdx.x == 0)
            *out = p;
    }

    __global__ __launch_bounds__(kBlock) void momentsCombineFKernel(MomentPartialF const* partials, uint32_t n,
                                                                   MomentPartialF* out)
    {
        MomentPartialF p = emptyMomentF();
        for (uint32_t i = threadIdx.x; i < n; i += kBlock)
            momentCombineF(p, partials[i]);
        momentBlockReduceF<kBlock / 64>(p);
        if (threadIdx.x == 0)
            *out = p;
    }

    // The first voxels of item `item` holding codes tmin / tmax, folded into *bMin / *bMax with
    // atomicMin (LDS or global).
    template <int BPV, bool CONTIG>
    __device__ __forceinline__ void findCodes(FastHistArgs const& h, uint64_t item, int32_t tmin, int32_t tmax,
                                              unsigned long long* bMin, unsigned long long* bMax)
    {
        uint32_t c[8];
        load8<BPV, true>(h.data, spanVoxel<CONTIG>(h, item), c);
        uint32_t const m = itemMask<CONTIG>(h, item);
        int jMin = 8, jMax = 8;
#pragma unroll
        for (int j = 7; j >= 0; --j)
            if ((m >> j) & 1u)
            {
                jMin = static_cast<int32_t>(c[j]) == tmin ? j : jMin;
                jMax = static_cast<int32_t>(c[j]) == tmax ? j : jMax;
            }
        if (jMin < 8)
            atomicMin(bMin, static_cast<unsigned long long>(spanGlobalIndex<CONTIG>(h, item, jMin)));
        if (jMax < 8)
            atomicMin(bMax, static_cast<unsigned long long>(spanGlobalIndex<CONTIG>(h, item, jMax)));
    }

    // First occurrence of codes targets[0] / targets[1] (the extremes' codes), stage 1: the first
    // `headItems` items of the range, one 1024-item step per workgroup (kFindHeadBlocks of them,
    // all in flight at once), each workgroup folding its first hits in LDS and then with one
    // global atomicMin per code into res[0].minIndex / maxIndex (kNoIndex before the launch).  On
    // varied data the codes occur in the first step.  (One workgroup walking the head in order
    // stopped early but paid one memory latency per step: 22-43 us for UInt16, whose extreme
    // codes first occur ~65 Ki voxels in; a whole-grid walk with global atomics and early exit
    // took 0.35 ms -- many waves folding into one global word serialise on it.)
    constexpr uint32_t kFindHeadBlocks = 64;
    template <int BPV, bool CONTIG>
    __global__ __launch_bounds__(1024) void aggregatesFindHeadKernel(FastHistArgs h, int32_t const* targets,
                                                                    vktHipAggregatePartial_t* res, uint64_t headItems)
    {
        int32_t const tmin = targets[0], tmax = targets[1];
        if (tmin < 0 || tmax < 0)
            return;
        __shared__ unsigned long long sMin, sMax;
        if (threadIdx.x == 0)
            sMin = sMax = kNoIndex;
        __syncthreads();
        uint64_t const end = headItems < h.items ? headItems : h.items;
        uint64_t const item = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
        if (item < end)
            findCodes<BPV, CONTIG>(h, item, tmin, tmax, &sMin, &sMax);
        __syncthreads();
        if (threadIdx.x == 0)
        {
            auto* const bMin = reinterpret_cast<unsigned long long*>(&res[0].minIndex);
            auto* const bMax = reinterpret_cast<unsigned long long*>(&res[0].maxIndex);
            if (sMin != kNoIndex)
                atomicMin(bMin, sMin);
            if (sMax != kNoIndex)
                atomicMin(bMax, sMax);
        }
    }

    // Stage 2, the whole grid over the items after the head -- only when stage 1 left a code
    // unfound (it then occurs rarely, so few lanes fold into the global words).
    template <int BPV, bool CONTIG>
    __global__ __launch_bounds__(kBlock) void aggregatesFindTailKernel(FastHistArgs h, int32_t const* targets,
                                                                      vktHipAggregatePartial_t* res, uint64_t headItems)
    {
        int32_t const tmin = targets[0], tmax = targets[1];
        if (tmin < 0 || tmax < 0 || (res[0].minIndex != kNoIndex && res[0].maxIndex != kNoIndex))
            return;   // (stage 1's stores are visible: a kernel boundary lies between)
        auto* const bMin = reinterpret_cast<unsigned long long*>(&res[0].minIndex);
        auto* const bMax = reinterpret_cast<unsigned long long*>(&res[0].maxIndex);
        uint64_t const stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
        for (uint64_t item = headItems + static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; item < h.items;
             item += stride)
            findCodes<BPV, CONTIG>(h, item, tmin, tmax, bMin, bMax);
    }

    __global__ void zeroU64Kernel(unsigned long long* p, uint64_t n)
    {
        uint64_t const i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
        if (i < n)
            p[i] = 0ull;
    }

    // ---- host helpers -------------------------------------------------------------------
    bool makeBox(vktHipVolumeView_t const& v, vktVec3i_t first, vktVec3i_t last, int64_t zGlobal, BoxArgs& a,
                 char const* what, vktError& err)
    {
        err = vktNoError;
        if (!validView(v))
        {
            err = rt::fail(what);
            return false;
        }
        int64_t nx = int64_t(last.x) - first.x, ny = int64_t(last.y) - first.y, nz = int64_t(last.z) - first.z;
        if (nx <= 0 || ny <= 0 || nz <= 0)
            return false;   // empty range: nothing to read
        if (first.x < 0 || first.y < 0 || first.z < 0 || last.x > v.dimX || last.y > v.dimY || last.z > v.dimZ)
        {
            err = rt::fail("range outside the volume (the reference reads out of bounds)");
            return false;
        }
        if (ny * nz >= (1ll << 32))
        {
            err = rt::fail("range has too many rows");
            return false;
        }
        a.data = v.data;
        a.dimX = v.dimX;
        a.dimY = v.dimY;
        a.fx = first.x;
        a.fy = first.y;
        a.fz = first.z;
        a.nx = static_cast<int32_t>(nx);
        a.rows = static_cast<uint32_t>(ny * nz);
        a.fdNy = makeFastDiv(static_cast<uint32_t>(ny));
        a.fmt = v.dataFormat;
        a.lo = v.mappingLo;
        a.hi = v.mappingHi;
        a.zGlobal = zGlobal;
        return true;
    }

    unsigned rowGrid(uint32_t rows) { return streamingGrid(rows, kBlock / 64, 8); }

    bool vecRows(BoxArgs const& a)
    {
        uint32_t const bpv = codec::bytesPerVoxel(a.fmt);
        return (bpv == 1 || bpv == 2 || bpv == 4) && a.fx % 8 == 0 && a.nx % 8 == 0 && a.dimX % 8 == 0 &&
               reinterpret_cast<uintptr_t>(a.data) % 16 == 0;
    }

    // dispatch on bytes per voxel and the vector-row condition
#define VKT_REDUCE_DISPATCH(KERNEL, ...)                                                                      \
    do {                                                                                                      \
        uint32_t const bpv_ = codec::bytesPerVoxel(a.fmt);                                                    \
        bool const vec_ = vecRows(a);                                                                         \
        if (bpv_ == 1) { if (vec_) KERNEL(1, true, __VA_ARGS__); else KERNEL(1, false, __VA_ARGS__); }        \
        else if (bpv_ == 2) { if (vec_) KERNEL(2, true, __VA_ARGS__); else KERNEL(2, false, __VA_ARGS__); }   \
        else { if (vec_) KERNEL(4, true, __VA_ARGS__); else KERNEL(4, false, __VA_ARGS__); }                  \
    } while (0)

#define VKT_AGG_LAUNCH(B, V, PASS, G, S, MEANPTR, MEANV, OUT) \
    hipLaunchKernelGGL((aggregatesKernel<PASS, B, V>), dim3(G), dim3(kBlock), 0, S, a, MEANPTR, MEANV, OUT)
#define VKT_HIST_LAUNCH(B, V, G, LDS, S) \
    hipLaunchKernelGGL((histogramKernel<B, V>), dim3(G), dim3(kBlock), LDS, S, a, h)

    // Item walk of the streaming kernels (histogramFastKernel, aggregatesFastKernel) over a
    // range: UInt8/UInt16/Float32 with 8-voxel-aligned rows; false if the range does not qualify.
    bool makeSpanArgs(BoxArgs const& a, FastHistArgs& h, bool& contig)
    {
        int32_t const fmt = a.fmt;
        if (fmt != codec::FmtUInt8 && fmt != codec::FmtUInt16 && fmt != codec::FmtFloat32)
            return false;
        // rows on the 8-voxel grid (16-B aligned base, dimX % 8 == 0); a range row that starts or
        // ends off it is padded to whole items, the extra voxels masked (itemMask)
        if (a.dimX % 8 != 0 || reinterpret_cast<uintptr_t>(a.data) % 16 != 0)
            return false;
        bool const padded = a.fx % 8 != 0 || a.nx % 8 != 0;
        int32_t const px0 = a.fx & ~7;
        int32_t const px1 = (a.fx + a.nx + 7) & ~7;
        uint32_t const bpv = codec::bytesPerVoxel(fmt);
        uint64_t const ny = a.fdNy.d;   // range rows = ny * nz
        uint64_t const nz = a.rows / ny;
        contig = !padded && a.nx == a.dimX && (ny == static_cast<uint64_t>(a.dimY) || nz == 1);
        uint64_t const ipr = static_cast<uint64_t>(px1 - px0) / 8;
        uint64_t const items = ipr * a.rows;
        if (!contig && items >= (1ull << 32))
            return false;
        h = FastHistArgs{};
        h.items = items;
        h.dimX = a.dimX;
        h.dimY = a.dimY;
        h.fx = a.fx;
        h.fy = a.fy;
        h.fz = a.fz;
        h.px0 = px0;
        h.rx0 = a.fx;
        h.rx1 = a.fx + a.nx;
        h.padded = padded ? 1u : 0u;
        h.fdIpr = makeFastDiv(static_cast<uint32_t>(ipr));
        h.fdNy = a.fdNy;
        uint64_t const start = (static_cast<uint64_t>(a.fz) * a.dimY + a.fy) * a.dimX;   // CONTIG: fx == 0
        h.data = contig ? a.data + start * bpv : a.data;
        h.lo = a.lo;
        h.hi = a.hi;
        h.zGlobal = a.zGlobal;
        h.giBase = start + static_cast<uint64_t>(a.zGlobal) * a.dimY * a.dimX;
        return true;
    }

    // fastBin of a UInt8 code, evaluated on the host with the kernel's float operations
    uint64_t hostBinU8(uint32_t c, float lo, float hi, float scale, float nbf, uint64_t nb)
    {
        volatile float v = codec::decode(c, codec::FmtUInt8, lo, hi);
        volatile float d = v - lo;
        volatile float f = d * scale;
        return (f > -1.0f && f < nbf) ? static_cast<uint64_t>(static_cast<int32_t>(f)) : nb;
    }

    // fastBin of a UInt16 code, evaluated on the host with the kernel's float operations
    // (histogramFastKernel's UInt16 decode: t = c * 2^-16, lerp as (1 - t) * lo + t * hi)
    uint64_t hostBinU16(uint32_t c, float lo, float hi, float scale, float nbf, uint64_t nb)
    {
        volatile float t = static_cast<float>(c) * (1.0f / 65536.0f);
        volatile float sm = 1.0f - t;
        volatile float p = sm * lo;
        volatile float q = t * hi;
        volatile float v = p + q;
        volatile float d = v - lo;
        volatile float f = d * scale;
        return (f > -1.0f && f < nbf) ? static_cast<uint64_t>(static_cast<int32_t>(f)) : nb;
    }

    // True when every UInt16 code's bin is (code * numBins) >> 16 (mul-shift bins).  The
    // 65 536-code check costs ~0.2 ms on the host, so the last answer is kept per thread.
    bool mulShiftBinsU16(float lo, float hi, float scale, uint64_t numBins)
    {
        if (numBins == 0 || numBins > 65536u)
            return false;
        struct Key
        {
            uint32_t lo, hi, scale;
            uint64_t nb;
            bool operator==(Key const& o) const { return lo == o.lo && hi == o.hi && scale == o.scale && nb == o.nb; }
        };
        Key const key{codec::floatToBits(lo), codec::floatToBits(hi), codec::floatToBits(scale), numBins};
        thread_local Key lastKey{0, 0, 0, 0};
        thread_local bool lastResult = false;
        if (key == lastKey)
            return lastResult;
        bool ok = true;
        float const nbf = static_cast<float>(numBins);
        for (uint32_t c = 0; c < 65536u && ok; ++c)
            ok = hostBinU16(c, lo, hi, scale, nbf, numBins) == ((static_cast<uint64_t>(c) * numBins) >> 16);
        lastKey = key;
        lastResult = ok;
        return ok;
    }

    // UInt8 code counts of a non-CONTIG span walk h added into h.bins (256 u64) by
    // codeCountsU8RowsKernel (16-voxel items over the rows); false (nothing launched) when the
    // volume's rows are not on the 16-voxel grid or knob reduce.u8_rows16 is 0.
    bool launchU8RowCounts(FastHistArgs const& h, hipStream_t s)
    {
        int64_t const k = rt::knob(rt::Knob::ReduceU8Rows16);
        if (h.dimX % 16 != 0 || k == 0)
            return false;
        uint64_t const rows = h.items / h.fdIpr.d;
        int32_t const px0 = h.rx0 & ~15, px1 = (h.rx1 + 15) & ~15;
        uint64_t const ipr = static_cast<uint64_t>(px1 - px0) / 16;
        FastHistArgs r = h;
        r.px0 = px0;
        r.fdIpr = makeFastDiv(static_cast<uint32_t>(ipr));
        r.items = ipr * rows;
        r.rows = static_cast<uint32_t>(rows);
        r.padded = px0 != h.rx0 || px1 != h.rx1 ? 1u : 0u;
        unsigned const g = streamingGrid(r.items, 64u * 4u * (kBlock / 64), 4);
        size_t const lds = 256u << 7;   // 32 copies of 256 counters
        // end bytes subtracted inside the main loop needs <= 32 rows per 256-item step
        if (r.padded && ipr >= 9 && k == 1)
            hipLaunchKernelGGL(codeCountsU8RowsKernel<true>, dim3(g), dim3(kBlock), lds, s, r);
        else
            hipLaunchKernelGGL(codeCountsU8RowsKernel<false>, dim3(g), dim3(kBlock), lds, s, r);
        return true;
    }

    // UInt8 histogram from code counts: bins[bin(c)] += counts[c] with the streaming kernel's own
    // bin formula (codes outside [0, numBins) dropped, as its trash row)
    __global__ __launch_bounds__(256) void histogramFromCodesKernel(unsigned long long const* counts, float lo,
                                                                  float hi, float scale, uint32_t nb,
                                                                  unsigned long long* bins)
    {
        uint32_t const c = threadIdx.x;
        float const v = codec::decode(c, codec::FmtUInt8, lo, hi);
        uint32_t const b = fastBin((v - lo) * scale, static_cast<float>(nb), nb);
        if (b < nb && counts[c] != 0ull)
            atomicAdd(&bins[b], counts[c]);
    }

    // bins += the workgroups' partial counter words (tiled histogram launches with
    // FastHistArgs::partials): one thread per word and slice of
    // kPartialRows workgroup rows (loads coalesced along the row, all of a thread's in flight),
    // one 64-bit atomic per nonzero count and slice; PACKED words hold two 16-bit counts.  The
    // data kernel's in-run flushes reached bins first (same stream).
    constexpr uint32_t kPartialRows = 32;
    template <bool PACKED>
    __global__ __launch_bounds__(256) void histogramPartialsKernel(uint32_t const* partials, uint32_t groups,
                                                                 uint32_t words, uint32_t tileBins,
                                                                 unsigned long long* bins)
    {
        uint32_t const w = blockIdx.x * 256u + threadIdx.x;
        if (w >= words)
            return;
        uint32_t const r0 = blockIdx.y * kPartialRows;
        uint32_t const r1 = min(groups, r0 + kPartialRows);
        uint32_t lo = 0, hi = 0;   // PACKED: <= 32 rows of 16-bit halves (< 2^16 each, the in-run flush) fit 32 bits
        unsigned long long wide = 0ull;
#pragma unroll 8
        for (uint32_t r = r0; r < r1; ++r)
        {
            uint32_t const v = __builtin_nontemporal_load(partials + static_cast<uint64_t>(r) * words + w);
            if constexpr (PACKED)
            {
                lo += v & 0xFFFFu;
                hi += v >> 16;
            }
            else
                wide += v;
        }
        if constexpr (PACKED)
        {
            if (lo != 0u)
                atomicAdd(&bins[2 * w], static_cast<unsigned long long>(lo));
            if (hi != 0u && 2 * w + 1 < tileBins)
                atomicAdd(&bins[2 * w + 1], static_cast<unsigned long long>(hi));
        }
        else if (wide != 0ull)
            atomicAdd(&bins[w], wide);
    }

    // A tiled (not PAIR) histogram launch of g workgroups over tileBins bins starting at
    // h.bins + h.tileBase: with knob histogram.partials (1, default: packed-16 launches; 2: every
    // tiled launch) the workgroups store their counter words and histogramPartialsKernel sums
    // them, instead of one global 64-bit atomic per nonzero counter and workgroup (256 x 65 536
    // for a packed-16 histogram: ~70 us of its ~0.5 ms at 1024^3, most of its time at 256^3).
    template <bool P16, typename Launch>
    void tiledWithPartials(FastHistArgs& h, unsigned g, hipStream_t s, Launch&& launch)
    {
        static rt::StreamScratch scratch;
        uint32_t* parts = nullptr;
        int64_t const k = rt::knob(rt::Knob::HistogramPartials);
        uint32_t const words = P16 ? (h.tileBins + 1) / 2 : h.tileBins;
        if (k == 2 || (k == 1 && P16))
            parts = static_cast<uint32_t*>(scratch.acquire(static_cast<size_t>(g) * words * sizeof(uint32_t), s));
        h.partials = parts;
        launch();
        if (parts != nullptr)
        {
            dim3 const grid((words + 255) / 256, (g + kPartialRows - 1) / kPartialRows);
            hipLaunchKernelGGL((histogramPartialsKernel<P16>), grid, dim3(256), 0, s, parts, g, words, h.tileBins,
                               h.bins + h.tileBase);
            scratch.release(s);
        }
        h.partials = nullptr;
    }

    // 16-bit histogram from code counts: bins[bin(c)] += counts[c] for the 65 536 codes (UInt16 or
    // Int16 `fmt`), with the reference's bin of the decoded value (binOf: any bin count,
    // out-of-range and NaN dropped).  A thread folds kFoldCodes consecutive codes, adding a run of
    // codes on one bin with one atomic (the decode is monotonic along a run of codes, so few bins
    // hold many codes: one atomic per code put ~256 adds on each of 256 bins, serialised).
    constexpr uint32_t kFoldCodes = 16;
    __global__ __launch_bounds__(256) void histogramFromCodesU16Kernel(unsigned long long const* counts, int32_t fmt,
                                                                     float lo, float hi, float scale,
                                                                     uint64_t numBins, unsigned long long* bins)
    {
        uint32_t const c0 = (blockIdx.x * 256u + threadIdx.x) * kFoldCodes;
        uint64_t runBin = ~0ull;
        unsigned long long run = 0ull;
        for (uint32_t c = c0; c < c0 + kFoldCodes; ++c)
        {
            unsigned long long const n = counts[c];
            if (n == 0ull)
                continue;
            uint64_t const b = binOf(codec::decode(c, fmt, lo, hi), lo, scale, numBins);
            if (b != runBin)
            {
                if (run != 0ull && runBin < numBins)
                    atomicAdd(&bins[runBin], run);
                runBin = b;
                run = 0ull;
            }
            run += n;
        }
        if (run != 0ull && runBin < numBins)
            atomicAdd(&bins[runBin], run);
    }

    // UInt16 bins that are not a function of code >> s / (code * n) >> 16 and do not fit the
    // replicated counters (knob histogram.u16_codes, default 2; 1: only beyond one LDS tile;
    // DESIGN §4.8 round 6): a UInt16 voxel holds one of 65 536
    // codes and its bin depends on the code alone, so the data pass counts codes -- the P16
    // kernel with the identity bin (SHIFT, code >> 0), one pass whatever the bin count -- and a
    // 65 536-thread kernel folds the counts into the bins.  Same counts as the per-voxel bin, by
    // construction.  Int16 volumes take the same counts of their raw 16-bit codes (the streaming
    // kernels below read only UInt8 / UInt16 / Float32).
    bool launchU16CodeHistogram(FastHistArgs const& h, bool contig, uint32_t tileCap, BoxArgs const& a,
                                HistArgs const& hh, hipStream_t s)
    {
        if (32768u > tileCap)   // 65 536 packed 16-bit counters in one workgroup's LDS
            return false;
        static rt::StreamScratch scratch;
        auto* const counts = static_cast<unsigned long long*>(scratch.acquire(65536 * sizeof(unsigned long long), s));
        if (!counts)
            return false;
        FastHistArgs c = h;
        c.bins = counts;
        c.nb = 65536u;
        c.nbf = 65536.0f;
        c.binShift = 0u;
        c.binMul = 1u;
        c.rShift = 0u;
        c.tileBase = 0u;
        c.tileBins = 65536u;
        c.pairTiles = 0u;
        c.p16Step = rt::knob(rt::Knob::HistogramP16Step) != 0 ? 1u : 0u;
        bool ok = hipMemsetAsync(counts, 0, 65536 * sizeof(unsigned long long), s) == hipSuccess;
        if (ok)
        {
            unsigned const g = streamingGrid(c.items, 64u * 4u * (kTileBlock / 64), 1);
            size_t const lds = 32768u * 4u;
            tiledWithPartials<true>(c, g, s, [&] {
                if (contig)
                    hipLaunchKernelGGL((histogramFastKernel<codec::FmtUInt16, true, true, kTileBlock, true, true>),
                                       dim3(g), dim3(kTileBlock), lds, s, c);
                else
                    hipLaunchKernelGGL((histogramFastKernel<codec::FmtUInt16, false, true, kTileBlock, true, true>),
                                       dim3(g), dim3(kTileBlock), lds, s, c);
            });
            hipLaunchKernelGGL(histogramFromCodesU16Kernel, dim3(65536 / (256 * kFoldCodes)), dim3(256), 0, s, counts,
                               a.fmt, a.lo, a.hi,
                               hh.scale, hh.numBins, hh.bins);
        }
        scratch.release(s);
        return ok;   // (a failed launch surfaces in the caller's finishLaunch)
    }

    // Launches histogramFastKernel when the range qualifies (see its comment); false otherwise.
    bool launchFastHistogram(BoxArgs const& a, HistArgs const& hh, hipStream_t s)
    {
        int32_t const fmt = a.fmt;
        // LDS counters of one 1024-thread workgroup (the device limit minus the static table)
        uint32_t const tileCap = (ldsBinCapacity() * 4u - 1024u) / 4u;
        uint64_t const tiles = (hh.numBins + tileCap - 1) / tileCap;
        FastHistArgs h;
        bool contig;
        BoxArgs a16 = a;   // (Int16: the span of its raw 16-bit codes)
        if (fmt == codec::FmtInt16)
            a16.fmt = codec::FmtUInt16;
        if (!makeSpanArgs(a16, h, contig))
            return false;
        // 16-bit code counts (knob histogram.u16_codes: 2 (default) UInt16 bins beyond the
        // replicated counters and every Int16 histogram, 1 only UInt16 bins beyond one LDS tile,
        // 0 off); integer UInt16 bins keep the streaming kernels below
        int64_t const u16k = rt::knob(rt::Knob::HistogramU16Codes);
        if (fmt == codec::FmtInt16)
            return u16k > 0 && launchU16CodeHistogram(h, contig, tileCap, a, hh, s);
        if (fmt == codec::FmtUInt16 && u16k > 0 && (tiles > 1 || (u16k == 2 && hh.numBins > kReplicatedMaxBins)))
        {
            bool integerBins = codec::isUnitMapping(a.lo, a.hi) && hh.numBins <= 65536u &&
                               (hh.numBins & (hh.numBins - 1)) == 0 && hh.scale == static_cast<float>(hh.numBins);
            if (!integerBins && rt::knob(rt::Knob::HistogramMulShift) != 0)
                integerBins = mulShiftBinsU16(a.lo, a.hi, hh.scale, hh.numBins);
            if (!integerBins && launchU16CodeHistogram(h, contig, tileCap, a, hh, s))
                return true;
        }
        if (tiles > kFastMaxTiles)
            return false;
        uint64_t const items = h.items;
        h.scale = hh.scale;
        h.nb = static_cast<uint32_t>(hh.numBins);
        h.nbf = static_cast<float>(hh.numBins);
        h.bins = hh.bins;
        // integer bins (SHIFT, see histogramFastKernel): unit mapping, numBins = 2^k, k <= 16
        uint32_t k = 0;
        while (k < 16 && (1ull << k) < hh.numBins)
            ++k;
        bool shift = fmt == codec::FmtUInt16 && codec::isUnitMapping(a.lo, a.hi) && (1ull << k) == hh.numBins &&
                     hh.scale == static_cast<float>(hh.numBins);
        h.binShift = 16u - k;
        h.binMul = 1u;
        h.p16Step = rt::knob(rt::Knob::HistogramP16Step) != 0 ? 1u : 0u;
        if (fmt == codec::FmtUInt16 && !shift && rt::knob(rt::Knob::HistogramMulShift) != 0 &&
            mulShiftBinsU16(a.lo, a.hi, hh.scale, hh.numBins))
        {
            shift = true;
            h.binShift = 16u;
            h.binMul = static_cast<uint32_t>(hh.numBins);
        }
        if (fmt == codec::FmtUInt8)
        {
            // the kernel's own bin formula for all 256 codes, on the host (volkit_codec.hpp is shared)
            for (uint32_t sh = 0; sh < 8 && !shift; ++sh)
            {
                shift = true;
                for (uint32_t c = 0; c < 256 && shift; ++c)
                    shift = hostBinU8(c, a.lo, a.hi, hh.scale, static_cast<float>(hh.numBins), hh.numBins) == (c >> sh);
                h.binShift = sh;
            }
        }
        if (fmt == codec::FmtUInt8 && !contig && h.dimX % 16 == 0 && rt::knob(rt::Knob::ReduceU8Rows16) != 0)
        {
            // range rows: count the 256 codes with the 16-voxel row walk, then fold the counts
            // into the bins (800^3 sub-box of 1024^3 at x0 = 100, 256 bins: DESIGN §4.8)
            static rt::StreamScratch scratch;
            auto* const counts = static_cast<unsigned long long*>(scratch.acquire(256 * sizeof(unsigned long long), s));
            if (!counts)
                return false;
            FastHistArgs c = h;
            c.bins = counts;
            bool const ok = hipMemsetAsync(counts, 0, 256 * sizeof(unsigned long long), s) == hipSuccess &&
                            launchU8RowCounts(c, s);
            if (ok)
                hipLaunchKernelGGL(histogramFromCodesKernel, dim3(1), dim3(256), 0, s, counts, a.lo, a.hi, h.scale, h.nb,
                                   h.bins);
            scratch.release(s);
            if (ok)
                return true;
        }
#define VKT_FAST_HIST(FMT, TILED, BLOCK, G, LDS)                                                                   \
    do {                                                                                                           \
        if (contig)                                                                                                \
            hipLaunchKernelGGL((histogramFastKernel<FMT, true, TILED, BLOCK>), dim3(G), dim3(BLOCK), LDS, s, h);    \
        else                                                                                                       \
            hipLaunchKernelGGL((histogramFastKernel<FMT, false, TILED, BLOCK>), dim3(G), dim3(BLOCK), LDS, s, h);   \
    } while (0)
#define VKT_FAST_HIST_FMT(TILED, BLOCK, G, LDS)                                                                    \
    do {                                                                                                           \
        if (fmt == codec::FmtUInt8 && shift) {                                                                     \
            if (contig)                                                                                            \
                hipLaunchKernelGGL((histogramFastKernel<codec::FmtUInt8, true, TILED, BLOCK, true>), dim3(G),      \
                                   dim3(BLOCK), LDS, s, h);                                                        \
            else                                                                                                   \
                hipLaunchKernelGGL((histogramFastKernel<codec::FmtUInt8, false, TILED, BLOCK, true>), dim3(G),     \
                                   dim3(BLOCK), LDS, s, h);                                                        \
        }                                                                                                          \
        else if (fmt == codec::FmtUInt8) VKT_FAST_HIST(codec::FmtUInt8, TILED, BLOCK, G, LDS);                     \
        else if (shift) {                                                                                          \
            if (contig)                                                                                            \
                hipLaunchKernelGGL((histogramFastKernel<codec::FmtUInt16, true, TILED, BLOCK, true>), dim3(G),     \
                                   dim3(BLOCK), LDS, s, h);                                                        \
            else                                                                                                   \
                hipLaunchKernelGGL((histogramFastKernel<codec::FmtUInt16, false, TILED, BLOCK, true>), dim3(G),    \
                                   dim3(BLOCK), LDS, s, h);                                                        \
        }                                                                                                          \
        else if (fmt == codec::FmtUInt16) VKT_FAST_HIST(codec::FmtUInt16, TILED, BLOCK, G, LDS);                   \
        else VKT_FAST_HIST(codec::FmtFloat32, TILED, BLOCK, G, LDS);                                               \
    } while (0)
        if (h.nb <= kReplicatedMaxBins)
        {
            // replicas: as many as fit in 40 KiB (4 workgroups per CU), at most one per bank (32)
            // (R = 32 keeps a constant or skewed volume -- empty space -- at the streaming rate:
            // 0.36 ms at 1024^3 UInt16 vs 0.89 ms with R = 4; uniform random data is ~flat in R)
            uint32_t rs = 5;
            while (rs > 0 && (static_cast<uint64_t>(h.nb) + 1) * (4ull << rs) > 40u * 1024u)
                --rs;
            h.rShift = rs;
            h.tileBase = 0;
            h.tileBins = h.nb;
            size_t const lds = (static_cast<size_t>(h.nb) + 1) * (4u << rs);
            unsigned const perCU = static_cast<unsigned>(std::min<size_t>(8, (160u * 1024u) / (lds + 1024u)));
            unsigned const g = streamingGrid(items, 64u * 4u * (kBlock / 64), std::max(1u, perCU));
            VKT_FAST_HIST_FMT(false, kBlock, g, lds);
        }
        else if (tiles > 1 && fmt != codec::FmtUInt8 && (hh.numBins + 1) / 2 > tileCap &&
                 rt::knob(rt::Knob::HistogramPacked16) == 2 &&
                 (hh.numBins + 2ull * tileCap - 1) / (2ull * tileCap) <= kFastMaxTiles)
        {
            // packed 16-bit counters in tiles of up to 2 tileCap bins, one pass per tile (more bins
            // than one packed-16 launch holds: Float32, UInt16 with the code counts off)
            uint64_t const t16 = (hh.numBins + 2ull * tileCap - 1) / (2ull * tileCap);
            uint32_t const per = static_cast<uint32_t>(((hh.numBins + t16 - 1) / t16 + 1) & ~1ull);   // even
            h.rShift = 0;
            unsigned const g = streamingGrid(items, 64u * 4u * (kTileBlock / 64), 1);
            for (uint64_t t = 0; t < t16; ++t)
            {
                h.tileBase = static_cast<uint32_t>(t * per);
                h.tileBins = static_cast<uint32_t>(std::min<uint64_t>(per, hh.numBins - h.tileBase));
                size_t const lds = static_cast<size_t>((h.tileBins + 1) / 2) * 4u;
                tiledWithPartials<true>(h, g, s, [&] {
#define VKT_P16T(FMT, SH)                                                                                          \
    do {                                                                                                           \
        if (contig)                                                                                                \
            hipLaunchKernelGGL((histogramFastKernel<FMT, true, true, kTileBlock, SH, true>), dim3(g),              \
                               dim3(kTileBlock), lds, s, h);                                                       \
        else                                                                                                       \
            hipLaunchKernelGGL((histogramFastKernel<FMT, false, true, kTileBlock, SH, true>), dim3(g),             \
                               dim3(kTileBlock), lds, s, h);                                                       \
    } while (0)
                    if (shift)
                        VKT_P16T(codec::FmtUInt16, true);
                    else if (fmt == codec::FmtUInt16)
                        VKT_P16T(codec::FmtUInt16, false);
                    else
                        VKT_P16T(codec::FmtFloat32, false);
#undef VKT_P16T
                });
            }
        }
        else if (tiles > 1 && tiles <= kPairMaxTiles && fmt != codec::FmtUInt8 &&
                 (rt::knob(rt::Knob::HistogramPairTiles) == 2 ||
                  (rt::knob(rt::Knob::HistogramPairTiles) == 1 &&
                   !((hh.numBins + 1) / 2 <= tileCap && rt::knob(rt::Knob::HistogramPacked16) != 0))))
        {
            // PAIR: the tiles side by side in one launch, workgroups of one group on one XCD
            uint32_t const T = static_cast<uint32_t>(tiles);
            h.rShift = 0;
            h.tileBase = 0;
            h.pairTiles = T;
            h.tileBins = (h.nb + T - 1) / T;
            unsigned const g0 = streamingGrid(items, 64u * 4u * (kTileBlock / 64), 1);
            unsigned const groups = std::max(8u, g0 / T / 8u * 8u);
            unsigned const g = groups * T;
            size_t const lds = static_cast<size_t>(h.tileBins) * 4u;
#define VKT_PAIR(FMT, SH)                                                                                          \
    do {                                                                                                           \
        if (contig)                                                                                                \
            hipLaunchKernelGGL((histogramFastKernel<FMT, true, true, kTileBlock, SH, false, true>), dim3(g),        \
                               dim3(kTileBlock), lds, s, h);                                                       \
        else                                                                                                       \
            hipLaunchKernelGGL((histogramFastKernel<FMT, false, true, kTileBlock, SH, false, true>), dim3(g),       \
                               dim3(kTileBlock), lds, s, h);                                                       \
    } while (0)
            if (shift)
                VKT_PAIR(codec::FmtUInt16, true);
            else if (fmt == codec::FmtUInt16)
                VKT_PAIR(codec::FmtUInt16, false);
            else
                VKT_PAIR(codec::FmtFloat32, false);
#undef VKT_PAIR
        }
        else if (tiles > 1 && fmt != codec::FmtUInt8 && (hh.numBins + 1) / 2 <= tileCap &&
                 rt::knob(rt::Knob::HistogramPacked16) != 0)
        {
            // P16: every bin in one pass, two 16-bit counters per LDS word
            h.rShift = 0;
            h.tileBase = 0;
            h.tileBins = h.nb;
            unsigned const g = streamingGrid(items, 64u * 4u * (kTileBlock / 64), 1);
            size_t const lds = static_cast<size_t>((h.nb + 1) / 2) * 4u;
#define VKT_P16(FMT, SH)                                                                                           \
    do {                                                                                                           \
        if (contig)                                                                                                \
            hipLaunchKernelGGL((histogramFastKernel<FMT, true, true, kTileBlock, SH, true>), dim3(g),              \
                               dim3(kTileBlock), lds, s, h);                                                       \
        else                                                                                                       \
            hipLaunchKernelGGL((histogramFastKernel<FMT, false, true, kTileBlock, SH, true>), dim3(g),             \
                               dim3(kTileBlock), lds, s, h);                                                       \
    } while (0)
            tiledWithPartials<true>(h, g, s, [&] {
                if (shift)
                    VKT_P16(codec::FmtUInt16, true);
                else if (fmt == codec::FmtUInt16)
                    VKT_P16(codec::FmtUInt16, false);
                else
                    VKT_P16(codec::FmtFloat32, false);
            });
#undef VKT_P16
        }
        else
        {
            h.rShift = 0;
            unsigned const g = streamingGrid(items, 64u * 4u * (kTileBlock / 64), 1);
            for (uint64_t t = 0; t < tiles; ++t)
            {
                h.tileBase = static_cast<uint32_t>(t * tileCap);
                h.tileBins = static_cast<uint32_t>(std::min<uint64_t>(tileCap, hh.numBins - h.tileBase));
                tiledWithPartials<false>(h, g, s, [&] { VKT_FAST_HIST_FMT(true, kTileBlock, g, static_cast<size_t>(h.tileBins) * 4u); });
            }
        }
#undef VKT_FAST_HIST_FMT
#undef VKT_FAST_HIST
        return true;
    }

    // Grid of one aggregates pass (= number of partials it writes) and its launch: the
    // streaming kernel when the range qualifies, else the row kernel.
    unsigned aggGrid(BoxArgs const& a)
    {
        FastHistArgs h;
        bool contig;
        if (makeSpanArgs(a, h, contig))
            return streamingGrid(h.items, 64u * 4u * (kBlock / 64), 8);
        return rowGrid(a.rows);
    }

    void launchAggregates(BoxArgs const& a, int pass, unsigned g, hipStream_t s, float const* meanPtr, float meanV,
                          vktHipAggregatePartial_t* out)
    {
        FastHistArgs h;
        bool contig;
        if (makeSpanArgs(a, h, contig))
        {
            bool const unit = codec::isUnitMapping(a.lo, a.hi);
#define VKT_AGG_FAST_U(PASS, FMT, U)                                                                             \
    do {                                                                                                         \
        if (contig)                                                                                              \
            hipLaunchKernelGGL((aggregatesFastKernel<PASS, FMT, true, U>), dim3(g), dim3(kBlock), 0, s, h, meanPtr, meanV, out); \
        else                                                                                                     \
            hipLaunchKernelGGL((aggregatesFastKernel<PASS, FMT, false, U>), dim3(g), dim3(kBlock), 0, s, h, meanPtr, meanV, out); \
    } while (0)
#define VKT_AGG_FAST(PASS, FMT)                                                                                  \
    do {                                                                                                         \
        if (unit) VKT_AGG_FAST_U(PASS, FMT, true); else VKT_AGG_FAST_U(PASS, FMT, false);                        \
    } while (0)
#define VKT_AGG_FAST_FMT(PASS)                                                                                   \
    do {                                                                                                         \
        if (a.fmt == codec::FmtUInt8) VKT_AGG_FAST(PASS, codec::FmtUInt8);                                       \
        else if (a.fmt == codec::FmtUInt16) VKT_AGG_FAST(PASS, codec::FmtUInt16);                                \
        else VKT_AGG_FAST_U(PASS, codec::FmtFloat32, false);                                                     \
    } while (0)
            if (pass == 1)
                VKT_AGG_FAST_FMT(1);
            else
                VKT_AGG_FAST_FMT(2);
#undef VKT_AGG_FAST_FMT
#undef VKT_AGG_FAST
#undef VKT_AGG_FAST_U
            return;
        }
        if (pass == 1)
            VKT_REDUCE_DISPATCH(VKT_AGG_LAUNCH, 1, g, s, meanPtr, meanV, out);
        else
            VKT_REDUCE_DISPATCH(VKT_AGG_LAUNCH, 2, g, s, meanPtr, meanV, out);
    }

    struct AggScratch
    {
        rt::StreamScratch dev;
        vktHipAggregatePartial_t* host = nullptr;   // pinned: [0] pass 1, [1] pass 2
    };

    AggScratch& aggScratch()
    {
        static AggScratch s;
        return s;
    }

    // Code counts of a span walk into the device array h.bins (256 or 65 536 u64, zeroed here):
    // UInt8 aggregatesFastKernel<CODES>; UInt16 the histogram kernel's one-pass packed-16
    // counters with bin = code.  g: codeAggGrid.
    bool launchCodeCounts(FastHistArgs h, bool contig, int32_t fmt, unsigned g, hipStream_t s)
    {
        bool const u8 = fmt == codec::FmtUInt8;
        uint32_t const codes = u8 ? 256u : 65536u;
        if (hipMemsetAsync(h.bins, 0, codes * sizeof(unsigned long long), s) != hipSuccess)
            return false;
        auto* const none = static_cast<vktHipAggregatePartial_t*>(nullptr);
        if (u8)
        {
            h.rShift = 5;   // 32 copies of each counter: lane groups never share a bank (as the histogram)
            size_t const lds = 256u << (h.rShift + 2);
            if (contig)
                hipLaunchKernelGGL((aggregatesFastKernel<1, codec::FmtUInt8, true, false, true>), dim3(g), dim3(kBlock),
                                   lds, s, h, static_cast<float const*>(nullptr), 0.f, none);
            else if (!launchU8RowCounts(h, s))
                hipLaunchKernelGGL((aggregatesFastKernel<1, codec::FmtUInt8, false, false, true>), dim3(g), dim3(kBlock),
                                   lds, s, h, static_cast<float const*>(nullptr), 0.f, none);
        }
        else
        {
            // bin = (code * 1) >> 0 over 65 536 bins in one tile of packed 16-bit counters
            h.nb = 65536u;
            h.nbf = 65536.0f;
            h.binShift = 0u;
            h.binMul = 1u;
            h.rShift = 0;
            h.tileBase = 0;
            h.tileBins = 65536u;
            h.p16Step = rt::knob(rt::Knob::HistogramP16Step) != 0 ? 1u : 0u;
            size_t const lds = 32768u * 4u;
            if (contig)
                hipLaunchKernelGGL((histogramFastKernel<codec::FmtUInt16, true, true, kTileBlock, true, true>), dim3(g),
                                   dim3(kTileBlock), lds, s, h);
            else
                hipLaunchKernelGGL((histogramFastKernel<codec::FmtUInt16, false, true, kTileBlock, true, true>), dim3(g),
                                   dim3(kTileBlock), lds, s, h);
        }
        return true;
    }

    // work: device scratch of sizeof(CodeFinalWork) bytes (UInt16; its ticket is zeroed here)
    bool launchCodesFinal(unsigned long long const* counts, int32_t fmt, float lo, float hi, double numElems,
                          vktHipAggregatePartial_t* res, int32_t* targets, CodeFinalWork* work, hipStream_t s)
    {
        if (fmt == codec::FmtUInt8)
            hipLaunchKernelGGL((aggregatesCodesFinalKernel<codec::FmtUInt8, 0>), dim3(1), dim3(256), 0, s, counts, lo,
                               hi, numElems, res, targets, work);
        else
        {
            if (hipMemsetAsync(work, 0, 8, s) != hipSuccess)
                return false;
            hipLaunchKernelGGL((aggregatesCodesFinalKernel<codec::FmtUInt16, 1>), dim3(kCodeFinalBlocks), dim3(1024), 0,
                               s, counts, lo, hi, numElems, res, targets, work);
            hipLaunchKernelGGL((aggregatesCodesFinalKernel<codec::FmtUInt16, 2>), dim3(kCodeFinalBlocks), dim3(1024), 0,
                               s, counts, lo, hi, numElems, res, targets, work);
        }
        return true;
    }

    // First occurrences of codes targets[0] / [1] in the walk h into res[0].minIndex / maxIndex.
    void launchFindCodes(FastHistArgs const& h, bool contig, int32_t fmt, int32_t const* targets,
                         vktHipAggregatePartial_t* res, hipStream_t s)
    {
        uint64_t const head = 1024u * kFindHeadBlocks;   // stage 1 covers the first 512 Ki voxels at most
        unsigned const gf = static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(2048, (h.items + kBlock - 1) / kBlock)));
        unsigned const gh = static_cast<unsigned>(std::max<uint64_t>(1, (std::min<uint64_t>(head, h.items) + 1023) / 1024));
#define VKT_FIND(B, CT)                                                                                          \
    do {                                                                                                         \
        hipLaunchKernelGGL((aggregatesFindHeadKernel<B, CT>), dim3(gh), dim3(1024), 0, s, h, targets, res, head);  \
        hipLaunchKernelGGL((aggregatesFindTailKernel<B, CT>), dim3(gf), dim3(kBlock), 0, s, h, targets, res, head); \
    } while (0)
        if (fmt == codec::FmtUInt8)
        {
            if (contig) VKT_FIND(1, true); else VKT_FIND(1, false);
        }
        else
        {
            if (contig) VKT_FIND(2, true); else VKT_FIND(2, false);
        }
#undef VKT_FIND
    }

    // UInt8 / UInt16 aggregates in one data pass: code counts, aggregatesCodesFinalKernel, then the
    // first-occurrence search, into res[0], res[1]; false when the range does not take the
    // streaming walk.  scratch: the code counts (256 or 65 536), 2 target codes
    // + 8 B, then the final kernel's CodeFinalWork.
    bool launchCodeAggregates(BoxArgs const& a, hipStream_t s, double numElems, void* scratch, unsigned g,
                              vktHipAggregatePartial_t* res)
    {
        FastHistArgs h;
        bool contig;
        if (!makeSpanArgs(a, h, contig))
            return false;
        uint32_t const codes = a.fmt == codec::FmtUInt8 ? 256u : 65536u;
        h.bins = static_cast<unsigned long long*>(scratch);
        auto* const targets = reinterpret_cast<int32_t*>(h.bins + codes);
        auto* const work = reinterpret_cast<CodeFinalWork*>(targets + 4);
        if (!launchCodeCounts(h, contig, a.fmt, g, s))
            return false;
        if (!launchCodesFinal(h.bins, a.fmt, a.lo, a.hi, numElems, res, targets, work, s))
            return false;
        launchFindCodes(h, contig, a.fmt, targets, res, s);
        return true;
    }

    // The integer-moments kernel variant (knob aggregates.moments_pipe: 0 one buffer, 4 items per
    // lane and step; 1 two buffers (next step's loads in flight during this step's arithmetic),
    // 4 items; 2 two buffers, 8 items; 3 one buffer, 8 items; 4 two buffers, 2 items; 5 as 1, bound to
    // 7 waves per SIMD for spans) and its grid: as many workgroups as the variant keeps
    // resident on every CU (hipOccupancyMaxActiveBlocksPerMultiprocessor, at most 8) -- a grid-
    // stride walk with more would leave a second partial wave of workgroups running alone.
    using MomentKernelU16 = void (*)(FastHistArgs, MomentPartialU16*);

    template <bool CONTIG>
    MomentKernelU16 momentKernelU16(int64_t v, int& itemsPerLane)
    {
        switch (v)
        {
        case 1: itemsPerLane = 4; return aggregatesMomentsU16Kernel<CONTIG, 4, true>;
        case 2: itemsPerLane = 8; return aggregatesMomentsU16Kernel<CONTIG, 8, true>;
        case 3: itemsPerLane = 8; return aggregatesMomentsU16Kernel<CONTIG, 8, false>;
        case 4: itemsPerLane = 2; return aggregatesMomentsU16Kernel<CONTIG, 2, true>;
        case 5: itemsPerLane = 4; return aggregatesMomentsU16Kernel<CONTIG, 4, true, CONTIG ? 7 : 0>;
        default: itemsPerLane = 4; return aggregatesMomentsU16Kernel<CONTIG, 4, false>;
        }
    }

    MomentKernelU16 momentKernelU16(bool contig, int& itemsPerLane)
    {
        int64_t const v = rt::knob(rt::Knob::AggregatesMomentsPipe);
        return contig ? momentKernelU16<true>(v, itemsPerLane) : momentKernelU16<false>(v, itemsPerLane);
    }

    unsigned residentBlocksPerCU(void const* fn)
    {
        static std::mutex mu;
        static std::unordered_map<void const*, unsigned> cache;
        std::lock_guard<std::mutex> lock(mu);
        auto it = cache.find(fn);
        if (it != cache.end())
            return it->second;
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kBlock, 0) != hipSuccess || n < 1)
        {
            (void)hipGetLastError();
            n = 4;
        }
        unsigned const r = static_cast<unsigned>(std::min(n, 8));
        cache.emplace(fn, r);
        return r;
    }

    unsigned momentGridItemsU16(uint64_t items, bool contig)
    {
        int u = 4;
        MomentKernelU16 const k = momentKernelU16(contig, u);
        return streamingGrid(items, 64u * static_cast<unsigned>(u) * (kBlock / 64),
                             residentBlocksPerCU(reinterpret_cast<void const*>(k)));
    }

    void launchMomentsU16Kernel(FastHistArgs const& h, bool contig, unsigned g, MomentPartialU16* parts, hipStream_t s)
    {
        int u = 4;
        hipLaunchKernelGGL(momentKernelU16(contig, u), dim3(g), dim3(kBlock), 0, s, h, parts);
    }

    // UInt16 under the unit mapping: ComputeAggregates from one pass of integer moments
    // (aggregatesMomentsU16Kernel + its final kernel) into res[0], res[1]; 0 when the range does
    // not take it, else the number of partials (scratch: that many MomentPartialU16).
    // Knob aggregates.moments, bit 0.
    unsigned momentGridU16(BoxArgs const& a, FastHistArgs& h, bool& contig)
    {
        if (a.fmt != codec::FmtUInt16 || !codec::isUnitMapping(a.lo, a.hi) ||
            (rt::knob(rt::Knob::AggregatesMoments) & 1) == 0 || !makeSpanArgs(a, h, contig))
            return 0;
        return momentGridItemsU16(h.items, contig);
    }

    // 1 when some UInt16 (Int16) code decodes to a nonzero |v| < 2^-40 under (lo, hi): every code
    // once on the host, the answer kept per thread for the last mapping
    uint32_t tinyCodesU16(float lo, float hi, int32_t fmt = codec::FmtUInt16)
    {
        thread_local uint64_t lastKey = ~0ull;
        thread_local uint32_t lastTiny = 0;
        uint64_t const key = (static_cast<uint64_t>(codec::floatToBits(lo)) << 32 | codec::floatToBits(hi)) ^
                             (fmt == codec::FmtInt16 ? 1ull << 63 | 1ull : 0ull);
        if (key != lastKey)
        {
            uint32_t t = 0;
            for (uint32_t c = 0; c < 65536u && !t; ++c)
            {
                float const v = std::fabs(codec::decode(c, fmt, lo, hi));
                t = v != 0.f && v < 0x1p-40f ? 1u : 0u;
            }
            lastKey = key;
            lastTiny = t;
        }
        return lastTiny;
    }

    // UInt16 under any other mapping and Float32: one pass of floating-point moments
    // (aggregatesMomentsFKernel); knob aggregates.moments bit 1.  0 when the range does not take
    // it, else the number of partials.  tiny: some UInt16 code decodes to a nonzero |v| < 2^-40.
    unsigned momentGridF(BoxArgs const& a, FastHistArgs& h, bool& contig, uint32_t& tiny)
    {
        tiny = 0;
        bool const fmtOk = (a.fmt == codec::FmtUInt16 && !codec::isUnitMapping(a.lo, a.hi)) || a.fmt == codec::FmtFloat32 ||
                           ((a.fmt == codec::FmtInt16 || a.fmt == codec::FmtUInt32) &&
                            (rt::knob(rt::Knob::AggregatesMoments) & 4) != 0);
        BoxArgs w = a;   // (Int16 / UInt32: the item walk of the 2- / 4-byte span)
        if (a.fmt == codec::FmtInt16)
            w.fmt = codec::FmtUInt16;
        else if (a.fmt == codec::FmtUInt32)
            w.fmt = codec::FmtFloat32;
        if (!fmtOk || (rt::knob(rt::Knob::AggregatesMoments) & 2) == 0 || !makeSpanArgs(w, h, contig))
            return 0;
        if (a.fmt == codec::FmtUInt16 || a.fmt == codec::FmtInt16)
            tiny = tinyCodesU16(a.lo, a.hi, a.fmt);
        return streamingGrid(h.items, 64u * 4u * (kBlock / 64), 8);
    }

    void launchMomentsF(FastHistArgs const& h, bool contig, int32_t fmt, unsigned g, double numElems, uint32_t tiny,
                        MomentPartialF* parts, vktHipAggregatePartial_t* res, hipStream_t s)
    {
#define VKT_MOMF(FMT)                                                                                            \
    do {                                                                                                         \
        if (contig)                                                                                              \
            hipLaunchKernelGGL((aggregatesMomentsFKernel<FMT, true>), dim3(g), dim3(kBlock), 0, s, h, parts);   \
        else                                                                                                     \
            hipLaunchKernelGGL((aggregatesMomentsFKernel<FMT, false>), dim3(g), dim3(kBlock), 0, s, h, parts);  \
    } while (0)
        if (fmt == codec::FmtUInt16)
            VKT_MOMF(codec::FmtUInt16);
        else if (fmt == codec::FmtInt16)
            VKT_MOMF(codec::FmtInt16);
        else if (fmt == codec::FmtUInt32)
            VKT_MOMF(codec::FmtUInt32);
        else
            VKT_MOMF(codec::FmtFloat32);
#undef VKT_MOMF
        hipLaunchKernelGGL(aggregatesMomentsFFinalKernel, dim3(1), dim3(kBlock), 0, s, parts, g, numElems, tiny, res);
    }

    void launchMomentsU16(FastHistArgs const& h, bool contig, unsigned g, double numElems, MomentPartialU16* parts,
                          vktHipAggregatePartial_t* res, hipStream_t s)
    {
        launchMomentsU16Kernel(h, contig, g, parts, s);
        hipLaunchKernelGGL(aggregatesMomentsU16FinalKernel, dim3(1), dim3(kBlock), 0, s, parts, g, numElems, res);
    }

    // Grid of the code-count pass (0 when the range does not take it): UInt8 32 KiB of counters
    // per workgroup, 4 per CU; UInt16 the packed-16 histogram's one 1024-thread workgroup per CU.
    // Knob aggregates.codes: bit 0 UInt8, bit 1 UInt16.
    unsigned codeAggGrid(BoxArgs const& a)
    {
        FastHistArgs h;
        bool contig;
        int64_t const k = rt::knob(rt::Knob::AggregatesCodes);
        bool const on = (a.fmt == codec::FmtUInt8 && (k & 1)) || (a.fmt == codec::FmtUInt16 && (k & 2));
        if (!on || !makeSpanArgs(a, h, contig))
            return 0;
        if (a.fmt == codec::FmtUInt8)
            return streamingGrid(h.items, 64u * 4u * (kBlock / 64), 4);
        return streamingGrid(h.items, 64u * 4u * (kTileBlock / 64), 1);
    }

} // hipk
} // vkt

using namespace vkt;
using namespace vkt::hipk;

extern "C" {

vktError vktHipAggregatePartialInit(vktHipAggregatePartial_t* p)
{
    if (!p)
        return rt::fail("vktHipAggregatePartialInit: null pointer");
    std::memset(p, 0, sizeof(*p));
    p->prod = 1.0;
    p->minValue = FLT_MAX;
    p->maxValue = -FLT_MAX;
    p->minIndex = kNoIndex;
    p->maxIndex = kNoIndex;
    return vktNoError;
}

vktError vktHipAggregatePartialCombine(vktHipAggregatePartial_t* acc, vktHipAggregatePartial_t const* other)
{
    if (!acc || !other)
        return rt::fail("vktHipAggregatePartialCombine: null pointer");
    vktHipAggregatePartial_t const& o = *other;
    if (o.minValue < acc->minValue || (o.minValue == acc->minValue && o.minIndex < acc->minIndex))
    {
        acc->minValue = o.minValue;
        acc->minIndex = o.minIndex;
    }
    if (o.maxValue > acc->maxValue || (o.maxValue == acc->maxValue && o.maxIndex < acc->maxIndex))
    {
        acc->maxValue = o.maxValue;
        acc->maxIndex = o.maxIndex;
    }
    acc->sum += o.sum;
    acc->prod *= o.prod;
    acc->sumSq += o.sumSq;
    acc->count += o.count;
    return vktNoError;
}

float vktHipAggregatesMean(vktHipAggregatePartial_t const* pass1, uint64_t numElems)
{
    return static_cast<float>(static_cast<double>(static_cast<float>(pass1->sum)) / static_cast<double>(numElems));
}

vktError vktHipAggregatesPass(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last, int32_t zGlobalOffset,
                              int32_t pass, float mean, vktHipAggregatePartial_t* out)
{
    if (!out || (pass != 1 && pass != 2))
        return rt::fail("vktHipAggregatesPass: bad arguments");
    vktHipAggregatePartialInit(out);
    BoxArgs a{};
    vktError e;
    if (!makeBox(volume, first, last, zGlobalOffset, a, "vktHipAggregatesPass: invalid volume view", e))
        return e;
    hipStream_t s = rt::computeStream();
    unsigned const g = aggGrid(a);
    AggScratch& sc = aggScratch();
    size_t const bytes = (static_cast<size_t>(g) + 1) * sizeof(vktHipAggregatePartial_t);
    auto* partials = static_cast<vktHipAggregatePartial_t*>(sc.dev.acquire(bytes, s));
    if (!partials)
        return vktInvalidValue;
    if (!sc.host && rt::check(hipHostMalloc(reinterpret_cast<void**>(&sc.host), 2 * sizeof(vktHipAggregatePartial_t)),
                              "hipHostMalloc") != vktNoError)
    {
        sc.dev.release(s);
        return vktInvalidValue;
    }
    launchAggregates(a, pass, g, s, nullptr, pass == 1 ? 0.f : mean, partials);
    hipLaunchKernelGGL(aggregatesFinalKernel, dim3(1), dim3(kBlock), 0, s, partials, g, partials + g,
                       static_cast<float*>(nullptr), 1.0);
    e = rt::check(hipMemcpyAsync(sc.host, partials + g, sizeof(vktHipAggregatePartial_t), hipMemcpyDeviceToHost, s),
                  "hipMemcpyAsync(aggregates)");
    sc.dev.release(s);
    if (e != vktNoError)
        return e;
    VKT_HIP_TRY(hipStreamSynchronize(s));
    *out = sc.host[0];
    return rt::finishLaunch("AggregatesPass_hip");
}

vktError vktHipAggregatesFinish(vktHipAggregatePartial_t const* pass1, vktHipAggregatePartial_t const* pass2,
                                uint64_t numElems, int32_t dimX, int32_t dimY, vktAggregates_t* out)
{
    if (!pass1 || !pass2 || !out)
        return rt::fail("vktHipAggregatesFinish: null pointer");
    std::memset(out, 0, sizeof(*out));   // Aggregates_serial.hpp:27
    auto coords = [&](uint64_t i) {
        uint64_t const px = static_cast<uint64_t>(dimX), py = static_cast<uint64_t>(dimY);
        return vktVec3i_t{static_cast<int>(i % px), static_cast<int>((i / px) % py), static_cast<int>(i / (px * py))};
    };
    out->min = pass1->minIndex == kNoIndex ? FLT_MAX : pass1->minValue;
    out->max = pass1->maxIndex == kNoIndex ? -FLT_MAX : pass1->maxValue;
    if (pass1->minIndex != kNoIndex)
        out->argmin = coords(pass1->minIndex);
    if (pass1->maxIndex != kNoIndex)
        out->argmax = coords(pass1->maxIndex);
    out->sum = static_cast<float>(pass1->sum);
    out->prod = pass1->count ? static_cast<float>(pass1->prod) : 1.f;
    double const n = static_cast<double>(numElems);
    out->mean = static_cast<float>(static_cast<double>(out->sum) / n);     // mean /= (double)numElems
    float const varAcc = static_cast<float>(pass2->sumSq);
    out->var = static_cast<float>(static_cast<double>(varAcc) / n);
    out->stddev = sqrtf(out->var);
    return vktNoError;
}

vktError vktHipAggregatesRange(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last, vktAggregates_t* out)
{
    if (!out)
        return rt::fail("vktHipAggregatesRange: null pointer");
    vktHipAggregatePartial_t p1, p2;
    vktHipAggregatePartialInit(&p1);
    vktHipAggregatePartialInit(&p2);
    uint64_t const numElems = static_cast<uint64_t>(volume.dimX > 0 ? volume.dimX : 0) *
                              static_cast<uint64_t>(volume.dimY > 0 ? volume.dimY : 0) *
                              static_cast<uint64_t>(volume.dimZ > 0 ? volume.dimZ : 0);
    BoxArgs a{};
    vktError e;
    bool done = false;
    bool const boxed = makeBox(volume, first, last, 0, a, "vktHipAggregatesRange: invalid volume view", e);
    FastHistArgs hm;
    bool contigM = false;
    uint32_t tiny = 0;
    unsigned const gm = boxed ? momentGridU16(a, hm, contigM) : 0u;
    unsigned const gf = boxed && gm == 0 ? momentGridF(a, hm, contigM, tiny) : 0u;
    unsigned const gc = boxed && gm == 0 && gf == 0 ? codeAggGrid(a) : 0u;
    if (gm != 0 || gf != 0)
    {
        // UInt16 under the unit mapping: one pass of exact integer moments, complete; other
        // mappings / Float32: one pass of float moments, the two passes below when it says so
        hipStream_t s = rt::computeStream();
        AggScratch& sc = aggScratch();
        size_t const bytes = 2 * sizeof(vktHipAggregatePartial_t) +
                             std::max(static_cast<size_t>(gm) * sizeof(MomentPartialU16),
                                      static_cast<size_t>(gf) * sizeof(MomentPartialF));
        auto* res = static_cast<vktHipAggregatePartial_t*>(sc.dev.acquire(bytes, s));
        if (!res)
            return vktInvalidValue;
        if (!sc.host && rt::check(hipHostMalloc(reinterpret_cast<void**>(&sc.host),
                                                2 * sizeof(vktHipAggregatePartial_t)),
                                  "hipHostMalloc") != vktNoError)
        {
            sc.dev.release(s);
            return vktInvalidValue;
        }
        if (gm != 0)
            launchMomentsU16(hm, contigM, gm, static_cast<double>(numElems),
                             reinterpret_cast<MomentPartialU16*>(res + 2), res, s);
        else
            launchMomentsF(hm, contigM, a.fmt, gf, static_cast<double>(numElems), tiny,
                           reinterpret_cast<MomentPartialF*>(res + 2), res, s);
        e = rt::check(hipMemcpyAsync(sc.host, res, 2 * sizeof(vktHipAggregatePartial_t), hipMemcpyDeviceToHost, s),
                      "hipMemcpyAsync(aggregates)");
        sc.dev.release(s);
        if (e != vktNoError)
            return e;
        VKT_HIP_TRY(hipStreamSynchronize(s));
        if ((e = rt::finishLaunch("AggregatesRange_hip")) != vktNoError)
            return e;
        if (sc.host[1].count == 1u)
        {
            p1 = sc.host[0];
            p2 = sc.host[1];
            done = true;
        }
    }
    else if (gc != 0)
    {
        // UInt8 / UInt16: one pass of code counts; the two float passes below only when the
        // counts cannot give the first occurrence of an extreme (aggregatesCodesFinalKernel)
        hipStream_t s = rt::computeStream();
        AggScratch& sc = aggScratch();
        size_t const bytes = 2 * sizeof(vktHipAggregatePartial_t) + 65536 * sizeof(unsigned long long) + 16 +
                             sizeof(CodeFinalWork);
        auto* res = static_cast<vktHipAggregatePartial_t*>(sc.dev.acquire(bytes, s));
        if (!res)
            return vktInvalidValue;
        if (!sc.host && rt::check(hipHostMalloc(reinterpret_cast<void**>(&sc.host),
                                                2 * sizeof(vktHipAggregatePartial_t)),
                                  "hipHostMalloc") != vktNoError)
        {
            sc.dev.release(s);
            return vktInvalidValue;
        }
        // layout: the two results, then the code counts and the 2 target codes
        bool const launched = launchCodeAggregates(a, s, static_cast<double>(numElems), res + 2, gc, res);
        e = launched ? rt::check(hipMemcpyAsync(sc.host, res, 2 * sizeof(vktHipAggregatePartial_t),
                                                hipMemcpyDeviceToHost, s),
                                 "hipMemcpyAsync(aggregates)")
                     : rt::fail("vktHipAggregatesRange: code-count launch failed");
        sc.dev.release(s);
        if (e != vktNoError)
            return e;
        VKT_HIP_TRY(hipStreamSynchronize(s));
        if ((e = rt::finishLaunch("AggregatesRange_hip")) != vktNoError)
            return e;
        if (sc.host[1].count == 1u)
        {
            p1 = sc.host[0];
            p2 = sc.host[1];
            done = true;
        }
    }
    if (!done && makeBox(volume, first, last, 0, a, "vktHipAggregatesRange: invalid volume view", e))
    {
        // both passes and the mean stay on the device: one host round trip at the end
        hipStream_t s = rt::computeStream();
        unsigned const g = aggGrid(a);
        AggScratch& sc = aggScratch();
        size_t const bytes = (2 * static_cast<size_t>(g) + 2) * sizeof(vktHipAggregatePartial_t) + 16;
        auto* partials = static_cast<vktHipAggregatePartial_t*>(sc.dev.acquire(bytes, s));
        if (!partials)
            return vktInvalidValue;
        if (!sc.host && rt::check(hipHostMalloc(reinterpret_cast<void**>(&sc.host),
                                                2 * sizeof(vktHipAggregatePartial_t)),
                                  "hipHostMalloc") != vktNoError)
        {
            sc.dev.release(s);
            return vktInvalidValue;
        }
        vktHipAggregatePartial_t* res = partials + 2 * g;   // [0] pass 1, [1] pass 2
        float* meanDev = reinterpret_cast<float*>(res + 2);
        launchAggregates(a, 1, g, s, nullptr, 0.f, partials);
        hipLaunchKernelGGL(aggregatesFinalKernel, dim3(1), dim3(kBlock), 0, s, partials, g, res, meanDev,
                           static_cast<double>(numElems));
        launchAggregates(a, 2, g, s, meanDev, 0.f, partials + g);
        hipLaunchKernelGGL(aggregatesFinalKernel, dim3(1), dim3(kBlock), 0, s, partials + g, g, res + 1,
                           static_cast<float*>(nullptr), 1.0);
        e = rt::check(hipMemcpyAsync(sc.host, res, 2 * sizeof(vktHipAggregatePartial_t), hipMemcpyDeviceToHost, s),
                      "hipMemcpyAsync(aggregates)");
        sc.dev.release(s);
        if (e != vktNoError)
            return e;
        VKT_HIP_TRY(hipStreamSynchronize(s));
        p1 = sc.host[0];
        p2 = sc.host[1];
        e = rt::finishLaunch("AggregatesRange_hip");
        if (e != vktNoError)
            return e;
    }
    else if (!done && e != vktNoError)
        return e;
    return vktHipAggregatesFinish(&p1, &p2, numElems, volume.dimX, volume.dimY, out);
}

int32_t vktHipAggregateMomentsSupported(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last)
{
    if (volume.dataFormat != codec::FmtUInt16 && volume.dataFormat != codec::FmtFloat32)
        return 0;
    BoxArgs a{};
    vktError e;
    if (!makeBox(volume, first, last, 0, a, "vktHipAggregateMomentsSupported: invalid volume view", e))
        return e == vktNoError ? 1 : 0;   // an empty range: count 0
    FastHistArgs h;
    bool contig;
    return makeSpanArgs(a, h, contig) ? 1 : 0;
}

vktError vktHipAggregateMoments(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last, int32_t zGlobalOffset,
                                vktHipMomentPartial_t* partial)
{
    if (partial == nullptr)
        return rt::fail("vktHipAggregateMoments: null partial");
    if (volume.dataFormat != codec::FmtUInt16 && volume.dataFormat != codec::FmtFloat32)
        return rt::fail("vktHipAggregateMoments: UInt16 / Float32 volumes only");
    bool const integer = volume.dataFormat == codec::FmtUInt16 && codec::isUnitMapping(volume.mappingLo, volume.mappingHi);
    vktHipMomentPartial_t& o = *partial;
    std::memset(&o, 0, sizeof(o));
    o.prod = 1.0;
    o.minValue = FLT_MAX;
    o.maxValue = -FLT_MAX;
    o.minIndex = o.maxIndex = kNoIndex;
    o.form = integer ? 1 : 2;
    o.flags = !integer && volume.dataFormat == codec::FmtUInt16 && tinyCodesU16(volume.mappingLo, volume.mappingHi)
                  ? 2u
                  : 0u;
    BoxArgs a{};
    vktError e;
    if (!makeBox(volume, first, last, zGlobalOffset, a, "vktHipAggregateMoments: invalid volume view", e))
        return e;   // empty range: the empty partial
    FastHistArgs h;
    bool contig;
    if (!makeSpanArgs(a, h, contig))
        return rt::fail("vktHipAggregateMoments: the range does not take the moments walk (16-B aligned volume with "
                        "dimX % 8 == 0 needed)");
    unsigned const g = integer ? momentGridItemsU16(h.items, contig) : streamingGrid(h.items, 64u * 4u * (kBlock / 64), 8);
    hipStream_t s = rt::computeStream();
    AggScratch& sc = aggScratch();
    size_t const unit = std::max(sizeof(MomentPartialU16), sizeof(MomentPartialF));
    auto* parts = static_cast<uint8_t*>(sc.dev.acquire((static_cast<size_t>(g) + 1) * unit, s));
    if (!parts)
        return vktInvalidValue;
    union
    {
        MomentPartialU16 u;
        MomentPartialF f;
    } host;
    if (integer)
    {
        auto* pp = reinterpret_cast<MomentPartialU16*>(parts);
        launchMomentsU16Kernel(h, contig, g, pp, s);
        hipLaunchKernelGGL(momentsCombineU16Kernel, dim3(1), dim3(kBlock), 0, s, pp, g, pp + g);
        e = rt::check(hipMemcpyAsync(&host.u, pp + g, sizeof(host.u), hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
    }
    else
    {
        auto* pp = reinterpret_cast<MomentPartialF*>(parts);
        if (a.fmt == codec::FmtUInt16)
        {
            if (contig)
                hipLaunchKernelGGL((aggregatesMomentsFKernel<codec::FmtUInt16, true>), dim3(g), dim3(kBlock), 0, s, h, pp);
            else
                hipLaunchKernelGGL((aggregatesMomentsFKernel<codec::FmtUInt16, false>), dim3(g), dim3(kBlock), 0, s, h,
                                   pp);
        }
        else if (contig)
            hipLaunchKernelGGL((aggregatesMomentsFKernel<codec::FmtFloat32, true>), dim3(g), dim3(kBlock), 0, s, h, pp);
        else
            hipLaunchKernelGGL((aggregatesMomentsFKernel<codec::FmtFloat32, false>), dim3(g), dim3(kBlock), 0, s, h, pp);
        hipLaunchKernelGGL(momentsCombineFKernel, dim3(1), dim3(kBlock), 0, s, pp, g, pp + g);
        e = rt::check(hipMemcpyAsync(&host.f, pp + g, sizeof(host.f), hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
    }
    sc.dev.release(s);
    if (e != vktNoError)
        return e;
    VKT_HIP_TRY(hipStreamSynchronize(s));
    if (integer)
    {
        MomentPartialU16 const& u = host.u;
        o.count = u.count;
        o.codeSum = u.sumC;
        o.codeSumSqLo = u.sumSqLo;
        o.codeSumSqHi = u.sumSqHi;
        o.prod = u.prod;
        if (u.cmin <= 0xFFFFu)
        {
            o.minValue = static_cast<float>(u.cmin) * 0x1p-16f;
            o.minIndex = u.minIndex;
        }
        if (u.cmax >= 0)
        {
            o.maxValue = static_cast<float>(u.cmax) * 0x1p-16f;
            o.maxIndex = u.maxIndex;
        }
    }
    else
    {
        MomentPartialF const& f = host.f;
        o.count = f.count;
        o.mean = f.mean;
        o.m2 = f.m2;
        o.sum = f.sum;
        o.prod = f.prod;
        o.minValue = f.minValue;
        o.maxValue = f.maxValue;
        o.minIndex = f.minIndex;
        o.maxIndex = f.maxIndex;
        o.flags |= f.flags;
    }
    return rt::finishLaunch("AggregateMoments_hip");
}

// Host combine of rank partials in the given order + the finish of the final kernels
// (aggregatesMomentsU16FinalKernel / aggregatesMomentsFFinalKernel: the same formulas).
vktError vktHipAggregatesFromMoments(vktHipMomentPartial_t const* partials, int32_t numPartials, uint64_t numElems,
                                     int32_t dimX, int32_t dimY, vktAggregates_t* aggregates, int32_t* complete)
{
    if (partials == nullptr || aggregates == nullptr || complete == nullptr || numPartials <= 0)
        return rt::fail("vktHipAggregatesFromMoments: null pointer or no partials");
    int32_t const form = partials[0].form;
    if (form != 1 && form != 2)
        return rt::fail("vktHipAggregatesFromMoments: unknown partial form");
    vktHipAggregatePartial_t one, two;
    vktHipAggregatePartialInit(&one);
    vktHipAggregatePartialInit(&two);
    double const N = static_cast<double>(numElems);
    uint64_t count = 0;
    bool ok = true;
    auto extremes = [&](vktHipMomentPartial_t const& q) {
        if (q.minIndex != kNoIndex &&
            (q.minValue < one.minValue || (q.minValue == one.minValue && q.minIndex < one.minIndex)))
        {
            one.minValue = q.minValue;
            one.minIndex = q.minIndex;
        }
        if (q.maxIndex != kNoIndex &&
            (q.maxValue > one.maxValue || (q.maxValue == one.maxValue && q.maxIndex < one.maxIndex)))
        {
            one.maxValue = q.maxValue;
            one.maxIndex = q.maxIndex;
        }
    };
    if (form == 1)
    {
        uint64_t sc = 0;
        unsigned __int128 sc2 = 0;
        for (int32_t i = 0; i < numPartials; ++i)
        {
            vktHipMomentPartial_t const& q = partials[i];
            if (q.form != form)
                return rt::fail("vktHipAggregatesFromMoments: partials of different forms");
            count += q.count;
            sc += q.codeSum;
            sc2 += (static_cast<unsigned __int128>(q.codeSumSqHi) << 64) | q.codeSumSqLo;
            one.prod *= q.prod;
            extremes(q);
        }
        one.sum = static_cast<double>(sc) * 0x1p-16;
        float const m = static_cast<float>(static_cast<double>(static_cast<float>(one.sum)) / N);
        double const mu = static_cast<double>(m) * 65536.0;
        unsigned __int128 const t = static_cast<unsigned __int128>(count) * sc2 - static_cast<unsigned __int128>(sc) * sc;
        double const td = static_cast<double>(static_cast<uint64_t>(t >> 64)) * 0x1p64 + static_cast<double>(static_cast<uint64_t>(t));
        double const dn = static_cast<double>(count);
        double const r = std::fma(-dn, mu, static_cast<double>(sc));
        two.sumSq = count ? (td + r * r) / dn * 0x1p-32 : 0.0;
    }
    else
    {
        double mean = 0.0, m2 = 0.0;
        uint32_t flags = 0;
        for (int32_t i = 0; i < numPartials; ++i)
        {
            vktHipMomentPartial_t const& q = partials[i];
            if (q.form != form)
                return rt::fail("vktHipAggregatesFromMoments: partials of different forms");
            flags |= q.flags;
            if (q.count != 0)
            {
                if (count == 0)
                {
                    mean = q.mean;
                    m2 = q.m2;
                }
                else
                {
                    double const na = static_cast<double>(count), nb = static_cast<double>(q.count);
                    double const n = na + nb, delta = q.mean - mean;
                    mean += delta * (nb / n);
                    m2 += q.m2 + delta * delta * (na * nb / n);
                }
            }
            count += q.count;
            one.sum += q.sum;
            one.prod *= q.prod;
            extremes(q);
        }
        float const m = static_cast<float>(static_cast<double>(static_cast<float>(one.sum)) / N);
        double const dm = static_cast<double>(m);
        ok = (flags & 1u) == 0 && std::fabs(one.sum) <= DBL_MAX && m2 <= DBL_MAX && (flags & 2u) == 0 &&
             (m == 0.f || std::fabs(m) >= 0x1p-40f);
        if (count != 0)
            ok = ok && std::fabs(static_cast<double>(one.maxValue) - dm) < 0x1p62 &&
                 std::fabs(static_cast<double>(one.minValue) - dm) < 0x1p62;
        double const dd = mean - dm;
        two.sumSq = count ? m2 + static_cast<double>(count) * dd * dd : 0.0;
    }
    one.count = count;
    *complete = ok ? 1 : 0;
    return vktHipAggregatesFinish(&one, &two, numElems, dimX, dimY, aggregates);
}

vktError vktHipAggregateCodeCounts(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last, uint64_t* counts)
{
    if (counts == nullptr)
        return rt::fail("vktHipAggregateCodeCounts: null counts");
    if (volume.dataFormat != codec::FmtUInt8 && volume.dataFormat != codec::FmtUInt16)
        return rt::fail("vktHipAggregateCodeCounts: UInt8 / UInt16 volumes only");
    uint32_t const codes = volume.dataFormat == codec::FmtUInt8 ? 256u : 65536u;
    hipStream_t s = rt::computeStream();
    BoxArgs a{};
    vktError e;
    if (!makeBox(volume, first, last, 0, a, "vktHipAggregateCodeCounts: invalid volume view", e))
    {
        if (e != vktNoError)
            return e;
        VKT_HIP_TRY(hipMemsetAsync(counts, 0, codes * sizeof(uint64_t), s));   // empty range
        return rt::finishLaunch("AggregateCodeCounts_hip");
    }
    FastHistArgs h;
    bool contig;
    if (!makeSpanArgs(a, h, contig))
        return rt::fail("vktHipAggregateCodeCounts: the range does not take the code-count walk (16-B aligned volume "
                        "with dimX % 8 == 0 needed)");
    h.bins = reinterpret_cast<unsigned long long*>(counts);
    unsigned const g = a.fmt == codec::FmtUInt8 ? streamingGrid(h.items, 64u * 4u * (kBlock / 64), 4)
                                                : streamingGrid(h.items, 64u * 4u * (kTileBlock / 64), 1);
    if (!launchCodeCounts(h, contig, a.fmt, g, s))
        return rt::check(hipGetLastError(), "vktHipAggregateCodeCounts");
    return rt::finishLaunch("AggregateCodeCounts_hip");
}

int32_t vktHipAggregateCodesSupported(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last)
{
    if (volume.dataFormat != codec::FmtUInt8 && volume.dataFormat != codec::FmtUInt16)
        return 0;
    BoxArgs a{};
    vktError e;
    if (!makeBox(volume, first, last, 0, a, "vktHipAggregateCodesSupported: invalid volume view", e))
        return e == vktNoError ? 1 : 0;   // an empty range counts nothing
    FastHistArgs h;
    bool contig;
    return makeSpanArgs(a, h, contig) ? 1 : 0;
}

vktError vktHipAggregatesFromCodes(uint64_t const* counts, int32_t dataFormat, float mappingLo, float mappingHi,
                                   uint64_t numElems, vktHipAggregatePartial_t* pass1, vktHipAggregatePartial_t* pass2,
                                   int32_t* codes)
{
    if (counts == nullptr || pass1 == nullptr || pass2 == nullptr || codes == nullptr)
        return rt::fail("vktHipAggregatesFromCodes: null pointer");
    if (dataFormat != codec::FmtUInt8 && dataFormat != codec::FmtUInt16)
        return rt::fail("vktHipAggregatesFromCodes: UInt8 / UInt16 only");
    hipStream_t s = rt::computeStream();
    AggScratch& sc = aggScratch();
    size_t const bytes = 2 * sizeof(vktHipAggregatePartial_t) + 16 + sizeof(CodeFinalWork);
    auto* res = static_cast<vktHipAggregatePartial_t*>(sc.dev.acquire(bytes, s));
    if (!res)
        return vktInvalidValue;
    auto* targets = reinterpret_cast<int32_t*>(res + 2);
    if (!launchCodesFinal(reinterpret_cast<unsigned long long const*>(counts), dataFormat, mappingLo, mappingHi,
                          static_cast<double>(numElems), res, targets, reinterpret_cast<CodeFinalWork*>(targets + 4), s))
    {
        sc.dev.release(s);
        return rt::check(hipGetLastError(), "vktHipAggregatesFromCodes");
    }
    struct
    {
        vktHipAggregatePartial_t r[2];
        int32_t t[2];
    } host;
    vktError e = rt::check(hipMemcpyAsync(&host, res, sizeof(host.r), hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
    if (e == vktNoError)
        e = rt::check(hipMemcpyAsync(host.t, targets, sizeof(host.t), hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
    sc.dev.release(s);
    if (e != vktNoError)
        return e;
    VKT_HIP_TRY(hipStreamSynchronize(s));
    *pass1 = host.r[0];
    *pass2 = host.r[1];
    pass2->count = 0;
    codes[0] = host.t[0];
    codes[1] = host.t[1];
    return rt::finishLaunch("AggregatesFromCodes_hip");
}

vktError vktHipAggregateFirstCodes(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last, int32_t zGlobalOffset,
                                   int32_t minCode, int32_t maxCode, uint64_t* indices)
{
    if (indices == nullptr)
        return rt::fail("vktHipAggregateFirstCodes: null indices");
    indices[0] = indices[1] = kNoIndex;
    if (minCode < 0 || maxCode < 0)
        return rt::fail("vktHipAggregateFirstCodes: negative code");
    BoxArgs a{};
    vktError e;
    if (!makeBox(volume, first, last, zGlobalOffset, a, "vktHipAggregateFirstCodes: invalid volume view", e))
        return e;
    FastHistArgs h;
    bool contig;
    if ((a.fmt != codec::FmtUInt8 && a.fmt != codec::FmtUInt16) || !makeSpanArgs(a, h, contig))
        return rt::fail("vktHipAggregateFirstCodes: the range does not take the code-count walk");
    hipStream_t s = rt::computeStream();
    AggScratch& sc = aggScratch();
    size_t const bytes = 2 * sizeof(vktHipAggregatePartial_t) + 16;
    auto* res = static_cast<vktHipAggregatePartial_t*>(sc.dev.acquire(bytes, s));
    if (!res)
        return vktInvalidValue;
    auto* targets = reinterpret_cast<int32_t*>(res + 2);
    int32_t const t[2] = {minCode, maxCode};
    uint64_t const none[2] = {kNoIndex, kNoIndex};   // the search folds into them with atomicMin
    e = rt::check(hipMemcpyAsync(targets, t, sizeof(t), hipMemcpyHostToDevice, s), "hipMemcpyAsync");
    if (e == vktNoError)
        e = rt::check(hipMemcpyAsync(&res[0].minIndex, none, sizeof(none), hipMemcpyHostToDevice, s), "hipMemcpyAsync");
    if (e == vktNoError)
        launchFindCodes(h, contig, a.fmt, targets, res, s);
    uint64_t out[2] = {kNoIndex, kNoIndex};
    if (e == vktNoError)
        e = rt::check(hipMemcpyAsync(out, &res[0].minIndex, sizeof(out), hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
    sc.dev.release(s);
    if (e != vktNoError)
        return e;
    VKT_HIP_TRY(hipStreamSynchronize(s));
    indices[0] = out[0];
    indices[1] = out[1];
    return rt::finishLaunch("AggregateFirstCodes_hip");
}

vktError vktHipHistogramRange(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last, uint64_t* bins,
                              uint64_t numBins, int32_t accumulate)
{
    if (numBins > 0 && bins == nullptr)
        return rt::fail("vktHipHistogramRange: null bins");
    hipStream_t s = rt::computeStream();
    if (!accumulate && numBins > 0)
    {
        unsigned const g = static_cast<unsigned>((numBins + kBlock - 1) / kBlock);
        hipLaunchKernelGGL(zeroU64Kernel, dim3(g), dim3(kBlock), 0, s, reinterpret_cast<unsigned long long*>(bins),
                           numBins);
    }
    BoxArgs a{};
    vktError e;
    if (numBins > 0 && makeBox(volume, first, last, 0, a, "vktHipHistogramRange: invalid volume view", e))
    {
        HistArgs h;
        h.bins = reinterpret_cast<unsigned long long*>(bins);
        h.numBins = numBins;
        volatile float range = volume.mappingHi - volume.mappingLo;
        volatile float nbf = static_cast<float>(numBins);          // size_t -> float
        h.scale = nbf / range;                                     // numBins / (hi - lo)
        if (launchFastHistogram(a, h, s))
            return rt::finishLaunch("HistogramRange_hip");
        // LDS counters in tiles of up to ldsBins bins, one pass over the range per tile (u32
        // per workgroup cannot overflow: a workgroup visits < 2^32 voxels); beyond 8 tiles the
        // counters go straight to global 64-bit atomics.
        uint32_t const ldsBins = ldsBinCapacity();
        uint64_t const tiles = (numBins + ldsBins - 1) / ldsBins;
        h.useLds = tiles <= 8;
        if (h.useLds)
        {
            uint32_t const tileBins = static_cast<uint32_t>(numBins < ldsBins ? numBins : ldsBins);
            size_t const lds = static_cast<size_t>(tileBins) * sizeof(uint32_t);
            // occupancy-limited by LDS: enough workgroups for every CU, no more
            unsigned const perCU = static_cast<unsigned>(std::max<size_t>(1, (160u * 1024u) / std::max<size_t>(lds, 1)));
            unsigned const g = streamingGrid(a.rows, kBlock / 64, std::min(8u, perCU));
            for (uint64_t t = 0; t < tiles; ++t)
            {
                h.tileBase = t * tileBins;
                h.tileBins = static_cast<uint32_t>(std::min<uint64_t>(tileBins, numBins - h.tileBase));
                VKT_REDUCE_DISPATCH(VKT_HIST_LAUNCH, g, lds, s);
            }
        }
        else
        {
            h.tileBase = 0;
            h.tileBins = 0;
            unsigned const g = rowGrid(a.rows);
            VKT_REDUCE_DISPATCH(VKT_HIST_LAUNCH, g, 0, s);
        }
    }
    else if (numBins > 0 && e != vktNoError)
        return e;
    return rt::finishLaunch("HistogramRange_hip");
}

} // extern "C"
