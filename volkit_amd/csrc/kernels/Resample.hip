// Resample.hip -- SV->SV Resample on gfx950 (replaces Resample_cuda,
// reference src/vkt/Resample_cuda.cu:19-43; semantics of Resample_serial,
// src/vkt/Resample_serial.hpp:26-71).
//
// Semantics restated:
//  * dst.dims == src.dims: per-voxel re-encode dst[i] = map_dst(unmap_src(src[i])), no index
//    math (serial branch :32-48, absent from the CUDA path) -> the pointwise convert kernel.
//  * otherwise, per axis, s = (int32)( (float)d / (float)Dd * (float)Ds ) -- computed ONCE on
//    the host into exact index tables; Nearest reads src[s]; "Linear" calls
//    sampleLinear(int,int,int) whose fractions are all 0, i.e. lerp chains v000 + 0*v100 ...
//    over the neighbours (hi.x = the next voxel in memory, unclamped; hi.y, hi.z clamped),
//    so for finite neighbours and an integer destination it equals Nearest exactly, while a
//    non-finite neighbour turns the result into NaN and -0 may become +0.
//
// MI355X design (source-row-centric): the y and z index tables are monotone, so every
// source row (sy, sz) that is read at all feeds a rectangle of destination rows
// [y0,y1) x [z0,z1).  One wave owns one source row: it reads the row once from HBM,
// converts each source voxel once, replicates along x in registers (integer x ratio) and
// streams the result into every destination row of its rectangle with 16-byte nontemporal
// stores.  HBM traffic is therefore N_src*b_src + N_dst*b_dst, the algorithmic minimum.
// General ratios use a gather through the exact x table; the float "Linear" chain reads its
// neighbours through the same tables (L2/MALL-resident rows).

#include "ResampleRow.hpp"
#include "../runtime/Runtime.hpp"
#include "volkit_hip.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

namespace vkt
{
namespace hipk
{
    vktError convertBox(vktHipVolumeView_t dst, vktHipVolumeView_t src, vktVec3i_t srcOrigin, bool clampSrc,
                        vktVec3i_t dstOrigin, int64_t nx, int64_t ny, int64_t nz);
    bool validView(vktHipVolumeView_t const& v);
    bool encodeWrites(int32_t fmt);
    bool overlaps(vktHipVolumeView_t const& a, vktHipVolumeView_t const& b);

    // ---- general gather path (any ratio, any formats, Nearest semantics) -------------
    // Wave-per-source-row again; lanes walk the destination x range and gather through the
    // exact x table (the source row stays in L1/L2 while the wave reads it).
    __global__ __launch_bounds__(kBlock) void resampleGatherKernel(ResampleArgs a, int32_t conv)
    {
        int const lane = threadIdx.x & 63;
        uint32_t const wavesPerBlock = blockDim.x >> 6;
        uint32_t const wave = xcdSwizzle(blockIdx.x, gridDim.x) * wavesPerBlock + (threadIdx.x >> 6);
        uint32_t const totalWaves = gridDim.x * wavesPerBlock;
        uint32_t const tasks = static_cast<uint32_t>(a.nRunsY) * static_cast<uint32_t>(a.nRunsZ);
        uint32_t const bs = codec::bytesPerVoxel(a.fs), bd = codec::bytesPerVoxel(a.fd);

        for (uint32_t t = wave; t < tasks; t += totalWaves)
        {
            Run const ry = runY(a, t % static_cast<uint32_t>(a.nRunsY));
            Run const rz = runZ(a, t / static_cast<uint32_t>(a.nRunsY));
            uint64_t const srow = srcRowIndex(a, ry.s, rz.s);
            for (int32_t x = lane; x < a.ddx; x += 64)
            {
                uint32_t c = loadCodeDyn(a.src, srow + static_cast<uint64_t>(a.xtab[x]), bs);
                if (conv)
                    c = convertCode<-1, -1>(c, a);
                for (int32_t zd = rz.d0; zd < rz.d1; ++zd)
                    for (int32_t yd = ry.d0; yd < ry.d1; ++yd)
                        storeCodeDyn(a.dst, dstRowIndex(a, yd, zd) + static_cast<uint64_t>(x), bd, c);
            }
        }
    }

    // ---- "Linear" with float semantics: the exact sampleLinear lerp chain -------------
    // Value depends only on the source position, so it is evaluated per destination voxel
    // from the 8 neighbours (StructuredVolumeView.hpp:80-119): lo = (sx,sy,sz); hi.x reads
    // the next voxel in memory (unclamped in the reference); hi.y, hi.z are clamped.
    __device__ __forceinline__ float flatValue(ResampleArgs const& a, uint64_t voxel, uint32_t bs)
    {
        if (voxel >= a.srcVoxels)
            voxel = a.srcVoxels - 1;   // reference reads past the buffer end (UB); clamp
        return codec::decode(loadCodeDyn(a.src, voxel, bs), a.fs, a.slo, a.shi);
    }

    // One task (source row (ry.s, rz.s) -> its dst rectangle) of the chain, lane-strided.
    __device__ __forceinline__ void chainTask(ResampleArgs const& a, Run const& ry, Run const& rz, int lane)
    {
        uint32_t const bs = codec::bytesPerVoxel(a.fs), bd = codec::bytesPerVoxel(a.fd);
        int32_t const hy = ry.s + 1 < a.sdy ? ry.s + 1 : a.sdy - 1;
        int32_t const hz = rz.s + 1 < a.srcGlobalDz ? rz.s + 1 : a.srcGlobalDz - 1;
        uint64_t const r00 = srcRowIndex(a, ry.s, rz.s), r10 = srcRowIndex(a, hy, rz.s);
        uint64_t const r01 = srcRowIndex(a, ry.s, hz), r11 = srcRowIndex(a, hy, hz);
        for (int32_t x = lane; x < a.ddx; x += 64)
        {
            uint64_t const sx = static_cast<uint64_t>(a.xtab[x]);
            float v0 = flatValue(a, r00 + sx, bs), v1 = flatValue(a, r00 + sx + 1, bs);
            float v2 = flatValue(a, r10 + sx, bs), v3 = flatValue(a, r10 + sx + 1, bs);
            float v4 = flatValue(a, r01 + sx, bs), v5 = flatValue(a, r01 + sx + 1, bs);
            float v6 = flatValue(a, r11 + sx, bs), v7 = flatValue(a, r11 + sx + 1, bs);
            float const f = 0.f;   // xf1 - lo.x etc.: lo is never clamped, so every fraction is 0
            float value = codec::lerp(codec::lerp(codec::lerp(v0, v1, f), codec::lerp(v2, v3, f), f),
                                      codec::lerp(codec::lerp(v4, v5, f), codec::lerp(v6, v7, f), f), f);
            bool w;
            uint32_t c = codec::encode(value, a.fd, a.dm, w);
            for (int32_t zd = rz.d0; zd < rz.d1; ++zd)
                for (int32_t yd = ry.d0; yd < ry.d1; ++yd)
                    storeCodeDyn(a.dst, dstRowIndex(a, yd, zd) + static_cast<uint64_t>(x), bd, c);
        }
    }

    __global__ __launch_bounds__(kBlock) void resampleChainKernel(ResampleArgs a)
    {
        int const lane = threadIdx.x & 63;
        uint32_t const wavesPerBlock = blockDim.x >> 6;
        uint32_t const wave = xcdSwizzle(blockIdx.x, gridDim.x) * wavesPerBlock + (threadIdx.x >> 6);
        uint32_t const totalWaves = gridDim.x * wavesPerBlock;
        uint32_t const tasks = static_cast<uint32_t>(a.nRunsY) * static_cast<uint32_t>(a.nRunsZ);
        for (uint32_t t = wave; t < tasks; t += totalWaves)
            chainTask(a, runY(a, t % static_cast<uint32_t>(a.nRunsY)), runZ(a, t / static_cast<uint32_t>(a.nRunsY)),
                      lane);
    }

    // Vectorised gather: lane l handles V = 16 / BPVD consecutive destination voxels, reads
    // their V exact x-table entries and V source codes (the row is L1/L2-resident while the
    // wave sweeps it) and writes one 16-byte nontemporal store per destination row.
    // CHAIN (Float32 "Linear", any ratio): a task whose source rows' chain neighbourhood holds
    // a non-finite value or a -0 (a.rowChain, from rowDirtyKernel + rowChainKernel) evaluates
    // the full lerp chain (chainTask); every other task's chain equals v000 exactly, so it is
    // a plain gather -- the 8 neighbour reads per voxel are skipped.
    template <int BPVD, bool CONV, bool CHAIN = false>
    __global__ __launch_bounds__(kBlock) void resampleGatherVecKernel(ResampleArgs a)
    {
        constexpr int V = 16 / BPVD;
        int const lane = threadIdx.x & 63;
        uint32_t const wavesPerBlock = blockDim.x >> 6;
        uint32_t const wave = __builtin_amdgcn_readfirstlane(xcdSwizzle(blockIdx.x, gridDim.x) * wavesPerBlock +
                                                             (threadIdx.x >> 6));
        uint32_t const totalWaves = gridDim.x * wavesPerBlock;
        uint32_t const tasks = static_cast<uint32_t>(a.nRunsY) * static_cast<uint32_t>(a.nRunsZ);
        uint32_t const bs = codec::bytesPerVoxel(a.fs);

        for (uint32_t t = wave; t < tasks; t += totalWaves)
        {
            Run const ry = runY(a, t % static_cast<uint32_t>(a.nRunsY));
            Run const rz = runZ(a, t / static_cast<uint32_t>(a.nRunsY));
            uint64_t const srow = srcRowIndex(a, ry.s, rz.s);
            if constexpr (CHAIN)
            {
                if (a.rowChain[srow / static_cast<uint64_t>(a.sdx)])   // wave-uniform
                {
                    chainTask(a, ry, rz, lane);
                    continue;
                }
            }
            for (int32_t dx = V * lane; dx < a.ddx; dx += 64 * V)
            {
                int32_t xs[V];
                if constexpr (V == 4)
                {
                    u32x4 q = *reinterpret_cast<u32x4 const*>(a.xtab + dx);
                    xs[0] = q.x; xs[1] = q.y; xs[2] = q.z; xs[3] = q.w;
                }
                else
                {
#pragma unroll
                    for (int i = 0; i < V; i += 4)
                    {
                        u32x4 q = *reinterpret_cast<u32x4 const*>(a.xtab + dx + i);
                        xs[i] = q.x; xs[i + 1] = q.y; xs[i + 2] = q.z; xs[i + 3] = q.w;
                    }
                }
                uint32_t code[V];
#pragma unroll
                for (int i = 0; i < V; ++i)
                {
                    uint32_t c = loadCodeDyn(a.src, srow + static_cast<uint64_t>(xs[i]), bs);
                    code[i] = CONV ? convertCode<-1, -1>(c, a) : c;
                }
                for (int32_t zd = rz.d0; zd < rz.d1; ++zd)
                    for (int32_t yd = ry.d0; yd < ry.d1; ++yd)
                        store16<BPVD>(a.dst, dstRowIndex(a, yd, zd) + static_cast<uint64_t>(dx), code);
            }
        }
    }

    // LDS-staged gather (any ratio): each wave copies its task's source row into its own LDS
    // slot with coalesced 16-byte loads (every source byte read from L2/HBM once, instead of
    // one 1-4-byte gather instruction per destination voxel), the workgroup keeps the exact x
    // table in LDS, and lane l assembles V = 16 / BPVD destination voxels from LDS reads and
    // writes one 16-byte nontemporal store per destination row of the task's rectangle.
    // Preconditions (host): rows are 16-byte multiples, 16-byte aligned buffers, 4 slots fit.
    // DETECT (Float32 "Linear", optimistic): every staged source row is also checked for values
    // that can make the lerp chain differ from v000 (chainSensitive); such a row's flag is set
    // in a.rowDirtyOut and resampleGatherFixupKernel later re-evaluates the affected tasks.
    // A 16-B vector at any byte address (source rows that are not 16-B multiples start anywhere).
    struct __attribute__((packed, aligned(1))) RowVec16
    {
        u32x4 v;
    };

    // Offset of a row's 16-B chunk starting at byte o (< rowBytes): rows of a whole number of
    // chunks keep o; otherwise the chunk that would run past the row end is taken at rowBytes - 16
    // instead (it overlaps its neighbour with the same bytes), so no load leaves the row.
    __device__ __forceinline__ uint32_t rowChunk(uint32_t o, uint32_t rowBytes)
    {
        return o + 16u <= rowBytes ? o : rowBytes - 16u;
    }

    // PREFETCH (knob resample.prefetch; rows <= 4 KiB, no chain / detect): a wave that loops over
    // tasks (the capped UInt8 grid) loads the NEXT task's source row into registers while it
    // gathers and stores the current one, instead of one load -> wait -> gather round trip per task.
    // PAD (knob resample.lds_pad; 16-B multiple rows): 16 bytes of padding after every 256 bytes
    // of a staged row, so the gather's per-lane reads -- lane l at source byte ~16 l r for a
    // ratio r -- spread over the LDS banks (UInt8 1024 -> 768: a 5.33-dword lane stride hit
    // each bank ~5 times per wave read; SQ_LDS_BANK_CONFLICT 85 M cycles per launch, 34 % of the
    // wave cycles waiting on LDS, profiles/r06/u8gather.pmc.jsonl).
    template <bool PAD>
    __device__ __forceinline__ uint32_t padOff(uint32_t o)
    {
        return PAD ? o + ((o >> 8) << 4) : o;
    }

    template <int BPVS, int BPVD, bool CONV, bool CHAIN, bool DETECT = false, bool PREFETCH = false, int NT = kBlock,
              bool PAD = false>
    __global__ __launch_bounds__(NT) void resampleGatherLdsKernel(ResampleArgs a, uint32_t slotBytes)
    {
        constexpr bool kPre = PREFETCH && !CHAIN && !DETECT;   // plain gathers only
        constexpr int V = 16 / BPVD;
        extern __shared__ u32x4 ldsRaw[];
        uint8_t* const lds = reinterpret_cast<uint8_t*>(ldsRaw);
        int32_t* const xt = reinterpret_cast<int32_t*>(lds);                  // ddx entries (padded)
        uint32_t const xtBytes = (static_cast<uint32_t>(a.ddx) * 4u + 15u) & ~15u;
        int const lane = threadIdx.x & 63;
        uint32_t const wib = threadIdx.x >> 6;
        uint8_t* const slot = lds + xtBytes + wib * slotBytes;
        for (uint32_t i = threadIdx.x * 4; i < static_cast<uint32_t>(a.ddx); i += NT * 4)
            *reinterpret_cast<u32x4*>(xt + i) = *reinterpret_cast<u32x4 const*>(a.xtab + i);
        __syncthreads();

        uint32_t const wavesPerBlock = blockDim.x >> 6;
        uint32_t const wave = __builtin_amdgcn_readfirstlane(xcdSwizzle(blockIdx.x, gridDim.x) * wavesPerBlock + wib);
        uint32_t const totalWaves = gridDim.x * wavesPerBlock;
        uint32_t const tasks = static_cast<uint32_t>(a.nRunsY) * static_cast<uint32_t>(a.nRunsZ);
        uint32_t const rowBytes = static_cast<uint32_t>(a.sdx) * BPVS;
        constexpr int kStage = 4;
        u32x4 pre[kStage];   // PREFETCH: the next task's row (lane l holds bytes 16 l + 1024 j)
        auto loadRow = [&](uint32_t tt) {
            Run const ny = runY(a, tt % static_cast<uint32_t>(a.nRunsY));
            Run const nz = runZ(a, tt / static_cast<uint32_t>(a.nRunsY));
            uint8_t const* const np = a.src + srcRowIndex(a, ny.s, nz.s) * BPVS;
#pragma unroll
            for (int j = 0; j < kStage; ++j)
                if (16u * lane + 1024u * j < rowBytes)
                    pre[j] = reinterpret_cast<RowVec16 const*>(np + rowChunk(16u * lane + 1024u * j, rowBytes))->v;
        };
        if constexpr (kPre)
        {
            if (wave < tasks)
                loadRow(wave);
        }
        for (uint32_t t = wave; t < tasks; t += totalWaves)
        {
            Run const ry = runY(a, t % static_cast<uint32_t>(a.nRunsY));
            Run const rz = runZ(a, t / static_cast<uint32_t>(a.nRunsY));
            uint64_t const srow = srcRowIndex(a, ry.s, rz.s);
            if constexpr (kPre)
            {
                // this task's row is in registers: to the slot, then the next row goes out
#pragma unroll
                for (int j = 0; j < kStage; ++j)
                    if (16u * lane + 1024u * j < rowBytes)
                        reinterpret_cast<RowVec16*>(slot + padOff<PAD>(rowChunk(16u * lane + 1024u * j, rowBytes)))->v =
                            pre[j];
                if (t + totalWaves < tasks)
                    loadRow(t + totalWaves);
            }
            if constexpr (CHAIN)
            {
                if (a.rowChain[srow / static_cast<uint64_t>(a.sdx)])   // wave-uniform
                {
                    chainTask(a, ry, rz, lane);
                    continue;
                }
            }
            uint8_t const* sp = a.src + srow * BPVS;
            bool sens = false;   // DETECT: the row holds a chain-sensitive value
            // stage: all of a lane's loads in flight before the first LDS write
            for (uint32_t o0 = 16u * lane; !kPre && o0 < rowBytes; o0 += 1024u * kStage)
            {
                u32x4 w[kStage];
#pragma unroll
                for (int j = 0; j < kStage; ++j)
                    if (o0 + 1024u * j < rowBytes)
                    {
                        uint32_t const oc = rowChunk(o0 + 1024u * j, rowBytes);
                        if (rowBytes % 16u == 0u)   // (wave-uniform) aligned rows: nontemporal vector loads
                            w[j] = __builtin_nontemporal_load(reinterpret_cast<u32x4 const*>(sp + oc));
                        else
                            w[j] = reinterpret_cast<RowVec16 const*>(sp + oc)->v;
                    }
#pragma unroll
                for (int j = 0; j < kStage; ++j)
                    if (o0 + 1024u * j < rowBytes)
                        reinterpret_cast<RowVec16*>(slot + padOff<PAD>(rowChunk(o0 + 1024u * j, rowBytes)))->v = w[j];
                if constexpr (DETECT)
                {
#pragma unroll
                    for (int j = 0; j < kStage; ++j)
                        if (o0 + 1024u * j < rowBytes)
                            sens = sens | int(chainSensitive(w[j].x)) | int(chainSensitive(w[j].y)) | int(chainSensitive(w[j].z)) |
                                   chainSensitive(w[j].w);
                }
            }
            if constexpr (DETECT)
            {
                // every staged row's flag is written (0 or 1): no per-call clearing of the flags
                bool const any = __ballot(sens) != 0;
                if (lane == 0)
                {
                    a.rowDirtyOut[srow / static_cast<uint64_t>(a.sdx)] = any;
                    if (any)
                        *a.anyDirtyOut = a.epoch;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (int32_t dx = V * lane; dx < a.ddx; dx += 64 * V)
            {
                uint32_t code[V];
#pragma unroll
                for (int i = 0; i < V; i += 4)
                {
                    u32x4 const q = *reinterpret_cast<u32x4 const*>(xt + dx + i);
                    int32_t const xs[4] = {static_cast<int32_t>(q.x), static_cast<int32_t>(q.y),
                                           static_cast<int32_t>(q.z), static_cast<int32_t>(q.w)};
#pragma unroll
                    for (int j = 0; j < 4 && i + j < V; ++j)
                    {
                        uint32_t const c =
                            PAD ? loadCode<BPVS>(slot + padOff<true>(static_cast<uint32_t>(xs[j]) * BPVS), 0)
                                : loadCode<BPVS>(slot, static_cast<uint64_t>(xs[j]));
                        code[i + j] = CONV ? convertCode<-1, -1>(c, a) : c;
                    }
                }
                for (int32_t zd = rz.d0; zd < rz.d1; ++zd)
                    for (int32_t yd = ry.d0; yd < ry.d1; ++yd)
                        store16<BPVD>(a.dst, dstRowIndex(a, yd, zd) + static_cast<uint64_t>(dx), code);
            }
            // the slot is rewritten by the next task: every lane's reads first
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }

    // ---- LDS gather over DESTINATION rows (round 6, knob resample.dst_rows) ---------------------
    // gfx950's vmcnt counts loads and stores in one in-order counter, and the compiler can wait for
    // a load without also waiting for the stores issued after it only when it knows how many were
    // issued.  A source-row task stores to 1..4 destination rows (its run rectangle): a dynamic
    // count, so resampleGatherLdsKernel's next row load always waited for the previous task's
    // stores.  Here a task is ONE destination row (plane-linear order: consecutive tasks share or
    // neighbour a source row, which the L2 serves again): exactly G 16-B store instructions per
    // task, every lane storing (lanes past the row end repeat the last lane's store: same address,
    // same bytes), and exactly KS 16-B loads per lane for the source row (clamped to its last 16 B).
    // The next task's row is loaded into registers before this task's gather and stores, and its
    // wait at the next iteration is vmcnt(G): the stores stay in flight.  Rows <= 64 G V voxels
    // (destination) and <= 1 KiB KS (source).
    template <int BPVS, int BPVD, bool CONV, bool PAD, int G, int KS>
    __global__ __launch_bounds__(kBlock) void resampleGatherDstRowKernel(ResampleArgs a, uint32_t slotBytes)
    {
        constexpr int V = 16 / BPVD;
        extern __shared__ u32x4 ldsRaw[];
        uint8_t* const lds = reinterpret_cast<uint8_t*>(ldsRaw);
        int32_t* const xt = reinterpret_cast<int32_t*>(lds);
        uint32_t const xtBytes = (static_cast<uint32_t>(a.ddx) * 4u + 15u) & ~15u;
        int const lane = threadIdx.x & 63;
        uint32_t const wib = threadIdx.x >> 6;
        uint8_t* const slot = lds + xtBytes + wib * slotBytes;
        for (uint32_t i = threadIdx.x * 4; i < static_cast<uint32_t>(a.ddx); i += kBlock * 4)
            *reinterpret_cast<u32x4*>(xt + i) = *reinterpret_cast<u32x4 const*>(a.xtab + i);
        __syncthreads();

        uint32_t const wave = __builtin_amdgcn_readfirstlane(xcdSwizzle(blockIdx.x, gridDim.x) * (kBlock / 64) + wib);
        uint32_t const totalWaves = gridDim.x * (kBlock / 64);
        uint32_t const ddy = static_cast<uint32_t>(a.ddy);
        uint32_t const tasks = ddy * static_cast<uint32_t>(a.dnz);
        uint32_t const rowBytes = static_cast<uint32_t>(a.sdx) * BPVS;
        bool const aligned = rowBytes % 16u == 0u;
        uint32_t off[KS];
#pragma unroll
        for (int j = 0; j < KS; ++j)
            off[j] = rowChunk(min(16u * lane + 1024u * j, rowBytes - 16u), rowBytes);
        int32_t dxs[G];
#pragma unroll
        for (int g = 0; g < G; ++g)
            dxs[g] = min(V * lane + 64 * V * g, a.ddx - V);
        typedef __attribute__((address_space(4))) int32_t const CI32;
        auto srcRow = [&](uint32_t t) -> uint8_t const* {
            uint32_t const zl = fdiv(t, a.fdDdy);
            uint32_t const yd = t - zl * ddy;
            int32_t const ys = ((CI32*)a.ysrc)[yd];
            int32_t const zs = ((CI32*)a.zsrc)[zl];
            return a.src + srcRowIndex(a, ys, zs) * BPVS;
        };
        u32x4 w[KS];
        auto load = [&](uint32_t t) {
            uint8_t const* const p = srcRow(t);
#pragma unroll
            for (int j = 0; j < KS; ++j)
                w[j] = aligned ? *reinterpret_cast<u32x4 const*>(p + off[j]) : reinterpret_cast<RowVec16 const*>(p + off[j])->v;
        };
        // one task: this row into the slot, the next row's loads out, gather, G stores.  The first
        // task is peeled so that every path into the loop issues the loads and then the stores,
        // and the wait at the top of the next task counts G younger stores: vmcnt(G), not 0.
        auto step = [&](uint32_t t) {
#pragma unroll
            for (int j = 0; j < KS; ++j)
                reinterpret_cast<RowVec16*>(slot + padOff<PAD>(off[j]))->v = w[j];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // the next task's row, in flight during this task's gather and stores
            load(t + totalWaves < tasks ? t + totalWaves : t);
            uint32_t const zl = fdiv(t, a.fdDdy);
            uint32_t const yd = t - zl * ddy;
            uint8_t* const drow = a.dst + dstRowIndex(a, static_cast<int32_t>(yd), a.dstZ0 + static_cast<int32_t>(zl)) * BPVD;
#pragma unroll
            for (int g = 0; g < G; ++g)
            {
                int32_t const dx = dxs[g];
                uint32_t code[V];
#pragma unroll
                for (int i = 0; i < V; i += 4)
                {
                    u32x4 const q = *reinterpret_cast<u32x4 const*>(xt + dx + i);
                    int32_t const xs[4] = {static_cast<int32_t>(q.x), static_cast<int32_t>(q.y),
                                           static_cast<int32_t>(q.z), static_cast<int32_t>(q.w)};
#pragma unroll
                    for (int j = 0; j < 4 && i + j < V; ++j)
                    {
                        uint32_t const c =
                            PAD ? loadCode<BPVS>(slot + padOff<true>(static_cast<uint32_t>(xs[j]) * BPVS), 0)
                                : loadCode<BPVS>(slot, static_cast<uint64_t>(xs[j]));
                        code[i + j] = CONV ? convertCode<-1, -1>(c, a) : c;
                    }
                }
                store16<BPVD>(drow, static_cast<uint64_t>(dx), code);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        };
        if (wave < tasks)
        {
            load(wave);
            step(wave);
            for (uint32_t t = wave + totalWaves; t < tasks; t += totalWaves)
                step(t);
        }
    }

    // Fix-up of the optimistic Float32 "Linear" gather: one wave per task; tasks whose source
    // row's chain neighbourhood holds a flagged row (a.rowChain, from rowChainKernel) rewrite
    // their destination rectangle with the full sampleLinear chain.
    __global__ __launch_bounds__(kBlock) void resampleGatherFixupKernel(ResampleArgs a)
    {
        // no flagged row anywhere (the common case): nothing to re-evaluate.  Scanning every
        // task's rowChain byte cost 92 us for 1024^3 -> 768^3 (589 824 tasks, dependent loads).
        if (a.anyChain != nullptr && *a.anyChain == 0u)
            return;
        if (a.anyDirtyOut != nullptr && *a.anyDirtyOut != a.epoch)
            return;
        int const lane = threadIdx.x & 63;
        uint32_t const wave = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
        uint32_t const totalWaves = gridDim.x * (kBlock / 64);
        uint32_t const tasks = static_cast<uint32_t>(a.nRunsY) * static_cast<uint32_t>(a.nRunsZ);
        for (uint32_t t = wave; t < tasks; t += totalWaves)
        {
            Run const ry = runY(a, t % static_cast<uint32_t>(a.nRunsY));
            Run const rz = runZ(a, t / static_cast<uint32_t>(a.nRunsY));
            bool flagged;
            if (a.rowChain != nullptr)
                flagged = a.rowChain[srcRowIndex(a, ry.s, rz.s) / static_cast<uint64_t>(a.sdx)] != 0;
            else
                flagged = taskFlagged(a, ry, rz);   // the chain's rows straight from rowDirty
            if (flagged)   // wave-uniform, rare
                chainTask(a, ry, rz, lane);
        }
    }

    // ---- Float32 "Linear": which source rows can make the chain differ from v000 ------
    // One wave per local source row; byte r of `dirty` = the row holds a non-finite value or
    // a -0 (chainSensitive).  One streaming read of the source (N_src * 4 bytes) lets the
    // row kernel skip the three neighbour-row reads for every clean task.
    template <bool VEC>
    __global__ __launch_bounds__(kBlock) void rowDirtyKernel(uint8_t const* src, int32_t sdx, uint64_t rows,
                                                             uint8_t* dirty)
    {
        int const lane = threadIdx.x & 63;
        uint64_t const row = static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
        if (row >= rows)
            return;
        uint32_t const* p = reinterpret_cast<uint32_t const*>(src) + row * static_cast<uint64_t>(sdx);
        bool d = false;
        if constexpr (VEC)
        {
            for (int32_t x = 4 * lane; x < sdx; x += 256)
            {
                u32x4 v = __builtin_nontemporal_load(reinterpret_cast<u32x4 const*>(p + x));
                d = d || chainSensitive(v.x) || chainSensitive(v.y) || chainSensitive(v.z) || chainSensitive(v.w);
            }
        }
        else
        {
            for (int32_t x = lane; x < sdx; x += 64)
                d = d || chainSensitive(p[x]);
        }
        uint64_t const any = __ballot(d);
        if (lane == 0)
            dirty[row] = any != 0;
    }

    // rowDirtyKernel over the local rows NO task stages (staged[y] && staged[sdy + global z]
    // skipped): the optimistic LDS gather flags the rows it stages itself, so together every
    // row a chain can read is classified with one read of each source row.
    __global__ __launch_bounds__(kBlock) void rowDirtyUnstagedKernel(uint8_t const* src, int32_t sdx, int32_t sdy,
                                                                     uint64_t rows, int32_t srcZ0, uint8_t const* staged,
                                                                     uint8_t* dirty, uint32_t* anyDirty, uint32_t epoch)
    {
        int const lane = threadIdx.x & 63;
        uint64_t const row = static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
        if (row >= rows)
            return;
        uint32_t const z = static_cast<uint32_t>(row / static_cast<uint64_t>(sdy));
        uint32_t const y = static_cast<uint32_t>(row - static_cast<uint64_t>(z) * static_cast<uint64_t>(sdy));
        if (staged[y] && staged[static_cast<uint32_t>(sdy) + static_cast<uint32_t>(srcZ0) + z])
            return;
        uint32_t const* p = reinterpret_cast<uint32_t const*>(src) + row * static_cast<uint64_t>(sdx);
        // all of a lane's loads in flight before the tests (4 KiB rows: one batch), no
        // short-circuit between them
        constexpr int kBatch = 4;
        bool d = false;
        for (int32_t x0 = 4 * lane; x0 < sdx; x0 += 256 * kBatch)
        {
            u32x4 v[kBatch];
#pragma unroll
            for (int j = 0; j < kBatch; ++j)
                if (x0 + 256 * j < sdx)
                    v[j] = __builtin_nontemporal_load(reinterpret_cast<u32x4 const*>(p + x0 + 256 * j));
#pragma unroll
            for (int j = 0; j < kBatch; ++j)
                if (x0 + 256 * j < sdx)
                    d = d | int(chainSensitive(v[j].x)) | int(chainSensitive(v[j].y)) | int(chainSensitive(v[j].z)) |
                        chainSensitive(v[j].w);
        }
        uint64_t const any = __ballot(d);
        if (lane == 0)
        {
            dirty[row] = any != 0;
            if (any != 0 && anyDirty != nullptr)
                *anyDirty = epoch;
        }
    }

    // rowChain[r] = OR of rowDirty over the rows the chain of row r's voxels reads:
    // (y,z), (y+1,z), (y,z+1), (y+1,z+1) -- y+1 / z+1 clamped like sampleLinear -- and the
    // row after each in memory (hi.x of the last voxel).  Indices are clamped into the local
    // buffer; rows whose neighbourhood leaves it are never read by a task (slab precondition).
    __global__ __launch_bounds__(kBlock) void rowChainKernel(uint8_t const* dirty, int32_t sdy, int32_t sdz,
                                                            int32_t srcZ0, int32_t srcGlobalDz, uint8_t* chain,
                                                            uint32_t* anyChain)
    {
        uint64_t const rows = static_cast<uint64_t>(sdy) * static_cast<uint64_t>(sdz);
        uint64_t const r = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
        if (r >= rows)
            return;
        int32_t const y = static_cast<int32_t>(r % static_cast<uint64_t>(sdy));
        int32_t const zl = static_cast<int32_t>(r / static_cast<uint64_t>(sdy));
        int32_t const hy = y + 1 < sdy ? y + 1 : sdy - 1;
        int32_t const zg = srcZ0 + zl;
        int32_t const hzl = (zg + 1 < srcGlobalDz ? zg + 1 : srcGlobalDz - 1) - srcZ0;
        uint64_t const last = rows - 1;
        auto at = [&](int32_t yy, int32_t zz) {
            uint64_t i = static_cast<uint64_t>(zz) * static_cast<uint64_t>(sdy) + static_cast<uint64_t>(yy);
            i = i < last ? i : last;
            return dirty[i] | dirty[i < last ? i + 1 : last];
        };
        bool const c = (at(y, zl) | at(hy, zl) | at(y, hzl) | at(hy, hzl)) != 0;
        chain[r] = c;
        if (c && anyChain != nullptr)
            *anyChain = 1u;   // vector store; every writer stores the same value
    }

    // ---- host planning -------------------------------------------------------------
    std::vector<Run> buildRuns(int32_t dstBegin, int32_t dstEnd, int32_t dd, int32_t sd)
    {
        std::vector<Run> runs;
        for (int32_t d = dstBegin; d < dstEnd; ++d)
        {
            int32_t s = srcIndex(d, dd, sd);
            if (!runs.empty() && runs.back().s == s)
                runs.back().d1 = d + 1;
            else
                runs.push_back(Run{s, d, d + 1});
        }
        return runs;
    }

    // Device copies of the per-geometry tables, cached for the life of the process (a
    // benchmark or pipeline resamples the same geometry repeatedly; uploading per call would
    // put a pageable H2D copy in every step).
    struct TableKey
    {
        int32_t v[9];
        bool operator<(TableKey const& o) const
        {
            for (int i = 0; i < 9; ++i)
                if (v[i] != o.v[i])
                    return v[i] < o.v[i];
            return false;
        }
    };

    struct Tables
    {
        int32_t* dev = nullptr;
        int32_t nRunsY = 0, nRunsZ = 0;
        int32_t k = 0;            // integer x ratio, 0 if none
        int32_t minSz = 0, maxSz = 0;
        Run const* runsY = nullptr;
        Run const* runsZ = nullptr;
        int32_t const* xtab = nullptr;
        int32_t const* zsrc = nullptr;   // source plane of every local dst plane
        int32_t const* ysrc = nullptr;   // source row of every dst row (ddy entries)
        uint8_t const* staged = nullptr; // sdy bytes (y) then sgz bytes (global z): 1 = a task reads it
        bool yAllRows = false;           // the y runs read every source row 0..sdy-1, in order
        bool zContiguous = false;        // the z runs read consecutive source planes
        int32_t aff[2][6] = {{0, 0, 0, 0, 0, 0}, {0, 0, 0, 0, 0, 0}};   // {aff, sa, da, dl, s0, d0}
    };

    // Do the runs follow {s0 + sa*i, d0 + da*i, +dl}?  (exact integer up/down-sampling)
    void affineOf(std::vector<Run> const& runs, int32_t (&out)[6])
    {
        out[0] = 0;
        if (runs.empty())
            return;
        int32_t s0 = runs[0].s, d0 = runs[0].d0, dl = runs[0].d1 - runs[0].d0;
        int32_t sa = runs.size() > 1 ? runs[1].s - runs[0].s : 1;
        int32_t da = runs.size() > 1 ? runs[1].d0 - runs[0].d0 : dl;
        for (size_t i = 0; i < runs.size(); ++i)
        {
            int32_t ii = static_cast<int32_t>(i);
            if (runs[i].s != s0 + sa * ii || runs[i].d0 != d0 + da * ii || runs[i].d1 != d0 + da * ii + dl)
                return;
        }
        out[0] = 1;
        out[1] = sa;
        out[2] = da;
        out[3] = dl;
        out[4] = s0;
        out[5] = d0;
    }

    vktError getTables(int32_t ddx, int32_t ddy, int32_t dgz, int32_t dz0, int32_t dnz, int32_t sdx, int32_t sdy,
                       int32_t sgz, Tables& out)
    {
        static std::mutex m;
        static std::map<std::pair<int, TableKey>, Tables> cache;
        TableKey key{{ddx, ddy, dgz, dz0, dnz, sdx, sdy, sgz, 0}};
        int dev = rt::device();
        std::lock_guard<std::mutex> lock(m);
        auto it = cache.find({dev, key});
        if (it != cache.end())
        {
            out = it->second;
            return vktNoError;
        }
        std::vector<Run> ry = buildRuns(0, ddy, ddy, sdy);
        std::vector<Run> rz = buildRuns(dz0, dz0 + dnz, dgz, sgz);
        std::vector<int32_t> xt(static_cast<size_t>(ddx));
        bool rep = ddx % sdx == 0;
        int32_t k = rep ? ddx / sdx : 0;
        for (int32_t x = 0; x < ddx; ++x)
        {
            xt[x] = srcIndex(x, ddx, sdx);
            if (rep && xt[x] != x / k)
                rep = false;
        }
        for (Run const& r : ry)
            if (r.s < 0 || r.s >= sdy)
                return rt::fail("Resample: y index table leaves the source (reference would read out of bounds)");
        for (int32_t s : xt)
            if (s < 0 || s >= sdx)
                return rt::fail("Resample: x index table leaves the source (reference would read out of bounds)");
        for (Run const& r : rz)
            if (r.s < 0 || r.s >= sgz)
                return rt::fail("Resample: z index table leaves the source (reference would read out of bounds)");
        Tables t;
        t.nRunsY = static_cast<int32_t>(ry.size());
        t.nRunsZ = static_cast<int32_t>(rz.size());
        t.k = rep ? k : 0;
        affineOf(ry, t.aff[0]);
        affineOf(rz, t.aff[1]);
        t.yAllRows = static_cast<int32_t>(ry.size()) == sdy;
        for (size_t i = 0; t.yAllRows && i < ry.size(); ++i)
            t.yAllRows = ry[i].s == static_cast<int32_t>(i);
        t.zContiguous = true;
        for (size_t i = 1; i < rz.size(); ++i)
            t.zContiguous = t.zContiguous && rz[i].s == rz[i - 1].s + 1;
        t.minSz = rz.empty() ? 0 : rz.front().s;
        t.maxSz = rz.empty() ? -1 : rz.back().s;
        // layout: x table first (16-byte aligned for vector reads, padded to 4 entries), runs after
        size_t xwords = (xt.size() + 3) / 4 * 4;
        size_t words = xwords + 3 * ry.size() + 3 * rz.size() + static_cast<size_t>(dnz) + static_cast<size_t>(ddy);
        std::vector<int32_t> host(xt.begin(), xt.end());
        host.resize(xwords, 0);
        for (Run const& r : ry) host.insert(host.end(), {r.s, r.d0, r.d1});
        for (Run const& r : rz) host.insert(host.end(), {r.s, r.d0, r.d1});
        for (Run const& r : rz)
            for (int32_t d = r.d0; d < r.d1; ++d)
                host.push_back(r.s);
        for (Run const& r : ry)
            for (int32_t d = r.d0; d < r.d1; ++d)
                host.push_back(r.s);
        VKT_HIP_TRY(hipMalloc(&t.dev, words * sizeof(int32_t) + 16));
        VKT_HIP_TRY(hipMemcpy(t.dev, host.data(), words * sizeof(int32_t), hipMemcpyHostToDevice));
        t.xtab = t.dev;
        t.runsY = reinterpret_cast<Run const*>(t.dev + xwords);
        t.runsZ = reinterpret_cast<Run const*>(t.dev + xwords + 3 * ry.size());
        t.zsrc = t.dev + xwords + 3 * ry.size() + 3 * rz.size();
        t.ysrc = t.zsrc + dnz;
        {
            // rows the tasks stage (the optimistic Float32 Linear gather flags those itself)
            std::vector<uint8_t> st(static_cast<size_t>(sdy) + static_cast<size_t>(sgz), 0);
            for (Run const& r : ry)
                st[static_cast<size_t>(r.s)] = 1;
            for (Run const& r : rz)
                st[static_cast<size_t>(sdy) + static_cast<size_t>(r.s)] = 1;
            uint8_t* d = nullptr;
            VKT_HIP_TRY(hipMalloc(&d, st.size()));
            VKT_HIP_TRY(hipMemcpy(d, st.data(), st.size(), hipMemcpyHostToDevice));
            t.staged = d;
        }
        cache[{dev, key}] = t;
        out = t;
        return vktNoError;
    }

    // Is map_dst(unmap_src(c)) == c for every code c?  (only <=16-bit formats are enumerable)
    bool identityConversionUncached(int32_t fs, float slo, float shi, int32_t fd, float dlo, float dhi)
    {
        if (fs != fd)
            return false;
        uint32_t n;
        if (fs == codec::FmtUInt8)
            n = 256;
        else if (fs == codec::FmtUInt16 || fs == codec::FmtInt16)
            n = 65536;
        else
            return false;
        MapParams dm = codec::makeMapParams(dlo, dhi);
        for (uint32_t c = 0; c < n; ++c)
        {
            bool w;
            if (codec::encode(codec::decode(c, fs, slo, shi), fd, dm, w) != c)
                return false;
        }
        return true;
    }

    // Are all unmapped source values finite, so that Linear's 0*neighbour terms vanish?
    bool allSourceValuesFiniteUncached(int32_t fs, float lo, float hi)
    {
        if (fs == codec::FmtUInt8 || fs == codec::FmtUInt16 || fs == codec::FmtInt16)
        {
            uint32_t n = fs == codec::FmtUInt8 ? 256u : 65536u;
            for (uint32_t c = 0; c < n; ++c)
                if (!std::isfinite(codec::decode(c, fs, lo, hi)))
                    return false;
            return true;
        }
        if (fs == codec::FmtUInt32)
            return std::isfinite(lo) && std::isfinite(hi) && std::fabs(lo) <= 1e38f && std::fabs(hi) <= 1e38f;
        if (fs == codec::FmtInt8 || fs == codec::FmtInt32)
            return true;   // unmap leaves 0.f
        return false;      // Float32: raw bits, anything goes
    }

    // Can an unmapped source value be -0?  (lerp(a, b, 0) = a + 0*b turns a = -0 into +0 for
    // b >= +0, which a Float32 destination stores differently.)  (1-t)*lo + t*hi is -0 only
    // when both products are -0, impossible if lo > 0 or hi > 0.
    bool negativeZeroPossibleUncached(int32_t fs, float lo, float hi)
    {
        if (fs == codec::FmtUInt8 || fs == codec::FmtUInt16 || fs == codec::FmtInt16)
        {
            uint32_t n = fs == codec::FmtUInt8 ? 256u : 65536u;
            for (uint32_t c = 0; c < n; ++c)
            {
                float const v = codec::decode(c, fs, lo, hi);
                if (v == 0.f && std::signbit(v))
                    return true;
            }
            return false;
        }
        if (fs == codec::FmtUInt32)
            return !(lo > 0.f || hi > 0.f);
        if (fs == codec::FmtInt8 || fs == codec::FmtInt32)
            return false;   // unmap leaves +0.f
        return true;        // Float32: raw bits
    }

    // All properties are enumerations over up to 65536 codes (~ms); cache them per mapping.
    struct ConvProps
    {
        bool identity;
        bool finite;
        bool negZero;
    };

    ConvProps conversionProperties(int32_t fs, float slo, float shi, int32_t fd, float dlo, float dhi)
    {
        static std::mutex m;
        static std::map<std::tuple<int32_t, uint32_t, uint32_t, int32_t, uint32_t, uint32_t>, ConvProps> cache;
        auto key = std::make_tuple(fs, codec::floatToBits(slo), codec::floatToBits(shi), fd, codec::floatToBits(dlo),
                                   codec::floatToBits(dhi));
        std::lock_guard<std::mutex> lock(m);
        auto it = cache.find(key);
        if (it != cache.end())
            return it->second;
        ConvProps p{identityConversionUncached(fs, slo, shi, fd, dlo, dhi), allSourceValuesFiniteUncached(fs, slo, shi),
                    negativeZeroPossibleUncached(fs, slo, shi)};
        cache[key] = p;
        return p;
    }

    bool launchRowKernel(ResampleArgs const& a, int32_t k, uint64_t tasks, uint32_t bs, uint32_t bd, bool identity,
                         bool chain, vktHipVolumeView_t const& src, vktHipVolumeView_t const& dst, hipStream_t s,
                         Tables const& tb)
    {
        if (!(k == 1 || k == 2 || k == 4))
            return false;
        uint32_t const v = 16 / bd;            // dst voxels per lane-store
        uint32_t const n = v / k;              // source voxels per lane-load
        if (bd > 4 || bs > 4 || dst.dimX % v != 0 || src.dimX % n != 0 || n * bs > 32)
            return false;
        if (reinterpret_cast<uintptr_t>(src.data) % 16 != 0 || reinterpret_cast<uintptr_t>(dst.data) % 16 != 0)
            return false;
        uint64_t const padded = chain && a.band ? (static_cast<uint64_t>(a.nRunsY) + a.band - 1) / a.band * a.band * a.nRunsZ
                                                : tasks;
        uint64_t blocks = (padded + 3) / 4;    // one task per wave (measured fastest)
        unsigned grid = static_cast<unsigned>(blocks < (1u << 30) ? blocks : (1u << 30));
        int32_t const instrPerRow = static_cast<int32_t>((dst.dimX + 64 * v - 1) / (64 * v));
        if (chain)
        {
            if (src.dataFormat != codec::FmtFloat32 || (bd == 1 && k == 1))
                return false;   // per-dst-voxel chain kernel handles these
            ResampleArgs b = a;
            b.srcRows = static_cast<uint64_t>(src.dimY) * static_cast<uint64_t>(src.dimZ);
            if (b.planeLayout && tb.yAllRows && tb.zContiguous)
            {
                // Optimistic path: the detect pass loads every source row of planes
                // [minSz, maxSz] anyway; only the local planes above maxSz (z+1 halo) are
                // scanned separately.  Then one fix-up pass over the few flagged tasks.
                static rt::StreamScratch flags;
                uint64_t const nTasks = static_cast<uint64_t>(a.nRunsY) * static_cast<uint64_t>(a.nRunsZ);
                uint64_t const flagBytes = (b.srcRows + 15) / 16 * 16;
                uint8_t* dirty = nTasks < (1ull << 31)
                                     ? static_cast<uint8_t*>(flags.acquire(flagBytes + 4 * (nTasks + 1), s))
                                     : nullptr;
                if (dirty)
                {
                    uint32_t* list = reinterpret_cast<uint32_t*>(dirty + flagBytes);
                    bool ok = hipMemsetAsync(dirty, 0, flagBytes + 4, s) == hipSuccess;   // flags + list count
                    int32_t const above = tb.maxSz + 1 - a.srcZ0;   // first local plane above the task planes
                    if (ok && above < src.dimZ)
                    {
                        uint64_t const row0 = static_cast<uint64_t>(above) * static_cast<uint64_t>(src.dimY);
                        uint64_t const nrows = b.srcRows - row0;
                        unsigned const g = static_cast<unsigned>((nrows + kBlock / 64 - 1) / (kBlock / 64));
                        uint8_t const* base = src.data + row0 * static_cast<uint64_t>(src.dimX) * 4u;
                        if (src.dimX % 4 == 0)
                            hipLaunchKernelGGL(rowDirtyKernel<true>, dim3(g), dim3(kBlock), 0, s, base, src.dimX, nrows,
                                               dirty + row0);
                        else
                            hipLaunchKernelGGL(rowDirtyKernel<false>, dim3(g), dim3(kBlock), 0, s, base, src.dimX,
                                               nrows, dirty + row0);
                    }
                    if (ok)
                    {
                        b.rowDirty = dirty;
                        b.rowDirtyOut = dirty;
                        launchLinearOptimistic(b, k, bd, instrPerRow, list, s);
                        flags.release(s);
                        return true;
                    }
                    (void)hipGetLastError();
                    flags.release(s);
                }
            }
            // rowDirty, then rowChain for the plane layout; without scratch every task takes
            // the chain (still exact)
            static rt::StreamScratch scratch;
            uint8_t* dirty = static_cast<uint8_t*>(scratch.acquire(2 * b.srcRows, s));
            if (dirty)
            {
                unsigned const g = static_cast<unsigned>((b.srcRows + kBlock / 64 - 1) / (kBlock / 64));
                bool const vec = src.dimX % 4 == 0;   // base is 16-B aligned (checked above)
                if (vec)
                    hipLaunchKernelGGL(rowDirtyKernel<true>, dim3(g), dim3(kBlock), 0, s, src.data, src.dimX, b.srcRows,
                                       dirty);
                else
                    hipLaunchKernelGGL(rowDirtyKernel<false>, dim3(g), dim3(kBlock), 0, s, src.data, src.dimX,
                                       b.srcRows, dirty);
                b.rowDirty = dirty;
                if (b.planeLayout)
                {
                    unsigned const gc = static_cast<unsigned>((b.srcRows + kBlock - 1) / kBlock);
                    hipLaunchKernelGGL(rowChainKernel, dim3(gc), dim3(kBlock), 0, s, dirty, src.dimY, src.dimZ, a.srcZ0,
                                       a.srcGlobalDz, dirty + b.srcRows, nullptr);
                    b.rowChain = dirty + b.srcRows;
                }
            }
            launchRowMode2(b, k, bd, grid, instrPerRow, s);
            if (dirty)
                scratch.release(s);
            return true;
        }
        if (bs != bd)
            return false;
        if (identity)
            launchRowMode0(a, k, bs, grid, instrPerRow, s);
        else
            launchRowMode1(a, k, bs, src.dataFormat, dst.dataFormat, grid, instrPerRow, s);
        return true;
    }

    bool gatherLdsEnabled()   // A/B tuning knob: VKT_GATHER=vec keeps the per-voxel gather
    {
        static bool const on = !(std::getenv("VKT_GATHER") && std::string(std::getenv("VKT_GATHER")) == "vec");
        return on;
    }

    // LDS-staged gather when the rows and tables fit (see resampleGatherLdsKernel).
    bool launchGatherLds(ResampleArgs const& b, uint32_t bs, uint32_t bd, bool identity, bool chain, uint64_t tasks,
                         hipStream_t s, bool detect = false)
    {
        if ((bs != 1 && bs != 2 && bs != 4) || (bd != 1 && bd != 2 && bd != 4) || ((chain || detect) && bs != 4))
            return false;
        uint64_t const rowBytes = static_cast<uint64_t>(b.sdx) * bs;
        uint64_t const xtBytes = (static_cast<uint64_t>(b.ddx) * 4 + 15) & ~uint64_t(15);
        // rows that are not 16-B multiples (>= 16 B) stage through rowChunk; slots stay 16-B aligned
        int64_t const padKnob = rt::knob(rt::Knob::ResampleLdsPad);
        bool const pad = rowBytes % 16 == 0 && (padKnob == 2 || (padKnob == 1 && bs == 1));
        uint64_t const slotBytes = pad ? rowBytes + (rowBytes >> 8) * 16 : (rowBytes + 15) & ~uint64_t(15);
        uint64_t const lds = xtBytes + (kBlock / 64) * slotBytes;
        if (rowBytes < 16 || (rowBytes % 16 != 0 && rt::knob(rt::Knob::ResampleAnyRows) == 0) ||
            reinterpret_cast<uintptr_t>(b.src) % 16 != 0 || lds > 65536)
            return false;
        // next-row prefetch (knob resample.prefetch): 1 for 2-byte destinations, 2 for every
        // destination, 0 (default since round 6) off.  Round 5 (profiles/r05/gatherp.jsonl): UInt16
        // 1024^3 -> 768^3 0.378 -> 0.358 ms with it, UInt8 lost.  Round 6, after the run tables
        // moved to scalar loads (profiles/r06/gatherp.jsonl): UInt16 1024^3 -> 768^3 0.343-0.346 ms
        // without vs 0.354-0.356 with, 768^3 -> 1024^3 0.500-0.503 vs 0.507-0.508; UInt8 equal.
        // The prefetched row's wait is a vmcnt(0) behind the task's stores either way (the store
        // count per task is not a compile-time constant).
        // destination-row tasks (knob resample.dst_rows: 0 off, 1 (default) UInt8 rows that are not
        // 16-B multiples with a 64 K-workgroup grid, >= 2 every eligible gather with a grid cap of
        // that many 1024s of workgroups).  In-process A/B (profiles/r06/dstab.jsonl): UInt8
        // 1000^3 -> 1024^3 0.407 -> 0.381 ms at cap 64; 768^3 -> 1024^3 and 1024^3 -> 768^3 UInt8
        // equal (0.305-0.318 / 0.201-0.216 vs 0.308 / 0.201), UInt16 15-25 % slower
        int64_t dr = rt::knob(rt::Knob::ResampleDstRows);
        if (dr == 1)
            dr = bs == 1 && bd == 1 && rowBytes % 16 != 0 ? 64 : 0;
        if (dr > 0 && !detect && !chain && bs == bd && bs <= 2 && rowBytes >= 16)
        {
            uint32_t const vd = 16 / bd;
            uint32_t const G = (static_cast<uint32_t>(b.ddx) + 64 * vd - 1) / (64 * vd);
            uint32_t const KS = static_cast<uint32_t>((rowBytes + 1023) / 1024);
            uint64_t const dtasks = static_cast<uint64_t>(b.ddy) * static_cast<uint64_t>(b.dnz);
            if (G <= 2 && KS <= 2 && b.ddx >= static_cast<int32_t>(vd) && dtasks < (1ull << 32))
            {
                uint64_t blocksD = (dtasks + 3) / 4;
                uint64_t const cap = static_cast<uint64_t>(dr) * 1024;
                unsigned const gd = static_cast<unsigned>(blocksD < cap ? blocksD : cap);
                uint32_t const slotd = static_cast<uint32_t>(slotBytes);
#define VKT_DR(S, C, P, GG, KK) hipLaunchKernelGGL((resampleGatherDstRowKernel<S, S, C, P, GG, KK>), dim3(gd), dim3(kBlock), lds, s, b, slotd)
#define VKT_DR_GK(S, C, P) do { if (G == 1) { if (KS == 1) VKT_DR(S, C, P, 1, 1); else VKT_DR(S, C, P, 1, 2); } \
                                else { if (KS == 1) VKT_DR(S, C, P, 2, 1); else VKT_DR(S, C, P, 2, 2); } } while (0)
                if (bs == 1)
                {
                    if (pad) { if (identity) VKT_DR_GK(1, false, true); else VKT_DR_GK(1, true, true); }
                    else { if (identity) VKT_DR_GK(1, false, false); else VKT_DR_GK(1, true, false); }
                }
                else
                {
                    if (identity) VKT_DR_GK(2, false, false); else VKT_DR_GK(2, true, false);
                }
#undef VKT_DR_GK
#undef VKT_DR
                return true;
            }
        }
        int64_t const pk = rt::knob(rt::Knob::ResamplePrefetch);
        bool const prefetch = (pk == 2 || (pk == 1 && bd == 2)) && !detect && !chain && rowBytes <= 4096;
        // one task per wave; for 1-byte destinations a task writes so little (one 1-KiB store
        // per dst row) that staging the x table per workgroup dominates: there the grid is
        // capped and waves loop over tasks (768^3 -> 1024^3 UInt8: 0.38 -> 0.29 ms; 2- and
        // 4-byte destinations ran 4-12 % slower capped)
        uint64_t blocks = (tasks + 3) / 4;
        if (bd == 1 && blocks > 16384)
            blocks = 16384;
        unsigned const g = static_cast<unsigned>(blocks < (1u << 30) ? blocks : (1u << 30));
        uint32_t const slot = static_cast<uint32_t>(slotBytes);
#define VKT_GL(S, D, C, H)                                                                                         \
    do {                                                                                                           \
        if (pad && !(H))                                                                                           \
        {                                                                                                          \
            if (prefetch)                                                                                          \
                hipLaunchKernelGGL((resampleGatherLdsKernel<S, D, C, false, false, true, kBlock, true>), dim3(g),  \
                                   dim3(kBlock), lds, s, b, slot);                                                \
            else                                                                                                   \
                hipLaunchKernelGGL((resampleGatherLdsKernel<S, D, C, false, false, false, kBlock, true>), dim3(g), \
                                   dim3(kBlock), lds, s, b, slot);                                                \
        }                                                                                                          \
        else if (prefetch && !(H))   /* (a chain instance with PREFETCH compiles as the plain one) */             \
            hipLaunchKernelGGL((resampleGatherLdsKernel<S, D, C, H, false, true>), dim3(g), dim3(kBlock), lds, s, b, \
                               slot);                                                                              \
        else                                                                                                       \
            hipLaunchKernelGGL((resampleGatherLdsKernel<S, D, C, H>), dim3(g), dim3(kBlock), lds, s, b, slot);     \
    } while (0)
#define VKT_GL_D(S, C, H) do { if (bd == 1) VKT_GL(S, 1, C, H); else if (bd == 2) VKT_GL(S, 2, C, H); else VKT_GL(S, 4, C, H); } while (0)
#define VKT_GLX(D, C) hipLaunchKernelGGL((resampleGatherLdsKernel<4, D, C, false, true>), dim3(g), dim3(kBlock), lds, s, b, slot)
        if (detect)
        {
            if (bd == 1) { if (identity) VKT_GLX(1, false); else VKT_GLX(1, true); }
            else if (bd == 2) { if (identity) VKT_GLX(2, false); else VKT_GLX(2, true); }
            else { if (identity) VKT_GLX(4, false); else VKT_GLX(4, true); }
        }
        else if (chain)
        {
            if (identity) VKT_GL_D(4, false, true); else VKT_GL_D(4, true, true);
        }
        else if (bs == 1)
        {
            if (identity) VKT_GL_D(1, false, false); else VKT_GL_D(1, true, false);
        }
        else if (bs == 2)
        {
            if (identity) VKT_GL_D(2, false, false); else VKT_GL_D(2, true, false);
        }
        else
        {
            if (identity) VKT_GL_D(4, false, false); else VKT_GL_D(4, true, false);
        }
#undef VKT_GLX
#undef VKT_GL_D
#undef VKT_GL
        return true;
    }

    vktError resampleSlab(vktHipVolumeView_t dst, vktHipVolumeView_t src, vktFilterMode fm, int32_t dgz, int32_t dz0,
                          int32_t sgz, int32_t sz0)
    {
        if (!validView(dst) || !validView(src))
            return rt::fail("Resample_hip: invalid volume view");
        if (fm != vktFilterModeNearest && fm != vktFilterModeLinear)
            return rt::fail("Resample_hip: unknown filter mode");
        if (dst.dimX == 0 || dst.dimY == 0 || dst.dimZ == 0)
            return vktNoError;
        if (src.dimX <= 0 || src.dimY <= 0 || src.dimZ <= 0)
            return rt::fail("Resample_hip: empty source");
        if (dz0 < 0 || dz0 + dst.dimZ > dgz || sz0 < 0 || sz0 + src.dimZ > sgz)
            return rt::fail("Resample_hip: slab outside the global volume");
        if (overlaps(dst, src) && dst.data != src.data)
            return rt::fail("Resample_hip: partially overlapping source and destination");
        if (!encodeWrites(dst.dataFormat))
            return vktNoError;

        hipStream_t s = rt::computeStream();
        // same-dims branch (Resample_serial.hpp:32-48)
        if (dst.dimX == src.dimX && dst.dimY == src.dimY && dgz == sgz)
        {
            if (dz0 < sz0 || dz0 + dst.dimZ > sz0 + src.dimZ)
                return rt::fail("Resample_hip: source slab does not hold the planes this dst slab reads");
            if (dst.data == src.data && dz0 != sz0)
                return rt::fail("Resample_hip: in-place same-dims resample needs aligned slabs");
            vktError e = convertBox(dst, src, vktVec3i_t{0, 0, dz0 - sz0}, false, vktVec3i_t{0, 0, 0}, dst.dimX,
                                    dst.dimY, dst.dimZ);
            return e != vktNoError ? e : rt::finishLaunch("Resample_hip(same dims)");
        }
        if (dst.data == src.data)
            return rt::fail("Resample_hip: in-place resample with different dims");

        Tables t;
        vktError e = getTables(dst.dimX, dst.dimY, dgz, dz0, dst.dimZ, src.dimX, src.dimY, sgz, t);
        if (e != vktNoError)
            return e;

        ConvProps const props = conversionProperties(src.dataFormat, src.mappingLo, src.mappingHi, dst.dataFormat,
                                                     dst.mappingLo, dst.mappingHi);
        bool const identity = props.identity;
        // "Linear" = the 8-neighbour lerp chain with every fraction 0; it differs
        // from v000 only through a non-finite neighbour, or a -0 v000 stored by a Float32
        // destination.  When the source mapping can produce neither, Linear IS Nearest.
        bool const chain = fm == vktFilterModeLinear &&
                           (!props.finite || (dst.dataFormat == codec::FmtFloat32 && props.negZero));
        // planes this dst slab reads: for the chain also the clamped z+1 neighbour plane and
        // the first voxel of the plane after it (hi.x of that plane's last voxel)
        int32_t needLo = t.minSz, needHi = t.maxSz;
        if (chain)
            needHi = needHi + 2 < sgz ? needHi + 2 : sgz - 1;
        if (needLo < sz0 || needHi >= sz0 + src.dimZ)
            return rt::fail("Resample_hip: source slab does not hold the planes this dst slab reads");

        ResampleArgs a{};
        a.dst = dst.data;
        a.src = src.data;
        a.ddx = dst.dimX;
        a.ddy = dst.dimY;
        a.sdx = src.dimX;
        a.sdy = src.dimY;
        a.sdz = src.dimZ;
        a.srcZ0 = sz0;
        a.srcGlobalDz = sgz;
        a.dstZ0 = dz0;
        a.nRunsY = t.nRunsY;
        a.nRunsZ = t.nRunsZ;
        a.runsY = t.runsY;
        a.runsZ = t.runsZ;
        a.xtab = t.xtab;
        a.affY = t.aff[0][0]; a.saY = t.aff[0][1]; a.daY = t.aff[0][2]; a.dlY = t.aff[0][3];
        a.s0Y = t.aff[0][4]; a.d0Y = t.aff[0][5];
        a.affZ = t.aff[1][0]; a.saZ = t.aff[1][1]; a.daZ = t.aff[1][2]; a.dlZ = t.aff[1][3];
        a.s0Z = t.aff[1][4]; a.d0Z = t.aff[1][5];
        a.k = t.k;
        a.zsrc = t.zsrc;
        a.ysrc = t.ysrc;
        a.fdDdy = makeFastDiv(static_cast<uint32_t>(dst.dimY));
        a.dnz = dst.dimZ;
        {
            static int const layout = [] {
                char const* e = std::getenv("VKT_RESAMPLE_LAYOUT");   // A/B tuning knob
                return e && std::string(e) == "row" ? 0 : 1;
            }();
            a.planeLayout = layout;
        }
        {
            uint32_t const bdv = codec::bytesPerVoxel(dst.dataFormat);
            uint32_t const vv = bdv <= 4 ? 16 / bdv : 1;
            uint32_t const instr = static_cast<uint32_t>((static_cast<uint64_t>(dst.dimX) + 64 * vv - 1) / (64 * vv));
            a.fdInstr = makeFastDiv(instr);
            a.fdRunsY = makeFastDiv(static_cast<uint32_t>(t.nRunsY));
            // plane layout computes the z run arithmetically only for contiguous affine runs
            if (t.aff[1][0] && t.aff[1][2] != t.aff[1][3])
                a.affZ = 0;
            a.fdDaZ = makeFastDiv(static_cast<uint32_t>(a.affZ ? a.daZ : 1));
            if (static_cast<uint64_t>(dst.dimZ) * static_cast<uint64_t>(t.nRunsY) * instr >= (1ull << 32))
                a.planeLayout = 0;
        }
        {
            // chain task order: bands of 8 rows (measured: equal time, 1.6x less HBM re-reading)
            a.band = 8;
        }
        a.fs = src.dataFormat;
        a.fd = dst.dataFormat;
        a.slo = src.mappingLo;
        a.shi = src.mappingHi;
        a.dm = codec::makeMapParams(dst.mappingLo, dst.mappingHi);
        a.srcVoxels = static_cast<uint64_t>(src.dimX) * src.dimY * src.dimZ;
        a.srcIsGlobalEnd = sz0 + src.dimZ == sgz;

        uint64_t tasks = static_cast<uint64_t>(t.nRunsY) * static_cast<uint64_t>(t.nRunsZ);
        if (tasks >= (1ull << 32))
            return rt::fail("Resample_hip: too many source rows");
        unsigned grid = streamingGrid(tasks, kBlock / 64);

        uint32_t const bs = codec::bytesPerVoxel(src.dataFormat), bd = codec::bytesPerVoxel(dst.dataFormat);
        if (launchRowKernel(a, t.k, tasks, bs, bd, identity, chain, src, dst, s, t))
            return rt::finishLaunch(chain ? "Resample_hip(row, linear chain)" : "Resample_hip(row)");
        uint32_t const v = bd <= 4 ? 16 / bd : 0;
        bool const vecDst = v != 0 && dst.dimX % v == 0 && reinterpret_cast<uintptr_t>(dst.data) % 16 == 0;
        if (chain && vecDst && src.dataFormat == codec::FmtFloat32 && reinterpret_cast<uintptr_t>(src.data) % 16 == 0)
        {
            // any ratio, Float32 source: flag the source rows holding a non-finite value or a
            // -0 (one streaming read of the source), OR the flags over each row's chain
            // neighbourhood, then gather -- only flagged tasks evaluate the chain
            static rt::StreamScratch scratch;
            uint64_t const srcRows = static_cast<uint64_t>(src.dimY) * static_cast<uint64_t>(src.dimZ);
            // [dirty: srcRows][chain: srcRows][pad to 4][anyChain word]
            uint64_t const anyOff = (2 * srcRows + 3) & ~uint64_t(3);
            uint8_t* dirty = static_cast<uint8_t*>(scratch.acquire(anyOff + 4, s));
            uint32_t* anyChain = dirty ? reinterpret_cast<uint32_t*>(dirty + anyOff) : nullptr;
            // Optimistic variant: the LDS gather flags the rows it stages itself, the local rows
            // no task stages (skipped rows when downsampling, the z+1 halo planes) are scanned
            // (rowDirtyUnstagedKernel), then rowChainKernel and a fix-up pass over the flagged
            // tasks -- every source row is read once (768^3 -> 1024^3 and 1024^3 -> 768^3
            // Float32 Linear: see DESIGN.md §4.2b)
            if (dirty && t.staged && src.dimX % 4 == 0 && gatherLdsEnabled())
            {
                // Every local row's flag is written this call -- the gather writes the rows it
                // stages, rowDirtyUnstagedKernel the rest (launched only when some local row is
                // not staged: downsampling, z+1 halo planes) -- so nothing is cleared first; the
                // fix-up reads the flags of each task's chain rows directly (taskFlagged) and
                // returns at once unless a pass wrote this call's epoch.  Clean upsampling
                // volumes: the gather and one early-exiting fix-up launch (round 6: two memsets,
                // a 147 k-workgroup unstaged scan and rowChainKernel gone).
                static std::atomic<uint32_t> epochs{0};
                ResampleArgs b = a;
                b.rowDirtyOut = dirty;
                b.rowDirty = dirty;
                b.srcRows = srcRows;
                b.rowChain = nullptr;
                b.anyDirtyOut = anyChain;
                b.epoch = epochs.fetch_add(1) + 1;
                bool const unstaged = static_cast<uint64_t>(t.nRunsY) * static_cast<uint64_t>(t.nRunsZ) < srcRows;
                if (unstaged)
                {
                    unsigned const gd = static_cast<unsigned>((srcRows + kBlock / 64 - 1) / (kBlock / 64));
                    hipLaunchKernelGGL(rowDirtyUnstagedKernel, dim3(gd), dim3(kBlock), 0, s, src.data, src.dimX,
                                       src.dimY, srcRows, a.srcZ0, t.staged, dirty, anyChain, b.epoch);
                }
                if (launchGatherLds(b, bs, bd, identity, false, tasks, s, true))
                {
                    unsigned const gf = streamingGrid(tasks, kBlock / 64, 8);
                    hipLaunchKernelGGL(resampleGatherFixupKernel, dim3(gf), dim3(kBlock), 0, s, b);
                    scratch.release(s);
                    return rt::finishLaunch("Resample_hip(linear chain, optimistic gather)");
                }
            }
            if (dirty)
            {
                unsigned const gd = static_cast<unsigned>((srcRows + kBlock / 64 - 1) / (kBlock / 64));
                if (src.dimX % 4 == 0)
                    hipLaunchKernelGGL(rowDirtyKernel<true>, dim3(gd), dim3(kBlock), 0, s, src.data, src.dimX, srcRows,
                                       dirty);
                else
                    hipLaunchKernelGGL(rowDirtyKernel<false>, dim3(gd), dim3(kBlock), 0, s, src.data, src.dimX, srcRows,
                                       dirty);
                unsigned const gc = static_cast<unsigned>((srcRows + kBlock - 1) / kBlock);
                hipLaunchKernelGGL(rowChainKernel, dim3(gc), dim3(kBlock), 0, s, dirty, src.dimY, src.dimZ, a.srcZ0,
                                   a.srcGlobalDz, dirty + srcRows, nullptr);
                ResampleArgs b = a;
                b.rowChain = dirty + srcRows;
                if (!gatherLdsEnabled() || !launchGatherLds(b, bs, bd, identity, true, tasks, s))
                {
                    uint64_t blocks = (tasks + 3) / 4;   // one task per wave
                    unsigned g = static_cast<unsigned>(blocks < (1u << 30) ? blocks : (1u << 30));
#define VKT_GVC(B, C) hipLaunchKernelGGL((resampleGatherVecKernel<B, C, true>), dim3(g), dim3(kBlock), 0, s, b)
                    if (bd == 1) { if (identity) VKT_GVC(1, false); else VKT_GVC(1, true); }
                    else if (bd == 2) { if (identity) VKT_GVC(2, false); else VKT_GVC(2, true); }
                    else { if (identity) VKT_GVC(4, false); else VKT_GVC(4, true); }
#undef VKT_GVC
                }
                scratch.release(s);
                return rt::finishLaunch("Resample_hip(linear chain, flagged gather)");
            }
            (void)hipGetLastError();
        }
        if (chain)
        {
            hipLaunchKernelGGL(resampleChainKernel, dim3(grid), dim3(kBlock), 0, s, a);
            return rt::finishLaunch("Resample_hip(linear chain, gather)");
        }
        if (vecDst && gatherLdsEnabled() && launchGatherLds(a, bs, bd, identity, false, tasks, s))
            return rt::finishLaunch("Resample_hip(gather, LDS)");
        if (vecDst)
        {
            uint64_t blocks = (tasks + 3) / 4;   // one task per wave
            unsigned g = static_cast<unsigned>(blocks < (1u << 30) ? blocks : (1u << 30));
#define VKT_GV(B, C) hipLaunchKernelGGL((resampleGatherVecKernel<B, C>), dim3(g), dim3(kBlock), 0, s, a)
            if (bd == 1) { if (identity) VKT_GV(1, false); else VKT_GV(1, true); }
            else if (bd == 2) { if (identity) VKT_GV(2, false); else VKT_GV(2, true); }
            else { if (identity) VKT_GV(4, false); else VKT_GV(4, true); }
#undef VKT_GV
            return rt::finishLaunch("Resample_hip(gather, vector)");
        }
        hipLaunchKernelGGL(resampleGatherKernel, dim3(grid), dim3(kBlock), 0, s, a, identity ? 0 : 1);
        return rt::finishLaunch("Resample_hip(gather)");
    }

} // hipk
} // vkt

using namespace vkt;

extern "C" {

vktError vktHipResample(vktHipVolumeView_t dst, vktHipVolumeView_t src, vktFilterMode fm)
{
    return hipk::resampleSlab(dst, src, fm, dst.dimZ, 0, src.dimZ, 0);
}

vktError vktHipResampleSlab(vktHipVolumeView_t dst, vktHipVolumeView_t src, vktFilterMode fm, int32_t dstGlobalDimZ,
                            int32_t dstZ0, int32_t srcGlobalDimZ, int32_t srcZ0)
{
    return hipk::resampleSlab(dst, src, fm, dstGlobalDimZ, dstZ0, srcGlobalDimZ, srcZ0);
}

vktError vktHipResampleSlabSourceRange(int32_t dstGlobalDimZ, int32_t dstZ0, int32_t dstZ1, int32_t srcGlobalDimZ,
                                       vktFilterMode fm, int32_t needsNeighbours, int32_t* srcZBegin,
                                       int32_t* srcZEnd)
{
    if (srcZBegin == nullptr || srcZEnd == nullptr)
        return rt::fail("vktHipResampleSlabSourceRange: null pointer");
    if (dstZ1 <= dstZ0)
    {
        *srcZBegin = *srcZEnd = 0;
        return vktNoError;
    }
    if (dstGlobalDimZ == srcGlobalDimZ)   // same-dims branch maps plane to plane
    {
        *srcZBegin = dstZ0;
        *srcZEnd = dstZ1;
        return vktNoError;
    }
    int32_t lo = hipk::srcIndex(dstZ0, dstGlobalDimZ, srcGlobalDimZ);
    int32_t hi = hipk::srcIndex(dstZ1 - 1, dstGlobalDimZ, srcGlobalDimZ);
    if (fm == vktFilterModeLinear && needsNeighbours)
        hi = hi + 2 < srcGlobalDimZ ? hi + 2 : srcGlobalDimZ - 1;
    *srcZBegin = lo;
    *srcZEnd = hi + 1;
    return vktNoError;
}

} // extern "C"
