// ResampleRow.hpp -- shared types of the Resample kernels and the integer-ratio row kernel
// template (instantiated per MODE in ResampleRow{0,1,2}.hip so that the ~100 instantiations
// compile in parallel).  Semantics and design: kernels/Resample.hip header comment.
#pragma once

#include "KernelCommon.hpp"
#include "volkit_c.h"

namespace vkt
{
namespace hipk
{
    using codec::MapParams;

    // Exact reference index formula (Resample_serial.hpp:60-62 + int32 truncation).
    inline int32_t srcIndex(int32_t d, int32_t dd, int32_t sd)
    {
        volatile float q = static_cast<float>(d) / static_cast<float>(dd);
        volatile float s = q * static_cast<float>(sd);
        return static_cast<int32_t>(s);
    }

    // One run: destination rows [d0, d1) all read source row `s`.
    struct Run
    {
        int32_t s, d0, d1;
    };

    struct ResampleArgs
    {
        uint8_t* dst;
        uint8_t const* src;
        int32_t ddx, ddy;          // dst dims x, y (dst slab depth implied by runs)
        int32_t sdx, sdy, sdz;     // src dims of the LOCAL source buffer
        int32_t srcZ0;             // global z of local plane 0
        int32_t srcGlobalDz;       // global source depth (hi.z clamp)
        int32_t dstZ0;             // global z of dst plane 0
        int32_t nRunsY, nRunsZ;
        Run const* runsY;          // device
        Run const* runsZ;          // device (s in GLOBAL source planes, d in GLOBAL dst planes)
        // Affine run generators (exact integer ratios, verified against the tables on the
        // host): run i = {s0 + sa*i, d0 + da*i, d0 + da*i + dl}; avoids a dependent table load
        // at the start of every task.
        int32_t affY, saY, daY, dlY, s0Y, d0Y;
        int32_t affZ, saZ, daZ, dlZ, s0Z, d0Z;
        int32_t band;              // chain task order: rows per band (0 = plain y-fastest order)
        int32_t const* xtab;       // device, ddx entries (gather/chain paths)
        int32_t k;                 // integer x ratio (replication path)
        int32_t fs, fd;
        float slo, shi;
        MapParams dm;
        uint64_t srcVoxels;        // voxels in the local source buffer (flat-read clamp)
        int32_t srcIsGlobalEnd;    // local buffer ends at the global end (clamp there)
        // MODE 2 only: one byte per local source row, nonzero if the row holds a value that
        // can make the lerp chain differ from its first term (non-finite, or -0); nullptr =
        // evaluate the chain everywhere.  Built by rowDirtyKernel just before the launch.
        uint8_t const* rowDirty;
        uint64_t srcRows;          // local source rows (sdy * sdz)
        // plane-linear layout (resamplePlaneKernel): source plane (global) of every local dst
        // plane, and the dst slab depth
        int32_t const* zsrc;       // device, dnz entries
        int32_t dnz;
        int32_t planeLayout;       // 1: resamplePlaneKernel, 0: resampleRowKernel
        FastDiv fdInstr, fdRunsY, fdDaZ;   // task decomposition without integer division
        uint8_t* rowDirtyOut;      // MODE 3: flags written by the detect pass (zeroed before)
        // MODE 2, plane layout: one byte per local source row r, nonzero if the chain of a
        // voxel in row r can differ from v000 (OR of rowDirty over the rows its chain reads);
        // built from rowDirty by rowChainKernel.  nullptr = chain everywhere.
        uint8_t const* rowChain;
        // resamplePlaneKernel: this launch runs tasks [taskBase, taskEnd) (planeChunks)
        uint32_t taskBase, taskEnd;
        // optimistic gather: nonzero iff any rowChain byte is set (written by rowChainKernel);
        // the fix-up pass returns at once when it is 0 (the common case).  nullptr = scan.
        uint32_t const* anyChain;
        // optimistic LDS gather (Float32 "Linear", any ratio): the passes that classify source
        // rows write this call's `epoch` here when they flag one; the fix-up runs only if the word
        // holds the epoch (no per-call zeroing: a stale equal value only costs a scan).
        uint32_t* anyDirtyOut;
        uint32_t epoch;
        // dst-row gather (resampleGatherDstRowKernel): source row y of every dst row y (ddy
        // entries) and a fast divisor by ddy
        int32_t const* ysrc;
        FastDiv fdDdy;
    };

    // Plane-layout launches are split into at most kMaxPlaneTasksPerLaunch one-wave workgroups
    // (as the pointwise engine's kMaxQuantaPerLaunch: multi-million-workgroup launches ran
    // ~10 % below the per-voxel rate of 1 M-workgroup ones on MI355X).
    constexpr uint64_t kMaxPlaneTasksPerLaunch = 1ull << 20;

    template <class Launch>
    void planeChunks(ResampleArgs a, uint64_t tasks, Launch&& launch)
    {
        uint64_t t0 = 0;
        do
        {
            uint64_t const n = tasks - t0 < kMaxPlaneTasksPerLaunch ? tasks - t0 : kMaxPlaneTasksPerLaunch;
            a.taskBase = static_cast<uint32_t>(t0);
            a.taskEnd = static_cast<uint32_t>(t0 + n);
            launch(a, static_cast<unsigned>(n > 0 ? n : 1));
            t0 += n;
        } while (t0 < tasks);
    }

    // A Float32 code that can make lerp(a, b, 0) = a + 0*b differ from a: b non-finite
    // (0*b = NaN) or a == -0 (-0 + +0 = +0).
    __device__ __forceinline__ bool chainSensitive(uint32_t bits)
    {
        return (bits & 0x7F800000u) == 0x7F800000u || bits == 0x80000000u;
    }

    // Run tables are read through the constant address space: with a wave-uniform index they
    // become scalar loads (lgkmcnt), not vector loads whose s_waitcnt vmcnt(0) would also wait
    // for every store the wave still has in flight (gfx950's vmcnt counts loads AND stores).
    typedef __attribute__((address_space(4))) int32_t const ConstI32;
    __device__ __forceinline__ Run loadRun(Run const* table, uint32_t i)
    {
        ConstI32* const p = (ConstI32*)table + 3u * i;
        return Run{p[0], p[1], p[2]};
    }

    __device__ __forceinline__ Run runY(ResampleArgs const& a, uint32_t i)
    {
        if (a.affY)
        {
            int32_t d0 = a.d0Y + a.daY * static_cast<int32_t>(i);
            return Run{a.s0Y + a.saY * static_cast<int32_t>(i), d0, d0 + a.dlY};
        }
        return loadRun(a.runsY, i);
    }

    __device__ __forceinline__ Run runZ(ResampleArgs const& a, uint32_t i)
    {
        if (a.affZ)
        {
            int32_t d0 = a.d0Z + a.daZ * static_cast<int32_t>(i);
            return Run{a.s0Z + a.saZ * static_cast<int32_t>(i), d0, d0 + a.dlZ};
        }
        return loadRun(a.runsZ, i);
    }

    template <int FS, int FD>
    __device__ __forceinline__ uint32_t convertCode(uint32_t c, ResampleArgs const& a)
    {
        float v = codec::decode(c, FS == -1 ? a.fs : FS, a.slo, a.shi);
        bool w;
        return codec::encode(v, FD == -1 ? a.fd : FD, a.dm, w);
    }

    __device__ __forceinline__ uint64_t dstRowIndex(ResampleArgs const& a, int32_t yd, int32_t zdGlobal)
    {
        return (static_cast<uint64_t>(zdGlobal - a.dstZ0) * static_cast<uint64_t>(a.ddy) + static_cast<uint64_t>(yd)) *
               static_cast<uint64_t>(a.ddx);
    }

    __device__ __forceinline__ uint64_t srcRowIndex(ResampleArgs const& a, int32_t ys, int32_t zsGlobal)
    {
        return (static_cast<uint64_t>(zsGlobal - a.srcZ0) * static_cast<uint64_t>(a.sdy) + static_cast<uint64_t>(ys)) *
               static_cast<uint64_t>(a.sdx);
    }

    // ---- integer-ratio row kernel (replication, conversion, and the Float32 lerp chain) ----
    // One wave per source row (task).  Destination rows are written as wave-instructions of
    // 64 lanes x 16 bytes: lane l of instruction g writes dst voxels [g*64V + V*l, +V) with
    // V = 16 / BPVD, so every wave-store is one contiguous KiB.  Those V voxels come from
    // N = V / K consecutive source voxels (one coalesced load per lane); each source voxel is
    // decoded / converted / chained ONCE and replicated K times in registers, and the same
    // registers are stored to every destination row of the task's rectangle.  Loads of all
    // NSLOT instructions are issued unconditionally (clamped into the row) before any store.
    // Measured (512^3 -> 1024^3 UInt16 identity): 0.35 ms = 6.9 TB/s; a half-strided store
    // layout (2 x 16 B per lane) ran at 2.6 TB/s.
    //
    // MODE 0: identity codes (verified on the host for every code); MODE 1: convert each
    // source code; MODE 2: "Linear" with float semantics -- the reference's sampleLinear
    // chain lerp(lerp(lerp(v000,v100,0),lerp(v010,v110,0),0), lerp(...), 0) over the
    // neighbours (x+1 = next voxel in memory, y+1 / z+1 clamped), evaluated per SOURCE voxel.
    template <int BPVS, int BPVD, int K, int MODE, int FS, int FD, int NSLOT>
    __global__ __launch_bounds__(kBlock) void resampleRowKernel(ResampleArgs a)
    {
        constexpr int V = 16 / BPVD;
        constexpr int N = V / K;
        constexpr int kInstr = 64 * V;
        int const lane = threadIdx.x & 63;
        uint32_t const wavesPerBlock = blockDim.x >> 6;
        // wave-uniform task index in SGPRs
        uint32_t const wave = __builtin_amdgcn_readfirstlane(xcdSwizzle(blockIdx.x, gridDim.x) * wavesPerBlock +
                                                             (threadIdx.x >> 6));
        uint32_t const totalWaves = gridDim.x * wavesPerBlock;
        int32_t const instrPerRow = (a.ddx + kInstr - 1) / kInstr;
        // Task order.  Replication/conversion: y fastest (the write stream sweeps each plane).
        // Chain: bands of kBand source rows, then z, then y within the band -- the workgroup
        // that handles plane sz+1 of a band runs right after the one for plane sz on the same
        // XCD (xcdSwizzle), so the z+1 neighbour rows are still in L2 (otherwise they were
        // evicted and re-read from HBM: 2x source traffic measured).
        uint32_t const kBand = MODE == 2 ? static_cast<uint32_t>(a.band) : 0u;
        uint32_t const nY = static_cast<uint32_t>(a.nRunsY), nZ = static_cast<uint32_t>(a.nRunsZ);
        uint32_t const tasks = kBand ? (nY + kBand - 1) / kBand * kBand * nZ : nY * nZ;

        for (uint32_t t = wave; t < tasks; t += totalWaves)
        {
            uint32_t iy, iz;
            if (kBand)
            {
                uint32_t const rest = t / kBand;
                iz = rest % nZ;
                iy = (rest / nZ) * kBand + t % kBand;
                if (iy >= nY)
                    continue;
            }
            else
            {
                iy = t % nY;
                iz = t / nY;
            }
            Run const ry = runY(a, iy);
            Run const rz = runZ(a, iz);
            uint64_t const r00 = srcRowIndex(a, ry.s, rz.s);
            uint64_t r10 = 0, r01 = 0, r11 = 0;
            bool chainTask = false;   // wave-uniform
            if constexpr (MODE == 2)
            {
                int32_t const hy = ry.s + 1 < a.sdy ? ry.s + 1 : a.sdy - 1;
                int32_t const hz = rz.s + 1 < a.srcGlobalDz ? rz.s + 1 : a.srcGlobalDz - 1;
                r10 = srcRowIndex(a, hy, rz.s);
                r01 = srcRowIndex(a, ry.s, hz);
                r11 = srcRowIndex(a, hy, hz);
                chainTask = true;
                if (a.rowDirty)
                {
                    // The chain of a voxel reads rows r00, r10, r01, r11 and, for the row's
                    // last voxel, the first voxel of the row after each in memory (clamped to
                    // the buffer's last voxel, i.e. its own row, at the end).  If none of
                    // them holds a sensitive value, every 0*neighbour term is +-0 and the
                    // chain returns v000 exactly: plain conversion, no neighbour reads.
                    uint64_t const lastRow = a.srcRows - 1;
                    uint64_t const sdx = static_cast<uint64_t>(a.sdx);
                    uint32_t dirty = 0;
                    for (uint64_t r : {r00 / sdx, r10 / sdx, r01 / sdx, r11 / sdx})
                        dirty |= a.rowDirty[r] | a.rowDirty[r < lastRow ? r + 1 : lastRow];
                    chainTask = __builtin_amdgcn_readfirstlane(dirty) != 0;
                }
            }
            for (int32_t g0 = 0; g0 < instrPerRow; g0 += NSLOT)
            {
                uint32_t code[NSLOT][V];
                bool active[NSLOT];
#pragma unroll
                for (int u = 0; u < NSLOT; ++u)
                {
                    int32_t dx = kInstr * (g0 + u) + V * lane;
                    active[u] = g0 + u < instrPerRow && dx < a.ddx;
                    dx = dx < a.ddx ? dx : a.ddx - V;
                    uint64_t const sx = static_cast<uint64_t>(dx / K);
                    uint32_t sc[N];
                    loadN<BPVS, N, true>(a.src, r00 + sx, sc);
                    if constexpr (MODE == 1)
                    {
#pragma unroll
                        for (int i = 0; i < N; ++i)
                            sc[i] = convertCode<FS, FD>(sc[i], a);
                    }
                    else if constexpr (MODE == 2)
                    {
                      if (!chainTask)
                      {
#pragma unroll
                        for (int i = 0; i < N; ++i)
                            sc[i] = convertCode<FS, FD>(sc[i], a);
                      }
                      else
                      {
                        uint32_t c10[N], c01[N], c11[N];
                        loadN<BPVS, N, true>(a.src, r10 + sx, c10);
                        loadN<BPVS, N, true>(a.src, r01 + sx, c01);
                        loadN<BPVS, N, true>(a.src, r11 + sx, c11);
                        // x+1 neighbour of the lane's last voxel = the next lane's first voxel:
                        // wave64 shuffle; lane 63 and the row's last group (whose neighbour is
                        // the next row's first voxel, or past the buffer end) read it directly.
                        uint32_t e00 = __shfl_down(sc[0], 1), e10 = __shfl_down(c10[0], 1);
                        uint32_t e01 = __shfl_down(c01[0], 1), e11 = __shfl_down(c11[0], 1);
                        if (lane == 63 || dx + V >= a.ddx)
                        {
                            uint64_t const last = a.srcVoxels - 1;   // reference reads past the end: clamp
                            auto flat = [&](uint64_t i) { return loadCode<BPVS>(a.src, i < last ? i : last); };
                            e00 = flat(r00 + sx + N);
                            e10 = flat(r10 + sx + N);
                            e01 = flat(r01 + sx + N);
                            e11 = flat(r11 + sx + N);
                        }
                        int32_t const fs = FS == -1 ? a.fs : FS;
                        auto dec = [&](uint32_t c) { return codec::decode(c, fs, a.slo, a.shi); };
                        float const f = 0.f;   // every fraction of sampleLinear(int,int,int) is 0
                        uint32_t out[N];
#pragma unroll
                        for (int i = 0; i < N; ++i)
                        {
                            float v0 = dec(sc[i]), v1 = dec(i + 1 < N ? sc[i + 1] : e00);
                            float v2 = dec(c10[i]), v3 = dec(i + 1 < N ? c10[i + 1] : e10);
                            float v4 = dec(c01[i]), v5 = dec(i + 1 < N ? c01[i + 1] : e01);
                            float v6 = dec(c11[i]), v7 = dec(i + 1 < N ? c11[i + 1] : e11);
                            float value = codec::lerp(codec::lerp(codec::lerp(v0, v1, f), codec::lerp(v2, v3, f), f),
                                                      codec::lerp(codec::lerp(v4, v5, f), codec::lerp(v6, v7, f), f), f);
                            bool w;
                            out[i] = codec::encode(value, FD == -1 ? a.fd : FD, a.dm, w);
                        }
#pragma unroll
                        for (int i = 0; i < N; ++i)
                            sc[i] = out[i];
                      }
                    }
#pragma unroll
                    for (int i = 0; i < V; ++i)
                        code[u][i] = sc[i / K];
                }
                for (int32_t zd = rz.d0; zd < rz.d1; ++zd)
                    for (int32_t yd = ry.d0; yd < ry.d1; ++yd)
                    {
                        uint64_t const drow = dstRowIndex(a, yd, zd) + static_cast<uint64_t>(V) * lane;
#pragma unroll
                        for (int u = 0; u < NSLOT; ++u)
                            if (active[u])
                                store16<BPVD>(a.dst, drow + static_cast<uint64_t>(kInstr) * (g0 + u), code[u]);
                    }
            }
        }
    }


    // The reference's sampleLinear chain for the N source voxels [sx, sx + N) of row r00
    // (codes in sc), with neighbour rows r10 (y+1), r01 (z+1), r11 and hi.x = the next voxel in
    // memory (from the next lane, or loaded directly at the lane / row end; past the buffer end
    // clamped to the last voxel).  Overwrites sc with the destination codes.
    template <int BPVS, int N, int FS, int FD>
    __device__ __forceinline__ void chainEval(ResampleArgs const& a, uint64_t r00, uint64_t r10, uint64_t r01,
                                              uint64_t r11, uint64_t sx, bool rowEnd, int lane, uint32_t (&sc)[N])
    {
        uint32_t c10[N], c01[N], c11[N];
        loadN<BPVS, N, true>(a.src, r10 + sx, c10);
        loadN<BPVS, N, true>(a.src, r01 + sx, c01);
        loadN<BPVS, N, true>(a.src, r11 + sx, c11);
        uint32_t e00 = __shfl_down(sc[0], 1), e10 = __shfl_down(c10[0], 1);
        uint32_t e01 = __shfl_down(c01[0], 1), e11 = __shfl_down(c11[0], 1);
        if (lane == 63 || rowEnd)
        {
            uint64_t const last = a.srcVoxels - 1;   // reference reads past the end: clamp
            auto flat = [&](uint64_t i) { return loadCode<BPVS>(a.src, i < last ? i : last); };
            e00 = flat(r00 + sx + N);
            e10 = flat(r10 + sx + N);
            e01 = flat(r01 + sx + N);
            e11 = flat(r11 + sx + N);
        }
        int32_t const fs = FS == -1 ? a.fs : FS;
        auto dec = [&](uint32_t c) { return codec::decode(c, fs, a.slo, a.shi); };
        float const f = 0.f;   // every fraction of sampleLinear(int,int,int) is 0
        uint32_t out[N];
#pragma unroll
        for (int i = 0; i < N; ++i)
        {
            float v0 = dec(sc[i]), v1 = dec(i + 1 < N ? sc[i + 1] : e00);
            float v2 = dec(c10[i]), v3 = dec(i + 1 < N ? c10[i + 1] : e10);
            float v4 = dec(c01[i]), v5 = dec(i + 1 < N ? c01[i + 1] : e01);
            float v6 = dec(c11[i]), v7 = dec(i + 1 < N ? c11[i + 1] : e11);
            float value = codec::lerp(codec::lerp(codec::lerp(v0, v1, f), codec::lerp(v2, v3, f), f),
                                      codec::lerp(codec::lerp(v4, v5, f), codec::lerp(v6, v7, f), f), f);
            bool w;
            out[i] = codec::encode(value, FD == -1 ? a.fd : FD, a.dm, w);
        }
#pragma unroll
        for (int i = 0; i < N; ++i)
            sc[i] = out[i];
    }

    // ---- plane-linear variant: the write stream sweeps the destination in memory order ----
    // One wave (and one 64-thread workgroup) per task = (dst plane, source-row run in y, one
    // 64-lane store instruction of x): it loads the N = V/K source voxels per lane that feed
    // its 64*V destination voxels, converts / chains them once, and stores the instruction
    // into every dst row of the y run (K_y rows of ONE plane).  Tasks are numbered x-fastest,
    // then y, then dst plane, so the grid writes memory in order; a source row is re-read by
    // the tasks of each dst plane it feeds (from L2 / MALL, not HBM: the source plane is
    // re-used within one dst plane's sweep).  Measured on 1024^3 -> 2048^3 Float32 (tools/
    // kbench6): 5.9 ms vs 7.4 ms for the source-row-rectangle layout -- many short one-wave
    // workgroups writing 2 KiB each keep more store streams in flight per channel than long
    // waves writing 32 KiB into 4 rows of 2 planes.
    template <int BPVS, int BPVD, int K, int MODE, int FS, int FD>
    __global__ __launch_bounds__(64) void resamplePlaneKernel(ResampleArgs a)
    {
        constexpr int V = 16 / BPVD;
        constexpr int N = V / K;
        constexpr int kInstr = 64 * V;
        int const lane = threadIdx.x & 63;
        uint32_t const instrPerRow = a.fdInstr.d;
        uint32_t const nY = a.fdRunsY.d;
        // tasks < 2^32 (checked on the host); this launch: [taskBase, taskEnd)
        for (uint32_t t = a.taskBase + blockIdx.x; t < a.taskEnd; t += gridDim.x)
        {
            // all task math is wave-uniform (scalar unit); no dependent table load before the
            // source load when the z runs are affine
            uint32_t const rest = fdiv(t, a.fdInstr);
            uint32_t const g = t - rest * instrPerRow;
            uint32_t const zlu = fdiv(rest, a.fdRunsY);
            uint32_t const iy = rest - zlu * nY;
            int32_t const zl = static_cast<int32_t>(zlu);           // local dst plane
            Run const ry = runY(a, iy);
            int32_t sz;                                             // global source plane
            if (a.affZ)
                sz = a.s0Z + a.saZ * static_cast<int32_t>(fdiv(static_cast<uint32_t>(a.dstZ0 + zl - a.d0Z), a.fdDaZ));
            else
                sz = a.zsrc[zl];
            uint64_t const r00 = srcRowIndex(a, ry.s, sz);
            int32_t dx = kInstr * static_cast<int32_t>(g) + V * lane;
            bool const active = dx < a.ddx;
            dx = active ? dx : a.ddx - V;
            uint64_t const sx = static_cast<uint64_t>(dx / K);
            uint32_t sc[N];
            loadN<BPVS, N, true>(a.src, r00 + sx, sc);
            if constexpr (MODE == 1)
            {
#pragma unroll
                for (int i = 0; i < N; ++i)
                    sc[i] = convertCode<FS, FD>(sc[i], a);
            }
            else if constexpr (MODE == 2)
            {
                int32_t const hy = ry.s + 1 < a.sdy ? ry.s + 1 : a.sdy - 1;
                int32_t const hz = sz + 1 < a.srcGlobalDz ? sz + 1 : a.srcGlobalDz - 1;
                uint64_t const r10 = srcRowIndex(a, hy, sz), r01 = srcRowIndex(a, ry.s, hz);
                uint64_t const r11 = srcRowIndex(a, hy, hz);
                bool chainTask = true;
                if (a.rowChain)
                {
                    uint64_t const row = static_cast<uint64_t>(sz - a.srcZ0) * static_cast<uint64_t>(a.sdy) +
                                         static_cast<uint64_t>(ry.s);
                    chainTask = __builtin_amdgcn_readfirstlane(a.rowChain[row]) != 0;
                }
                if (!chainTask)
                {
#pragma unroll
                    for (int i = 0; i < N; ++i)
                        sc[i] = convertCode<FS, FD>(sc[i], a);
                }
                else
                    chainEval<BPVS, N, FS, FD>(a, r00, r10, r01, r11, sx, dx + V >= a.ddx, lane, sc);
            }
            else if constexpr (MODE == 3)
            {
                // optimistic Float32 "Linear": write the conversion of v000 and flag the source
                // row if it holds a value that can make the chain differ (resampleFixupKernel
                // then rewrites the tasks next to flagged rows)
                bool sens = false;
#pragma unroll
                for (int i = 0; i < N; ++i)
                    sens = sens || chainSensitive(sc[i]);
                if (sens)   // rare; any lane may set the row's flag
                    a.rowDirtyOut[static_cast<uint64_t>(sz - a.srcZ0) * static_cast<uint64_t>(a.sdy) +
                                  static_cast<uint64_t>(ry.s)] = 1;
#pragma unroll
                for (int i = 0; i < N; ++i)
                    sc[i] = convertCode<FS, FD>(sc[i], a);
            }
            uint32_t code[V];
#pragma unroll
            for (int i = 0; i < V; ++i)
                code[i] = sc[i / K];
            if (active)
            {
                int32_t const zd = a.dstZ0 + zl;
                for (int32_t yd = ry.d0; yd < ry.d1; ++yd)
                    store16<BPVD>(a.dst, dstRowIndex(a, yd, zd) + static_cast<uint64_t>(dx), code);
            }
        }
    }

    // After a MODE 3 pass.  Scan: one THREAD per task (y run, z run) ORs the flags of the rows
    // its chain reads (r00, r10, r01, r11 and the row after each in memory) and appends the
    // flagged tasks to a work list.  Fix-up: a fixed grid of waves drains the list, re-evaluating
    // the chain for each listed task and overwriting what MODE 3 wrote there.
    __device__ __forceinline__ bool taskFlagged(ResampleArgs const& a, Run const& ry, Run const& rz)
    {
        int32_t const hy = ry.s + 1 < a.sdy ? ry.s + 1 : a.sdy - 1;
        int32_t const hz = rz.s + 1 < a.srcGlobalDz ? rz.s + 1 : a.srcGlobalDz - 1;
        uint64_t const sdy = static_cast<uint64_t>(a.sdy);
        uint64_t const z0 = static_cast<uint64_t>(rz.s - a.srcZ0) * sdy, z1 = static_cast<uint64_t>(hz - a.srcZ0) * sdy;
        uint64_t const lastRow = a.srcRows - 1;
        uint32_t dirty = 0;
        for (uint64_t r : {z0 + ry.s, z0 + hy, z1 + ry.s, z1 + hy})
            dirty |= a.rowDirty[r] | a.rowDirty[r < lastRow ? r + 1 : lastRow];
        return dirty != 0;
    }

    template <int BPVD, int K>
    __global__ __launch_bounds__(64) void resampleFixupKernel(ResampleArgs a, uint32_t const* list)
    {
        constexpr int BPVS = 4;
        constexpr int V = 16 / BPVD;
        constexpr int N = V / K;
        constexpr int kInstr = 64 * V;
        int const lane = threadIdx.x & 63;
        uint32_t const nY = static_cast<uint32_t>(a.nRunsY);
        uint32_t const instrPerRow = a.fdInstr.d;
        uint32_t const count = __builtin_amdgcn_readfirstlane(list[0]);
        for (uint32_t w = blockIdx.x; w < count; w += gridDim.x)
        {
            uint32_t const t = __builtin_amdgcn_readfirstlane(list[1 + w]);
            uint32_t const iz = t / nY, iy = t - iz * nY;
            Run const ry = runY(a, iy);
            Run const rz = runZ(a, iz);
            int32_t const hy = ry.s + 1 < a.sdy ? ry.s + 1 : a.sdy - 1;
            int32_t const hz = rz.s + 1 < a.srcGlobalDz ? rz.s + 1 : a.srcGlobalDz - 1;
            uint64_t const r00 = srcRowIndex(a, ry.s, rz.s), r10 = srcRowIndex(a, hy, rz.s);
            uint64_t const r01 = srcRowIndex(a, ry.s, hz), r11 = srcRowIndex(a, hy, hz);
            for (uint32_t g = 0; g < instrPerRow; ++g)
            {
                int32_t dx = kInstr * static_cast<int32_t>(g) + V * lane;
                bool const active = dx < a.ddx;
                dx = active ? dx : a.ddx - V;
                uint64_t const sx = static_cast<uint64_t>(dx / K);
                uint32_t sc[N];
                loadN<BPVS, N, true>(a.src, r00 + sx, sc);
                chainEval<BPVS, N, codec::FmtFloat32, -1>(a, r00, r10, r01, r11, sx, dx + V >= a.ddx, lane, sc);
                uint32_t code[V];
#pragma unroll
                for (int i = 0; i < V; ++i)
                    code[i] = sc[i / K];
                if (active)
                    for (int32_t zd = rz.d0; zd < rz.d1; ++zd)
                        for (int32_t yd = ry.d0; yd < ry.d1; ++yd)
                            store16<BPVD>(a.dst, dstRowIndex(a, yd, zd) + static_cast<uint64_t>(dx), code);
            }
        }
    }

    // Float32 "Linear", optimistic: MODE 3 plane pass (convert + flag) then the fix-up
    // (ResampleRow2.hip).  grid of the fix-up: one wave per (y run, z run), capped.
    // `list`: device work list of 1 + nRunsY*nRunsZ uint32 (count first, zeroed by the caller).
    void launchLinearOptimistic(ResampleArgs const& a, int32_t k, uint32_t bpvd, int32_t instrPerRow, uint32_t* list,
                                hipStream_t s);

    // Row-kernel launchers, one translation unit per MODE (0 identity, 1 convert, 2 chain).
    // k: integer x ratio; instrPerRow: 64-lane 16-byte store instructions per dst row.
    void launchRowMode0(ResampleArgs const& a, int32_t k, uint32_t bpv, unsigned grid, int32_t instrPerRow,
                        hipStream_t s);
    void launchRowMode1(ResampleArgs const& a, int32_t k, uint32_t bpv, int32_t fs, int32_t fd, unsigned grid,
                        int32_t instrPerRow, hipStream_t s);
    void launchRowMode2(ResampleArgs const& a, int32_t k, uint32_t bpvd, unsigned grid, int32_t instrPerRow,
                        hipStream_t s);

    template <int BPVS, int BPVD, int MODE, int FS, int FD>
    void launchRowK(ResampleArgs const& a, int32_t k, unsigned grid, int32_t instrPerRow, hipStream_t s)
    {
#define VKT_ROW_NS(K)                                                                                        \
    do {                                                                                                     \
        if (a.planeLayout)                                                                                   \
        {                                                                                                    \
            uint64_t const tasks = static_cast<uint64_t>(a.dnz) * a.nRunsY * instrPerRow;                    \
            planeChunks(a, tasks, [&](ResampleArgs const& c, unsigned g) {                                   \
                hipLaunchKernelGGL((resamplePlaneKernel<BPVS, BPVD, K, MODE, FS, FD>), dim3(g), dim3(64), 0, s, c); \
            });                                                                                              \
        }                                                                                                    \
        else if (instrPerRow == 1)                                                                                \
            hipLaunchKernelGGL((resampleRowKernel<BPVS, BPVD, K, MODE, FS, FD, 1>), dim3(grid), dim3(kBlock), 0, s, a); \
        else if (instrPerRow == 2)                                                                           \
            hipLaunchKernelGGL((resampleRowKernel<BPVS, BPVD, K, MODE, FS, FD, 2>), dim3(grid), dim3(kBlock), 0, s, a); \
        else                                                                                                 \
            hipLaunchKernelGGL((resampleRowKernel<BPVS, BPVD, K, MODE, FS, FD, 4>), dim3(grid), dim3(kBlock), 0, s, a); \
    } while (0)
        if (k == 1)
        {
            if constexpr ((16 / BPVD) * BPVS <= 32)
                VKT_ROW_NS(1);
        }
        else if (k == 2)
            VKT_ROW_NS(2);
        else
            VKT_ROW_NS(4);
#undef VKT_ROW_NS
    }

} // hipk
} // vkt
