// Pointwise.hpp -- the pointwise streaming engine behind Fill, Copy, Arithmetic and the
// same-dims branch of Resample.
//
// Iteration space: a box of extent (nx, ny, nz) voxels.  Every operand maps box voxel
// (i, j, k) to its own voxel origin + (i, j, k) (optionally clamped to its dims, as
// CopyRange_serial clamps its source, reference src/vkt/Copy_serial.hpp:38-40).
//
// Two device paths, chosen on the host:
//  * vector path: the box is collapsed (rows that are contiguous in every operand merge
//    into longer rows, whole-volume ops become one row of dimX*dimY*dimZ voxels), every
//    lane moves 8 consecutive voxels per operand with 8/16/32-byte loads and a nontemporal
//    store; rows whose length is not a multiple of 8 finish with a scalar tail.
//  * scalar path: one voxel per lane-iteration with full 3-D coordinates (clamping,
//    unaligned operands, mixed voxel sizes).
#pragma once

#include "KernelCommon.hpp"
#include "../runtime/Runtime.hpp"

#include <type_traits>
#include <utility>
#include "volkit_c.h"

namespace vkt
{
namespace hipk
{
    struct Operand
    {
        uint8_t* data;
        // vector path (after collapsing): voxel index = base + k*sz + j*sy + i
        int64_t base;
        int64_t sy;
        int64_t sz;
        // scalar path
        int32_t dims[3];
        int32_t origin[3];
        int32_t clamp;
        int32_t fmt;
        uint32_t bpv;
        float lo;
        float hi;
    };

    struct Geom
    {
        int64_t nx, ny, nz;      // raw extents (scalar path)
        int64_t vnx, vny, vnz;   // collapsed extents (vector path)
        int64_t vnx8;            // end of the 8-aligned middle of each row: vhead + 8 * chunks
        int64_t vhead;           // scalar head voxels per row (common misalignment phase);
                                 // padded rows: -(phase), the row's first item starts before it
        int32_t fast32;          // all index arithmetic fits 32 bits -> magic-number division
        int32_t padded;          // rows > 1: every row is covered by whole 8-voxel items from the
                                 // 8-aligned voxel at or below its start; items that straddle the
                                 // row ends load the whole vector and store only the row's voxels
        FastDiv divCpr, divVny;  // vector path: items -> (row, chunk), row -> (j, k)
        FastDiv divNx, divNy;    // scalar path: voxel -> (i, j, k)
        // padded rows with 64-B sector completion (Pointwise.hip planPointwise): items cover the
        // destination's whole end sectors [vhead, vnx8); sources are read only inside the rows'
        // 8-aligned items [vhead0, vend0) (item x clamped there), the chunks outside the box are
        // the destination's own bytes loaded and stored back whole
        int32_t merge;
        int64_t vhead0, vend0;
        // UInt8 rows (several) on a 16-voxel grid: every row holds an even number of items and
        // its first item starts 16-B aligned, so items 2l, 2l + 1 form one 16-B access (the
        // contiguous-lane shape below) with byte-range stores at the row ends
        int32_t pair16;
        // 4-byte voxels: padded rows take the contiguous-lane shape too, 16-B halves masked
        int32_t f32halves;
    };

    struct PassF;   // PointwiseOps.hpp: dst = source code (bytewise CopyRange)

    // Sentinel for "format known only at run time".
    constexpr int kDyn = -1;

    // ---- operand index helpers ----------------------------------------------------------
    __device__ __forceinline__ int32_t clampRefI(int32_t x, int32_t lo, int32_t hi)
    {
        int32_t m = hi < x ? hi : x;   // reference clamp = max(lo, min(x, hi)), linalg.hpp:38-41
        return lo < m ? m : lo;
    }

    __device__ __forceinline__ uint64_t scalarIndex(Operand const& o, int64_t i, int64_t j, int64_t k)
    {
        int32_t x = o.origin[0] + static_cast<int32_t>(i);
        int32_t y = o.origin[1] + static_cast<int32_t>(j);
        int32_t z = o.origin[2] + static_cast<int32_t>(k);
        if (o.clamp)
        {
            x = clampRefI(x, 0, o.dims[0] - 1);
            y = clampRefI(y, 0, o.dims[1] - 1);
            z = clampRefI(z, 0, o.dims[2] - 1);
        }
        return (static_cast<uint64_t>(z) * static_cast<uint64_t>(o.dims[1]) + static_cast<uint64_t>(y)) *
                   static_cast<uint64_t>(o.dims[0]) + static_cast<uint64_t>(x);
    }

    // ---- kernels ---------------------------------------------------------------------
    // Vector path.  Work items are 8-voxel chunks of the collapsed rows.  Each workgroup owns
    // one contiguous span of items (measured on MI355X: 5.3-5.4 TB/s for a 3-stream UInt16
    // op against 4.5-4.7 TB/s for a grid-stride sweep), keeps kUnroll items per lane in
    // flight (all loads issued before the first store), and uses nontemporal loads and
    // stores: every byte is touched once.
    //
    // Quantum per workgroup: ONE wave.  First measured for the 3-stream UInt16 Sum at 1024^3
    // (dev/kbench/kbench7.hip, kbench9.hip): 2 KiB per operand ran 0.98-0.99 ms (6.5 TB/s) against
    // 1.01-1.08 ms for 4 waves x 4 items (16 KiB per operand): small one-shot workgroups keep
    // more distinct DRAM pages in flight per CU while the moving window stays compact.
    //
    // Quantum size per stream count, measured with dev/kbench/kbench_fill.hip on 2 GiB buffers
    // (MI355X, one-wave workgroups, 16-B nontemporal accesses): pure stores run best at 4 KiB
    // per workgroup (6.4-6.5 TB/s vs 5.1-5.3 at 2 KiB and 5.7-5.9 at 8 KiB); copies and the
    // 3-stream sum at 1 KiB of each stream (copy 6.82 vs 6.55 TB/s at 2 KiB, sum 6.34 vs 6.14).
    // Items are 8 voxels, so Float32 (32-B items) cannot go below 2 KiB per stream.
    constexpr int kVecBlock = 64;
    template <int NS, int BPV>
    constexpr int vecUnroll()
    {
        if constexpr (NS == 0)
            return BPV == 1 ? 8 : BPV == 2 ? 4 : 2;   // 4 KiB of stores
        else
            return BPV == 1 ? 4 : BPV == 2 ? 2 : 1;  // 2 KiB per stream
    }

    // MODE 0: one collapsed row; 1: rows, 32-bit magic division; 2: rows, 64-bit division.
    template <int NS, int BPV, int MODE, class F>
    __device__ __forceinline__ void pointwiseVecItem(Operand const& d, Operand const& s1, Operand const& s2,
                                                     Geom const& g, uint64_t it, uint64_t& o1, uint64_t& o2,
                                                     uint64_t& od, int64_t* rowX = nullptr, int64_t span = 8)
    {
        if constexpr (MODE == 0)
        {
            uint64_t x = static_cast<uint64_t>(g.vhead) + (it << 3);
            o1 = s1.base + x;
            o2 = s2.base + x;
            od = d.base + x;
        }
        else
        {
            uint64_t j, k, x;   // x wraps below 0 for a padded row's first item: the sums below
                                // are taken modulo 2^64 and land on the 8-aligned voxel
            if constexpr (MODE == 1)
            {
                uint32_t r = fdiv(static_cast<uint32_t>(it), g.divCpr);
                x = static_cast<uint64_t>(g.vhead) +
                    (static_cast<uint64_t>(static_cast<uint32_t>(it) - r * g.divCpr.d) << 3);
                uint32_t kk = fdiv(r, g.divVny);
                k = kk;
                j = r - kk * g.divVny.d;
            }
            else
            {
                uint64_t const cpr = static_cast<uint64_t>(g.vnx8 - g.vhead) >> 3, ny = static_cast<uint64_t>(g.vny);
                uint64_t r = it / cpr;
                x = static_cast<uint64_t>(g.vhead) + ((it - r * cpr) << 3);
                j = r % ny;
                k = r / ny;
            }
            od = d.base + k * d.sz + j * d.sy + x;
            if (rowX)
                *rowX = static_cast<int64_t>(x);
            if (g.merge)
            {
                // sector completion: sources only inside the rows' own 8-aligned items
                int64_t xl = static_cast<int64_t>(x);
                xl = xl < g.vhead0 ? g.vhead0 : (xl > g.vend0 - span ? g.vend0 - span : xl);
                x = static_cast<uint64_t>(xl);
            }
            o1 = s1.base + k * s1.sz + j * s1.sy + x;
            o2 = s2.base + k * s2.sz + j * s2.sy + x;
        }
    }

    // Sector completion: an edge item (straddling a row end, or wholly outside the box inside
    // an end sector) is stored whole, its voxels outside [0, vnx) being the destination's own.
    template <int BPV>
    __device__ __forceinline__ void loadDstChunk(uint8_t const* base, uint64_t od, uint32_t (&c)[8])
    {
        load8<BPV, false>(base, od, c);
    }

    // One workgroup's span [beg, end) of 8-voxel items.  The main loop is branch-free so that
    // the compiler keeps all kUnroll x NS loads in flight (a guard per item made hipcc wait
    // vmcnt(0) after every item); the remainder loop handles the last partial quantum.
    // Functors with kPacked16 work on raw dwords of two UInt16 codes (F::pk).
    template <class F, class = void>
    struct IsPacked16 { static constexpr bool value = false; };
    template <class F>
    struct IsPacked16<F, decltype(void(F::kPacked16))> { static constexpr bool value = F::kPacked16; };

    // Store the 8 codes of an item whose row-relative start is x; only voxels inside [0, vnx)
    // of the row are written when the item straddles a row end.
    template <int BPV>
    __device__ __forceinline__ void storeItemMasked(uint8_t* base, uint64_t od, int64_t x, int64_t vnx,
                                                    uint32_t const (&c)[8], bool merge = false,
                                                    uint32_t const* own = nullptr)
    {
        if (x >= 0 && x + 8 <= vnx)
            store8<BPV, true>(base, od, c);
        else if (merge)
        {
            uint32_t m[8];
#pragma unroll
            for (int v = 0; v < 8; ++v)
                m[v] = x + v >= 0 && x + v < vnx ? c[v] : own[v];
            store8<BPV, true>(base, od, m);
        }
        else
        {
#pragma unroll
            for (int v = 0; v < 8; ++v)
                if (x + v >= 0 && x + v < vnx)
                    storeCode<BPV>(base, od + v, c[v]);
        }
    }

    template <int NS, int BPV, int MODE, int U, class F>
    __device__ __forceinline__ void pointwiseVecSpan(Operand const& d, Operand const& s1, Operand const& s2,
                                                     Geom const& g, uint64_t beg, uint64_t end, F const& f)
    {
        constexpr int kUnroll = U;
        constexpr uint64_t kQ = static_cast<uint64_t>(kVecBlock) * kUnroll;
        uint64_t it = beg + threadIdx.x;
        if constexpr (BPV == 2 && NS == 2 && IsPacked16<F>::value)
        {
            // same schedule as below (all loads of a quantum before its stores), no unpacking:
            // 16 B of each source -> 16 B of dst
            auto apply = [&](u32x4 const& a, u32x4 const& b, uint64_t od, int64_t x, uint32_t const* own) {
                u32x4 r;
                r.x = f.pk(a.x, b.x);
                r.y = f.pk(a.y, b.y);
                r.z = f.pk(a.z, b.z);
                r.w = f.pk(a.w, b.w);
                if constexpr (MODE != 0)
                {
                    if (g.padded)
                    {
                        if (x < 0 || x + 8 > g.vnx)
                        {
                            uint32_t c[8] = {r.x & 0xFFFFu, r.x >> 16, r.y & 0xFFFFu, r.y >> 16,
                                             r.z & 0xFFFFu, r.z >> 16, r.w & 0xFFFFu, r.w >> 16};
                            storeItemMasked<2>(d.data, od, x, g.vnx, c, g.merge != 0, own);
                            return;
                        }
                    }
                }
                __builtin_nontemporal_store(r, reinterpret_cast<u32x4*>(d.data + 2 * od));
            };
            for (; it + (kUnroll - 1) * static_cast<uint64_t>(kVecBlock) < end; it += kQ)
            {
                u32x4 a[kUnroll], b[kUnroll];
                uint64_t od[kUnroll];
                int64_t xr[kUnroll];
                uint32_t own[kUnroll][8];
#pragma unroll
                for (int u = 0; u < kUnroll; ++u)
                {
                    uint64_t o1, o2;
                    xr[u] = 0;
                    pointwiseVecItem<NS, BPV, MODE, F>(d, s1, s2, g, it + static_cast<uint64_t>(u) * kVecBlock, o1, o2,
                                                       od[u], &xr[u]);
                    a[u] = loadVec<u32x4, true>(s1.data + 2 * o1);
                    b[u] = loadVec<u32x4, true>(s2.data + 2 * o2);
                    if constexpr (MODE != 0)
                        if (g.merge && (xr[u] < 0 || xr[u] + 8 > g.vnx))
                            loadDstChunk<2>(d.data, od[u], own[u]);
                }
#pragma unroll
                for (int u = 0; u < kUnroll; ++u)
                    apply(a[u], b[u], od[u], xr[u], own[u]);
            }
            for (; it < end; it += kVecBlock)
            {
                uint64_t o1, o2, od;
                int64_t xr = 0;
                uint32_t own[8];
                pointwiseVecItem<NS, BPV, MODE, F>(d, s1, s2, g, it, o1, o2, od, &xr);
                if constexpr (MODE != 0)
                    if (g.merge && (xr < 0 || xr + 8 > g.vnx))
                        loadDstChunk<2>(d.data, od, own);
                apply(loadVec<u32x4, true>(s1.data + 2 * o1), loadVec<u32x4, true>(s2.data + 2 * o2), od, xr, own);
            }
            return;
        }
        // Contiguous lanes for UInt8 and Float32 (a whole quantum, rows without padded edges,
        // 16-B aligned rows in every operand): every load / store instruction of a wave covers
        // one contiguous KiB, lane l bytes [16l, 16l + 16).  The per-item loop below moves 8 B per
        // lane for UInt8 (8-B loads run below the 16-B rate) and, for Float32, two 16-B halves of
        // a 32-B item per lane (each instruction every other 16 B of 2 KiB): 1024^3 Copy UInt8
        // 0.73 and Float32 0.51 of 8 TB/s against 0.82 for UInt16.  Here UInt8 items 2l, 2l + 1
        // of a 128-item pair of blocks share one 16-B access (one collapsed row), and Float32
        // lane l takes half 4(l mod 2) of items l/2 and 32 + l/2 of its 64-item block (a half
        // never leaves its item, so never its row; every operand uses the same voxels, and
        // without padded edges no item needs a mask).
        if constexpr (BPV == 4 || (BPV == 1 && kUnroll % 2 == 0))
        {
            uint64_t const lane = threadIdx.x;
            auto aligned = [&](Operand const& op) {
                uint64_t const rowStart = reinterpret_cast<uintptr_t>(op.data) +
                                          static_cast<uint64_t>(op.base + g.vhead) * BPV;
                if constexpr (MODE == 0)
                    return ((rowStart + (beg << 3) * BPV) & 15u) == 0;
                else
                    return ((rowStart | static_cast<uint64_t>(op.sy) * BPV | static_cast<uint64_t>(op.sz) * BPV) & 15u) == 0;
            };
            // multi-row boxes: Float32 without padded rows; UInt8 on the 16-voxel grid (pair16),
            // byte-range stores at the row ends (the per-item loop stored a straddling item
            // voxel by voxel: 8 byte stores, 24 store instructions per wave on an 800^3 sub-box
            // at x0 = 100, 0.30 of 8 TB/s)
            // Float32 rows with padded edges: each 16-B half (4 voxels) is stored whole, as its
            // row's dwords (storeByteRange16), or -- sector completion -- merged with the
            // destination's own dwords (g.f32halves, knob pointwise.f32_halves)
            bool const shape = MODE == 0 || (BPV == 4 && (!g.padded || g.f32halves)) || (BPV == 1 && g.pair16);
            if (end - beg == kQ && shape && aligned(d) && (NS < 1 || aligned(s1)) && (NS < 2 || aligned(s2)))
            {
                uint32_t a[kUnroll][8], b[kUnroll][8];
                int64_t xr[kUnroll][2];   // row-relative x of the lane's access (Float32: of the half)
                // voxel offsets (d, s1, s2) of the lane's 16-B access number q of block u
                auto at = [&](int u, int q, uint64_t& od, uint64_t& o1, uint64_t& o2) {
                    uint64_t item;
                    uint64_t sub = 0;
                    xr[u][q] = 0;
                    if constexpr (BPV == 4)
                    {
                        item = beg + static_cast<uint64_t>(u) * 64u + 32u * static_cast<uint64_t>(q) + lane / 2;
                        sub = 4u * (lane & 1u);
                    }
                    else
                        item = beg + static_cast<uint64_t>(u / 2) * 128u + 2u * lane;
                    pointwiseVecItem<NS, BPV, MODE, F>(d, s1, s2, g, item, o1, o2, od, &xr[u][q], BPV == 1 ? 16 : 8);
                    xr[u][q] += static_cast<int64_t>(sub);
                    od += sub;
                    o1 += sub;
                    o2 += sub;
                };
                uint64_t od[kUnroll][2], o1[kUnroll][2], o2[kUnroll][2];
#pragma unroll
                for (int u = 0; u < kUnroll; ++u)
                {
                    if constexpr (BPV == 4)
                    {
                        at(u, 0, od[u][0], o1[u][0], o2[u][0]);
                        at(u, 1, od[u][1], o1[u][1], o2[u][1]);
                    }
                    else if (u % 2 == 0)
                        at(u, 0, od[u][0], o1[u][0], o2[u][0]);
                }
                auto load = [&](Operand const& op, uint64_t const (&off)[kUnroll][2], uint32_t (&c)[kUnroll][8]) {
#pragma unroll
                    for (int u = 0; u < kUnroll; ++u)
                    {
                        if constexpr (BPV == 4)
                        {
                            u32x4 const x = loadVec<u32x4, true>(op.data + off[u][0] * 4u);
                            u32x4 const y = loadVec<u32x4, true>(op.data + off[u][1] * 4u);
                            c[u][0] = x.x; c[u][1] = x.y; c[u][2] = x.z; c[u][3] = x.w;
                            c[u][4] = y.x; c[u][5] = y.y; c[u][6] = y.z; c[u][7] = y.w;
                        }
                        else if (u % 2 == 0)
                        {
                            u32x4 const x = loadVec<u32x4, true>(op.data + off[u][0]);
                            uint32_t const w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                            for (int i = 0; i < 8; ++i)
                            {
                                c[u][i] = (w[i / 4] >> (8 * (i % 4))) & 0xFFu;
                                c[u + 1][i] = (w[2 + i / 4] >> (8 * (i % 4))) & 0xFFu;
                            }
                        }
                    }
                };
                if constexpr (NS >= 1)
                    load(s1, o1, a);
                if constexpr (NS >= 2)
                    load(s2, o2, b);
                // UInt8 pairs with 64-B sector completion: a pair outside the box row (inside an
                // end sector) or straddling its end is stored whole, its bytes outside the row
                // being the destination's own
                u32x4 own[kUnroll][2];
                if constexpr (BPV == 1 && MODE != 0)
                {
#pragma unroll
                    for (int u = 0; u < kUnroll; u += 2)
                        if (g.merge && (xr[u][0] < 0 || xr[u][0] + 16 > g.vnx))
                            own[u][0] = *reinterpret_cast<u32x4 const*>(d.data + od[u][0]);
                }
                if constexpr (BPV == 4 && MODE != 0)
                {
#pragma unroll
                    for (int u = 0; u < kUnroll; ++u)
#pragma unroll
                        for (int q = 0; q < 2; ++q)
                            if (g.merge && (xr[u][q] < 0 || xr[u][q] + 4 > g.vnx))
                                own[u][q] = *reinterpret_cast<u32x4 const*>(d.data + od[u][q] * 4u);
                }
                uint32_t o[kUnroll][8];
#pragma unroll
                for (int u = 0; u < kUnroll; ++u)
#pragma unroll
                    for (int v = 0; v < 8; ++v)
                        o[u][v] = f(NS >= 1 ? a[u][v] : 0u, NS >= 2 ? b[u][v] : 0u);
#pragma unroll
                for (int u = 0; u < kUnroll; ++u)
                {
                    if constexpr (BPV == 4)
                    {
#pragma unroll
                        for (int q = 0; q < 2; ++q)
                        {
                            u32x4 v{o[u][4 * q], o[u][4 * q + 1], o[u][4 * q + 2], o[u][4 * q + 3]};
                            uint8_t* const p = d.data + od[u][q] * 4u;
                            if constexpr (MODE != 0)
                            {
                                int64_t const x = xr[u][q];
                                if (g.padded && (x < 0 || x + 4 > g.vnx))
                                {
                                    // a half straddling or outside a row end: the row's dwords
                                    int const lo = 4 * static_cast<int>(x < 0 ? (x < -4 ? 4 : -x) : 0);
                                    int const hi = 4 * static_cast<int>(g.vnx - x < 4 ? (g.vnx - x < 0 ? 0 : g.vnx - x) : 4);
                                    if (g.merge)
                                        v = mergeBytes16(v, own[u][q], lo, hi);   // (stored below, with the rest)
                                    else
                                    {
                                        if (hi > lo)
                                            storeByteRange16(p, v, lo, hi);
                                        continue;
                                    }
                                }
                            }
                            // one store statement for whole and merged halves: a wave holding both
                            // issues it once (two statements: both, in nearly every wave of a sub-box)
                            __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
                        }
                    }
                    else if (u % 2 == 0)
                    {
                        uint32_t w[4];
#pragma unroll
                        for (int i = 0; i < 2; ++i)
                        {
                            w[i] = o[u][4 * i] | o[u][4 * i + 1] << 8 | o[u][4 * i + 2] << 16 | o[u][4 * i + 3] << 24;
                            w[2 + i] = o[u + 1][4 * i] | o[u + 1][4 * i + 1] << 8 | o[u + 1][4 * i + 2] << 16 |
                                       o[u + 1][4 * i + 3] << 24;
                        }
                        u32x4 v{w[0], w[1], w[2], w[3]};
                        if constexpr (MODE != 0)
                        {
                            int64_t const x = xr[u][0];
                            if (g.padded && (x < 0 || x + 16 > g.vnx))
                            {
                                // the pair straddles a row end (or, merging, lies in an end
                                // sector): the row's bytes only, or the whole 16 B merged with
                                // the destination's own bytes (stored below, with the rest)
                                int const lo = x < 0 ? static_cast<int>(x < -16 ? 16 : -x) : 0;
                                int const hi = g.vnx - x < 16 ? static_cast<int>(g.vnx - x < 0 ? 0 : g.vnx - x) : 16;
                                if (g.merge)
                                    v = mergeBytes16(v, own[u][0], lo, hi);
                                else
                                {
                                    storeByteRange16(d.data + od[u][0], v, lo, hi);
                                    continue;
                                }
                            }
                        }
                        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(d.data + od[u][0]));
                    }
                }
                return;
            }
        }
        for (; it + (kUnroll - 1) * static_cast<uint64_t>(kVecBlock) < end; it += kQ)
        {
            uint32_t a[kUnroll][8], b[kUnroll][8], own[kUnroll][8];
            uint64_t od[kUnroll];
            int64_t xr[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u)
            {
                uint64_t o1, o2;
                xr[u] = 0;
                pointwiseVecItem<NS, BPV, MODE, F>(d, s1, s2, g, it + static_cast<uint64_t>(u) * kVecBlock, o1, o2,
                                                   od[u], &xr[u]);
                if constexpr (NS >= 1)
                    load8<BPV, true>(s1.data, o1, a[u]);
                if constexpr (NS >= 2)
                    load8<BPV, true>(s2.data, o2, b[u]);
                if constexpr (MODE != 0)
                    if (g.merge && (xr[u] < 0 || xr[u] + 8 > g.vnx))
                        loadDstChunk<BPV>(d.data, od[u], own[u]);
            }
#pragma unroll
            for (int u = 0; u < kUnroll; ++u)
            {
                uint32_t o[8];
#pragma unroll
                for (int v = 0; v < 8; ++v)
                    o[v] = f(NS >= 1 ? a[u][v] : 0u, NS >= 2 ? b[u][v] : 0u);
                if constexpr (MODE != 0)
                {
                    if (g.padded)
                    {
                        storeItemMasked<BPV>(d.data, od[u], xr[u], g.vnx, o, g.merge != 0, own[u]);
                        continue;
                    }
                }
                store8<BPV, true>(d.data, od[u], o);
            }
        }
        for (; it < end; it += kVecBlock)
        {
            uint32_t a[8], b[8], o[8], own[8];
            uint64_t o1, o2, od;
            int64_t xr = 0;
            pointwiseVecItem<NS, BPV, MODE, F>(d, s1, s2, g, it, o1, o2, od, &xr);
            if constexpr (NS >= 1)
                load8<BPV, true>(s1.data, o1, a);
            if constexpr (NS >= 2)
                load8<BPV, true>(s2.data, o2, b);
            if constexpr (MODE != 0)
                if (g.merge && (xr < 0 || xr + 8 > g.vnx))
                    loadDstChunk<BPV>(d.data, od, own);
#pragma unroll
            for (int v = 0; v < 8; ++v)
                o[v] = f(NS >= 1 ? a[v] : 0u, NS >= 2 ? b[v] : 0u);
            if constexpr (MODE != 0)
            {
                if (g.padded)
                {
                    storeItemMasked<BPV>(d.data, od, xr, g.vnx, o, g.merge != 0, own);
                    continue;
                }
            }
            store8<BPV, true>(d.data, od, o);
        }
    }

    // One collapsed row (whole-volume ops: every operand contiguous, no row edges, no scalar
    // head / tail): the same span code instantiated for MODE 0 alone.  The general kernel below
    // carries the multi-row, padded-row and sector-completion paths in one body, so its VGPR
    // count (85 for UInt16 SumRange, 118 for UInt8) is set by code a collapsed row never runs
    // and caps the waves per SIMD (5 / 4) -- the bytes each SIMD keeps in flight.
    // MODE 1 (knob pointwise.rows_kernel): the same for multi-row boxes on 32-bit row math
    // without scalar edges (padded rows or rows of whole items).
    template <int NS, int BPV, int MODE, int U, class F>
    __global__ __launch_bounds__(kVecBlock) void pointwiseRowKernel(Operand d, Operand s1, Operand s2, Geom g, F f,
                                                                   uint64_t qBase, uint64_t qEnd, uint32_t runs)
    {
        uint64_t const items = (static_cast<uint64_t>(g.vnx8 - g.vhead) >> 3) * static_cast<uint64_t>(g.vny) *
                               static_cast<uint64_t>(g.vnz);
        constexpr uint64_t kQ = static_cast<uint64_t>(kVecBlock) * U;
        // workgroup b runs on XCD b mod 8; runs > 0 (knob pointwise.row_swizzle) gives each XCD
        // runs of `runs` consecutive quanta instead of every 8th one
        uint32_t b = blockIdx.x;
        if (runs > 0u)
        {
            uint32_t const span = 8u * runs, whole = gridDim.x / span * span;
            if (b < whole)
            {
                uint32_t const l = b >> 3;
                b = (l / runs) * span + (b & 7u) * runs + l % runs;
            }
        }
        for (uint64_t q = qBase + b; q < qEnd; q += gridDim.x)
        {
            uint64_t const beg = q * kQ;
            if (beg >= items)
                break;
            pointwiseVecSpan<NS, BPV, MODE, U>(d, s1, s2, g, beg, beg + kQ < items ? beg + kQ : items, f);
        }
    }

    // Work distribution: workgroup q handles the q-th quantum of kVecBlock*kUnroll items and
    // the grid holds one workgroup per quantum (grid-stride only beyond 2^30 quanta).  Short
    // one-shot workgroups dispatched in order make the whole chip sweep memory as one
    // compact moving window: measured 1.05 ms (6.1 TB/s) for UInt16 Sum at 1024^3 against
    // 1.20 ms for 4096 persistent workgroups that each stream their own span (16-KiB quanta;
    // the 2-KiB quanta above gain another ~5%).
    //
    // Large ranges are split into launches of at most kMaxQuantaPerLaunch workgroups (quanta
    // [qBase, qEnd) per launch): measured on MI355X, SumRange over 2048^3 UInt16 took 8.9 ms
    // as one launch of 8 M workgroups and 8.3 ms as 1 M-workgroup launches (the per-voxel rate
    // of the 1024^3 case); launches of 4 M workgroups were as slow as one.  Row edges are
    // handled by the first launch only.
    constexpr uint64_t kMaxQuantaPerLaunch = 1ull << 20;   // default of the knob below
    static_assert(kMaxQuantaPerLaunch > 0, "");

    template <int NS, int BPV, int U, class F>
    __global__ __launch_bounds__(kVecBlock) void pointwiseVecKernel(Operand d, Operand s1, Operand s2, Geom g, F f,
                                                                   uint64_t qBase, uint64_t qEnd, int32_t edges)
    {
        uint64_t const cpr = static_cast<uint64_t>(g.vnx8 - g.vhead) >> 3;   // chunks per row
        uint64_t const rows = static_cast<uint64_t>(g.vny) * static_cast<uint64_t>(g.vnz);
        uint64_t const items = cpr * rows;
        uint64_t const ny = static_cast<uint64_t>(g.vny);
        constexpr uint64_t kQ = static_cast<uint64_t>(kVecBlock) * U;
        for (uint64_t q = qBase + blockIdx.x; q < qEnd; q += gridDim.x)
        {
            uint64_t const beg = q * kQ;
            if (beg >= items)
                break;
            uint64_t const end = beg + kQ < items ? beg + kQ : items;
            if (rows == 1)
                pointwiseVecSpan<NS, BPV, 0, U>(d, s1, s2, g, beg, end, f);
            else if (g.fast32)
                pointwiseVecSpan<NS, BPV, 1, U>(d, s1, s2, g, beg, end, f);
            else
                pointwiseVecSpan<NS, BPV, 2, U>(d, s1, s2, g, beg, end, f);
        }

        // scalar edges of every row: head [0, vhead) and tail [vnx8, vnx)
        if (g.padded || !edges)
            return;
        uint64_t const head = static_cast<uint64_t>(g.vhead);
        uint64_t const tailLen = head + static_cast<uint64_t>(g.vnx - g.vnx8);
        if (tailLen == 0)
            return;
        uint64_t const tid = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x;
        uint64_t const stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
        uint64_t const tailItems = tailLen * rows;
        for (uint64_t it = tid; it < tailItems; it += stride)
        {
            uint64_t r = it / tailLen;
            uint64_t e = it - r * tailLen;
            uint64_t x = e < head ? e : static_cast<uint64_t>(g.vnx8) + (e - head);
            uint64_t j = r % ny, k = r / ny;
            uint32_t a = 0, b = 0;
            if constexpr (NS >= 1)
                a = loadCode<BPV>(s1.data, s1.base + k * s1.sz + j * s1.sy + x);
            if constexpr (NS >= 2)
                b = loadCode<BPV>(s2.data, s2.base + k * s2.sz + j * s2.sy + x);
            storeCode<BPV>(d.data, d.base + k * d.sz + j * d.sy + x, f(a, b));
        }
    }

    // ---- general vector path ---------------------------------------------------------
    // For boxes the aligned path above cannot take: operands at different 8-voxel phases (a
    // CopyRange from x0 = 3 to x0 = 0, an arithmetic dstOffset), row pitches that are not
    // multiples of 8, clamped CopyRange sources (halo copies past the border), and sources of a
    // different voxel size than the destination (CopyRange with format conversion).
    //
    // Items are 8 destination voxels aligned to the destination's memory: row (j, k) of the
    // box is covered by cpr = ceil((vnx + 7) / 8) chunks starting at x = -(phase of the row
    // start), so every item stores 8*BD aligned bytes (one 16-B vector for UInt16) and items
    // that straddle a row end store only the row's voxels.  A source's 8 voxels start at any
    // byte offset s: the lane loads the aligned 16-B words covering them (2 words, 3 for
    // 4-byte voxels; a neighbour lane's words are the same lines, served by L1) and shifts
    // them in registers -- a per-lane barrel shifter: select by 8 bytes, by 4 bytes, then
    // v_alignbyte_b32 by s & 3 (~15 VALU ops per 16 B).  Items whose source voxels leave the
    // source row (clamped x at the volume border) or the box row (straddling items) go voxel
    // by voxel with the reference clamp (Copy_serial.hpp:38-40); y and z clamp per row.
    // Traffic = the algorithmic bytes: each source line is fetched from HBM once (the words
    // a lane shares with its neighbour hit L1 / L2).
    struct GenGeom
    {
        int64_t vnx, vny, vnz;   // box (collapsed when no operand clamps)
        uint64_t cpr;            // chunks per row: ceil((vnx + 7) / 8)
        uint64_t items;          // rows * cpr
        int32_t dph;             // (d.data / BD) & 7: phase of destination voxel 0
        int32_t fast32;          // items and rows fit 32 bits
        int32_t anyClamp;        // some source clamps (then rows are not collapsed)
        int32_t fast;            // 32-bit addressing (pointwiseGenSpanFast): every operand < 4 GiB,
                                 // row / plane pitches and box rows / planes < 2^24 (24-bit muls)
        int32_t merge;           // complete the 64-B sectors at the row ends (fast path only)
        int32_t sv;              // voxels per 64-B sector (64 / BD)
        int32_t dph64;           // (d.data / BD) mod sv
        int32_t wide;            // every operand 1 or every operand 4 B/voxel, fast path: 16-B items
                                 // (pointwiseGenSpanFast16; cpr / dph in 16/B-voxel units)
        int32_t dword;           // every operand 4 B/voxel at a 4-B aligned address: every window
                                 // offset is a whole dword, the byte-align stage is the identity
        FastDiv divCpr, divVny;
    };

    // 8 consecutive codes starting at voxel `voxel` of a B-byte-per-voxel volume at any byte
    // offset: out = 2*B dwords of the little-endian byte stream.  Only words holding needed bytes
    // are loaded (an unneeded trailing word is replaced by the last needed one), so no load
    // leaves the 16-B blocks of the valid voxels.  The shifter's selects use constant indices
    // only (index_sequence folds): a select between two elements of a loop-indexed array is
    // folded into a dynamically indexed load before unrolling, which sends the array to scratch.
    template <std::size_t... T>
    __device__ __forceinline__ void shiftSel(uint32_t const* in, uint32_t* out, bool c, int by,
                                             std::index_sequence<T...>)
    {
        ((out[T] = c ? in[T + by] : in[T]), ...);
    }

    template <std::size_t... T>
    __device__ __forceinline__ void shiftAlign(uint32_t const* in, uint32_t* out, uint32_t r,
                                               std::index_sequence<T...>)
    {
        ((out[T] = __builtin_amdgcn_alignbyte(in[T + 1], in[T], r)), ...);
    }

    // The window is split in two halves so that a lane issues the loads of all its items
    // before it shifts the first one (the shift waits for its words).
    template <int B>
    struct Window
    {
        static constexpr int NW = B == 4 ? 3 : 2;   // 16-B words covering 8*B bytes at any offset
        uint32_t w[4 * NW];
        uint32_t s;                                 // byte offset of the first voxel in word 0
    };

    // Voxels [lo, hi) of the 8 (0 <= lo < hi <= 8) are the valid ones (an item straddling a row
    // end): words are clamped to the ones holding valid voxels, the other codes are garbage.
    template <int B>
    __device__ __forceinline__ void loadWindow(uint8_t const* data, int64_t voxel, int32_t lo, int32_t hi,
                                               Window<B>& win)
    {
        uint8_t const* const p = data + voxel * B;   // may lie before the row (x < 0): address only
        uint32_t const s = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p) & 15u);
        uint8_t const* const p0 = p - s;
        uint8_t const* const vf = p + lo * B;
        uint8_t const* const vl = p + hi * B - 1;
        uint8_t const* const pf = vf - (reinterpret_cast<uintptr_t>(vf) & 15u);
        uint8_t const* const pl = vl - (reinterpret_cast<uintptr_t>(vl) & 15u);
        auto word = [&](int i) {
            uint8_t const* a = p0 + 16 * i;
            a = a < pf ? pf : a;
            return *reinterpret_cast<u32x4 const*>(a < pl ? a : pl);
        };
        win.s = s;
        u32x4 const v0 = word(0);
        u32x4 const v1 = word(1);
        win.w[0] = v0.x; win.w[1] = v0.y; win.w[2] = v0.z; win.w[3] = v0.w;
        win.w[4] = v1.x; win.w[5] = v1.y; win.w[6] = v1.z; win.w[7] = v1.w;
        if constexpr (Window<B>::NW == 3)
        {
            u32x4 const v2 = word(2);
            win.w[8] = v2.x; win.w[9] = v2.y; win.w[10] = v2.z; win.w[11] = v2.w;
        }
    }

    // dword (GenGeom::dword, 4-byte voxels only): the offset is a multiple of 4, the two dword
    // selects finish the shift (wave-uniform branch around the v_alignbyte stage)
    template <int B>
    __device__ __forceinline__ void shiftWindow(Window<B> const& win, uint32_t (&out)[2 * B], bool dword = false)
    {
        constexpr int NO = 2 * B;   // output dwords
        uint32_t a[NO + 2], b[NO + 1];
        shiftSel(win.w, a, (win.s & 8u) != 0, 2, std::make_index_sequence<NO + 2>{});
        shiftSel(a, b, (win.s & 4u) != 0, 1, std::make_index_sequence<NO + 1>{});
        if (B == 4 && dword)
        {
#pragma unroll
            for (int i = 0; i < NO; ++i)
                out[i] = b[i];
        }
        else
            shiftAlign(b, out, win.s & 3u, std::make_index_sequence<NO>{});
    }

    template <int B>
    __device__ __forceinline__ void unpack8(uint32_t const (&w)[2 * B], uint32_t (&c)[8])
    {
#pragma unroll
        for (int v = 0; v < 8; ++v)
        {
            if constexpr (B == 1)
                c[v] = (w[v / 4] >> (8 * (v % 4))) & 0xFFu;
            else if constexpr (B == 2)
                c[v] = (w[v / 2] >> (16 * (v % 2))) & 0xFFFFu;
            else
                c[v] = w[v];
        }
    }

    // Voxel index of box x = 0 in row (j, k) of operand o, and of x = 0 of the volume row it
    // reads (clamped rows: the reference clamps y and z, x per voxel).
    __device__ __forceinline__ int64_t genRowStart(Operand const& o, uint64_t j, uint64_t k, int64_t& row0)
    {
        if (!o.clamp)
        {
            int64_t const r = o.base + static_cast<int64_t>(k) * o.sz + static_cast<int64_t>(j) * o.sy;
            row0 = r - o.origin[0];
            return r;
        }
        int32_t const y = clampRefI(o.origin[1] + static_cast<int32_t>(j), 0, o.dims[1] - 1);
        int32_t const z = clampRefI(o.origin[2] + static_cast<int32_t>(k), 0, o.dims[2] - 1);
        row0 = (static_cast<int64_t>(z) * o.dims[1] + y) * static_cast<int64_t>(o.dims[0]);
        return row0 + o.origin[0];
    }

    template <int BS>
    __device__ __forceinline__ uint32_t genLoadOne(Operand const& o, int64_t rowStart, int64_t row0, int64_t x)
    {
        if (!o.clamp)
            return loadCode<BS>(o.data, static_cast<uint64_t>(rowStart + x));
        int32_t const sx = clampRefI(o.origin[0] + static_cast<int32_t>(x), 0, o.dims[0] - 1);
        return loadCode<BS>(o.data, static_cast<uint64_t>(row0 + sx));
    }

    __device__ __forceinline__ bool genInterior(Operand const& o, int64_t x)
    {
        return !o.clamp || (o.origin[0] + x >= 0 && o.origin[0] + x + 8 <= o.dims[0]);
    }

    // 8 codes -> 2*B dwords of packed codes
    template <int B, std::size_t... V>
    __device__ __forceinline__ void packCodes(uint32_t const (&c)[8], Window<B>& win, std::index_sequence<V...>)
    {
        ((win.w[V] = B == 1 ? c[4 * V] | c[4 * V + 1] << 8 | c[4 * V + 2] << 16 | c[4 * V + 3] << 24
                   : B == 2 ? c[2 * V] | c[2 * V + 1] << 16 : c[V]), ...);
    }

    // Clamped x-border item (a clamped source reads voxels left of x = 0 or right of dimX - 1):
    // voxel by voxel with the reference clamp, in a pass after the streamed items (its loads
    // would otherwise be merged with the window registers and make the wave wait early).
    template <int B>
    __device__ __forceinline__ void loadBorder(Operand const& o, int64_t rowStart, int64_t row0, int64_t x,
                                               uint32_t (&c)[8])
    {
#pragma unroll
        for (int v = 0; v < 8; ++v)
            c[v] = genLoadOne<B>(o, rowStart, row0, x + v);
    }

    // MODE 1/2: items [beg, end) packed across rows (32-bit / 64-bit division).
    template <int NS, int BD, int B1, int B2, int MODE, int U, class F>
    __device__ __forceinline__ void pointwiseGenSpan(Operand const& d, Operand const& s1, Operand const& s2,
                                                     GenGeom const& g, uint64_t beg, uint64_t end, F const& f)
    {
        constexpr bool kPack = BD == 2 && B1 == 2 && B2 == 2 && NS == 2 && IsPacked16<F>::value;
        constexpr bool kPass = NS == 1 && BD == B1 && std::is_same<F, PassF>::value;
        Window<B1> wa[U];
        Window<NS >= 2 ? B2 : 1> wb[U];
        int64_t xs[U], od[U], r1[U], r10[U], r2[U], r20[U];
        bool win[U], border[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            uint64_t j, k, c;
            uint64_t const it = beg + threadIdx.x + static_cast<uint64_t>(u) * kVecBlock;
            bool live = it < end;
            uint64_t const ii = live ? it : beg;
            if constexpr (MODE == 1)
            {
                uint32_t const rr = fdiv(static_cast<uint32_t>(ii), g.divCpr);
                c = static_cast<uint32_t>(ii) - rr * g.divCpr.d;
                uint32_t const kk = fdiv(rr, g.divVny);
                k = kk;
                j = rr - kk * g.divVny.d;
            }
            else
            {
                uint64_t const r = ii / g.cpr;
                c = ii - r * g.cpr;
                j = r % static_cast<uint64_t>(g.vny);
                k = r / static_cast<uint64_t>(g.vny);
            }
            int64_t const dr = d.base + static_cast<int64_t>(k) * d.sz + static_cast<int64_t>(j) * d.sy;
            int64_t const x = 8 * static_cast<int64_t>(c) - ((g.dph + dr) & 7);
            xs[u] = x;
            od[u] = dr + x;
            live = live && x < g.vnx;
            r1[u] = r10[u] = r2[u] = r20[u] = 0;
            if constexpr (NS >= 1)
                r1[u] = genRowStart(s1, j, k, r10[u]);
            if constexpr (NS >= 2)
                r2[u] = genRowStart(s2, j, k, r20[u]);
            bool const clampX = NS >= 1 && g.anyClamp && !(genInterior(s1, x) && (NS < 2 || genInterior(s2, x)));
            border[u] = live && clampX;
            win[u] = live && !clampX;
            // voxels of the item inside the box row
            int32_t const lo = x < 0 ? static_cast<int32_t>(-x) : 0;
            int32_t const hi = x + 8 > g.vnx ? static_cast<int32_t>(g.vnx - x) : 8;
            if (win[u])
            {
                if constexpr (NS >= 1)
                    loadWindow<B1>(s1.data, r1[u] + x, lo, hi, wa[u]);
                if constexpr (NS >= 2)
                    loadWindow<B2>(s2.data, r2[u] + x, lo, hi, wb[u]);
            }
        }
        auto result = [&](uint32_t const* a, uint32_t const* b, uint32_t (&rd)[2 * BD]) {
            if constexpr (kPass)
            {
#pragma unroll
                for (int m = 0; m < 2 * BD; ++m)
                    rd[m] = a[m];
            }
            else if constexpr (kPack)
            {
#pragma unroll
                for (int m = 0; m < 4; ++m)
                    rd[m] = f.pk(a[m], b[m]);
            }
            else
            {
                uint32_t aa[2 * B1], bb[2 * (NS >= 2 ? B2 : 1)];
#pragma unroll
                for (int m = 0; m < 2 * B1; ++m)
                    aa[m] = NS >= 1 ? a[m] : 0u;
#pragma unroll
                for (int m = 0; m < 2 * (NS >= 2 ? B2 : 1); ++m)
                    bb[m] = NS >= 2 ? b[m] : 0u;
                uint32_t ca[8], cb[8] = {0, 0, 0, 0, 0, 0, 0, 0}, oc[8];
                unpack8<B1>(aa, ca);
                if constexpr (NS >= 2)
                    unpack8<B2>(bb, cb);
#pragma unroll
                for (int v = 0; v < 8; ++v)
                    oc[v] = f(NS >= 1 ? ca[v] : 0u, cb[v]);
                Window<BD> t;
                packCodes<BD>(oc, t, std::make_index_sequence<2 * BD>{});
#pragma unroll
                for (int m = 0; m < 2 * BD; ++m)
                    rd[m] = t.w[m];
            }
        };
        auto store = [&](int u, uint32_t const (&rd)[2 * BD]) {
            uint64_t const o = static_cast<uint64_t>(od[u]);
            if (xs[u] >= 0 && xs[u] + 8 <= g.vnx)
            {
                if constexpr (BD == 1)
                    *reinterpret_cast<u32x2*>(d.data + o) = u32x2{rd[0], rd[1]};
                else if constexpr (BD == 2)
                    __builtin_nontemporal_store(u32x4{rd[0], rd[1], rd[2], rd[3]},
                                                reinterpret_cast<u32x4*>(d.data + 2 * o));
                else
                {
                    __builtin_nontemporal_store(u32x4{rd[0], rd[1], rd[2], rd[3]}, reinterpret_cast<u32x4*>(d.data + 4 * o));
                    __builtin_nontemporal_store(u32x4{rd[4], rd[5], rd[6], rd[7]},
                                                reinterpret_cast<u32x4*>(d.data + 4 * o + 16));
                }
            }
            else
            {
                // an item straddling a row end: only the row's voxels
                uint32_t oc[8];
                unpack8<BD>(rd, oc);
#pragma unroll
                for (int v = 0; v < 8; ++v)
                    if (xs[u] + v >= 0 && xs[u] + v < g.vnx)
                        storeCode<BD>(d.data, o + v, oc[v]);
            }
        };
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            if (!win[u])
                continue;
            uint32_t a[2 * B1], b[2 * (NS >= 2 ? B2 : 1)], rd[2 * BD];
            if constexpr (NS >= 1)
                shiftWindow<B1>(wa[u], a);
            if constexpr (NS >= 2)
                shiftWindow<B2>(wb[u], b);
            result(a, b, rd);
            store(u, rd);
        }
        if (!g.anyClamp)
            return;
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            if (!border[u])
                continue;
            uint32_t ca[8], cb[8], a[2 * B1], b[2 * (NS >= 2 ? B2 : 1)], rd[2 * BD];
            loadBorder<B1>(s1, r1[u], r10[u], xs[u], ca);
            if constexpr (NS >= 2)
                loadBorder<B2>(s2, r2[u], r20[u], xs[u], cb);
            Window<B1> ta;
            packCodes<B1>(ca, ta, std::make_index_sequence<2 * B1>{});
#pragma unroll
            for (int m = 0; m < 2 * B1; ++m)
                a[m] = ta.w[m];
            if constexpr (NS >= 2)
            {
                Window<B2> tb;
                packCodes<B2>(cb, tb, std::make_index_sequence<2 * B2>{});
#pragma unroll
                for (int m = 0; m < 2 * B2; ++m)
                    b[m] = tb.w[m];
            }
            result(a, b, rd);
            store(u, rd);
        }
    }

    // ---- the same with 32-bit addressing (GenGeom::fast) ----------------------------------
    // Measured: the 64-bit version issues ~136 VALU per item (64-bit multiplies, 64-bit pointer
    // compares for the word clamps) and is VALU-bound (SQ_ACTIVE_INST_VALU x 4 cycles ~ 97 % of
    // the SIMD cycles for a phase-shifted copy).  Here row offsets are 24-bit multiply-adds,
    // window words are 32-bit byte offsets from the operand's 16-B aligned base clamped with one
    // v_med3_i32, and loads / stores address base (scalar) + 32-bit offset.
    struct FastOp
    {
        uint8_t const* abase;   // data & ~15
        int32_t mis;            // data & 15
        uint32_t base, sy, sz;  // voxel index of box (0,0,0), row and plane pitch
    };

    __device__ __forceinline__ FastOp fastOp(Operand const& o)
    {
        FastOp r;
        uintptr_t const a = reinterpret_cast<uintptr_t>(o.data);
        r.abase = o.data - (a & 15u);
        r.mis = static_cast<int32_t>(a & 15u);
        r.base = static_cast<uint32_t>(o.base);
        r.sy = static_cast<uint32_t>(o.sy);
        r.sz = static_cast<uint32_t>(o.sz);
        return r;
    }

    // voxel index of box x = 0 in row (j, k); clamped rows as genRowStart
    __device__ __forceinline__ int32_t fastRowStart(Operand const& o, FastOp const& f, uint32_t j, uint32_t k)
    {
        if (!o.clamp)
            return static_cast<int32_t>(f.base + __umul24(k, f.sz) + __umul24(j, f.sy));
        uint32_t const y = static_cast<uint32_t>(clampRefI(o.origin[1] + static_cast<int32_t>(j), 0, o.dims[1] - 1));
        uint32_t const z = static_cast<uint32_t>(clampRefI(o.origin[2] + static_cast<int32_t>(k), 0, o.dims[2] - 1));
        return static_cast<int32_t>(__umul24(z, f.sz) + __umul24(y, f.sy)) + o.origin[0];
    }

    // voxel: index of the item's first voxel, modulo 2^32 (it lies before voxel 0 for an item
    // that starts left of the row at the very start of the volume); the words actually loaded
    // hold valid voxels [lo, hi) only, so their offsets are true non-negative offsets < 2^32.
    template <int B>
    __device__ __forceinline__ void loadWindowFast(FastOp const& f, uint32_t voxel, int32_t lo, int32_t hi,
                                                   Window<B>& win)
    {
        uint32_t const bo = voxel * B + static_cast<uint32_t>(f.mis);    // byte offset from abase
        uint32_t const fo = (bo + static_cast<uint32_t>(lo * B)) & ~15u;   // first / last word holding
        uint32_t const lw = (bo + static_cast<uint32_t>(hi * B - 1)) & ~15u;   // a valid voxel
        int32_t const dw = static_cast<int32_t>((bo & ~15u) - fo);         // word 0 relative to fo: -16 or 0
        int32_t const span = static_cast<int32_t>(lw - fo);
        win.s = bo & 15u;
        auto word = [&](int i) {
            int32_t const o = min(max(dw + 16 * i, 0), span);
            return *reinterpret_cast<u32x4 const*>(f.abase + (fo + static_cast<uint32_t>(o)));
        };
        u32x4 const v0 = word(0);
        u32x4 const v1 = word(1);
        win.w[0] = v0.x; win.w[1] = v0.y; win.w[2] = v0.z; win.w[3] = v0.w;
        win.w[4] = v1.x; win.w[5] = v1.y; win.w[6] = v1.z; win.w[7] = v1.w;
        if constexpr (Window<B>::NW == 3)
        {
            u32x4 const v2 = word(2);
            win.w[8] = v2.x; win.w[9] = v2.y; win.w[10] = v2.z; win.w[11] = v2.w;
        }
    }

    template <int NS, int BD, int B1, int B2, int U, class F>
    __device__ __forceinline__ void pointwiseGenSpanFast(Operand const& d, Operand const& s1, Operand const& s2,
                                                         GenGeom const& g, uint32_t beg, uint32_t end, F const& f)
    {
        constexpr bool kPack = BD == 2 && B1 == 2 && B2 == 2 && NS == 2 && IsPacked16<F>::value;
        constexpr bool kPass = NS == 1 && BD == B1 && std::is_same<F, PassF>::value;
        FastOp const fd = fastOp(d), f1 = fastOp(s1), f2 = fastOp(s2);
        int32_t const vnx = static_cast<int32_t>(g.vnx);
        Window<B1> wa[U];
        Window<NS >= 2 ? B2 : 1> wb[U];
        uint32_t dd[U][2 * BD];   // merge: the destination's own codes of an edge item
        int32_t xs[U];
        uint32_t od[U], r1[U], r2[U], js[U], ks[U];
        bool win[U], border[U], pad[U];
        // items start on 8-voxel (merge: 64-B sector) boundaries of the destination
        uint32_t const unitMask = g.merge ? static_cast<uint32_t>(g.sv - 1) : 7u;
        uint32_t const dphU = g.merge ? static_cast<uint32_t>(g.dph64) : static_cast<uint32_t>(g.dph);
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            uint32_t const it = beg + threadIdx.x + static_cast<uint32_t>(u) * kVecBlock;
            bool live = it < end;
            uint32_t const ii = live ? it : beg;
            uint32_t const rr = fdiv(ii, g.divCpr);
            uint32_t const c = ii - rr * g.divCpr.d;
            uint32_t const k = fdiv(rr, g.divVny);
            uint32_t const j = rr - k * g.divVny.d;
            js[u] = j;
            ks[u] = k;
            uint32_t const dr = fd.base + __umul24(k, fd.sz) + __umul24(j, fd.sy);
            int32_t const ps = static_cast<int32_t>((dphU + dr) & unitMask);
            int32_t const x = static_cast<int32_t>(8 * c) - ps;
            xs[u] = x;
            od[u] = dr + static_cast<uint32_t>(x);   // modulo 2^32, like the window voxels
            // row's item range: [-ps, vnx) rounded up to the unit (a whole 64-B sector when merging)
            int32_t const rowEnd = static_cast<int32_t>((static_cast<uint32_t>(ps + vnx) + unitMask) & ~unitMask) - ps;
            live = live && x < (g.merge ? rowEnd : vnx);
            bool const boxPart = x + 8 > 0 && x < vnx;   // the item holds voxels of the box row
            pad[u] = live && !boxPart;                   // merge only: sector completion, no box voxel
            r1[u] = r2[u] = 0;
            if constexpr (NS >= 1)
                r1[u] = static_cast<uint32_t>(fastRowStart(s1, f1, j, k));
            if constexpr (NS >= 2)
                r2[u] = static_cast<uint32_t>(fastRowStart(s2, f2, j, k));
            bool const clampX = NS >= 1 && g.anyClamp && !(genInterior(s1, x) && (NS < 2 || genInterior(s2, x)));
            border[u] = live && boxPart && clampX;
            win[u] = live && boxPart && !clampX;
            int32_t const lo = x < 0 ? -x : 0;
            int32_t const hi = x + 8 > vnx ? vnx - x : 8;
            if (win[u])
            {
                if constexpr (NS >= 1)
                    loadWindowFast<B1>(f1, r1[u] + static_cast<uint32_t>(x), lo, hi, wa[u]);
                if constexpr (NS >= 2)
                    loadWindowFast<B2>(f2, r2[u] + static_cast<uint32_t>(x), lo, hi, wb[u]);
            }
            if (g.merge && live && !(x >= 0 && x + 8 <= vnx))
            {
                // edge or pad item: the destination chunk itself (8*BD aligned bytes)
                uint8_t const* const q = d.data + od[u] * BD;
                if constexpr (BD == 1)
                {
                    u32x2 const v = *reinterpret_cast<u32x2 const*>(q);
                    dd[u][0] = v.x; dd[u][1] = v.y;
                }
                else
                {
#pragma unroll
                    for (int h = 0; h < BD / 2; ++h)
                    {
                        u32x4 const v = *reinterpret_cast<u32x4 const*>(q + 16 * h);
                        dd[u][4 * h] = v.x; dd[u][4 * h + 1] = v.y; dd[u][4 * h + 2] = v.z; dd[u][4 * h + 3] = v.w;
                    }
                }
            }
        }
        auto result = [&](uint32_t const* a, uint32_t const* b, uint32_t (&rd)[2 * BD]) {
            if constexpr (kPass)
            {
#pragma unroll
                for (int m = 0; m < 2 * BD; ++m)
                    rd[m] = a[m];
            }
            else if constexpr (kPack)
            {
#pragma unroll
                for (int m = 0; m < 4; ++m)
                    rd[m] = f.pk(a[m], b[m]);
            }
            else
            {
                uint32_t aa[2 * B1], bb[2 * (NS >= 2 ? B2 : 1)];
#pragma unroll
                for (int m = 0; m < 2 * B1; ++m)
                    aa[m] = NS >= 1 ? a[m] : 0u;
#pragma unroll
                for (int m = 0; m < 2 * (NS >= 2 ? B2 : 1); ++m)
                    bb[m] = NS >= 2 ? b[m] : 0u;
                uint32_t ca[8], cb[8] = {0, 0, 0, 0, 0, 0, 0, 0}, oc[8];
                unpack8<B1>(aa, ca);
                if constexpr (NS >= 2)
                    unpack8<B2>(bb, cb);
#pragma unroll
                for (int v = 0; v < 8; ++v)
                    oc[v] = f(NS >= 1 ? ca[v] : 0u, cb[v]);
                Window<BD> t;
                packCodes<BD>(oc, t, std::make_index_sequence<2 * BD>{});
#pragma unroll
                for (int m = 0; m < 2 * BD; ++m)
                    rd[m] = t.w[m];
            }
        };
        auto storeFull = [&](int u, uint32_t const (&rd)[2 * BD]) {
            uint8_t* const p = d.data + od[u] * BD;
            if constexpr (BD == 1)
                *reinterpret_cast<u32x2*>(p) = u32x2{rd[0], rd[1]};
            else if constexpr (BD == 2)
                __builtin_nontemporal_store(u32x4{rd[0], rd[1], rd[2], rd[3]}, reinterpret_cast<u32x4*>(p));
            else
            {
                __builtin_nontemporal_store(u32x4{rd[0], rd[1], rd[2], rd[3]}, reinterpret_cast<u32x4*>(p));
                __builtin_nontemporal_store(u32x4{rd[4], rd[5], rd[6], rd[7]}, reinterpret_cast<u32x4*>(p + 16));
            }
        };
        // Full items, merged row-end items and sector-completion pads share ONE store statement
        // (see pointwiseGenSpanFast16: separate statements cost a wave both instruction sets
        // whenever it holds both kinds of item -- 2.3x the store instructions on a sub-box)
        auto store = [&](int u, uint32_t const (&rd)[2 * BD]) {
            bool const full = xs[u] >= 0 && xs[u] + 8 <= vnx;
            if (g.merge || full)
            {
                uint32_t m[2 * BD];
#pragma unroll
                for (int i = 0; i < 2 * BD; ++i)
                    m[i] = rd[i];
                if (!full)
                {
                    // the row's voxels from rd, the rest of the chunk from the destination itself:
                    // one whole-chunk store, so every 64-B sector of the row ends is written completely
                    uint32_t oc[8], dc[8];
                    unpack8<BD>(rd, oc);
                    unpack8<BD>(dd[u], dc);
#pragma unroll
                    for (int v = 0; v < 8; ++v)
                        oc[v] = xs[u] + v >= 0 && xs[u] + v < vnx ? oc[v] : dc[v];
                    Window<BD> t;
                    packCodes<BD>(oc, t, std::make_index_sequence<2 * BD>{});
#pragma unroll
                    for (int i = 0; i < 2 * BD; ++i)
                        m[i] = t.w[i];
                }
                storeFull(u, m);
            }
            else
            {
                uint32_t oc[8];
                unpack8<BD>(rd, oc);
#pragma unroll
                for (int v = 0; v < 8; ++v)
                    if (xs[u] + v >= 0 && xs[u] + v < vnx)
                        storeCode<BD>(d.data + (od[u] + v) * BD, 0, oc[v]);
            }
        };
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            if (!win[u] && !pad[u])
                continue;
            uint32_t rd[2 * BD];
#pragma unroll
            for (int i = 0; i < 2 * BD; ++i)
                rd[i] = dd[u][i];   // pad: sector completion, the destination's own bytes
            if (win[u])
            {
                uint32_t a[2 * B1], b[2 * (NS >= 2 ? B2 : 1)];
                if constexpr (NS >= 1)
                    shiftWindow<B1>(wa[u], a, g.dword != 0);
                if constexpr (NS >= 2)
                    shiftWindow<B2>(wb[u], b, g.dword != 0);
                result(a, b, rd);
            }
            store(u, rd);   // (a pad lies outside its row: merged, every voxel is the destination's own)
        }
        if (!g.anyClamp)
            return;
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            if (!border[u])
                continue;
            // clamped x border: voxel by voxel (rows as genRowStart: x = 0 of the volume row)
            int64_t r10 = 0, r20 = 0;
            int64_t const q1 = genRowStart(s1, js[u], ks[u], r10);
            int64_t q2 = 0;
            if constexpr (NS >= 2)
                q2 = genRowStart(s2, js[u], ks[u], r20);
            uint32_t ca[8], cb[8], a[2 * B1], b[2 * (NS >= 2 ? B2 : 1)], rd[2 * BD];
            loadBorder<B1>(s1, q1, r10, xs[u], ca);
            if constexpr (NS >= 2)
                loadBorder<B2>(s2, q2, r20, xs[u], cb);
            Window<B1> ta;
            packCodes<B1>(ca, ta, std::make_index_sequence<2 * B1>{});
#pragma unroll
            for (int m = 0; m < 2 * B1; ++m)
                a[m] = ta.w[m];
            if constexpr (NS >= 2)
            {
                Window<B2> tb;
                packCodes<B2>(cb, tb, std::make_index_sequence<2 * B2>{});
#pragma unroll
                for (int m = 0; m < 2 * B2; ++m)
                    b[m] = tb.w[m];
            }
            result(a, b, rd);
            store(u, rd);
        }
    }

    // ---- 16-B items for 1- and 4-byte voxels (GenGeom::wide) ------------------------------
    // The 8-voxel items above move 8 B per lane for UInt8 (and load a 32-B window per 8 B of
    // output) and 32 B per lane for 4-byte voxels (each store instruction every other 16 B of
    // 2 KiB).  Here an item is 16 destination bytes whatever the voxel size -- 16 voxels of
    // UInt8, 4 of Float32: one aligned 16-B store per lane, its source window the two aligned
    // 16-B words around the 16 source bytes (the UInt16 item's window) shifted once into four
    // dwords.  Row ends: byte-range stores (storeByteRange16), or with sector completion the
    // whole 16 B merged with the destination's own bytes (mergeBytes16).
    template <int B>
    __device__ __forceinline__ bool genInteriorW(Operand const& o, int32_t x)
    {
        return !o.clamp || (o.origin[0] + x >= 0 && o.origin[0] + x + 16 / B <= o.dims[0]);
    }

    __device__ __forceinline__ void shiftWindow16(Window<1> const& win, uint32_t (&out)[4], bool dword = false)
    {
        uint32_t a[6], b[5];
        shiftSel(win.w, a, (win.s & 8u) != 0, 2, std::make_index_sequence<6>{});
        shiftSel(a, b, (win.s & 4u) != 0, 1, std::make_index_sequence<5>{});
        if (dword)
        {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                out[i] = b[i];
        }
        else
            shiftAlign(b, out, win.s & 3u, std::make_index_sequence<4>{});
    }

    // the two aligned words around voxels [lo, hi) of the 16 / B voxels at `voxel` (as
    // loadWindowFast, two words for any voxel size)
    template <int B>
    __device__ __forceinline__ void loadWindowFast2(FastOp const& f, uint32_t voxel, int32_t lo, int32_t hi,
                                                    Window<1>& win)
    {
        uint32_t const bo = voxel * B + static_cast<uint32_t>(f.mis);
        uint32_t const fo = (bo + static_cast<uint32_t>(lo * B)) & ~15u;
        uint32_t const lw = (bo + static_cast<uint32_t>(hi * B - 1)) & ~15u;
        int32_t const dw = static_cast<int32_t>((bo & ~15u) - fo);
        int32_t const span = static_cast<int32_t>(lw - fo);
        win.s = bo & 15u;
        auto word = [&](int i) {
            int32_t const o = min(max(dw + 16 * i, 0), span);
            return *reinterpret_cast<u32x4 const*>(f.abase + (fo + static_cast<uint32_t>(o)));
        };
        u32x4 const v0 = word(0);
        u32x4 const v1 = word(1);
        win.w[0] = v0.x; win.w[1] = v0.y; win.w[2] = v0.z; win.w[3] = v0.w;
        win.w[4] = v1.x; win.w[5] = v1.y; win.w[6] = v1.z; win.w[7] = v1.w;
    }

    template <int NS, int B, int U, class F>
    __device__ __forceinline__ void pointwiseGenSpanFast16(Operand const& d, Operand const& s1, Operand const& s2,
                                                           GenGeom const& g, uint32_t beg, uint32_t end, F const& f)
    {
        constexpr int V = 16 / B;   // voxels per item
        constexpr bool kPass = NS == 1 && std::is_same<F, PassF>::value;
        FastOp const fd = fastOp(d), f1 = fastOp(s1), f2 = fastOp(s2);
        int32_t const vnx = static_cast<int32_t>(g.vnx);
        Window<1> wa[U];
        Window<1> wb[NS >= 2 ? U : 1];
        u32x4 dd[U];
        int32_t xs[U];
        int64_t od[U];   // signed: the first item of a row at voxel 0 of a destination view that
                         // starts inside a 16-B word lies before the view (only its row bytes are stored)
        uint32_t js[U], ks[U];
        bool win[U], border[U], pad[U];
        // items start on V-voxel (merge: 64-B sector) boundaries of the destination
        uint32_t const unitMask = g.merge ? static_cast<uint32_t>(64 / B - 1) : static_cast<uint32_t>(V - 1);
        uint32_t const dphU = static_cast<uint32_t>(g.merge ? g.dph64 : g.dph);
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            uint32_t const it = beg + threadIdx.x + static_cast<uint32_t>(u) * kVecBlock;
            bool live = it < end;
            uint32_t const ii = live ? it : beg;
            uint32_t const rr = fdiv(ii, g.divCpr);
            uint32_t const c = ii - rr * g.divCpr.d;
            uint32_t const k = fdiv(rr, g.divVny);
            uint32_t const j = rr - k * g.divVny.d;
            js[u] = j;
            ks[u] = k;
            uint32_t const dr = fd.base + __umul24(k, fd.sz) + __umul24(j, fd.sy);
            int32_t const ps = static_cast<int32_t>((dphU + dr) & unitMask);
            int32_t const x = static_cast<int32_t>(V * c) - ps;
            xs[u] = x;
            od[u] = static_cast<int64_t>(dr) + x;
            int32_t const rowEnd = static_cast<int32_t>((static_cast<uint32_t>(ps + vnx) + unitMask) & ~unitMask) - ps;
            live = live && x < (g.merge ? rowEnd : vnx);
            bool const boxPart = x + V > 0 && x < vnx;
            pad[u] = live && !boxPart;
            bool const clampX = NS >= 1 && g.anyClamp && !(genInteriorW<B>(s1, x) && (NS < 2 || genInteriorW<B>(s2, x)));
            border[u] = live && boxPart && clampX;
            win[u] = live && boxPart && !clampX;
            int32_t const lo = x < 0 ? -x : 0;
            int32_t const hi = x + V > vnx ? vnx - x : V;
            if (win[u])
            {
                if constexpr (NS >= 1)
                    loadWindowFast2<B>(f1, static_cast<uint32_t>(fastRowStart(s1, f1, j, k)) + static_cast<uint32_t>(x),
                                       lo, hi, wa[u]);
                if constexpr (NS >= 2)
                    loadWindowFast2<B>(f2, static_cast<uint32_t>(fastRowStart(s2, f2, j, k)) + static_cast<uint32_t>(x),
                                       lo, hi, wb[u]);
            }
            if (g.merge && live && !(x >= 0 && x + V <= vnx))
                dd[u] = *reinterpret_cast<u32x4 const*>(d.data + od[u] * B);
        }
        auto result = [&](uint32_t const (&a)[4], uint32_t const (&b)[4], u32x4& rd) {
            if constexpr (kPass)
                rd = u32x4{a[0], a[1], a[2], a[3]};
            else
            {
                uint32_t r[4];
#pragma unroll
                for (int m = 0; m < 4; ++m)
                {
                    if constexpr (B == 4)
                        r[m] = f(NS >= 1 ? a[m] : 0u, NS >= 2 ? b[m] : 0u);
                    else
                    {
                        uint32_t o = 0;
#pragma unroll
                        for (int v = 0; v < 4; ++v)
                            o |= (f(NS >= 1 ? (a[m] >> (8 * v)) & 0xFFu : 0u, NS >= 2 ? (b[m] >> (8 * v)) & 0xFFu : 0u) &
                                  0xFFu) << (8 * v);
                        r[m] = o;
                    }
                }
                rd = u32x4{r[0], r[1], r[2], r[3]};
            }
        };
        // Whole-item stores (full items, merged row-end items, sector-completion pads) go through
        // ONE store instruction per item slot: separate store statements per case issue each as
        // its own wave instruction whenever a wave holds both kinds of item -- nearly every wave of
        // a sub-box, whose rows end every ~100 items (PMC: 2.3x the store instructions of an
        // edge-free box).  Only the byte-range stores of unmerged row ends stay apart.
        auto store = [&](int u, u32x4 const& rd) {
            uint8_t* const p = d.data + od[u] * B;
            int32_t const x = xs[u];
            bool const full = x >= 0 && x + V <= vnx;
            if (full || g.merge)
            {
                u32x4 v = rd;
                if (!full)
                    v = mergeBytes16(rd, dd[u], B * (x < 0 ? -x : 0), B * (x + V > vnx ? vnx - x : V));
                __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
            }
            else
                storeByteRange16(p, rd, B * (x < 0 ? -x : 0), B * (x + V > vnx ? vnx - x : V));
        };
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            if (!win[u] && !pad[u])
                continue;
            u32x4 rd = dd[u];   // pad: sector completion with the destination's own bytes
            if (win[u])
            {
                uint32_t a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
                if constexpr (NS >= 1)
                    shiftWindow16(wa[u], a, B == 4 && g.dword != 0);
                if constexpr (NS >= 2)
                    shiftWindow16(wb[u], b, B == 4 && g.dword != 0);
                result(a, b, rd);
            }
            store(u, rd);   // (a pad lies outside its row: merged, every byte is the destination's own)
        }
        if (!g.anyClamp)
            return;
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            if (!border[u])
                continue;
            // clamped x border: voxel by voxel (rows as genRowStart: x = 0 of the volume row)
            int64_t r10 = 0, r20 = 0;
            int64_t const q1 = genRowStart(s1, js[u], ks[u], r10);
            int64_t q2 = 0;
            if constexpr (NS >= 2)
                q2 = genRowStart(s2, js[u], ks[u], r20);
            uint32_t a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
#pragma unroll
            for (int v = 0; v < V; ++v)
            {
                constexpr int kBits = 8 * B;
                a[(v * B) / 4] |= genLoadOne<B>(s1, q1, r10, xs[u] + v) << ((v * kBits) % 32);
                if constexpr (NS >= 2)
                    b[(v * B) / 4] |= genLoadOne<B>(s2, q2, r20, xs[u] + v) << ((v * kBits) % 32);
            }
            u32x4 rd;
            result(a, b, rd);
            store(u, rd);
        }
    }

    template <int NS, int BD, int B1, int B2, int U, class F>
    __global__ __launch_bounds__(kVecBlock) void pointwiseGenKernel(Operand d, Operand s1, Operand s2, GenGeom g, F f,
                                                                   uint64_t qBase, uint64_t qEnd)
    {
        constexpr uint64_t kQ = static_cast<uint64_t>(kVecBlock) * U;
        for (uint64_t q = qBase + blockIdx.x; q < qEnd; q += gridDim.x)
        {
            uint64_t const beg = q * kQ;
            if (beg >= g.items)
                break;
            uint64_t const end = beg + kQ < g.items ? beg + kQ : g.items;
            if constexpr ((BD == 1 || BD == 4) && B1 == BD && (NS < 2 || B2 == BD))
            {
                if (g.wide)
                {
                    pointwiseGenSpanFast16<NS, BD, U>(d, s1, s2, g, static_cast<uint32_t>(beg), static_cast<uint32_t>(end),
                                                      f);
                    continue;
                }
            }
            if (g.fast)
                pointwiseGenSpanFast<NS, BD, B1, B2, U>(d, s1, s2, g, static_cast<uint32_t>(beg),
                                                        static_cast<uint32_t>(end), f);
            else if (g.fast32)
                pointwiseGenSpan<NS, BD, B1, B2, 1, U>(d, s1, s2, g, beg, end, f);
            else
                pointwiseGenSpan<NS, BD, B1, B2, 2, U>(d, s1, s2, g, beg, end, f);
        }
    }

    // One span path of the general kernel per instantiation (PATH 0 wide 16-B items, 1 32-bit
    // addressing, 2 64-bit rows on 32-bit division, 3 64-bit division), chosen on the host from the
    // same GenGeom flags: the combined kernel's register count is set by its largest path (152
    // VGPRs for UInt8 SumRange) whichever one a launch takes.
    template <int NS, int BD, int B1, int B2, int U, int PATH, class F>
    __global__ __launch_bounds__(kVecBlock) void pointwiseGenPathKernel(Operand d, Operand s1, Operand s2, GenGeom g,
                                                                       F f, uint64_t qBase, uint64_t qEnd)
    {
        constexpr uint64_t kQ = static_cast<uint64_t>(kVecBlock) * U;
        for (uint64_t q = qBase + blockIdx.x; q < qEnd; q += gridDim.x)
        {
            uint64_t const beg = q * kQ;
            if (beg >= g.items)
                break;
            uint64_t const end = beg + kQ < g.items ? beg + kQ : g.items;
            if constexpr (PATH == 0)
                pointwiseGenSpanFast16<NS, BD, U>(d, s1, s2, g, static_cast<uint32_t>(beg), static_cast<uint32_t>(end), f);
            else if constexpr (PATH == 1)
                pointwiseGenSpanFast<NS, BD, B1, B2, U>(d, s1, s2, g, static_cast<uint32_t>(beg),
                                                        static_cast<uint32_t>(end), f);
            else
                pointwiseGenSpan<NS, BD, B1, B2, PATH - 1, U>(d, s1, s2, g, beg, end, f);
        }
    }

    template <int NS, class F>
    __global__ __launch_bounds__(kBlock) void pointwiseScalarKernel(Operand d, Operand s1, Operand s2, Geom g, F f)
    {
        uint64_t const tid = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x;
        uint64_t const stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
        uint64_t const nx = static_cast<uint64_t>(g.nx), ny = static_cast<uint64_t>(g.ny);
        uint64_t const total = nx * ny * static_cast<uint64_t>(g.nz);
        for (uint64_t l = tid; l < total; l += stride)
        {
            uint64_t i, j, k;
            if (g.fast32)
            {
                uint32_t t = fdiv(static_cast<uint32_t>(l), g.divNx);
                i = static_cast<uint32_t>(l) - t * g.divNx.d;
                uint32_t kk = fdiv(t, g.divNy);
                k = kk;
                j = t - kk * g.divNy.d;
            }
            else
            {
                i = l % nx;
                uint64_t t = l / nx;
                j = t % ny;
                k = t / ny;
            }
            uint32_t a = 0, b = 0;
            if constexpr (NS >= 1)
                a = loadCodeDyn(s1.data, scalarIndex(s1, i, j, k), s1.bpv);
            if constexpr (NS >= 2)
                b = loadCodeDyn(s2.data, scalarIndex(s2, i, j, k), s2.bpv);
            storeCodeDyn(d.data, scalarIndex(d, i, j, k), d.bpv, f(a, b));
        }
    }

    // ---- host-side planning (Pointwise.hip) -----------------------------------------
    struct PwPlan
    {
        Operand d, s1, s2;
        Geom g;
        GenGeom gg;
        bool vec;        // vector path eligible (aligned, unclamped, uniform voxel size)
        bool gen;        // general vector path eligible (any phase / pitch / clamp)
        bool uniform;    // every operand has the destination's voxel size
        uint32_t bpv;    // destination bytes per voxel
    };

    // General vector path launch (operand voxel sizes BD, B1, B2 fixed at compile time).
    template <int NS, int BD, int B1, int B2, int U, class F>
    vktError launchGenU(PwPlan const& p, F const& f, hipStream_t stream)
    {
        constexpr uint64_t kQ = static_cast<uint64_t>(kVecBlock) * U;
        // (measured and rejected: one row segment per workgroup, row coordinates on the scalar
        // unit -- 1021-voxel rows split into two 65-chunk segments, SumRange with dstOffset x = 3
        // at 1021 x 1024^2: 1.15 -> 1.62 ms; half-size quanta cost more than the index math saved)
        GenGeom const& gg = p.gg;
        uint64_t const quanta = (gg.items + kQ - 1) / kQ;
        uint64_t const maxQ = static_cast<uint64_t>(rt::knob(rt::Knob::PointwiseMaxQuanta));
        // 1- and 4-byte destinations: one kernel per span path (pointwiseGenPathKernel); 2-byte:
        // the combined kernel.  In-process A/B on 1024^3-class boxes (profiles/r05/gensplit.jsonl):
        // UInt8 SumRange dstOffset -97 0.431-0.516 -> 0.393-0.396 ms, UInt8 shifted copies -3 ..
        // -5 %, Float32 SumRange -1 %, copies -2 % (one +2 %); UInt16 +1 .. +2 % (the clamped
        // halo copy -6 %), so UInt16 keeps the combined kernel.
        constexpr bool kSplit = BD == 1 || BD == 4;
        constexpr bool kWideOk = (BD == 1 || BD == 4) && B1 == BD && (NS < 2 || B2 == BD);
        int const path = kWideOk && gg.wide ? 0 : gg.fast ? 1 : gg.fast32 ? 2 : 3;
        uint64_t q0 = 0;
        do
        {
            uint64_t const n = quanta - q0 < maxQ ? quanta - q0 : maxQ;
            dim3 const grid(static_cast<unsigned>(n > 0 ? n : 1));
            if constexpr (!kSplit)
                hipLaunchKernelGGL((pointwiseGenKernel<NS, BD, B1, B2, U, F>), grid, dim3(kVecBlock), 0, stream, p.d,
                                   p.s1, p.s2, gg, f, q0, q0 + n);
            else if (path == 0)
            {
                if constexpr (kWideOk)
                    hipLaunchKernelGGL((pointwiseGenPathKernel<NS, BD, B1, B2, U, 0, F>), grid, dim3(kVecBlock), 0,
                                       stream, p.d, p.s1, p.s2, gg, f, q0, q0 + n);
            }
            else if (path == 1)
                hipLaunchKernelGGL((pointwiseGenPathKernel<NS, BD, B1, B2, U, 1, F>), grid, dim3(kVecBlock), 0, stream,
                                   p.d, p.s1, p.s2, gg, f, q0, q0 + n);
            else if (path == 2)
                hipLaunchKernelGGL((pointwiseGenPathKernel<NS, BD, B1, B2, U, 2, F>), grid, dim3(kVecBlock), 0, stream,
                                   p.d, p.s1, p.s2, gg, f, q0, q0 + n);
            else
                hipLaunchKernelGGL((pointwiseGenPathKernel<NS, BD, B1, B2, U, 3, F>), grid, dim3(kVecBlock), 0, stream,
                                   p.d, p.s1, p.s2, gg, f, q0, q0 + n);
            q0 += n;
        } while (q0 < quanta);
        return vktNoError;
    }

    template <int NS, int BD, int B1, int B2, class F>
    vktError launchGen(PwPlan const& p, F const& f, hipStream_t stream)
    {
        constexpr int U = NS == 0 ? 2 : vecUnroll<NS, BD>();
        // 16-B items of 4-byte voxels are half the 8-voxel items: twice the items per lane
        // keep the bytes in flight
        if constexpr (BD == 4 && B1 == 4 && (NS < 2 || B2 == 4))
            if (p.gg.wide)
                return launchGenU<NS, BD, B1, B2, 2 * U>(p, f, stream);
        return launchGenU<NS, BD, B1, B2, U>(p, f, stream);
    }

    // Builds the plan for `ns` sources over a box of extent n (all > 0).
    PwPlan planPointwise(int ns, Operand d, Operand s1, Operand s2, int64_t nx, int64_t ny, int64_t nz);

    // Launch the plan with functor f: vector kernel if eligible and BPV matches, else scalar.
    template <int NS, int BPV, class F>
    vktError launchPointwise(PwPlan const& p, F const& f, hipStream_t stream)
    {
        if constexpr (BPV != 0)
        {
            if (p.vec && p.bpv == BPV)
            {
                uint64_t const rows = static_cast<uint64_t>(p.g.vny) * static_cast<uint64_t>(p.g.vnz);
                uint64_t items = rows * static_cast<uint64_t>((p.g.vnx8 - p.g.vhead) / 8);
                // enough threads for the scalar row edges too (narrow boxes are all edge)
                uint64_t edgeItems = p.g.padded ? 0 : rows * static_cast<uint64_t>(p.g.vhead + (p.g.vnx - p.g.vnx8));
                uint64_t edgeBlocks = (edgeItems + kVecBlock - 1) / kVecBlock;
                edgeBlocks = edgeBlocks < 4096 ? edgeBlocks : 4096;
                // one collapsed row without scalar edges -- UInt8 copies and arithmetic, UInt16
                // arithmetic: the MODE-0-only kernel (knob pointwise.row_kernel bits 0 / 1), with
                // 1 KiB per stream per one-wave workgroup and the waves per CU capped by dynamic
                // LDS (knobs pointwise.u8_unroll / u16_unroll, row_lds_u8 / row_lds).  In-process
                // A/Bs on the same 1024^3 allocations (profiles/r05/u8row.jsonl, u16row.jsonl):
                // UInt8 Copy 0.368 -> 0.326 ms, SumRange 0.540 -> 0.495 ms; UInt16 SumRange
                // 0.995 -> 0.968 ms (29 workgroups per CU; 32 -- no cap -- 0.986, 24: 0.986).
                // UInt16 copies (0.650 vs 0.660 ms), fills and Float32 stay on the general kernel.
                constexpr bool kRowCapable = (BPV == 1 && NS >= 1) || (BPV == 2 && NS == 2);   // (the only instantiations)
                bool const rowOnly = kRowCapable && rows == 1 && edgeItems == 0 &&
                                     (rt::knob(rt::Knob::PointwiseRowKernel) & (BPV == 1 ? 1 : 2)) != 0;
                // multi-row boxes on the MODE-1-only kernel (knob pointwise.rows_kernel, same bits)
                bool const rowsOnly = kRowCapable && rows > 1 && p.g.fast32 && edgeItems == 0 &&
                                      (rt::knob(rt::Knob::PointwiseRowsKernel) & (BPV == 1 ? 1 : 2)) != 0;
                // dynamic LDS per one-wave workgroup: caps the waves per CU at 160 KiB / rowLds
                // (knob pointwise.row_lds; the kernel does not touch it)
                uint32_t const rowRuns = static_cast<uint32_t>(rt::knob(rt::Knob::PointwiseRowSwizzle));
                unsigned const rowLds =
                    static_cast<unsigned>(rt::knob(BPV == 1 ? rt::Knob::PointwiseRowLdsU8 : rt::Knob::PointwiseRowLds));
                auto launch = [&](auto unroll, auto rowKernelOnly) {
                    constexpr int U = decltype(unroll)::value;
                    constexpr bool kRowOnly = decltype(rowKernelOnly)::value;
                    constexpr uint64_t kQ = static_cast<uint64_t>(kVecBlock) * U;
                    // (row-aligned quanta -- no 128-B line of a row shared by two workgroups --
                    // measured no better in an in-process A/B: 800^3 sub-box of 1024^3 at x0 = 100
                    // 0.603 vs 0.589 ms flat, at x0 = 96 0.537 vs 0.551 ms)
                    uint64_t const quanta = (items + kQ - 1) / kQ;
                    // the launch split counts quanta of the default unroll (knob
                    // pointwise.max_quanta_per_launch, default kMaxQuantaPerLaunch)
                    uint64_t const maxQ = static_cast<uint64_t>(rt::knob(rt::Knob::PointwiseMaxQuanta)) *
                                              vecUnroll<NS, BPV>() / U;
                    uint64_t q0 = 0;
                    do
                    {
                        uint64_t const n = quanta - q0 < maxQ ? quanta - q0 : maxQ;
                        uint64_t const g = q0 == 0 && n < edgeBlocks ? edgeBlocks : n;
                        if constexpr (kRowCapable)
                        {
                            if (rowsOnly)
                            {
                                hipLaunchKernelGGL((pointwiseRowKernel<NS, BPV, 1, U, F>),
                                                   dim3(static_cast<unsigned>(n > 0 ? n : 1)), dim3(kVecBlock), rowLds,
                                                   stream, p.d, p.s1, p.s2, p.g, f, q0, q0 + n, rowRuns);
                                q0 += n;
                                continue;
                            }
                            if (kRowOnly || rowOnly)
                            {
                                hipLaunchKernelGGL((pointwiseRowKernel<NS, BPV, 0, U, F>),
                                                   dim3(static_cast<unsigned>(n > 0 ? n : 1)), dim3(kVecBlock), rowLds,
                                                   stream, p.d, p.s1, p.s2, p.g, f, q0, q0 + n, rowRuns);
                                q0 += n;
                                continue;
                            }
                        }
                        if constexpr (!kRowOnly)
                            hipLaunchKernelGGL((pointwiseVecKernel<NS, BPV, U, F>), dim3(static_cast<unsigned>(g > 0 ? g : 1)),
                                               dim3(kVecBlock), 0, stream, p.d, p.s1, p.s2, p.g, f, q0, q0 + n,
                                               static_cast<int32_t>(q0 == 0));
                        q0 += n;
                    } while (q0 < quanta);
                };
                // (a 1-KiB quantum for the one-row 3-stream UInt16 ops measured the same as 2 KiB
                // in an in-process A/B, 0.985 vs 0.986 ms for 1024^3 SumRange: one unroll for all)
                // items per lane: the whole-volume kernel per knob (pointwise.u8_unroll / u16_unroll:
                // 1 KiB per stream measured best); the multi-row kernel 1 KiB per stream for UInt8
                // copies, the default 2 KiB otherwise (profiles/r05/rowsk.jsonl)
                int64_t u = vecUnroll<NS, BPV>();
                if (rowOnly)
                    u = rt::knob(BPV == 1 ? rt::Knob::PointwiseU8Unroll : rt::Knob::PointwiseU16Unroll);
                else if (rowsOnly && BPV == 1 && NS == 1)
                    u = 2;
                if constexpr (BPV == 1 && NS >= 1)
                {
                    if ((rowOnly || rowsOnly) && u == 2 && vecUnroll<NS, BPV>() != 2)
                    {
                        launch(std::integral_constant<int, 2>{}, std::true_type{});
                        return vktNoError;
                    }
                    if ((rowOnly || rowsOnly) && u == 8)
                    {
                        launch(std::integral_constant<int, 8>{}, std::true_type{});
                        return vktNoError;
                    }
                }
                if constexpr (BPV == 2 && NS == 2)
                {
                    if ((rowOnly || rowsOnly) && u == 1)
                    {
                        launch(std::integral_constant<int, 1>{}, std::true_type{});
                        return vktNoError;
                    }
                }
                launch(std::integral_constant<int, vecUnroll<NS, BPV>()>{}, std::false_type{});
                return vktNoError;
            }
            if (p.gen && p.uniform && p.bpv == BPV)
                return launchGen<NS, BPV, BPV, BPV>(p, f, stream);
        }
        uint64_t total = static_cast<uint64_t>(p.g.nx) * static_cast<uint64_t>(p.g.ny) * static_cast<uint64_t>(p.g.nz);
        unsigned grid = streamingGrid(total, kBlock);
        hipLaunchKernelGGL((pointwiseScalarKernel<NS, F>), dim3(grid), dim3(kBlock), 0, stream, p.d, p.s1, p.s2,
                           p.g, f);
        return vktNoError;
    }

} // hipk
} // vkt
