// volkit_transform.hpp -- Transform / TransformRange with __device__ functors (HIP only).
//
// The reference's Transform API takes HOST function pointers (include/cpp/vkt/Transform.hpp:
// 16-62) and its GPU backend is an empty stub (src/vkt/Transform_cuda.hpp:12-30).  Host
// callbacks cannot run on the GPU, so those overloads stage the range through host memory
// (volkit_amd/csrc/kernels/Transform.cpp).  This header adds the same overload set for
// callables that CAN run on the GPU -- a functor with a __device__ operator(), or a
// `[=] __device__ (...)` lambda -- with the reference's call signatures:
//
//     op(int32_t x, int32_t y, int32_t z, vkt::VoxelView voxel)                  unary
//     op(int32_t x, int32_t y, int32_t z, vkt::VoxelView v1, vkt::VoxelView v2)  binary
//
// Semantics are those of TransformRange_serial (src/vkt/Transform_serial.hpp:15-101): for
// every voxel of [first, last) the functor gets an 8-byte scratch (GetMaxBytesPerVoxel)
// zeroed and then filled with the voxel's bytes, the voxel's format and mapping; after the
// call the first bytesPerVoxel scratch bytes are stored back (binary: volume1, then
// volume2 -- for two handles on the SAME volume the volume2 bytes win, as in the serial
// loop).  The functor sees only its own voxel, so the visit order is unobservable and the
// kernel visits voxels in parallel.  vkt::device::MapVoxel / UnmapVoxel give the codec of
// the reference (src/vkt/VoxelMapping.hpp) on the device, bit-exact with the host.
//
// Kernels: for rows that are 16-byte aligned in every operand each lane moves 16-byte
// vectors (16 UInt8 / 8 UInt16 / 4 four-byte voxels), 4 per lane with all loads in flight
// before the first functor call, nontemporal loads and stores, one 256-lane workgroup per
// 16 KiB; every other range takes a one-voxel-per-lane row kernel.  They are compiled into
// the caller's translation unit (the functor is a template argument, so it is inlined and
// the scratch lives in registers) and run on volkit's compute stream in stream order with
// every library call.  Under the CPU policy the calls return InvalidValue, like every
// algorithm of this GPU backend.  Requires hipcc (--offload-arch=gfx950).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <type_traits>

#include "volkit.hpp"
#include "volkit_codec.hpp"
#include "volkit_hip.h"

namespace vkt
{
namespace device
{
    // The codec for device functors (also callable on the host, where it is the same code
    // libvolkit's vkt::MapVoxel / UnmapVoxel run).
    //! MapVoxel (reference src/vkt/Voxel.cpp:19-29 -> VoxelMapping.hpp:15-95)
    __host__ __device__ inline Error MapVoxel(uint8_t* dst, float value, DataFormat dataFormat, float mappingLo,
                                     float mappingHi)
    {
        codec::MapParams m;
        m.lo = mappingLo;
        m.hi = mappingHi;
        m.range = mappingHi - mappingLo;
        m.invRange = 0.f;
        m.rangeIsPow2 = 0;
        bool write = false;
        uint32_t code = codec::encode<2>(value, static_cast<int32_t>(dataFormat), m, write);
        if (write)
        {
            uint32_t n = codec::bytesPerVoxel(static_cast<int32_t>(dataFormat));
            for (uint32_t i = 0; i < n; ++i)
                dst[i] = static_cast<uint8_t>(code >> (8 * i));
        }
        return NoError;
    }

    //! UnmapVoxel (reference src/vkt/Voxel.cpp:31-42 -> VoxelMapping.hpp:98-177); formats the
    //! reference does not decode leave `value` untouched.
    __host__ __device__ inline Error UnmapVoxel(float& value, uint8_t const* src, DataFormat dataFormat, float mappingLo,
                                       float mappingHi)
    {
        uint32_t n = codec::bytesPerVoxel(static_cast<int32_t>(dataFormat));
        uint32_t code = 0;
        for (uint32_t i = 0; i < n && i < 4; ++i)
            code |= static_cast<uint32_t>(src[i]) << (8 * i);
        value = codec::decode(code, static_cast<int32_t>(dataFormat), mappingLo, mappingHi, value);
        return NoError;
    }
} // device

namespace transform_detail
{
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

    constexpr int kBlock = 256;           // 4 waves
    constexpr int kUnroll = 4;            // 16-byte items per lane (vector kernels)
    constexpr uint64_t kMaxItemsPerLaunch = uint64_t(1) << 30;

    // n / d for 32-bit n by multiply-high (d >= 1): l = ceil(log2 d), m = 2^32(2^l - d)/d + 1.
    struct FastDiv
    {
        uint32_t d, m, l;
    };

    inline FastDiv makeFastDiv(uint32_t d)
    {
        FastDiv f{d, 0u, 0u};
        uint32_t l = 0;
        while ((uint64_t(1) << l) < d)
            ++l;
        f.l = l;
        f.m = static_cast<uint32_t>(((uint64_t(1) << 32) * ((uint64_t(1) << l) - d)) / d + 1);
        return f;
    }

    __device__ __forceinline__ uint32_t fdiv(uint32_t n, FastDiv const& f)
    {
        return static_cast<uint32_t>((static_cast<uint64_t>(__umulhi(n, f.m)) + n) >> f.l);
    }

    struct Vol
    {
        uint8_t* data;
        uint64_t dimX, dimY;
        DataFormat format;
        float lo, hi;
    };

    // A launch covers box rows [row0, row0 + rows); a row is one (y, z) line of nx voxels,
    // split into `perRow` items (16-byte vectors, or 256-voxel segments).
    struct Rows
    {
        int32_t x0, y0, z0;
        uint32_t nx;
        int32_t rx0, rx1;   // padded launches: the range's own x [rx0, rx1) inside [x0, x0 + nx)
        uint32_t row0;
        uint64_t items;
        FastDiv perRow;   // items per row
        FastDiv ny;       // rows per plane
    };

    __device__ __forceinline__ void rowOf(Rows const& g, uint32_t local, uint32_t& c, int32_t& y, int32_t& z)
    {
        uint32_t rl = fdiv(local, g.perRow);
        c = local - rl * g.perRow.d;
        uint32_t r = g.row0 + rl;
        uint32_t zq = fdiv(r, g.ny);
        y = g.y0 + static_cast<int32_t>(r - zq * g.ny.d);
        z = g.z0 + static_cast<int32_t>(zq);
    }

    __device__ __forceinline__ uint64_t byteOf(Vol const& v, int32_t x, int32_t y, int32_t z, uint32_t bpv)
    {
        return ((static_cast<uint64_t>(z) * v.dimY + static_cast<uint64_t>(y)) * v.dimX + static_cast<uint64_t>(x)) *
               bpv;
    }

    // voxel k of a 16-byte vector <-> zeroed 8-byte scratch (Transform_serial.hpp:27-35)
    template <int BPV>
    __device__ __forceinline__ void unpack(u32x4 const& w, int k, uint8_t (&b)[8])
    {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            b[i] = 0;
        uint32_t word = w[(k * BPV) >> 2];
        int sh = ((k * BPV) & 3) * 8;
#pragma unroll
        for (int i = 0; i < BPV; ++i)
            b[i] = static_cast<uint8_t>(word >> (sh + 8 * i));
    }

    template <int BPV>
    __device__ __forceinline__ void pack(u32x4& w, int k, uint8_t const (&b)[8])
    {
        uint32_t bits = 0;
#pragma unroll
        for (int i = 0; i < BPV; ++i)
            bits |= static_cast<uint32_t>(b[i]) << (8 * i);
        int sh = ((k * BPV) & 3) * 8;
        w[(k * BPV) >> 2] |= bits << sh;
    }

    template <int BPV>
    __device__ __forceinline__ void loadVoxel(uint8_t const* p, uint8_t (&b)[8])
    {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            b[i] = 0;
        if constexpr (BPV == 1)
            b[0] = *p;
        else if constexpr (BPV == 2)
        {
            uint16_t c = *reinterpret_cast<uint16_t const*>(p);
            b[0] = static_cast<uint8_t>(c);
            b[1] = static_cast<uint8_t>(c >> 8);
        }
        else
        {
            uint32_t c = *reinterpret_cast<uint32_t const*>(p);
#pragma unroll
            for (int i = 0; i < 4; ++i)
                b[i] = static_cast<uint8_t>(c >> (8 * i));
        }
    }

    template <int BPV>
    __device__ __forceinline__ void storeVoxel(uint8_t* p, uint8_t const (&b)[8])
    {
        if constexpr (BPV == 1)
            *p = b[0];
        else if constexpr (BPV == 2)
            *reinterpret_cast<uint16_t*>(p) = static_cast<uint16_t>(b[0] | (b[1] << 8));
        else
            *reinterpret_cast<uint32_t*>(p) = static_cast<uint32_t>(b[0]) | (static_cast<uint32_t>(b[1]) << 8) |
                                               (static_cast<uint32_t>(b[2]) << 16) |
                                               (static_cast<uint32_t>(b[3]) << 24);
    }

    // ---- unary, 16-byte vectors: item = one 16-byte vector of one row -------------------
    // GUARD = false: the launch holds whole workgroups of valid items only (no per-item
    // branch between the loads; with one, hipcc waits for each load before the next).
    // PAD: the launch covers each row from the aligned chunk at or below the range start to
    // the one at or above its end (16-B, or 64-B sectors where the rows allow: a partly written
    // 64-B sector costs HBM a read-modify-write); voxels outside [rx0, rx1) are stored back as
    // they were loaded, without calling the functor.
    // Workgroup shape (NT threads x U 16-B items per lane): knob transform.shape (vecShape below).
    template <int BPV, bool GUARD, bool PAD, int NT, int U, class Op>
    __global__ void __launch_bounds__(NT) unaryVecKernel(Vol v, Rows g, uint32_t itemBase, Op op)
    {
        constexpr int V = 16 / BPV;
        constexpr int kUnroll = U;
        uint32_t base = itemBase + blockIdx.x * (NT * kUnroll) + threadIdx.x;
        u32x4 w[kUnroll];
        uint64_t at[kUnroll];
        int32_t xs[kUnroll], ys[kUnroll], zs[kUnroll];
        bool ok[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u)
        {
            uint32_t local = base + u * NT;
            ok[u] = !GUARD || local < g.items;
            if (GUARD && !ok[u])
                local = 0;
            uint32_t c;
            rowOf(g, local, c, ys[u], zs[u]);
            xs[u] = g.x0 + static_cast<int32_t>(c) * V;
            at[u] = byteOf(v, xs[u], ys[u], zs[u], BPV);
            w[u] = __builtin_nontemporal_load(reinterpret_cast<u32x4 const*>(v.data + at[u]));
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u)
        {
            u32x4 out = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int k = 0; k < V; ++k)
            {
                uint8_t bytes[8];
                unpack<BPV>(w[u], k, bytes);
                if (!PAD || (xs[u] + k >= g.rx0 && xs[u] + k < g.rx1))
                {
                    VoxelView voxel{bytes, v.format, v.lo, v.hi};
                    op(xs[u] + k, ys[u], zs[u], voxel);
                }
                pack<BPV>(out, k, bytes);
            }
            if (!GUARD || ok[u])
                __builtin_nontemporal_store(out, reinterpret_cast<u32x4*>(v.data + at[u]));
        }
    }

    // ---- unary, one voxel per lane: item = one 256-voxel segment of one row -------------
    template <int BPV, class Op>
    __global__ void __launch_bounds__(kBlock) unaryRowKernel(Vol v, Rows g, Op op)
    {
        uint32_t c;
        int32_t y, z;
        rowOf(g, blockIdx.x, c, y, z);
        uint32_t xr = c * kBlock + threadIdx.x;
        if (xr >= g.nx)
            return;
        int32_t x = g.x0 + static_cast<int32_t>(xr);
        uint8_t* p = v.data + byteOf(v, x, y, z, BPV);
        uint8_t bytes[8];
        loadVoxel<BPV>(p, bytes);
        VoxelView voxel{bytes, v.format, v.lo, v.hi};
        op(x, y, z, voxel);
        storeVoxel<BPV>(p, bytes);
    }

    // ---- binary, 16-byte vectors (both formats of the same size) ------------------------
    // ALIAS: both handles name one buffer with one layout: the voxel is loaded once, both
    // scratches start from it, and volume2's bytes are stored (the serial loop stores
    // volume1's, then volume2's, to the same address).
    template <int BPV, bool GUARD, bool ALIAS, bool PAD, int NT, int U, class Op>
    __global__ void __launch_bounds__(NT) binaryVecKernel(Vol v1, Vol v2, Rows g, uint32_t itemBase, Op op)
    {
        constexpr int V = 16 / BPV;
        constexpr int kUnroll = U;
        uint32_t base = itemBase + blockIdx.x * (NT * kUnroll) + threadIdx.x;
        u32x4 w1[kUnroll], w2[kUnroll];
        uint64_t at1[kUnroll], at2[kUnroll];
        int32_t xs[kUnroll], ys[kUnroll], zs[kUnroll];
        bool ok[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u)
        {
            uint32_t local = base + u * NT;
            ok[u] = !GUARD || local < g.items;
            if (GUARD && !ok[u])
                local = 0;
            uint32_t c;
            rowOf(g, local, c, ys[u], zs[u]);
            xs[u] = g.x0 + static_cast<int32_t>(c) * V;
            at1[u] = byteOf(v1, xs[u], ys[u], zs[u], BPV);
            w1[u] = __builtin_nontemporal_load(reinterpret_cast<u32x4 const*>(v1.data + at1[u]));
            if constexpr (!ALIAS)
            {
                at2[u] = byteOf(v2, xs[u], ys[u], zs[u], BPV);
                w2[u] = __builtin_nontemporal_load(reinterpret_cast<u32x4 const*>(v2.data + at2[u]));
            }
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u)
        {
            u32x4 o1 = {0u, 0u, 0u, 0u}, o2 = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int k = 0; k < V; ++k)
            {
                uint8_t b1[8], b2[8];
                unpack<BPV>(w1[u], k, b1);
                unpack<BPV>(ALIAS ? w1[u] : w2[u], k, b2);
                if (!PAD || (xs[u] + k >= g.rx0 && xs[u] + k < g.rx1))
                {
                    VoxelView voxel1{b1, v1.format, v1.lo, v1.hi};
                    VoxelView voxel2{b2, v2.format, v2.lo, v2.hi};
                    op(xs[u] + k, ys[u], zs[u], voxel1, voxel2);
                }
                if constexpr (!ALIAS)
                    pack<BPV>(o1, k, b1);
                pack<BPV>(o2, k, b2);
            }
            if (!GUARD || ok[u])
            {
                if constexpr (ALIAS)
                    __builtin_nontemporal_store(o2, reinterpret_cast<u32x4*>(v1.data + at1[u]));
                else
                {
                    __builtin_nontemporal_store(o1, reinterpret_cast<u32x4*>(v1.data + at1[u]));
                    __builtin_nontemporal_store(o2, reinterpret_cast<u32x4*>(v2.data + at2[u]));
                }
            }
        }
    }

    // ---- binary, one voxel per lane (any formats) ----------------------------------------
    template <int B1, int B2, bool ALIAS, class Op>
    __global__ void __launch_bounds__(kBlock) binaryRowKernel(Vol v1, Vol v2, Rows g, Op op)
    {
        uint32_t c;
        int32_t y, z;
        rowOf(g, blockIdx.x, c, y, z);
        uint32_t xr = c * kBlock + threadIdx.x;
        if (xr >= g.nx)
            return;
        int32_t x = g.x0 + static_cast<int32_t>(xr);
        uint8_t* p1 = v1.data + byteOf(v1, x, y, z, B1);
        uint8_t* p2 = v2.data + byteOf(v2, x, y, z, B2);
        uint8_t b1[8], b2[8];
        loadVoxel<B1>(p1, b1);
        if constexpr (ALIAS)
        {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                b2[i] = b1[i];
        }
        else
            loadVoxel<B2>(p2, b2);
        VoxelView voxel1{b1, v1.format, v1.lo, v1.hi};
        VoxelView voxel2{b2, v2.format, v2.lo, v2.hi};
        op(x, y, z, voxel1, voxel2);
        if constexpr (!ALIAS)
            storeVoxel<B1>(p1, b1);
        storeVoxel<B2>(p2, b2);
    }

    // ---- host side -----------------------------------------------------------------------
    inline int bytesPerVoxel(DataFormat f) { return static_cast<int>(codec::bytesPerVoxel(static_cast<int32_t>(f))); }

    inline Vol volOf(StructuredVolume& s)
    {
        Vol v;
        // migrates to the device first (GPU policy); nullptr when that failed (bytes stay on the host)
        v.data = s.getDataFor(GetThreadExecutionPolicy());
        Vec3i d = s.getDims();
        v.dimX = static_cast<uint64_t>(d.x);
        v.dimY = static_cast<uint64_t>(d.y);
        v.format = s.getDataFormat();
        Vec2f m = s.getVoxelMapping();
        v.lo = m.x;
        v.hi = m.y;
        return v;
    }

    inline bool inside(StructuredVolume& s, Vec3i first, Vec3i last)
    {
        Vec3i d = s.getDims();
        return first.x >= 0 && first.y >= 0 && first.z >= 0 && last.x <= d.x && last.y <= d.y && last.z <= d.z;
    }

    inline bool vec16(Vol const& v, int32_t x0, uint32_t nx, int bpv)
    {
        return (reinterpret_cast<uintptr_t>(v.data) & 15u) == 0 && (static_cast<uint64_t>(x0) * bpv) % 16 == 0 &&
               (static_cast<uint64_t>(nx) * bpv) % 16 == 0 && (v.dimX * bpv) % 16 == 0;
    }

    // A 16-B-aligned range whose rows do not start and end on 64-B sectors still takes the
    // padded launch when the layout allows sectors: a partly written sector costs HBM a
    // read-modify-write (measured, TransformRange x 16..1008 of 1024^3 UInt8: 0.51 of peak on
    // 16-B items vs 0.74 for the sector-padded 2..1022).
    inline int padUnit(Vol const& v, int bpv);
    inline bool sectorAligned(Vol const& v, int32_t x0, uint32_t nx, int bpv)
    {
        return padUnit(v, bpv) != 64 ||
               ((static_cast<uint64_t>(x0) * bpv) % 64 == 0 && (static_cast<uint64_t>(nx) * bpv) % 64 == 0);
    }

    // Padding unit for a range that vec16 refuses: rows start on 16-B (64-B) boundaries, so a
    // row's chunks belong to that row alone; 0 = no padded launch.
    inline int padUnit(Vol const& v, int bpv)
    {
        uintptr_t const a = reinterpret_cast<uintptr_t>(v.data);
        if (a % 64 == 0 && (v.dimX * bpv) % 64 == 0)
            return 64;
        if (a % 16 == 0 && (v.dimX * bpv) % 16 == 0)
            return 16;
        return 0;
    }

    // first/last widened to whole units of the row (x in voxels)
    inline void padRange(Vec3i& first, Vec3i& last, int unit, int bpv)
    {
        int const vu = unit / bpv;
        first.x = first.x / vu * vu;
        last.x = (last.x + vu - 1) / vu * vu;
    }

    // Calls launch(Rows, grid) for row ranges of at most kMaxItemsPerLaunch items.
    template <class Launch>
    hipError_t forRows(Vec3i first, Vec3i last, uint32_t perRow, Launch&& launch)
    {
        uint32_t nx = static_cast<uint32_t>(last.x - first.x);
        uint32_t ny = static_cast<uint32_t>(last.y - first.y);
        uint64_t rows = static_cast<uint64_t>(ny) * static_cast<uint32_t>(last.z - first.z);
        uint64_t rowsPerLaunch = kMaxItemsPerLaunch / perRow;
        if (rowsPerLaunch < 1)
            rowsPerLaunch = 1;
        for (uint64_t r0 = 0; r0 < rows; r0 += rowsPerLaunch)
        {
            uint64_t nr = rows - r0 < rowsPerLaunch ? rows - r0 : rowsPerLaunch;
            Rows g;
            g.x0 = first.x;
            g.y0 = first.y;
            g.z0 = first.z;
            g.nx = nx;
            g.rx0 = first.x;
            g.rx1 = last.x;
            g.row0 = static_cast<uint32_t>(r0);
            g.items = nr * perRow;
            g.perRow = makeFastDiv(perRow);
            g.ny = makeFastDiv(ny);
            hipError_t e = launch(g);
            if (e != hipSuccess)
                return e;
        }
        return hipSuccess;
    }

    // Workgroup shape of the 16-B vector kernels, knob transform.shape: 0 = 256 threads x 4 items
    // (16 KiB per stream per workgroup), 1 = one wave x 2 items (2 KiB), 2 = one wave x 1 item
    // (1 KiB) -- the pointwise engine's measured sweet spot for streaming ops is one-wave
    // workgroups of 1-2 KiB per stream.
    inline int vecShape()
    {
        int64_t k = 0;
        if (vktHipGetTuningKnob("transform.shape", &k) != vktNoError || k < 0 || k > 2)
            k = 0;
        return static_cast<int>(k);
    }

    // Whole workgroups without guards, then the remainder with guards:
    // launch(guarded, itemBase, blocks, NT, U) enqueues one kernel (NT / U as integral constants).
    template <class Launch>
    void launchVec(Rows const& g, Launch&& launch)
    {
        auto run = [&](auto nt, auto u) {
            constexpr uint64_t perBlock = uint64_t(decltype(nt)::value) * decltype(u)::value;
            uint64_t full = g.items / perBlock;
            if (full > 0)
                launch(false, 0u, static_cast<uint32_t>(full), nt, u);
            uint64_t done = full * perBlock;
            if (done < g.items)
                launch(true, static_cast<uint32_t>(done), static_cast<uint32_t>((g.items - done + perBlock - 1) / perBlock),
                       nt, u);
        };
        switch (vecShape())
        {
        case 1: run(std::integral_constant<int, 64>{}, std::integral_constant<int, 2>{}); break;
        case 2: run(std::integral_constant<int, 64>{}, std::integral_constant<int, 1>{}); break;
        default: run(std::integral_constant<int, kBlock>{}, std::integral_constant<int, kUnroll>{}); break;
        }
    }

    struct Scope
    {
        vktHipKernelScope h = nullptr;
        hipStream_t stream = nullptr;
        Error begin(char const* name)
        {
            void* s = nullptr;
            if (vktHipKernelScopeBegin(name, &h, &s) != vktNoError)
                return InvalidValue;
            stream = static_cast<hipStream_t>(s);
            return NoError;
        }
        Error end() { return static_cast<Error>(vktHipKernelScopeEnd(h)); }
    };
} // transform_detail

    // Callables that are not function pointers/references: functors with a __device__
    // operator() and __device__ lambdas.  Function pointers keep the library overloads.
    template <class Op>
    using EnableIfDeviceOp =
        typename std::enable_if<!std::is_pointer<typename std::decay<Op>::type>::value &&
                                    !std::is_function<typename std::remove_reference<Op>::type>::value,
                                int>::type;

    //! TransformRange with a device functor (unary; reference Transform.hpp:42-46)
    template <class Op, EnableIfDeviceOp<Op> = 0>
    Error TransformRange(StructuredVolume& volume, Vec3i first, Vec3i last, Op op)
    {
        using namespace transform_detail;
        Scope scope;
        if (scope.begin("TransformRange_hip") != NoError)
            return InvalidValue;
        if (!inside(volume, first, last))
        {
            scope.end();
            return static_cast<Error>(vktHipReportError("TransformRange_hip: range outside the volume"));
        }
        if (last.x <= first.x || last.y <= first.y || last.z <= first.z)
            return scope.end();
        Vol v = volOf(volume);
        if (v.data == nullptr)
        {
            scope.end();
            return static_cast<Error>(vktHipReportError("TransformRange_hip: the volume is not in HBM (its migration failed)"));
        }
        int bpv = bytesPerVoxel(v.format);
        if (bpv != 1 && bpv != 2 && bpv != 4)
        {
            scope.end();
            return static_cast<Error>(vktHipReportError("TransformRange_hip: unsupported data format"));
        }
        uint32_t nx = static_cast<uint32_t>(last.x - first.x);
        hipStream_t s = scope.stream;
        hipError_t err = hipSuccess;
        bool const aligned = vec16(v, first.x, nx, bpv) && sectorAligned(v, first.x, nx, bpv);
        int const unit = aligned ? 0 : padUnit(v, bpv);
        if (aligned || unit != 0)
        {
            Vec3i pf = first, pl = last;
            if (!aligned)
                padRange(pf, pl, unit, bpv);
            uint32_t perRow = static_cast<uint32_t>(pl.x - pf.x) * bpv / 16;
            err = forRows(pf, pl, perRow, [&](Rows const& gp) {
                Rows g = gp;
                g.rx0 = first.x;
                g.rx1 = last.x;
                launchVec(g, [&](bool guard, uint32_t base, uint32_t blocks, auto ntc, auto uc) {
                    constexpr int NT = decltype(ntc)::value, U = decltype(uc)::value;
                    dim3 grid(blocks), block(NT);
#define VKT_UN_VEC_(B, G, P) unaryVecKernel<B, G, P, NT, U><<<grid, block, 0, s>>>(v, g, base, op)
#define VKT_UN_VEC_B_(B)                                                               \
    (aligned ? (guard ? VKT_UN_VEC_(B, true, false) : VKT_UN_VEC_(B, false, false))    \
             : (guard ? VKT_UN_VEC_(B, true, true) : VKT_UN_VEC_(B, false, true)))
                    if (bpv == 1)
                        VKT_UN_VEC_B_(1);
                    else if (bpv == 2)
                        VKT_UN_VEC_B_(2);
                    else
                        VKT_UN_VEC_B_(4);
#undef VKT_UN_VEC_B_
#undef VKT_UN_VEC_
                });
                return hipPeekAtLastError();
            });
        }
        else
        {
            uint32_t perRow = (nx + kBlock - 1) / kBlock;
            err = forRows(first, last, perRow, [&](Rows const& g) {
                dim3 grid(static_cast<uint32_t>(g.items)), block(kBlock);
                if (bpv == 1)
                    unaryRowKernel<1><<<grid, block, 0, s>>>(v, g, op);
                else if (bpv == 2)
                    unaryRowKernel<2><<<grid, block, 0, s>>>(v, g, op);
                else
                    unaryRowKernel<4><<<grid, block, 0, s>>>(v, g, op);
                return hipPeekAtLastError();
            });
        }
        (void)err;   // launch errors stay pending (peeked, not cleared) for scope.end()
        return scope.end();
    }

    template <class Op, EnableIfDeviceOp<Op> = 0>
    Error TransformRange(StructuredVolume& volume, int32_t firstX, int32_t firstY, int32_t firstZ, int32_t lastX,
                         int32_t lastY, int32_t lastZ, Op op)
    {
        return TransformRange(volume, Vec3i{firstX, firstY, firstZ}, Vec3i{lastX, lastY, lastZ}, op);
    }

    //! Transform with a device functor over the whole volume (reference Transform.hpp:30-31)
    template <class Op, EnableIfDeviceOp<Op> = 0>
    Error Transform(StructuredVolume& volume, Op op)
    {
        return TransformRange(volume, Vec3i{0, 0, 0}, volume.getDims(), op);
    }

    //! TransformRange with a device functor (binary; reference Transform.hpp:48-62): volume2
    //! is visited at the same (x, y, z) as volume1.
    template <class Op, EnableIfDeviceOp<Op> = 0>
    Error TransformRange(StructuredVolume& volume1, StructuredVolume& volume2, Vec3i first, Vec3i last, Op op)
    {
        using namespace transform_detail;
        Scope scope;
        if (scope.begin("TransformRange_hip") != NoError)
            return InvalidValue;
        if (!inside(volume1, first, last) || !inside(volume2, first, last))
        {
            scope.end();
            return static_cast<Error>(vktHipReportError("TransformRange_hip: range outside a volume"));
        }
        if (last.x <= first.x || last.y <= first.y || last.z <= first.z)
            return scope.end();
        Vol a = volOf(volume1);
        Vol b = volOf(volume2);
        if (a.data == nullptr || b.data == nullptr)
        {
            scope.end();
            return static_cast<Error>(vktHipReportError("TransformRange_hip: a volume is not in HBM (its migration failed)"));
        }
        int b1 = bytesPerVoxel(a.format), b2 = bytesPerVoxel(b.format);
        if ((b1 != 1 && b1 != 2 && b1 != 4) || (b2 != 1 && b2 != 2 && b2 != 4))
        {
            scope.end();
            return static_cast<Error>(vktHipReportError("TransformRange_hip: unsupported data format"));
        }
        bool alias = a.data == b.data;
        if (alias && (a.dimX != b.dimX || a.dimY != b.dimY || b1 != b2))
        {
            scope.end();
            return static_cast<Error>(vktHipReportError("TransformRange_hip: aliased volumes with different layouts"));
        }
        uint32_t nx = static_cast<uint32_t>(last.x - first.x);
        hipStream_t s = scope.stream;
        bool const aligned = b1 == b2 && vec16(a, first.x, nx, b1) && vec16(b, first.x, nx, b2) &&
                             sectorAligned(a, first.x, nx, b1) && sectorAligned(b, first.x, nx, b2);
        int const ua = b1 == b2 && !aligned ? padUnit(a, b1) : 0, ub = b1 == b2 && !aligned ? padUnit(b, b2) : 0;
        int const unit = ua < ub ? ua : ub;
        if (aligned || unit != 0)
        {
            Vec3i pf = first, pl = last;
            if (!aligned)
                padRange(pf, pl, unit, b1);
            uint32_t perRow = static_cast<uint32_t>(pl.x - pf.x) * b1 / 16;
            (void)forRows(pf, pl, perRow, [&](Rows const& gp) {
                Rows g = gp;
                g.rx0 = first.x;
                g.rx1 = last.x;
                launchVec(g, [&](bool guard, uint32_t base, uint32_t blocks, auto ntc, auto uc) {
                    constexpr int NT = decltype(ntc)::value, U = decltype(uc)::value;
                    dim3 grid(blocks), block(NT);
#define VKT_BIN_VEC_(B, G, A, P) binaryVecKernel<B, G, A, P, NT, U><<<grid, block, 0, s>>>(a, b, g, base, op)
#define VKT_BIN_VEC_P_(B, P)                                                                    \
    (alias ? (guard ? VKT_BIN_VEC_(B, true, true, P) : VKT_BIN_VEC_(B, false, true, P))         \
           : (guard ? VKT_BIN_VEC_(B, true, false, P) : VKT_BIN_VEC_(B, false, false, P)))
#define VKT_BIN_VEC_B_(B) (aligned ? VKT_BIN_VEC_P_(B, false) : VKT_BIN_VEC_P_(B, true))
                    if (b1 == 1)
                        VKT_BIN_VEC_B_(1);
                    else if (b1 == 2)
                        VKT_BIN_VEC_B_(2);
                    else
                        VKT_BIN_VEC_B_(4);
#undef VKT_BIN_VEC_B_
#undef VKT_BIN_VEC_P_
#undef VKT_BIN_VEC_
                });
                return hipPeekAtLastError();
            });
        }
        else
        {
            uint32_t perRow = (nx + kBlock - 1) / kBlock;
            (void)forRows(first, last, perRow, [&](Rows const& g) {
                dim3 grid(static_cast<uint32_t>(g.items)), block(kBlock);
                auto run = [&](auto B1c, auto B2c) {
                    constexpr int B1 = decltype(B1c)::value, B2 = decltype(B2c)::value;
                    if constexpr (B1 == B2)
                    {
                        if (alias)
                        {
                            binaryRowKernel<B1, B2, true><<<grid, block, 0, s>>>(a, b, g, op);
                            return;
                        }
                    }
                    binaryRowKernel<B1, B2, false><<<grid, block, 0, s>>>(a, b, g, op);
                };
                using I1 = std::integral_constant<int, 1>;
                using I2 = std::integral_constant<int, 2>;
                using I4 = std::integral_constant<int, 4>;
                auto second = [&](auto B1c) {
                    if (b2 == 1)
                        run(B1c, I1{});
                    else if (b2 == 2)
                        run(B1c, I2{});
                    else
                        run(B1c, I4{});
                };
                if (b1 == 1)
                    second(I1{});
                else if (b1 == 2)
                    second(I2{});
                else
                    second(I4{});
                return hipPeekAtLastError();
            });
        }
        return scope.end();
    }

    template <class Op, EnableIfDeviceOp<Op> = 0>
    Error TransformRange(StructuredVolume& volume1, StructuredVolume& volume2, int32_t firstX, int32_t firstY,
                         int32_t firstZ, int32_t lastX, int32_t lastY, int32_t lastZ, Op op)
    {
        return TransformRange(volume1, volume2, Vec3i{firstX, firstY, firstZ}, Vec3i{lastX, lastY, lastZ}, op);
    }

    //! Transform with a device functor over volume1's dims (binary)
    template <class Op, EnableIfDeviceOp<Op> = 0>
    Error Transform(StructuredVolume& volume1, StructuredVolume& volume2, Op op)
    {
        return TransformRange(volume1, volume2, Vec3i{0, 0, 0}, volume1.getDims(), op);
    }

    //! A functor seen through a Z shift: z + dz is passed on (a slab's first global plane).
    template <class Op>
    struct ZShifted
    {
        Op op;
        int32_t dz;
        __device__ void operator()(int32_t x, int32_t y, int32_t z, VoxelView voxel) { op(x, y, z + dz, voxel); }
    };

    //! TransformRange with a device functor over a Z-slab partitioned volume (Transform shards
    //! with no exchange).  `slab` holds global planes [z0, z0 + dimZ) of a volume
    //! globalDimZ deep, split over nranks by the ceil partition of vktHipSlabExchangeHalo; rank
    //! `rank` transforms the planes it OWNS of the GLOBAL range [first, last), and the functor
    //! sees global coordinates.  Host-callback twin: vktHipSlabTransformRange1.
    template <class Op, EnableIfDeviceOp<Op> = 0>
    Error TransformRangeSlab(int32_t nranks, int32_t rank, StructuredVolume& slab, int32_t z0, int32_t globalDimZ,
                             Vec3i first, Vec3i last, Op op)
    {
        if (nranks <= 0 || rank < 0 || rank >= nranks || globalDimZ < 0)
            return static_cast<Error>(vktHipReportError("TransformRangeSlab: invalid rank / nranks"));
        if (last.x <= first.x || last.y <= first.y || last.z <= first.z)
            return NoError;
        if (first.z < 0 || last.z > globalDimZ)
            return static_cast<Error>(vktHipReportError("TransformRangeSlab: range outside the volume"));
        int64_t const size = (static_cast<int64_t>(globalDimZ) + nranks - 1) / nranks;
        int64_t const d0 = std::min<int64_t>(rank * size, globalDimZ), d1 = std::min<int64_t>(d0 + size, globalDimZ);
        int64_t const zb = std::max<int64_t>(first.z, d0), ze = std::min<int64_t>(last.z, d1);
        if (ze <= zb)
            return NoError;
        if (zb < z0 || ze > static_cast<int64_t>(z0) + slab.getDims().z)
            return static_cast<Error>(vktHipReportError("TransformRangeSlab: slab does not hold its owned planes"));
        return TransformRange(slab, Vec3i{first.x, first.y, static_cast<int32_t>(zb - z0)},
                              Vec3i{last.x, last.y, static_cast<int32_t>(ze - z0)}, ZShifted<Op>{op, z0});
    }
} // vkt
