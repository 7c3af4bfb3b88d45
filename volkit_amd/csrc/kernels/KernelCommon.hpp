// KernelCommon.hpp -- device-side helpers shared by the gfx950 kernels.
//
// All kernels are bandwidth-bound byte/integer/f32 streams (no MFMA): they are written for
// 64-lane waves, 16-byte-per-lane coalesced accesses where alignment allows, grid-stride
// loops sized to fill 256 CUs, and nontemporal stores for outputs that are not re-read.
#pragma once

#include <cstdint>
#include <hip/hip_runtime.h>

#include "volkit_codec.hpp"

namespace vkt
{
namespace hipk
{
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

    constexpr int kBlock = 256;          // 4 waves of 64
    constexpr int kNumCUs = 256;         // MI355X: 8 XCDs x 32 CUs

    // Grid for a grid-stride streaming kernel: enough workgroups for ~8 per CU, never more
    // than the work needs.
    inline unsigned streamingGrid(uint64_t items, unsigned itemsPerBlock, unsigned maxBlocksPerCU = 8)
    {
        uint64_t need = (items + itemsPerBlock - 1) / itemsPerBlock;
        uint64_t cap = static_cast<uint64_t>(kNumCUs) * maxBlocksPerCU;
        if (need < 1)
            need = 1;
        return static_cast<unsigned>(need < cap ? need : cap);
    }

    // Division by a run-time constant for 32-bit operands: q = (umulhi(n, m) + n) >> l with
    // l = ceil(log2 d), m = floor(2^32 (2^l - d) / d) + 1 (exact for every 32-bit n).  Replaces
    // the ~40-instruction 64-bit divide in per-item index decomposition.
    struct FastDiv
    {
        uint32_t d, m, l;
    };

    __host__ __device__ inline FastDiv makeFastDiv(uint32_t d)
    {
        FastDiv f{d, 0u, 0u};
        if (d == 0)
            return f;
        uint32_t const l = d <= 1 ? 0u : 32u - static_cast<uint32_t>(__builtin_clz(d - 1));   // ceil(log2 d)
        f.l = l;
        f.m = static_cast<uint32_t>(((1ull << 32) * ((1ull << l) - d)) / d + 1);
        return f;
    }

    __device__ __forceinline__ uint32_t fdiv(uint32_t n, FastDiv const& f)
    {
        uint64_t hi = __umulhi(n, f.m);
        return static_cast<uint32_t>((hi + n) >> f.l);
    }

    // ---- scalar code access -----------------------------------------------------------
    template <int BPV>
    __device__ __forceinline__ uint32_t loadCode(uint8_t const* base, uint64_t voxel)
    {
        if constexpr (BPV == 1)
            return base[voxel];
        else if constexpr (BPV == 2)
            return reinterpret_cast<uint16_t const*>(base)[voxel];
        else
            return reinterpret_cast<uint32_t const*>(base)[voxel];
    }

    template <int BPV>
    __device__ __forceinline__ void storeCode(uint8_t* base, uint64_t voxel, uint32_t code)
    {
        if constexpr (BPV == 1)
            base[voxel] = static_cast<uint8_t>(code);
        else if constexpr (BPV == 2)
            reinterpret_cast<uint16_t*>(base)[voxel] = static_cast<uint16_t>(code);
        else
            reinterpret_cast<uint32_t*>(base)[voxel] = code;
    }

    // Runtime bytes-per-voxel versions (wave-uniform branch).
    __device__ __forceinline__ uint32_t loadCodeDyn(uint8_t const* base, uint64_t voxel, uint32_t bpv)
    {
        return bpv == 1 ? loadCode<1>(base, voxel) : bpv == 2 ? loadCode<2>(base, voxel) : loadCode<4>(base, voxel);
    }

    __device__ __forceinline__ void storeCodeDyn(uint8_t* base, uint64_t voxel, uint32_t bpv, uint32_t code)
    {
        if (bpv == 1)
            storeCode<1>(base, voxel, code);
        else if (bpv == 2)
            storeCode<2>(base, voxel, code);
        else
            storeCode<4>(base, voxel, code);
    }

    // ---- 8 consecutive codes per lane ------------------------------------------------
    // BPV 1: one 8-byte load; BPV 2: one 16-byte load; BPV 4: two 16-byte loads.
    // Nontemporal only for 16-byte vectors: narrower nt/sc1 loads run at 0.54-0.70x the
    // 16-byte rate on gfx950 (MI355X_MICROARCH.md, inter-workgroup visibility table), and a
    // resample source read with 8-byte nt loads measured 0.44 ms vs 0.35 ms with plain loads.
    template <class V, bool NT>
    __device__ __forceinline__ V loadVec(void const* p)
    {
        if constexpr (NT && sizeof(V) >= 16)
            return __builtin_nontemporal_load(reinterpret_cast<V const*>(p));
        else
            return *reinterpret_cast<V const*>(p);
    }

    template <int BPV, bool NT = false>
    __device__ __forceinline__ void load8(uint8_t const* base, uint64_t voxel, uint32_t (&c)[8])
    {
        if constexpr (BPV == 1)
        {
            u32x2 v = loadVec<u32x2, NT>(base + voxel);
#pragma unroll
            for (int i = 0; i < 4; ++i)
            {
                c[i] = (v.x >> (8 * i)) & 0xFFu;
                c[4 + i] = (v.y >> (8 * i)) & 0xFFu;
            }
        }
        else if constexpr (BPV == 2)
        {
            u32x4 v = loadVec<u32x4, NT>(base + 2 * voxel);
            c[0] = v.x & 0xFFFFu; c[1] = v.x >> 16;
            c[2] = v.y & 0xFFFFu; c[3] = v.y >> 16;
            c[4] = v.z & 0xFFFFu; c[5] = v.z >> 16;
            c[6] = v.w & 0xFFFFu; c[7] = v.w >> 16;
        }
        else
        {
            u32x4 a = loadVec<u32x4, NT>(base + 4 * voxel);
            u32x4 b = loadVec<u32x4, NT>(base + 4 * voxel + 16);
            c[0] = a.x; c[1] = a.y; c[2] = a.z; c[3] = a.w;
            c[4] = b.x; c[5] = b.y; c[6] = b.z; c[7] = b.w;
        }
    }

    // N consecutive codes (N*BPV bytes in {1,2,4,8,16,32}, naturally aligned) -> c[0..N)
    template <int BPV, int N, bool NT>
    __device__ __forceinline__ void loadN(uint8_t const* base, uint64_t voxel, uint32_t* c)
    {
        constexpr int kBytes = BPV * N;
        uint8_t const* p = base + voxel * BPV;
        uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if constexpr (kBytes == 32)
        {
            u32x4 x = loadVec<u32x4, NT>(p), y = loadVec<u32x4, NT>(p + 16);
            w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w;
            w[4] = y.x; w[5] = y.y; w[6] = y.z; w[7] = y.w;
        }
        else if constexpr (kBytes == 16)
        {
            u32x4 x = loadVec<u32x4, NT>(p);
            w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w;
        }
        else if constexpr (kBytes == 8)
        {
            u32x2 x = loadVec<u32x2, NT>(p);
            w[0] = x.x; w[1] = x.y;
        }
        else if constexpr (kBytes == 4)
            w[0] = loadVec<uint32_t, NT>(p);
        else if constexpr (kBytes == 2)
            w[0] = *reinterpret_cast<uint16_t const*>(p);
        else
            w[0] = *p;
        constexpr uint32_t kMask = BPV == 4 ? 0xFFFFFFFFu : ((1u << (8 * BPV)) - 1u);
#pragma unroll
        for (int i = 0; i < N; ++i)
        {
            constexpr int kBits = 8 * BPV;
            int off = i * kBits;
            c[i] = (w[off / 32] >> (off % 32)) & kMask;
        }
    }

    template <int BPV, bool NT>
    __device__ __forceinline__ void store8(uint8_t* base, uint64_t voxel, uint32_t const (&c)[8])
    {
        if constexpr (BPV == 1)
        {
            u32x2 v;
            v.x = c[0] | c[1] << 8 | c[2] << 16 | c[3] << 24;
            v.y = c[4] | c[5] << 8 | c[6] << 16 | c[7] << 24;
            u32x2* p = reinterpret_cast<u32x2*>(base + voxel);
            if constexpr (NT) __builtin_nontemporal_store(v, p); else *p = v;
        }
        else if constexpr (BPV == 2)
        {
            u32x4 v;
            v.x = c[0] | c[1] << 16; v.y = c[2] | c[3] << 16;
            v.z = c[4] | c[5] << 16; v.w = c[6] | c[7] << 16;
            u32x4* p = reinterpret_cast<u32x4*>(base + 2 * voxel);
            if constexpr (NT) __builtin_nontemporal_store(v, p); else *p = v;
        }
        else
        {
            u32x4 a, b;
            a.x = c[0]; a.y = c[1]; a.z = c[2]; a.w = c[3];
            b.x = c[4]; b.y = c[5]; b.z = c[6]; b.w = c[7];
            u32x4* p = reinterpret_cast<u32x4*>(base + 4 * voxel);
            if constexpr (NT) { __builtin_nontemporal_store(a, p); __builtin_nontemporal_store(b, p + 1); }
            else { p[0] = a; p[1] = b; }
        }
    }

    // 16 bytes of codes per lane (V = 16 / BPV voxels), nontemporal: the store layout of
    // every streaming writer -- lane l of a wave-instruction writes bytes [16l, 16l + 16) of
    // one contiguous KiB.
    template <int BPV>
    __device__ __forceinline__ void store16(uint8_t* base, uint64_t voxel, uint32_t const* c)
    {
        u32x4 v;
        if constexpr (BPV == 1)
        {
            uint32_t w[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                w[i] = c[4 * i] | c[4 * i + 1] << 8 | c[4 * i + 2] << 16 | c[4 * i + 3] << 24;
            v.x = w[0]; v.y = w[1]; v.z = w[2]; v.w = w[3];
        }
        else if constexpr (BPV == 2)
        {
            v.x = c[0] | c[1] << 16; v.y = c[2] | c[3] << 16;
            v.z = c[4] | c[5] << 16; v.w = c[6] | c[7] << 16;
        }
        else
        {
            v.x = c[0]; v.y = c[1]; v.z = c[2]; v.w = c[3];
        }
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(base + voxel * BPV));
    }

    // Bytes [lo, hi) (0 <= lo < hi <= 16) of the 16-B vector v to the 16-B aligned address p,
    // as naturally aligned 1/2/4/8-B pieces (at most 4 leading pieces that align the start, then
    // at most 4 trailing ones): no byte outside the range is written.  A row end of a UInt8 box
    // costs 1-3 stores instead of one byte store per voxel; the byte extraction is shifts of
    // the two 64-bit halves (no dynamically indexed register array).
    __device__ __forceinline__ void storeByteRange16(uint8_t* p, u32x4 v, int lo, int hi)
    {
        uint64_t const q0 = static_cast<uint64_t>(v.x) | static_cast<uint64_t>(v.y) << 32;
        uint64_t const q1 = static_cast<uint64_t>(v.z) | static_cast<uint64_t>(v.w) << 32;
        auto at = [&](int a) -> uint64_t {   // the (up to) 8 bytes starting at byte a
            uint64_t const l = (a & 8) ? q1 : q0, h = (a & 8) ? 0ull : q1;
            uint32_t const s = static_cast<uint32_t>(a & 7) * 8u;
            return s ? (l >> s) | (h << (64u - s)) : l;
        };
        int a = lo;
        if ((a & 1) && a < hi)
        {
            __builtin_nontemporal_store(static_cast<uint8_t>(at(a)), p + a);
            a += 1;
        }
        if ((a & 2) && a + 2 <= hi)
        {
            __builtin_nontemporal_store(static_cast<uint16_t>(at(a)), reinterpret_cast<uint16_t*>(p + a));
            a += 2;
        }
        if ((a & 4) && a + 4 <= hi)
        {
            __builtin_nontemporal_store(static_cast<uint32_t>(at(a)), reinterpret_cast<uint32_t*>(p + a));
            a += 4;
        }
        if ((a & 8) && a + 8 <= hi)
        {
            __builtin_nontemporal_store(at(a), reinterpret_cast<uint64_t*>(p + a));
            a += 8;
        }
        if (hi - a >= 8)
        {
            __builtin_nontemporal_store(at(a), reinterpret_cast<uint64_t*>(p + a));
            a += 8;
        }
        if (hi - a >= 4)
        {
            __builtin_nontemporal_store(static_cast<uint32_t>(at(a)), reinterpret_cast<uint32_t*>(p + a));
            a += 4;
        }
        if (hi - a >= 2)
        {
            __builtin_nontemporal_store(static_cast<uint16_t>(at(a)), reinterpret_cast<uint16_t*>(p + a));
            a += 2;
        }
        if (hi - a >= 1)
            __builtin_nontemporal_store(static_cast<uint8_t>(at(a)), p + a);
    }

    // Bytes [lo, hi) of v, the others from own (0 <= lo <= hi <= 16; lo == hi: own only).
    __device__ __forceinline__ u32x4 mergeBytes16(u32x4 v, u32x4 own, int lo, int hi)
    {
        auto m = [&](int dw) -> uint32_t {   // byte mask of dword dw: bytes 4dw..4dw+3 in [lo, hi)
            int const a = lo - 4 * dw, b = hi - 4 * dw;
            uint32_t const ma = a <= 0 ? 0xFFFFFFFFu : (a >= 4 ? 0u : 0xFFFFFFFFu << (8 * a));
            uint32_t const mb = b >= 4 ? 0xFFFFFFFFu : (b <= 0 ? 0u : 0xFFFFFFFFu >> (8 * (4 - b)));
            return ma & mb;
        };
        uint32_t const m0 = m(0), m1 = m(1), m2 = m(2), m3 = m(3);
        return u32x4{(v.x & m0) | (own.x & ~m0), (v.y & m1) | (own.y & ~m1), (v.z & m2) | (own.z & ~m2),
                     (v.w & m3) | (own.w & ~m3)};
    }

    // XCD-aware block order (guide §5.5 T1): hardware deals workgroups round-robin over the
    // 8 XCDs, so block b and b+8 share an L2.  Remap so each XCD walks one contiguous band of
    // logical blocks -- neighbouring rows then hit the same L2.  Speed only, never correctness.
    __device__ __forceinline__ uint32_t xcdSwizzle(uint32_t b, uint32_t nblocks)
    {
        uint32_t per = nblocks / 8u;
        if (per == 0u || b >= per * 8u)
            return b;
        return (b % 8u) * per + b / 8u;
    }

} // hipk
} // vkt
