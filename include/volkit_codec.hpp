// volkit_codec.hpp -- float <-> stored-code mapping, bit-exact with the reference serial path.
//
// Restates MapVoxelImpl / UnmapVoxelImpl (reference src/vkt/VoxelMapping.hpp:15-95, 98-177)
// with every implementation-defined step made explicit, so host code (gcc/clang x86-64)
// and gfx950 device code produce the same bits:
//  * float -> int conversions: the reference assigns floats to int8/int16/uint32 lvalues,
//    which gcc on x86-64 compiles to cvttss2si (32-bit; 64-bit for uint32) and keeps the
//    low bits.  Out-of-range and NaN give the "integer indefinite" value INT_MIN.  gfx950's
//    v_cvt_i32_f32 saturates and maps NaN to 0 instead, hence cvtt_i32/cvtt_i64 below.
//  * lerp(a,b,t) = (1-t)*a + t*b and clamp(x,lo,hi) = max(lo, min(x,hi)) with the
//    reference's `b < a ? b : a` min / `a < b ? b : a` max (src/vkt/linalg.hpp:18-41):
//    NaN clamps to lo, and +-0 ordering follows the ternaries, not fminf/fmaxf.
//  * no FMA contraction anywhere (built with -ffp-contract=off) and IEEE division.
//
// Everything here is __host__ __device__ and header-only; it is compiled by hipcc only.
#pragma once

#include <cstdint>
#include <hip/hip_runtime.h>

#define VKT_HD __host__ __device__ __forceinline__
// The reference rounds every f32 operation separately (x86 SSE, no FMA).  The library is
// built with -ffp-contract=off; this header is also included by user translation units
// (volkit_transform.hpp), where hipcc contracts a*b+c into FMAs by default, so every
// function with a multiply feeding an add turns contraction off for its own body.
#define VKT_NO_CONTRACT _Pragma("clang fp contract(off)")

namespace vkt
{
namespace codec
{
    // DataFormat values (reference include/cpp/vkt/common.hpp:53-66).
    enum : int32_t
    {
        FmtUnspecified = 0, FmtInt8 = 1, FmtInt16 = 2, FmtInt32 = 3,
        FmtUInt8 = 4, FmtUInt16 = 5, FmtUInt32 = 6, FmtFloat32 = 7,
    };

    // Bytes per voxel (reference src/vkt/DataFormatInfo.hpp:34-47; 255 for unknown).
    VKT_HD constexpr uint32_t bytesPerVoxel(int32_t fmt)
    {
        return (fmt == FmtInt8 || fmt == FmtUInt8) ? 1u
             : (fmt == FmtInt16 || fmt == FmtUInt16) ? 2u
             : (fmt == FmtInt32 || fmt == FmtUInt32 || fmt == FmtFloat32) ? 4u
             : 255u;
    }

    VKT_HD int32_t cvtt_i32(float f)
    {
        // x86 cvttss2si: truncate; NaN or |f| >= 2^31 -> 0x80000000.  (-2^31 itself takes the
        // fallback, which is its own conversion: one compare with an |.| source modifier.)
        return fabsf(f) < 2147483648.0f ? static_cast<int32_t>(f) : INT32_MIN;
    }

    VKT_HD int64_t cvtt_i64(float f)
    {
        return (f >= -9223372036854775808.0f && f < 9223372036854775808.0f) ? static_cast<int64_t>(f)
                                                                             : INT64_MIN;
    }

    VKT_HD float lerp(float a, float b, float t)
    {
        VKT_NO_CONTRACT
        float s = 1.0f - t;
        float p = s * a;
        float q = t * b;
        return p + q;
    }

    VKT_HD float rmin(float a, float b) { return b < a ? b : a; }
    VKT_HD float rmax(float a, float b) { return a < b ? b : a; }
    VKT_HD float clampRef(float x, float lo, float hi) { return rmax(lo, rmin(x, hi)); }

    VKT_HD float bitsToFloat(uint32_t u)
    {
        union { uint32_t u; float f; } c;
        c.u = u;
        return c.f;
    }

    VKT_HD uint32_t floatToBits(float f)
    {
        union { float f; uint32_t u; } c;
        c.f = f;
        return c.u;
    }

    // Parameters of one volume's forward mapping, precomputed on the host:
    // v = (value - lo) / (hi - lo).  When (hi - lo) is a power of two whose reciprocal is
    // a normal float, the division equals the multiplication by that reciprocal in every
    // case (both round the same exact real), so the kernel can skip the IEEE divide.
    struct MapParams
    {
        float lo;
        float hi;
        float range;      // hi - lo, rounded as the reference rounds it
        float invRange;   // exact reciprocal when rangeIsPow2
        int32_t rangeIsPow2;
    };

    // DIV selects the division at compile time where the caller has dispatched on
    // m.rangeIsPow2 (1: multiply by the exact reciprocal, 2: IEEE divide; 0: test at run
    // time -- a uniform branch per voxel that keeps hipcc from interleaving voxels;
    // 3: the unit mapping lo = +0, hi = 1 (isUnitMapping), where (value - 0) / 1 == value for
    // every float including -0, +-inf and NaN, so normalising is the identity).
    template <int DIV = 0>
    VKT_HD float normalise(float value, MapParams const& m)
    {
        VKT_NO_CONTRACT
        if constexpr (DIV == 3)
            return value;
        float v = value - m.lo;
        if constexpr (DIV == 1)
            return v * m.invRange;
        else if constexpr (DIV == 2)
            return v / m.range;
        else
            return m.rangeIsPow2 ? v * m.invRange : v / m.range;
    }

    // ---- encode (MapVoxelImpl) -------------------------------------------------------
    // Returns the stored code in the low bytesPerVoxel(fmt) bytes; `write` is false for
    // the formats the reference's switch skips (Int8, Int32, Unspecified).
    template <int DIV = 0>
    VKT_HD uint32_t encode(float value, int32_t fmt, MapParams const& m, bool& write)
    {
        VKT_NO_CONTRACT
        float v = normalise<DIV>(value, m);
        write = true;
        switch (fmt)
        {
        case FmtInt16:   // VoxelMapping.hpp:28-38
            return static_cast<uint32_t>(cvtt_i32(v * 65535.999f - 32767.f)) & 0xFFFFu;
        case FmtUInt8:   // VoxelMapping.hpp:41-46
            return static_cast<uint32_t>(cvtt_i32(v * 255.999f)) & 0xFFu;
        case FmtUInt16:  // VoxelMapping.hpp:48-59 (65535.999f == 65536.0f: 1.0 wraps to 0)
            return static_cast<uint32_t>(cvtt_i32(v * 65535.999f)) & 0xFFFFu;
        case FmtUInt32:  // VoxelMapping.hpp:62-76 (cvttss2si with a 64-bit register)
            return static_cast<uint32_t>(static_cast<uint64_t>(cvtt_i64(v * 4294967295.999f)));
        case FmtFloat32: // VoxelMapping.hpp:79-94 (stores the normalised value)
            return floatToBits(v);
        default:
            write = false;
            return 0u;
        }
    }

    // ---- decode (UnmapVoxelImpl) -----------------------------------------------------
    // float(1 / 255.999f) = 0x3B800021; c / 255.999f == c * kInv255999 for c = 0..255
    constexpr float kInv255999 = 0x1.000042p-8f;

    // `prior` is the value the reference leaves untouched for Int8/Int32/Unspecified
    // (getValue initialises it to 0.f, src/vkt/StructuredVolume.cpp:196).
    VKT_HD float decode(uint32_t code, int32_t fmt, float lo, float hi, float prior = 0.f)
    {
        VKT_NO_CONTRACT
        switch (fmt)
        {
        case FmtInt16:   // VoxelMapping.hpp:107-119
        {
            float f = static_cast<float>(static_cast<int16_t>(static_cast<uint16_t>(code)));
            return lerp(lo, hi, (f + 32767.f) / 65535.999f);
        }
        case FmtUInt8:   // VoxelMapping.hpp:122-127: an IEEE division by 255.999f, which for
                         // each of the 256 codes rounds to the same float as the product with
                         // kInv255999 (checked exhaustively: tests/test_host_codec.py), so the
                         // ~10-instruction gfx950 division sequence is not needed
            return lerp(lo, hi, static_cast<float>(code & 0xFFu) * kInv255999);
        case FmtUInt16:  // VoxelMapping.hpp:130-142 (divisor rounds to 2^16: exact)
            return lerp(lo, hi, static_cast<float>(code & 0xFFFFu) / 65535.999f);
        case FmtUInt32:  // VoxelMapping.hpp:145-160
            return lerp(lo, hi, static_cast<float>(code) / 4294967295.999f);
        case FmtFloat32: // VoxelMapping.hpp:163-175 (raw bits, no mapping)
            return bitsToFloat(code);
        default:
            return prior;
        }
    }

    // decode() for a volume whose mapping is the unit mapping (isUnitMapping): lerp(+0, 1, t)
    // = (1 - t) * +0 + t * 1 = +0 + t = t exactly for every t the integer formats produce
    // (finite, t > -1, 1 - t > 0 so the first product is +0; t = +0 gives +0 + +0 = +0), so
    // the four lerp operations drop out.
    VKT_HD float decodeUnit(uint32_t code, int32_t fmt, float prior = 0.f)
    {
        VKT_NO_CONTRACT
        switch (fmt)
        {
        case FmtInt16:
            return (static_cast<float>(static_cast<int16_t>(static_cast<uint16_t>(code))) + 32767.f) / 65535.999f;
        case FmtUInt8:
            return static_cast<float>(code & 0xFFu) * kInv255999;
        case FmtUInt16:
            return static_cast<float>(code & 0xFFFFu) / 65535.999f;
        case FmtUInt32:
            return static_cast<float>(code) / 4294967295.999f;
        case FmtFloat32:
            return bitsToFloat(code);
        default:
            return prior;
        }
    }

    // Mapping (lo, hi) is exactly (+0, 1): bit compare, since lo = -0 makes
    // normalise(-0) = -0 - -0 = +0 (not the identity).
    VKT_HD bool isUnitMapping(float lo, float hi)
    {
        return floatToBits(lo) == 0u && floatToBits(hi) == 0x3F800000u;
    }

    // Host helper: build MapParams for a volume's mapping.
    inline MapParams makeMapParams(float lo, float hi)
    {
        MapParams m;
        m.lo = lo;
        m.hi = hi;
        volatile float r = hi - lo;   // keep the float rounding of the reference
        m.range = r;
        m.invRange = 0.f;
        m.rangeIsPow2 = 0;
        uint32_t bits = floatToBits(m.range);
        uint32_t expo = (bits >> 23) & 0xFFu;
        uint32_t mant = bits & 0x7FFFFFu;
        // normal, power of two (mantissa 0), and reciprocal exponent also normal
        if (mant == 0 && expo >= 1 && expo <= 253 && expo != 0)
        {
            int32_t e = static_cast<int32_t>(expo) - 127;   // range = +-2^e
            int32_t re = -e + 127;                          // biased exponent of 2^-e
            if (re >= 1 && re <= 254)
            {
                m.invRange = bitsToFloat((bits & 0x80000000u) | (static_cast<uint32_t>(re) << 23));
                m.rangeIsPow2 = 1;
            }
        }
        return m;
    }

} // codec
} // vkt
