// PointwiseOps.hpp -- functors of the pointwise engine (fill, copy, convert, the ten
// arithmetic lambdas of reference src/vkt/Arithmetic_serial.hpp:63-258) and the per-op
// dispatch template; the arithmetic instantiations live in PointwiseArith{0..4}.hip (two ops
// per translation unit, compiled in parallel).
#pragma once

#include "Pointwise.hpp"
#include "volkit_hip.h"

namespace vkt
{
namespace hipk
{
    using codec::MapParams;

    // ---- functors ------------------------------------------------------------------
    struct FillF
    {
        uint32_t code;
        __device__ __forceinline__ uint32_t operator()(uint32_t, uint32_t) const { return code; }
    };

    struct PassF
    {
        __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t) const { return a; }
    };

    // dst = map_dst(unmap_src(code))  (CopyRange by value, Copy_serial.hpp:69-70;
    // Resample same-dims branch, Resample_serial.hpp:32-48)
    template <int FS, int FD, int DIV = 0>
    struct ConvertF
    {
        int32_t fs, fd;
        float slo, shi;
        MapParams dm;
        __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t) const
        {
            // DIV 3: source and destination mappings are both the unit mapping
            float v = DIV == 3 ? codec::decodeUnit(a, FS == kDyn ? fs : FS) : codec::decode(a, FS == kDyn ? fs : FS, slo, shi);
            bool w;
            return codec::encode<DIV>(v, FD == kDyn ? fd : FD, dm, w);
        }
    };

    // The ten lambdas of reference src/vkt/Arithmetic_serial.hpp:63-258.
    template <int OP>
    __device__ __forceinline__ float applyOp(float a, float b, float lo, float hi)
    {
        if constexpr (OP == vktHipOpSum) return a + b;
        else if constexpr (OP == vktHipOpDiff) return a - b;
        else if constexpr (OP == vktHipOpProd) return a * b;
        else if constexpr (OP == vktHipOpQuot) return a / b;
        else if constexpr (OP == vktHipOpAbsDiff) return fabsf(a - b);
        else if constexpr (OP == vktHipOpSafeSum) return codec::clampRef(a + b, lo, hi);
        else if constexpr (OP == vktHipOpSafeDiff) return codec::clampRef(a - b, lo, hi);
        else if constexpr (OP == vktHipOpSafeProd) return codec::clampRef(a * b, lo, hi);
        else if constexpr (OP == vktHipOpSafeQuot) return codec::clampRef(a / b, lo, hi);
        else return codec::clampRef(fabsf(a - b), lo, hi);
    }

    template <int OP, int FS1, int FS2, int FD, int DIV = 0>
    struct ArithF
    {
        int32_t fs1, fs2, fd;
        float lo1, hi1, lo2, hi2;
        MapParams dm;
        __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t b) const
        {
            // DIV 3: all three mappings are the unit mapping (codec::isUnitMapping)
            float v1 = DIV == 3 ? codec::decodeUnit(a, FS1 == kDyn ? fs1 : FS1) : codec::decode(a, FS1 == kDyn ? fs1 : FS1, lo1, hi1);
            float v2 = DIV == 3 ? codec::decodeUnit(b, FS2 == kDyn ? fs2 : FS2) : codec::decode(b, FS2 == kDyn ? fs2 : FS2, lo2, hi2);
            float r = applyOp<OP>(v1, v2, dm.lo, dm.hi);
            bool w;
            return codec::encode<DIV>(r, FD == kDyn ? fd : FD, dm, w);
        }
    };

    // UInt16 codes with the unit mapping on all three volumes: decodeUnit(c) = c * 2^-16
    // exactly, so a + b, a - b and |a - b| are exact in f32 (at most 17 significant bits),
    // normalise<3> is the identity, and * 65535.999f (== 65536.0f), cvtt, & 0xFFFF give back
    // the integer result modulo 2^16.  Hence, bit for bit:
    //   Sum (a + b) mod 2^16, Diff (a - b) mod 2^16, AbsDiff and SafeAbsDiff |a - b| (< 1,
    //   never clamped), SafeDiff max(a - b, 0), SafeSum a + b < 2^16 ? a + b : 0 (the clamp to
    //   1.0 encodes to 65536 & 0xFFFF = 0).
    // Prod/Quot round in f32 and keep the float path.  Checked against the oracle for every
    // code as either operand (tests/test_gpu_parity.py::test_arithmetic_unit_mapping_*).
    // kPacked16: pointwiseVecSpan applies pk() to whole dwords (two voxels; v_pk_*_u16).
    template <int OP>
    struct IntArithU16F
    {
        static constexpr bool kPacked16 = true;
        typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));

        __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t b) const
        {
            if constexpr (OP == vktHipOpSum) return (a + b) & 0xFFFFu;
            else if constexpr (OP == vktHipOpDiff) return (a - b) & 0xFFFFu;
            else if constexpr (OP == vktHipOpSafeSum) return a + b < 0x10000u ? a + b : 0u;
            else if constexpr (OP == vktHipOpSafeDiff) return a > b ? a - b : 0u;
            else return a > b ? a - b : b - a;   // AbsDiff, SafeAbsDiff
        }

        __device__ __forceinline__ uint32_t pk(uint32_t a, uint32_t b) const
        {
            u16x2 const x = __builtin_bit_cast(u16x2, a), y = __builtin_bit_cast(u16x2, b);
            u16x2 r;
            if constexpr (OP == vktHipOpSum) r = x + y;
            else if constexpr (OP == vktHipOpDiff) r = x - y;
            else if constexpr (OP == vktHipOpSafeSum)
            {
                u16x2 const s = x + y;   // wrapped; it overflowed iff s < x
                r = s & ~__builtin_bit_cast(u16x2, s < x);
            }
            else if constexpr (OP == vktHipOpSafeDiff) r = __builtin_elementwise_sub_sat(x, y);
            else r = __builtin_elementwise_sub_sat(x, y) | __builtin_elementwise_sub_sat(y, x);
            return __builtin_bit_cast(uint32_t, r);
        }
    };

    // UInt8 codes with the unit mapping on all three volumes: the same IEEE operations as
    // ArithF<OP, UInt8, UInt8, UInt8, 3> (t = c * kInv255999, the op, * 255.999f, truncate), with
    // what the value ranges make redundant dropped: t in [0, 1), so Sum / Prod / SafeSum /
    // SafeProd results are >= +0 and Diff-type results are in (-1, 1) and never -0 (x - x = +0);
    // hence the reference clamp max(0, min(x, 1)) is min(x, 1) for SafeSum, max(x, 0) for
    // SafeDiff and the identity for SafeAbsDiff / SafeProd, and |x * 255.999f| < 512 makes the
    // x86 cvttss2si range check dead (plain v_cvt_i32_f32).  Quot / SafeQuot (inf, NaN) keep
    // ArithF.  Checked against the oracle on every code pair.
    template <int OP>
    struct UnitArithU8F
    {
        __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t b) const
        {
            float const x = static_cast<float>(a & 0xFFu) * codec::kInv255999;
            float const y = static_cast<float>(b & 0xFFu) * codec::kInv255999;
            float r;
            if constexpr (OP == vktHipOpSum) r = x + y;
            else if constexpr (OP == vktHipOpDiff) r = x - y;
            else if constexpr (OP == vktHipOpProd || OP == vktHipOpSafeProd) r = x * y;
            else if constexpr (OP == vktHipOpAbsDiff || OP == vktHipOpSafeAbsDiff) r = fabsf(x - y);
            else if constexpr (OP == vktHipOpSafeSum) r = fminf(x + y, 1.0f);
            else r = fmaxf(x - y, 0.0f);   // SafeDiff
            return static_cast<uint32_t>(static_cast<int32_t>(r * 255.999f)) & 0xFFu;
        }
    };

    template <int OP>
    constexpr bool hasUnitArithU8()
    {
        return OP != vktHipOpQuot && OP != vktHipOpSafeQuot;
    }

    template <int OP>
    constexpr bool hasIntArithU16()
    {
        return OP == vktHipOpSum || OP == vktHipOpDiff || OP == vktHipOpAbsDiff || OP == vktHipOpSafeSum ||
               OP == vktHipOpSafeDiff || OP == vktHipOpSafeAbsDiff;
    }

    template <int NS, class F>
    vktError launchByBpv(PwPlan const& p, F const& f, hipStream_t s)
    {
        switch (p.bpv)
        {
        case 1: return launchPointwise<NS, 1>(p, f, s);
        case 2: return launchPointwise<NS, 2>(p, f, s);
        case 4: return launchPointwise<NS, 4>(p, f, s);
        default: return launchPointwise<NS, 0>(p, f, s);
        }
    }

    // ---- arithmetic dispatch ---------------------------------------------------------
    template <int OP>
    vktError arithmetic(PwPlan const& p, vktHipVolumeView_t const& d, vktHipVolumeView_t const& a,
                        vktHipVolumeView_t const& b, hipStream_t s)
    {
        MapParams dm = codec::makeMapParams(d.mappingLo, d.mappingHi);
        int32_t f1 = a.dataFormat, f2 = b.dataFormat, fd = d.dataFormat;
        if ((p.vec || (p.gen && p.uniform)) && f1 == f2 && f1 == fd)
        {
        // unit mappings everywhere (the canonical [0, 1] inputs): the codec's lerp and
        // normalisation are identities (codec::decodeUnit / normalise<3>)
        bool const unit = codec::isUnitMapping(a.mappingLo, a.mappingHi) &&
                          codec::isUnitMapping(b.mappingLo, b.mappingHi) &&
                          codec::isUnitMapping(d.mappingLo, d.mappingHi);
#define VKT_ARITH_LAUNCH(FMT, BPV, DIV)                                                                        \
    launchPointwise<2, BPV>(p, ArithF<OP, FMT, FMT, FMT, DIV>{f1, f2, fd, a.mappingLo, a.mappingHi, b.mappingLo, \
                                                              b.mappingHi, dm}, s)
#define VKT_ARITH_FIXED(FMT, BPV)                                                                              \
    return unit ? VKT_ARITH_LAUNCH(FMT, BPV, 3)                                                                \
                : dm.rangeIsPow2 ? VKT_ARITH_LAUNCH(FMT, BPV, 1) : VKT_ARITH_LAUNCH(FMT, BPV, 2)
            if constexpr (hasIntArithU16<OP>())
                if (fd == codec::FmtUInt16 && unit)
                    return launchPointwise<2, 2>(p, IntArithU16F<OP>{}, s);
            if constexpr (hasUnitArithU8<OP>())
                if (fd == codec::FmtUInt8 && unit)
                    return launchPointwise<2, 1>(p, UnitArithU8F<OP>{}, s);
            if (fd == codec::FmtUInt16)
                VKT_ARITH_FIXED(codec::FmtUInt16, 2);
            if (fd == codec::FmtUInt8)
                VKT_ARITH_FIXED(codec::FmtUInt8, 1);
            if (fd == codec::FmtFloat32)
                VKT_ARITH_FIXED(codec::FmtFloat32, 4);
            if (fd == codec::FmtInt16)   // (round 6: the runtime-format functor ran Int16 at 0.62-0.65 of 8 TB/s)
                VKT_ARITH_FIXED(codec::FmtInt16, 2);
#undef VKT_ARITH_FIXED
#undef VKT_ARITH_LAUNCH
        }
        return launchByBpv<2>(p, ArithF<OP, kDyn, kDyn, kDyn>{f1, f2, fd, a.mappingLo, a.mappingHi, b.mappingLo,
                                                               b.mappingHi, dm}, s);
    }


    // op dispatchers, one per translation unit: ops {2i, 2i+1}
    vktError arithmeticPair0(int op, PwPlan const& p, vktHipVolumeView_t const& d, vktHipVolumeView_t const& a,
                             vktHipVolumeView_t const& b, hipStream_t s);
    vktError arithmeticPair1(int op, PwPlan const& p, vktHipVolumeView_t const& d, vktHipVolumeView_t const& a,
                             vktHipVolumeView_t const& b, hipStream_t s);
    vktError arithmeticPair2(int op, PwPlan const& p, vktHipVolumeView_t const& d, vktHipVolumeView_t const& a,
                             vktHipVolumeView_t const& b, hipStream_t s);
    vktError arithmeticPair3(int op, PwPlan const& p, vktHipVolumeView_t const& d, vktHipVolumeView_t const& a,
                             vktHipVolumeView_t const& b, hipStream_t s);
    vktError arithmeticPair4(int op, PwPlan const& p, vktHipVolumeView_t const& d, vktHipVolumeView_t const& a,
                             vktHipVolumeView_t const& b, hipStream_t s);

} // hipk
} // vkt
