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
            float v = codec::decode(a, FS == kDyn ? fs : FS, slo, shi);
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
            float v1 = codec::decode(a, FS1 == kDyn ? fs1 : FS1, lo1, hi1);
            float v2 = codec::decode(b, FS2 == kDyn ? fs2 : FS2, lo2, hi2);
            float r = applyOp<OP>(v1, v2, dm.lo, dm.hi);
            bool w;
            return codec::encode<DIV>(r, FD == kDyn ? fd : FD, dm, w);
        }
    };

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
        if (p.vec && f1 == f2 && f1 == fd)
        {
#define VKT_ARITH_FIXED(FMT, BPV)                                                                              \
    return dm.rangeIsPow2                                                                                      \
               ? launchPointwise<2, BPV>(p, ArithF<OP, FMT, FMT, FMT, 1>{f1, f2, fd, a.mappingLo, a.mappingHi,  \
                                                                         b.mappingLo, b.mappingHi, dm}, s)      \
               : launchPointwise<2, BPV>(p, ArithF<OP, FMT, FMT, FMT, 2>{f1, f2, fd, a.mappingLo, a.mappingHi,  \
                                                                         b.mappingLo, b.mappingHi, dm}, s)
            if (fd == codec::FmtUInt16)
                VKT_ARITH_FIXED(codec::FmtUInt16, 2);
            if (fd == codec::FmtUInt8)
                VKT_ARITH_FIXED(codec::FmtUInt8, 1);
            if (fd == codec::FmtFloat32)
                VKT_ARITH_FIXED(codec::FmtFloat32, 4);
#undef VKT_ARITH_FIXED
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
