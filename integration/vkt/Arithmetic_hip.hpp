// Arithmetic_hip.hpp -- include in src/vkt/Arithmetic.cpp instead of Arithmetic_cuda.hpp
// (reference src/vkt/Arithmetic.cpp:16-18, with VKT_HAVE_CUDA 1): every *Range_cuda the
// VKT_LEGACY_CALL__ seam pastes (src/vkt/Callable.hpp:82-113; declarations
// src/vkt/Arithmetic_cuda.hpp:10-98) forwards to vktHipArithmeticRange.
#pragma once
#include "HipView.hpp"

namespace vkt
{
#define VKT_HIP_ARITH_(NAME, OP)                                                               \
    inline void NAME##Range_cuda(StructuredVolume& dest, StructuredVolume& source1,            \
                                 StructuredVolume& source2, Vec3i first, Vec3i last,           \
                                 Vec3i dstOffset)                                              \
    {                                                                                          \
        vktHipArithmeticRange(OP, HipView(dest), HipView(source1), HipView(source2), C3(first), \
                              C3(last), C3(dstOffset));                                        \
    }
    VKT_HIP_ARITH_(Sum, vktHipOpSum)
    VKT_HIP_ARITH_(Diff, vktHipOpDiff)
    VKT_HIP_ARITH_(Prod, vktHipOpProd)
    VKT_HIP_ARITH_(Quot, vktHipOpQuot)
    VKT_HIP_ARITH_(AbsDiff, vktHipOpAbsDiff)
    VKT_HIP_ARITH_(SafeSum, vktHipOpSafeSum)
    VKT_HIP_ARITH_(SafeDiff, vktHipOpSafeDiff)
    VKT_HIP_ARITH_(SafeProd, vktHipOpSafeProd)
    VKT_HIP_ARITH_(SafeQuot, vktHipOpSafeQuot)
    VKT_HIP_ARITH_(SafeAbsDiff, vktHipOpSafeAbsDiff)
#undef VKT_HIP_ARITH_
} // vkt
