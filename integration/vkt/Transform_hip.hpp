// Transform_hip.hpp -- replaces src/vkt/Transform_cuda.hpp (:12-30, two empty stubs) in
// src/vkt/Transform.cpp.  The host callbacks run in the serial visit order on planes staged
// through host memory; vkt::VoxelView and vktVoxelView_t have the same layout
// ({uint8_t*, 4-byte format enum, float, float}), so the callback types are ABI-identical.
#pragma once
#include <vkt/Transform.hpp>
#include "HipView.hpp"

namespace vkt
{
    static_assert(sizeof(VoxelView) == sizeof(vktVoxelView_t), "VoxelView layout");

    inline void TransformRange_cuda(StructuredVolume& volume, Vec3i first, Vec3i last, TransformUnaryOp unaryOp)
    {
        vktHipTransformRange1(HipView(volume), C3(first), C3(last), reinterpret_cast<vktTransformUnaryOp>(unaryOp));
    }

    inline void TransformRange_cuda(StructuredVolume& volume1, StructuredVolume& volume2, Vec3i first, Vec3i last,
                                    TransformBinaryOp binaryOp)
    {
        vktHipTransformRange2(HipView(volume1), HipView(volume2), C3(first), C3(last), vktVec3i_t{0, 0, 0},
                              reinterpret_cast<vktTransformBinaryOp>(binaryOp));
    }
} // vkt
