// Copy_hip.hpp -- replaces src/vkt/Copy_cuda.hpp (declaration :11-17) in src/vkt/Copy.cpp.
#pragma once
#include "HipView.hpp"

namespace vkt
{
    inline void CopyRange_cuda(StructuredVolume& dest, StructuredVolume& source, Vec3i first, Vec3i last,
                               Vec3i dstOffset)
    {
        vktHipCopyRange(HipView(dest), HipView(source), C3(first), C3(last), C3(dstOffset));
    }
} // vkt
