// Resample_hip.hpp -- replaces the StructuredVolume overload of src/vkt/Resample_cuda.hpp
// (:12-17) in src/vkt/Resample.cpp (the HierarchicalVolume and CLAHE overloads stay on the
// reference's CUDA path; they are out of scope).
#pragma once
#include <vkt/Resample.hpp>
#include "HipView.hpp"

namespace vkt
{
    inline void Resample_cuda(StructuredVolume& dst, StructuredVolume& src, FilterMode fm)
    {
        vktHipResample(HipView(dst), HipView(src), static_cast<vktFilterMode>(fm));
    }
} // vkt
