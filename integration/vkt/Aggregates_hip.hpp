// Aggregates_hip.hpp -- replaces src/vkt/Aggregates_cuda.hpp (an empty function there) in
// src/vkt/Aggregates.cpp.  vkt::Aggregates and vktAggregates_t have the same layout.
#pragma once
#include <vkt/Aggregates.hpp>
#include "HipView.hpp"

namespace vkt
{
    static_assert(sizeof(Aggregates) == sizeof(vktAggregates_t), "Aggregates layout");

    inline void ComputeAggregatesRange_cuda(StructuredVolume& volume, Aggregates& aggregates, Vec3i first, Vec3i last)
    {
        vktHipAggregatesRange(HipView(volume), C3(first), C3(last), reinterpret_cast<vktAggregates_t*>(&aggregates));
    }
} // vkt
