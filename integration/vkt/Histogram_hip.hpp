// Histogram_hip.hpp -- replaces src/vkt/Histogram_cuda.hpp in src/vkt/Histogram.cpp
// (reference kernel src/vkt/Histogram_cuda.cu:45-76).  getBinCounts() migrates the bins to the
// thread's device; the backend zeroes and fills them (64-bit counters, size_t on LP64).
#pragma once
#include <vkt/Histogram.hpp>
#include "HipView.hpp"

namespace vkt
{
    static_assert(sizeof(std::size_t) == sizeof(uint64_t), "64-bit bin counters");

    inline void ComputeHistogramRange_cuda(StructuredVolume& volume, Histogram& histogram, Vec3i first, Vec3i last)
    {
        vktHipHistogramRange(HipView(volume), C3(first), C3(last),
                             reinterpret_cast<uint64_t*>(histogram.getBinCounts()), histogram.getNumBins(), 0);
    }
} // vkt
