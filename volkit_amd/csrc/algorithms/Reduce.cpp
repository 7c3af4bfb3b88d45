// Reduce.cpp -- ComputeAggregates / ComputeHistogram front-ends (C++ and C) and the Histogram
// container.
//
// Reference: src/vkt/Aggregates.cpp:20-120 (C++ overloads and vktComputeAggregates*SV, which
// memcpy the C++ struct into the C one), src/vkt/Histogram.cpp:20-95 (Histogram is a
// ManagedBuffer<size_t> of bin counts; C++ only).  Under the GPU policy the work is the
// vktHip* reduction backend (kernels/Reduce.hip); the CPU policy returns InvalidValue like
// every algorithm of this GPU backend.

#include "../runtime/Runtime.hpp"
#include "../StructuredVolume_impl.hpp"
#include "volkit_hip.h"

#include <cstring>

namespace vkt
{
namespace
{
    vktHipVolumeView_t viewOf(StructuredVolume& v)
    {
        vktHipVolumeView_t out;
        out.data = rt::deviceData(v);
        Vec3i d = v.getDims();
        out.dimX = d.x;
        out.dimY = d.y;
        out.dimZ = d.z;
        out.dataFormat = static_cast<int32_t>(v.getDataFormat());
        Vec2f m = v.getVoxelMapping();
        out.mappingLo = m.x;
        out.mappingHi = m.y;
        return out;
    }

    bool gpuPolicy(char const* name)
    {
        (void)rt::takeMigrationFailure();   // (only this call's migrations explain its errors)
        if (GetThreadExecutionPolicy().device == ExecutionPolicy::Device::GPU)
            return true;
        rt::setLastError(std::string(name) + ": CPU execution policy");
        VKT_LOG(rt::LogLevel::Error) << "When calling algorithm: " << name
                                     << " -- volkit-amd implements the GPU (HIP/gfx950) backend only; set "
                                        "ExecutionPolicy::Device::GPU";
        return false;
    }

    static_assert(sizeof(Aggregates) == sizeof(vktAggregates_t), "C and C++ Aggregates layouts must match");
} // namespace

//--- Aggregates ------------------------------------------------------------------------------
Error ComputeAggregates(StructuredVolume& volume, Aggregates& aggregates)
{
    return ComputeAggregatesRange(volume, aggregates, Vec3i{0, 0, 0}, volume.getDims());
}

Error ComputeAggregatesRange(StructuredVolume& volume, Aggregates& aggregates, int32_t fx, int32_t fy, int32_t fz,
                             int32_t lx, int32_t ly, int32_t lz)
{
    return ComputeAggregatesRange(volume, aggregates, Vec3i{fx, fy, fz}, Vec3i{lx, ly, lz});
}

Error ComputeAggregatesRange(StructuredVolume& volume, Aggregates& aggregates, Vec3i first, Vec3i last)
{
    if (!gpuPolicy("ComputeAggregatesRange_hip"))
        return InvalidValue;
    rt::ScopedKernelTimer timer("ComputeAggregatesRange_hip", GetThreadExecutionPolicy().printPerformance != False);
    vktAggregates_t out;
    vktError e = rt::explainFailure(vktHipAggregatesRange(viewOf(volume), vktVec3i_t{first.x, first.y, first.z},
                                                          vktVec3i_t{last.x, last.y, last.z}, &out),
                                    "ComputeAggregatesRange_hip");
    if (e == vktNoError)
        std::memcpy(&aggregates, &out, sizeof(out));
    return static_cast<Error>(e);
}

//--- Histogram -------------------------------------------------------------------------------
Histogram::Histogram(std::size_t numBins) { resize(numBins); }

std::size_t Histogram::getNumBins() const { return size_; }

std::size_t* Histogram::getBinCounts()
{
    migrate();
    return data_;
}

Error ComputeHistogram(StructuredVolume& volume, Histogram& histogram)
{
    return ComputeHistogramRange(volume, histogram, Vec3i{0, 0, 0}, volume.getDims());
}

Error ComputeHistogramRange(StructuredVolume& volume, Histogram& histogram, int32_t fx, int32_t fy, int32_t fz,
                            int32_t lx, int32_t ly, int32_t lz)
{
    return ComputeHistogramRange(volume, histogram, Vec3i{fx, fy, fz}, Vec3i{lx, ly, lz});
}

Error ComputeHistogramRange(StructuredVolume& volume, Histogram& histogram, Vec3i first, Vec3i last)
{
    if (!gpuPolicy("ComputeHistogramRange_hip"))
        return InvalidValue;
    rt::ScopedKernelTimer timer("ComputeHistogramRange_hip", GetThreadExecutionPolicy().printPerformance != False);
    static_assert(sizeof(std::size_t) == sizeof(uint64_t), "bin counters are 64-bit");
    uint64_t* bins = reinterpret_cast<uint64_t*>(histogram.getBinCounts());   // migrates to HBM
    if (!histogram.residentOn(GetThreadExecutionPolicy()))
    {
        rt::fail(("ComputeHistogramRange_hip: " + rt::takeMigrationFailure()).c_str());
        return InvalidValue;
    }
    return static_cast<Error>(rt::explainFailure(
        vktHipHistogramRange(viewOf(volume), vktVec3i_t{first.x, first.y, first.z}, vktVec3i_t{last.x, last.y, last.z},
                             bins, histogram.getNumBins(), 0),
        "ComputeHistogramRange_hip"));
}

} // vkt

//--- C API -----------------------------------------------------------------------------------
struct vktHistogram_impl
{
    explicit vktHistogram_impl(std::size_t n) : histogram(n) {}
    vkt::Histogram histogram;
};

extern "C" {

vktError vktComputeAggregatesSV(vktStructuredVolume volume, vktAggregates_t* aggregates)
{
    if (!volume || !aggregates)
        return vktInvalidValue;
    vkt::Aggregates a;
    vkt::Error e = vkt::ComputeAggregates(volume->volume, a);
    if (e == vkt::NoError)
        std::memcpy(aggregates, &a, sizeof(a));
    return static_cast<vktError>(e);
}

vktError vktComputeAggregatesRangeSV(vktStructuredVolume volume, vktAggregates_t* aggregates, int32_t fx, int32_t fy,
                                     int32_t fz, int32_t lx, int32_t ly, int32_t lz)
{
    if (!volume || !aggregates)
        return vktInvalidValue;
    vkt::Aggregates a;
    vkt::Error e = vkt::ComputeAggregatesRange(volume->volume, a, fx, fy, fz, lx, ly, lz);
    if (e == vkt::NoError)
        std::memcpy(aggregates, &a, sizeof(a));
    return static_cast<vktError>(e);
}

void vktHistogramCreate(vktHistogram* histogram, size_t numBins) { *histogram = new vktHistogram_impl(numBins); }

void vktHistogramDestroy(vktHistogram histogram) { delete histogram; }

size_t vktHistogramGetNumBins(vktHistogram histogram) { return histogram->histogram.getNumBins(); }

size_t* vktHistogramGetBinCounts(vktHistogram histogram) { return histogram->histogram.getBinCounts(); }

vktError vktComputeHistogramSV(vktStructuredVolume volume, vktHistogram histogram)
{
    if (!volume || !histogram)
        return vktInvalidValue;
    return static_cast<vktError>(vkt::ComputeHistogram(volume->volume, histogram->histogram));
}

vktError vktComputeHistogramRangeSV(vktStructuredVolume volume, vktHistogram histogram, int32_t fx, int32_t fy,
                                    int32_t fz, int32_t lx, int32_t ly, int32_t lz)
{
    if (!volume || !histogram)
        return vktInvalidValue;
    return static_cast<vktError>(
        vkt::ComputeHistogramRange(volume->volume, histogram->histogram, fx, fy, fz, lx, ly, lz));
}

} // extern "C"
