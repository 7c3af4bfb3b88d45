// HipView.hpp -- shared helper of the reference-side shims: the backend's kernel-argument
// view of a reference vkt::StructuredVolume (fields of StructuredVolumeView,
// src/vkt/StructuredVolumeView.hpp:221-225).  getData() migrates the volume to the thread's
// device first, as the reference's _cuda functions expect.
#pragma once
#include <vkt/StructuredVolume.hpp>
#include <volkit_hip.h>

namespace vkt
{
    inline vktHipVolumeView_t HipView(StructuredVolume& v)
    {
        Vec3i d = v.getDims();
        Vec2f m = v.getVoxelMapping();
        return {v.getData(), d.x, d.y, d.z, static_cast<int32_t>(v.getDataFormat()), m.x, m.y};
    }

    inline vktVec3i_t C3(Vec3i v) { return {v.x, v.y, v.z}; }
} // vkt
