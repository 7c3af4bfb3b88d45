// Fill_hip.hpp -- replaces src/vkt/Fill_cuda.hpp (:13) in src/vkt/Fill.cpp.  Its argument is
// the reference's internal StructuredVolumeView (src/vkt/StructuredVolumeView.hpp, which pulls
// in the CMake-generated vkt/config.h), so this shim only compiles inside the reference build;
// also give Call() its missing GPU branch (src/vkt/Callable.cpp:53-66), where SV Fill is a
// silent no-op today.
#pragma once
#include <volkit_hip.h>
#include "StructuredVolumeView.hpp"

namespace vkt
{
    inline void FillRange_cuda(StructuredVolumeView volume, Vec3i first, Vec3i last, float value)
    {
        Vec3i d = volume.getDims();
        Vec2f m = volume.getVoxelMapping();
        vktHipVolumeView_t v{const_cast<uint8_t*>(volume.getData()), d.x, d.y, d.z,
                             static_cast<int32_t>(volume.getDataFormat()), m.x, m.y};
        vktHipFillRange(v, vktVec3i_t{first.x, first.y, first.z}, vktVec3i_t{last.x, last.y, last.z}, value);
    }
} // vkt
