// Transform.cpp -- TransformRange for the GPU policy.
//
// The reference's TransformRange_cuda is an empty stub (src/vkt/Transform_cuda.hpp:12-30),
// so under the GPU policy Transform silently does nothing there.  The user operation is a
// host function pointer (include/cpp/vkt/Transform.hpp:16-25) and cannot execute on the GPU,
// so this backend stages the z-planes covering the range to host memory (one D2H copy on the
// copy stream, ordered after pending kernels), runs the callback over the range in the serial
// path's order and with its 8-byte zeroed scratch per voxel (src/vkt/Transform_serial.hpp:15-101),
// and writes the planes back (one H2D copy).  Two views of the same buffer share one staging
// copy, so aliasing behaves exactly as in the serial loop.

#include "../runtime/Runtime.hpp"
#include "volkit_codec.hpp"
#include "volkit_hip.h"

#include <algorithm>
#include <cstring>
#include <vector>

namespace vkt
{
namespace hipk
{
    bool validView(vktHipVolumeView_t const& v);
    bool boxInside(vktHipVolumeView_t const& v, vktVec3i_t o, int64_t nx, int64_t ny, int64_t nz);

    namespace
    {
        struct Staged
        {
            vktHipVolumeView_t view;
            int32_t z0 = 0, z1 = 0;      // staged planes [z0, z1)
            std::vector<uint8_t> host;
            size_t planeBytes = 0;

            vktError load()
            {
                planeBytes = static_cast<size_t>(view.dimX) * view.dimY * codec::bytesPerVoxel(view.dataFormat);
                host.resize(planeBytes * static_cast<size_t>(z1 - z0));
                return detail::memcpyHip(host.data(), view.data + planeBytes * z0, host.size(), CopyKind::DeviceToHost);
            }

            vktError store()
            {
                return detail::memcpyHip(view.data + planeBytes * z0, host.data(), host.size(), CopyKind::HostToDevice);
            }

            uint8_t* voxel(int32_t x, int32_t y, int32_t z)
            {
                size_t bpv = codec::bytesPerVoxel(view.dataFormat);
                return host.data() + planeBytes * static_cast<size_t>(z - z0) +
                       (static_cast<size_t>(y) * view.dimX + x) * bpv;
            }
        };
    } // namespace
} // hipk
} // vkt

namespace vkt
{
namespace hipk
{
    // The unary host-callback transform; the callback sees z + zShift (a Z-slab of a larger
    // volume passes its first global plane, runtime/Slab.cpp).
    vktError transformRange1Shifted(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last,
                                    vktTransformUnaryOp unaryOp, int32_t zShift);
} // hipk
} // vkt

using namespace vkt;
using namespace vkt::hipk;

vktError vkt::hipk::transformRange1Shifted(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last,
                                           vktTransformUnaryOp unaryOp, int32_t zShift)
{
    if (!validView(volume) || unaryOp == nullptr)
        return rt::fail("vktHipTransformRange1: invalid arguments");
    int64_t nx = int64_t(last.x) - first.x, ny = int64_t(last.y) - first.y, nz = int64_t(last.z) - first.z;
    if (nx <= 0 || ny <= 0 || nz <= 0)
        return vktNoError;
    if (!boxInside(volume, first, nx, ny, nz))
        return rt::fail("vktHipTransformRange1: range outside the volume");
    Staged s;
    s.view = volume;
    s.z0 = first.z;
    s.z1 = last.z;
    vktError e = s.load();
    if (e != vktNoError)
        return e;
    uint32_t bpv = codec::bytesPerVoxel(volume.dataFormat);
    for (int32_t z = first.z; z != last.z; ++z)
        for (int32_t y = first.y; y != last.y; ++y)
            for (int32_t x = first.x; x != last.x; ++x)
            {
                uint8_t bytes[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                uint8_t* p = s.voxel(x, y, z);
                std::memcpy(bytes, p, bpv);
                vktVoxelView_t vv{bytes, static_cast<vktDataFormat>(volume.dataFormat), volume.mappingLo,
                                  volume.mappingHi};
                unaryOp(x, y, z + zShift, vv);
                std::memcpy(p, bytes, bpv);
            }
    return s.store();
}

extern "C" {

vktError vktHipTransformRange1(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last,
                               vktTransformUnaryOp unaryOp)
{
    return transformRange1Shifted(volume, first, last, unaryOp, 0);
}

vktError vktHipTransformRange2(vktHipVolumeView_t volume1, vktHipVolumeView_t volume2, vktVec3i_t first,
                               vktVec3i_t last, vktVec3i_t off, vktTransformBinaryOp binaryOp)
{
    if (!validView(volume1) || !validView(volume2) || binaryOp == nullptr)
        return rt::fail("vktHipTransformRange2: invalid arguments");
    int64_t nx = int64_t(last.x) - first.x, ny = int64_t(last.y) - first.y, nz = int64_t(last.z) - first.z;
    if (nx <= 0 || ny <= 0 || nz <= 0)
        return vktNoError;
    vktVec3i_t first2{first.x + off.x, first.y + off.y, first.z + off.z};
    if (!boxInside(volume1, first, nx, ny, nz) || !boxInside(volume2, first2, nx, ny, nz))
        return rt::fail("vktHipTransformRange2: range outside a volume");
    bool same = volume1.data == volume2.data;
    if (same && (volume1.dimX != volume2.dimX || volume1.dimY != volume2.dimY ||
                 volume1.dataFormat != volume2.dataFormat))
        return rt::fail("vktHipTransformRange2: aliased volumes with different layouts");
    Staged s1, s2;
    s1.view = volume1;
    s2.view = volume2;
    if (same)
    {
        s1.z0 = std::min(first.z, first2.z);
        s1.z1 = std::max(last.z, last.z + off.z);
    }
    else
    {
        s1.z0 = first.z;
        s1.z1 = last.z;
        s2.z0 = first2.z;
        s2.z1 = last.z + off.z;
    }
    vktError e = s1.load();
    if (e == vktNoError && !same)
        e = s2.load();
    if (e != vktNoError)
        return e;
    Staged& t2 = same ? s1 : s2;
    uint32_t b1 = codec::bytesPerVoxel(volume1.dataFormat), b2 = codec::bytesPerVoxel(volume2.dataFormat);
    for (int32_t z = first.z; z != last.z; ++z)
        for (int32_t y = first.y; y != last.y; ++y)
            for (int32_t x = first.x; x != last.x; ++x)
            {
                uint8_t bytes1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, bytes2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                uint8_t* p1 = s1.voxel(x, y, z);
                uint8_t* p2 = t2.voxel(x + off.x, y + off.y, z + off.z);
                std::memcpy(bytes1, p1, b1);
                std::memcpy(bytes2, p2, b2);
                vktVoxelView_t v1{bytes1, static_cast<vktDataFormat>(volume1.dataFormat), volume1.mappingLo,
                                  volume1.mappingHi};
                vktVoxelView_t v2{bytes2, static_cast<vktDataFormat>(volume2.dataFormat), volume2.mappingLo,
                                  volume2.mappingHi};
                binaryOp(x, y, z, v1, v2);
                std::memcpy(p1, bytes1, b1);   // setBytes volume1 then volume2 (Transform_serial.hpp:96-97)
                std::memcpy(p2, bytes2, b2);
            }
    e = s1.store();
    if (e == vktNoError && !same)
        e = s2.store();
    return e;
}

} // extern "C"
