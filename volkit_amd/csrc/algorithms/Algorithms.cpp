// Algorithms.cpp -- C++ and C front-ends of the StructuredVolume core algorithms.
//
// Reference front-ends: src/vkt/Fill.cpp:32-186, src/vkt/Copy.cpp:26-123,
// src/vkt/Arithmetic.cpp:26-1161, src/vkt/Transform.cpp:26-153, src/vkt/Resample.cpp:22-31.
// There, VKT_LEGACY_CALL__ (src/vkt/Callable.hpp:82-113) reads the thread policy and calls
// FUNC##_serial or FUNC##_cuda.  Here the GPU branch calls the vktHip* backend
// (include/volkit_hip.h) on views of the migrated volumes; the CPU branch is not part of
// this library -- it logs an error and returns InvalidValue rather than silently running a
// host loop (the reference's own GPU Fill is a silent no-op, src/vkt/Callable.cpp:53-66).
// printPerformance wraps the call in hipEvents on the compute stream and logs the time,
// like VKT_CALL_CUDA_TIMER_ (Callable.hpp:37-47).

#include "../runtime/Runtime.hpp"
#include "../StructuredVolume_impl.hpp"
#include "volkit_hip.h"

#include <cstring>
#include <vector>

namespace vkt
{
namespace
{
    vktHipVolumeView_t view(StructuredVolume& v)
    {
        vktHipVolumeView_t out;
        out.data = rt::deviceData(v);   // migrates to the thread's device first (nullptr if that failed)
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

    vktVec3i_t c3(Vec3i v) { return vktVec3i_t{v.x, v.y, v.z}; }

    template <class Fn>
    Error dispatch(char const* name, Fn&& fn)
    {
        ExecutionPolicy ep = GetThreadExecutionPolicy();
        if (ep.device != ExecutionPolicy::Device::GPU)
        {
            rt::setLastError(std::string(name) + ": CPU execution policy");
            VKT_LOG(rt::LogLevel::Error) << "When calling algorithm: " << name
                                         << " -- volkit-amd implements the GPU (HIP/gfx950) backend only; set "
                                            "ExecutionPolicy::Device::GPU";
            return InvalidValue;
        }
        rt::ScopedKernelTimer timer(name, ep.printPerformance != False);
        (void)rt::takeMigrationFailure();
        return static_cast<Error>(rt::explainFailure(static_cast<vktError>(fn()), name));
    }
} // namespace

//--- Fill ----------------------------------------------------------------------------------
Error Fill(StructuredVolume& volume, float value) { return FillRange(volume, Vec3i{0, 0, 0}, volume.getDims(), value); }

Error FillRange(StructuredVolume& volume, int32_t fx, int32_t fy, int32_t fz, int32_t lx, int32_t ly, int32_t lz,
                float value)
{
    return FillRange(volume, Vec3i{fx, fy, fz}, Vec3i{lx, ly, lz}, value);
}

Error FillRange(StructuredVolume& volume, Vec3i first, Vec3i last, float value)
{
    return dispatch("FillRange_hip", [&] { return vktHipFillRange(view(volume), c3(first), c3(last), value); });
}

//--- Copy ----------------------------------------------------------------------------------
Error Copy(StructuredVolume& dst, StructuredVolume& src)
{
    return CopyRange(dst, src, Vec3i{0, 0, 0}, dst.getDims(), Vec3i{0, 0, 0});
}

Error CopyRange(StructuredVolume& dst, StructuredVolume& src, int32_t fx, int32_t fy, int32_t fz, int32_t lx,
                int32_t ly, int32_t lz, int32_t ox, int32_t oy, int32_t oz)
{
    return CopyRange(dst, src, Vec3i{fx, fy, fz}, Vec3i{lx, ly, lz}, Vec3i{ox, oy, oz});
}

Error CopyRange(StructuredVolume& dst, StructuredVolume& src, Vec3i first, Vec3i last, Vec3i dstOffset)
{
    return dispatch("CopyRange_hip", [&] {
        vktHipVolumeView_t d = view(dst);
        vktHipVolumeView_t s = view(src);
        return vktHipCopyRange(d, s, c3(first), c3(last), c3(dstOffset));
    });
}

//--- Arithmetic ----------------------------------------------------------------------------
namespace
{
    Error arith(char const* name, vktHipArithmeticOp op, StructuredVolume& dest, StructuredVolume& s1,
                StructuredVolume& s2, Vec3i first, Vec3i last, Vec3i off)
    {
        return dispatch(name, [&] {
            vktHipVolumeView_t d = view(dest);
            vktHipVolumeView_t a = view(s1);
            vktHipVolumeView_t b = view(s2);
            return vktHipArithmeticRange(op, d, a, b, c3(first), c3(last), c3(off));
        });
    }
} // namespace

// Whole-volume ops use dest's dims as the range (reference Arithmetic.cpp:26-42).
#define VKT_DEFINE_ARITHMETIC_(NAME, OP)                                                                        \
    Error NAME(StructuredVolume& dest, StructuredVolume& source1, StructuredVolume& source2)                   \
    {                                                                                                         \
        return arith(#NAME "Range_hip", OP, dest, source1, source2, Vec3i{0, 0, 0}, dest.getDims(),            \
                     Vec3i{0, 0, 0});                                                                         \
    }                                                                                                         \
    Error NAME##Range(StructuredVolume& dest, StructuredVolume& source1, StructuredVolume& source2, int32_t fx, \
                      int32_t fy, int32_t fz, int32_t lx, int32_t ly, int32_t lz, int32_t ox, int32_t oy,       \
                      int32_t oz)                                                                             \
    {                                                                                                         \
        return arith(#NAME "Range_hip", OP, dest, source1, source2, Vec3i{fx, fy, fz}, Vec3i{lx, ly, lz},      \
                     Vec3i{ox, oy, oz});                                                                      \
    }                                                                                                         \
    Error NAME##Range(StructuredVolume& dest, StructuredVolume& source1, StructuredVolume& source2, Vec3i first, \
                      Vec3i last, Vec3i dstOffset)                                                            \
    {                                                                                                         \
        return arith(#NAME "Range_hip", OP, dest, source1, source2, first, last, dstOffset);                   \
    }

VKT_DEFINE_ARITHMETIC_(Sum, vktHipOpSum)
VKT_DEFINE_ARITHMETIC_(Diff, vktHipOpDiff)
VKT_DEFINE_ARITHMETIC_(Prod, vktHipOpProd)
VKT_DEFINE_ARITHMETIC_(Quot, vktHipOpQuot)
VKT_DEFINE_ARITHMETIC_(AbsDiff, vktHipOpAbsDiff)
VKT_DEFINE_ARITHMETIC_(SafeSum, vktHipOpSafeSum)
VKT_DEFINE_ARITHMETIC_(SafeDiff, vktHipOpSafeDiff)
VKT_DEFINE_ARITHMETIC_(SafeProd, vktHipOpSafeProd)
VKT_DEFINE_ARITHMETIC_(SafeQuot, vktHipOpSafeQuot)
VKT_DEFINE_ARITHMETIC_(SafeAbsDiff, vktHipOpSafeAbsDiff)
#undef VKT_DEFINE_ARITHMETIC_

//--- Transform -----------------------------------------------------------------------------
Error Transform(StructuredVolume& volume, TransformUnaryOp op)
{
    return TransformRange(volume, Vec3i{0, 0, 0}, volume.getDims(), op);
}

Error Transform(StructuredVolume& v1, StructuredVolume& v2, TransformBinaryOp op)
{
    return TransformRange(v1, v2, Vec3i{0, 0, 0}, v1.getDims(), op);
}

Error TransformRange(StructuredVolume& volume, int32_t fx, int32_t fy, int32_t fz, int32_t lx, int32_t ly,
                     int32_t lz, TransformUnaryOp op)
{
    return TransformRange(volume, Vec3i{fx, fy, fz}, Vec3i{lx, ly, lz}, op);
}

Error TransformRange(StructuredVolume& volume, Vec3i first, Vec3i last, TransformUnaryOp op)
{
    return dispatch("TransformRange_hip", [&] {
        return vktHipTransformRange1(view(volume), c3(first), c3(last), reinterpret_cast<vktTransformUnaryOp>(op));
    });
}

Error TransformRange(StructuredVolume& v1, StructuredVolume& v2, int32_t fx, int32_t fy, int32_t fz, int32_t lx,
                     int32_t ly, int32_t lz, TransformBinaryOp op)
{
    return TransformRange(v1, v2, Vec3i{fx, fy, fz}, Vec3i{lx, ly, lz}, op);
}

Error TransformRange(StructuredVolume& v1, StructuredVolume& v2, Vec3i first, Vec3i last, TransformBinaryOp op)
{
    return dispatch("TransformRange_hip", [&] {
        vktHipVolumeView_t a = view(v1);
        vktHipVolumeView_t b = view(v2);
        return vktHipTransformRange2(a, b, c3(first), c3(last), vktVec3i_t{0, 0, 0},
                                     reinterpret_cast<vktTransformBinaryOp>(op));
    });
}

//--- Resample ------------------------------------------------------------------------------
Error Resample(StructuredVolume& dst, StructuredVolume& src, FilterMode fm)
{
    return dispatch("Resample_hip", [&] {
        vktHipVolumeView_t d = view(dst);
        vktHipVolumeView_t s = view(src);
        return vktHipResample(d, s, static_cast<vktFilterMode>(fm));
    });
}

} // vkt

//--- C API ---------------------------------------------------------------------------------
using vkt::Vec3i;

extern "C" {

vktError vktFillSV(vktStructuredVolume volume, float value)
{
    return static_cast<vktError>(vkt::Fill(volume->volume, value));
}

vktError vktFillRangeSV(vktStructuredVolume volume, int32_t fx, int32_t fy, int32_t fz, int32_t lx, int32_t ly,
                        int32_t lz, float value)
{
    return static_cast<vktError>(vkt::FillRange(volume->volume, Vec3i{fx, fy, fz}, Vec3i{lx, ly, lz}, value));
}

vktError vktCopySV(vktStructuredVolume dst, vktStructuredVolume src)
{
    return static_cast<vktError>(vkt::Copy(dst->volume, src->volume));
}

vktError vktCopyRangeSV(vktStructuredVolume dst, vktStructuredVolume src, int32_t fx, int32_t fy, int32_t fz,
                        int32_t lx, int32_t ly, int32_t lz, int32_t ox, int32_t oy, int32_t oz)
{
    return static_cast<vktError>(
        vkt::CopyRange(dst->volume, src->volume, Vec3i{fx, fy, fz}, Vec3i{lx, ly, lz}, Vec3i{ox, oy, oz}));
}

#define VKT_DEFINE_ARITHMETIC_C_(NAME)                                                                          \
    vktError vkt##NAME##SV(vktStructuredVolume dest, vktStructuredVolume s1, vktStructuredVolume s2)          \
    {                                                                                                         \
        return static_cast<vktError>(vkt::NAME(dest->volume, s1->volume, s2->volume));                        \
    }                                                                                                         \
    vktError vkt##NAME##RangeSV(vktStructuredVolume dest, vktStructuredVolume s1, vktStructuredVolume s2,     \
                                int32_t fx, int32_t fy, int32_t fz, int32_t lx, int32_t ly, int32_t lz,       \
                                int32_t ox, int32_t oy, int32_t oz)                                           \
    {                                                                                                         \
        return static_cast<vktError>(vkt::NAME##Range(dest->volume, s1->volume, s2->volume, Vec3i{fx, fy, fz}, \
                                                      Vec3i{lx, ly, lz}, Vec3i{ox, oy, oz}));                 \
    }
VKT_DEFINE_ARITHMETIC_C_(Sum)
VKT_DEFINE_ARITHMETIC_C_(Diff)
VKT_DEFINE_ARITHMETIC_C_(Prod)
VKT_DEFINE_ARITHMETIC_C_(Quot)
VKT_DEFINE_ARITHMETIC_C_(AbsDiff)
VKT_DEFINE_ARITHMETIC_C_(SafeSum)
VKT_DEFINE_ARITHMETIC_C_(SafeDiff)
VKT_DEFINE_ARITHMETIC_C_(SafeProd)
VKT_DEFINE_ARITHMETIC_C_(SafeQuot)
VKT_DEFINE_ARITHMETIC_C_(SafeAbsDiff)
#undef VKT_DEFINE_ARITHMETIC_C_

vktError vktTransformSV1(vktStructuredVolume volume, vktTransformUnaryOp op)
{
    return static_cast<vktError>(vkt::Transform(volume->volume, reinterpret_cast<vkt::TransformUnaryOp>(op)));
}

vktError vktTransformSV2(vktStructuredVolume v1, vktStructuredVolume v2, vktTransformBinaryOp op)
{
    return static_cast<vktError>(vkt::Transform(v1->volume, v2->volume, reinterpret_cast<vkt::TransformBinaryOp>(op)));
}

vktError vktTransformRangeSV1(vktStructuredVolume volume, int32_t fx, int32_t fy, int32_t fz, int32_t lx, int32_t ly,
                              int32_t lz, vktTransformUnaryOp op)
{
    return static_cast<vktError>(vkt::TransformRange(volume->volume, Vec3i{fx, fy, fz}, Vec3i{lx, ly, lz},
                                                     reinterpret_cast<vkt::TransformUnaryOp>(op)));
}

// 12-argument form of the reference header (include/c/vkt/Transform.h:45-56): volume2 is
// visited at (x,y,z) + volume2Offset.
vktError vktTransformRangeSV2(vktStructuredVolume v1, vktStructuredVolume v2, int32_t fx, int32_t fy, int32_t fz,
                              int32_t lx, int32_t ly, int32_t lz, int32_t ox, int32_t oy, int32_t oz,
                              vktTransformBinaryOp op)
{
    vkt::ExecutionPolicy ep = vkt::GetThreadExecutionPolicy();
    if (ep.device != vkt::ExecutionPolicy::Device::GPU)
        return vkt::rt::fail("TransformRange_hip: CPU execution policy (volkit-amd implements the GPU backend only)");
    vkt::rt::ScopedKernelTimer timer("TransformRange_hip", ep.printPerformance != vkt::False);
    (void)vkt::rt::takeMigrationFailure();
    auto mk = [](vkt::StructuredVolume& v) {
        vktHipVolumeView_t o;
        o.data = vkt::rt::deviceData(v);
        vkt::Vec3i d = v.getDims();
        o.dimX = d.x;
        o.dimY = d.y;
        o.dimZ = d.z;
        o.dataFormat = static_cast<int32_t>(v.getDataFormat());
        o.mappingLo = v.getVoxelMapping().x;
        o.mappingHi = v.getVoxelMapping().y;
        return o;
    };
    vktHipVolumeView_t a = mk(v1->volume);
    vktHipVolumeView_t b = mk(v2->volume);
    return vkt::rt::explainFailure(
        vktHipTransformRange2(a, b, vktVec3i_t{fx, fy, fz}, vktVec3i_t{lx, ly, lz}, vktVec3i_t{ox, oy, oz}, op),
        "TransformRange_hip");
}

vktError vktResampleSV(vktStructuredVolume dst, vktStructuredVolume src, vktFilterMode fm)
{
    return static_cast<vktError>(vkt::Resample(dst->volume, src->volume, static_cast<vkt::FilterMode>(fm)));
}

} // extern "C"
