// Render.cpp -- LookupTable, the headless Render front-ends and their C API.
//
// Reference: src/vkt/Render.cpp:770-987 (viewer setup: bbox = [0, dims * dist], default
// camera = 45 deg perspective, lens radius .05, focal distance 10, view_all(bbox); or the
// user's initialCamera), src/vkt/LookupTable.cpp (RGBA32F lookup table as a ManagedBuffer).
// The reference opens an interactive visionaray viewer; there is no display here, so Render
// accumulates a fixed number of frames headless and writes the snapshot file if one is
// requested.  The per-pixel work is vktHipRender (kernels/Render.hip).

#include "../runtime/Runtime.hpp"
#include "../StructuredVolume_impl.hpp"
#include "volkit_hip.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace vkt
{
//--- LookupTable -----------------------------------------------------------------------------
namespace
{
    std::size_t colorBytes(ColorFormat cf)
    {
        switch (cf)
        {
        case ColorFormat::R8: return 1;
        case ColorFormat::RG8: return 2;
        case ColorFormat::RGB8: return 3;
        case ColorFormat::RGBA8: return 4;
        case ColorFormat::R16UI: return 2;
        case ColorFormat::RG16UI: return 4;
        case ColorFormat::RGB16UI: return 6;
        case ColorFormat::RGBA16UI: return 8;
        case ColorFormat::R32UI: return 4;
        case ColorFormat::RG32UI: return 8;
        case ColorFormat::RGB32UI: return 12;
        case ColorFormat::RGBA32UI: return 16;
        case ColorFormat::R32F: return 4;
        case ColorFormat::RG32F: return 8;
        case ColorFormat::RGB32F: return 12;
        case ColorFormat::RGBA32F: return 16;
        default: return 0;
        }
    }

    std::size_t lutBytes(Vec3i d, ColorFormat cf)
    {
        return static_cast<std::size_t>(d.x > 0 ? d.x : 0) * static_cast<std::size_t>(d.y > 0 ? d.y : 0) *
               static_cast<std::size_t>(d.z > 0 ? d.z : 0) * colorBytes(cf);
    }
} // namespace

LookupTable::LookupTable() : ManagedBuffer(0) {}

LookupTable::LookupTable(int32_t dimX, int32_t dimY, int32_t dimZ, ColorFormat format)
    : ManagedBuffer(lutBytes(Vec3i{dimX, dimY, dimZ}, format)), dims_{dimX, dimY, dimZ}, format_(format)
{
}

void LookupTable::setDims(int32_t dimX, int32_t dimY, int32_t dimZ) { setDims(Vec3i{dimX, dimY, dimZ}); }

void LookupTable::getDims(int32_t& dimX, int32_t& dimY, int32_t& dimZ)
{
    dimX = dims_.x;
    dimY = dims_.y;
    dimZ = dims_.z;
}

void LookupTable::setDims(Vec3i dims)
{
    dims_ = dims;
    resize(getSizeInBytes());
}

Vec3i LookupTable::getDims() const { return dims_; }

void LookupTable::setColorFormat(ColorFormat cf)
{
    format_ = cf;
    resize(getSizeInBytes());
}

ColorFormat LookupTable::getColorFormat() const { return format_; }

void LookupTable::setData(uint8_t* data)
{
    std::size_t n = getSizeInBytes();
    if (n == 0 || data == nullptr)
        return;
    uint8_t* dst = getData();
    if (GetThreadExecutionPolicy().device == ExecutionPolicy::Device::GPU)
        (void)detail::memcpyHip(dst, data, n, CopyKind::HostToDevice);
    else
        std::memcpy(dst, data, n);
}

uint8_t* LookupTable::getData()
{
    migrate();
    return data_;
}

std::size_t LookupTable::getSizeInBytes() const { return lutBytes(dims_, format_); }

//--- camera (reference Render.cpp:838-866; visionaray pinhole/thin-lens camera, restated) --------
namespace
{
    struct F3
    {
        float x, y, z;
    };
    F3 sub(F3 a, F3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
    F3 scale(F3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
    F3 cross(F3 a, F3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
    F3 norm(F3 a)
    {
        float l = std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
        return {a.x / l, a.y / l, a.z / l};
    }

    struct Camera
    {
        F3 eye, center, up;
        float fovyDeg, lensRadius, focalDistance;
    };

    Camera cameraFor(RenderState const& rs, F3 box)
    {
        Camera c;
        if (rs.initialCamera.isSet)
        {
            c.eye = {rs.initialCamera.eye.x, rs.initialCamera.eye.y, rs.initialCamera.eye.z};
            c.center = {rs.initialCamera.center.x, rs.initialCamera.center.y, rs.initialCamera.center.z};
            c.up = {rs.initialCamera.up.x, rs.initialCamera.up.y, rs.initialCamera.up.z};
            c.fovyDeg = rs.initialCamera.fovy;
            c.lensRadius = rs.initialCamera.lensRadius;
            c.focalDistance = rs.initialCamera.focalDistance;
            return c;
        }
        // perspective(45 deg), lens radius .05, focal distance 10, view_all(bbox):
        // eye = center + (0, 0, r + r / atan(fovy)), r = |box| / 2
        c.fovyDeg = 45.f;
        c.lensRadius = 0.05f;
        c.focalDistance = 10.f;
        float const fovy = 45.f * 3.14159265f / 180.f;
        F3 const center{box.x * 0.5f, box.y * 0.5f, box.z * 0.5f};
        float const r = 0.5f * std::sqrt(box.x * box.x + box.y * box.y + box.z * box.z);
        c.center = center;
        c.eye = {center.x, center.y, center.z + r + r / std::atan(fovy)};
        c.up = {0.f, 1.f, 0.f};
        return c;
    }

    void fill3(float* dst, F3 v)
    {
        dst[0] = v.x;
        dst[1] = v.y;
        dst[2] = v.z;
    }

    vktHipRenderParams_t makeParams(RenderState const& rs, Camera const& c, F3 box)
    {
        vktHipRenderParams_t p;
        std::memset(&p, 0, sizeof(p));
        p.algo = static_cast<int32_t>(rs.renderAlgo);
        p.width = rs.viewportWidth;
        p.height = rs.viewportHeight;
        F3 const W = norm(sub(c.center, c.eye));
        F3 const right = norm(cross(W, c.up));
        F3 const up = cross(right, W);
        float const t = std::tan(0.5f * c.fovyDeg * 3.14159265f / 180.f);
        float const aspect = static_cast<float>(rs.viewportWidth) / static_cast<float>(rs.viewportHeight);
        fill3(p.eye, c.eye);
        fill3(p.W, W);
        fill3(p.U, scale(right, t * aspect));
        fill3(p.V, scale(up, t));
        fill3(p.right, right);
        fill3(p.up, up);
        p.lensRadius = c.lensRadius;
        p.focalDistance = c.focalDistance;
        fill3(p.bbox, box);
        p.dtRayMarching = rs.dtRayMarching;
        p.dtImplicitIso = rs.dtImplicitIso;
        p.majorant = rs.majorant;
        p.numIsoSurfaces = rs.numIsoSurfaces;
        for (int i = 0; i < 10; ++i)
            p.isoSurfaces[i] = rs.isoSurfaces[i];
        p.sRGB = rs.sRGB ? 1 : 0;
        return p;
    }

    // Renders numFrames frames into host RGBA floats; returns the camera used.
    Error renderImage(StructuredVolume& volume, RenderState const& rs, unsigned numFrames, float* rgba, Camera* used)
    {
        if (GetThreadExecutionPolicy().device != ExecutionPolicy::Device::GPU)
        {
            rt::setLastError("Render_hip: CPU execution policy");
            VKT_LOG(rt::LogLevel::Error) << "When calling algorithm: Render_hip -- volkit-amd implements the GPU "
                                            "(HIP/gfx950) backend only; set ExecutionPolicy::Device::GPU";
            return InvalidValue;
        }
        if (rs.viewportWidth <= 0 || rs.viewportHeight <= 0)
        {
            rt::fail("Render: empty viewport");
            return InvalidValue;
        }
        Vec3i d = volume.getDims();
        Vec3f dist = volume.getDist();
        F3 const box{d.x * dist.x, d.y * dist.y, d.z * dist.z};
        Camera cam = cameraFor(rs, box);
        if (used)
            *used = cam;
        vktHipRenderParams_t p = makeParams(rs, cam, box);
        if (rs.rgbaLookupTable != ResourceHandle(-1))
        {
            auto* lut = static_cast<LookupTable*>(GetManagedResource(rs.rgbaLookupTable));
            if (lut == nullptr || lut->getColorFormat() != ColorFormat::RGBA32F || lut->getDims().x <= 0)
            {
                rt::fail("Render: rgbaLookupTable must be an RGBA32F LookupTable");
                return InvalidValue;
            }
            p.lut = reinterpret_cast<float const*>(rt::deviceData(*lut));   // migrates to HBM
            if (p.lut == nullptr)
            {
                rt::fail(("Render: " + rt::takeMigrationFailure()).c_str());
                return InvalidValue;
            }
            p.lutSize = lut->getDims().x;
        }
        Vec2f m = volume.getVoxelMapping();
        vktHipVolumeView_t v{rt::deviceData(volume), d.x, d.y, d.z, static_cast<int32_t>(volume.getDataFormat()), m.x, m.y};
        std::size_t const n = static_cast<std::size_t>(p.width) * static_cast<std::size_t>(p.height) * 4;
        float* dev = nullptr;
        if (rt::check(hipMalloc(&dev, 2 * n * sizeof(float)), "hipMalloc(render target)") != vktNoError)
            return InvalidValue;
        vktError e = vktHipRender(v, &p, dev, dev + n, static_cast<int32_t>(numFrames));
        if (e == vktNoError)
            e = detail::memcpyHip(rgba, dev + n, n * sizeof(float), CopyKind::DeviceToHost);
        (void)hipFree(dev);
        return static_cast<Error>(e);
    }

    // binary PPM, origin top-left (the reference flips the GL read-back the same way)
    bool writePPM(char const* name, float const* rgba, int w, int h)
    {
        FILE* f = std::fopen(name, "wb");
        if (!f)
            return false;
        std::fprintf(f, "P6\n%d %d\n255\n", w, h);
        std::vector<uint8_t> row(static_cast<std::size_t>(w) * 3);
        for (int y = h - 1; y >= 0; --y)
        {
            for (int x = 0; x < w; ++x)
                for (int k = 0; k < 3; ++k)
                {
                    float c = rgba[(static_cast<std::size_t>(y) * w + x) * 4 + k];
                    c = c < 0.f ? 0.f : (c > 1.f ? 1.f : c);
                    row[static_cast<std::size_t>(x) * 3 + k] = static_cast<uint8_t>(c * 255.f + 0.5f);
                }
            std::fwrite(row.data(), 1, row.size(), f);
        }
        return std::fclose(f) == 0;
    }

    unsigned headlessFrames()
    {
        char const* s = std::getenv("VKT_RENDER_FRAMES");
        int n = s ? std::atoi(s) : 64;
        return n > 0 ? static_cast<unsigned>(n) : 64u;
    }
} // namespace

Error RenderToImage(StructuredVolume& volume, RenderState const& renderState, unsigned numFrames, float* rgba)
{
    if (rgba == nullptr)
    {
        rt::fail("RenderToImage: null image");
        return InvalidValue;
    }
    return renderImage(volume, renderState, numFrames, rgba, nullptr);
}

Error Render(StructuredVolume& volume, RenderState const& renderState, RenderState* newRenderState)
{
    std::vector<float> img(static_cast<std::size_t>(renderState.viewportWidth > 0 ? renderState.viewportWidth : 0) *
                           static_cast<std::size_t>(renderState.viewportHeight > 0 ? renderState.viewportHeight : 0) * 4);
    Camera cam;
    Error e = renderImage(volume, renderState, headlessFrames(), img.data(), &cam);
    if (e != NoError)
        return e;
    if (renderState.snapshotTool.enabled && renderState.snapshotTool.fileName && renderState.snapshotTool.fileName[0])
    {
        if (writePPM(renderState.snapshotTool.fileName, img.data(), renderState.viewportWidth,
                     renderState.viewportHeight))
        {
            std::string msg(renderState.snapshotTool.message ? renderState.snapshotTool.message : "");
            if (!msg.empty())
                VKT_LOG(rt::LogLevel::Info) << msg;
        }
        else
        {
            rt::fail("Render: error taking snapshot");
            return WriteError;
        }
    }
    if (newRenderState != nullptr)
    {
        *newRenderState = renderState;
        newRenderState->initialCamera.isSet = 1;
        newRenderState->initialCamera.eye = {cam.eye.x, cam.eye.y, cam.eye.z};
        newRenderState->initialCamera.center = {cam.center.x, cam.center.y, cam.center.z};
        newRenderState->initialCamera.up = {cam.up.x, cam.up.y, cam.up.z};
        newRenderState->initialCamera.fovy = cam.fovyDeg;
        newRenderState->initialCamera.lensRadius = cam.lensRadius;
        newRenderState->initialCamera.focalDistance = cam.focalDistance;
    }
    return NoError;
}

Error RenderFrames(StructuredVolume* volumes, std::size_t numAnimationFrames, RenderState const& renderState,
                   RenderState* newRenderState)
{
    if (volumes == nullptr || renderState.animationFrame >= numAnimationFrames)
    {
        rt::fail("RenderFrames: animationFrame outside the volume list");
        return InvalidValue;
    }
    return Render(volumes[renderState.animationFrame], renderState, newRenderState);
}

} // vkt

//--- C API -----------------------------------------------------------------------------------
struct vktLookupTable_impl
{
    template <typename... A>
    explicit vktLookupTable_impl(A&&... a) : lut(std::forward<A>(a)...)
    {
    }
    vkt::LookupTable lut;
};

namespace
{
    vkt::RenderState toCpp(vktRenderState_t const& c)
    {
        vkt::RenderState r;
        r.renderAlgo = static_cast<vkt::RenderAlgo>(c.renderAlgo);
        r.dtRayMarching = c.dtRayMarching;
        r.numIsoSurfaces = c.numIsoSurfaces;
        for (int i = 0; i < 10; ++i)
            r.isoSurfaces[i] = c.isoSurfaces[i];
        r.dtImplicitIso = c.dtImplicitIso;
        r.majorant = c.majorant;
        r.animationFrame = c.animationFrame;
        r.rgbaLookupTable = c.rgbaLookupTable;
        r.histogram = c.histogram;
        r.viewportWidth = c.viewportWidth;
        r.viewportHeight = c.viewportHeight;
        r.sRGB = c.sRGB;
        r.initialCamera.isSet = c.initialCamera.isSet;
        r.initialCamera.eye = {c.initialCamera.eye.x, c.initialCamera.eye.y, c.initialCamera.eye.z};
        r.initialCamera.center = {c.initialCamera.center.x, c.initialCamera.center.y, c.initialCamera.center.z};
        r.initialCamera.up = {c.initialCamera.up.x, c.initialCamera.up.y, c.initialCamera.up.z};
        r.initialCamera.fovy = c.initialCamera.fovy;
        r.initialCamera.lensRadius = c.initialCamera.lensRadius;
        r.initialCamera.focalDistance = c.initialCamera.focalDistance;
        r.snapshotTool.enabled = c.snapshotTool.enabled;
        r.snapshotTool.fileName = c.snapshotTool.fileName;
        r.snapshotTool.takeOnClose = c.snapshotTool.takeOnClose;
        r.snapshotTool.key = c.snapshotTool.key;
        r.snapshotTool.message = c.snapshotTool.message;
        return r;
    }

    void toC(vkt::RenderState const& r, vktRenderState_t& c)
    {
        c.initialCamera.isSet = r.initialCamera.isSet;
        c.initialCamera.eye = {r.initialCamera.eye.x, r.initialCamera.eye.y, r.initialCamera.eye.z};
        c.initialCamera.center = {r.initialCamera.center.x, r.initialCamera.center.y, r.initialCamera.center.z};
        c.initialCamera.up = {r.initialCamera.up.x, r.initialCamera.up.y, r.initialCamera.up.z};
        c.initialCamera.fovy = r.initialCamera.fovy;
        c.initialCamera.lensRadius = r.initialCamera.lensRadius;
        c.initialCamera.focalDistance = r.initialCamera.focalDistance;
    }
} // namespace

extern "C" {

void vktLookupTableCreate(vktLookupTable* lut, int32_t dimX, int32_t dimY, int32_t dimZ, vktColorFormat format)
{
    *lut = new vktLookupTable_impl(dimX, dimY, dimZ, static_cast<vkt::ColorFormat>(format));
}

void vktLookupTableDestroy(vktLookupTable lut) { delete lut; }

void vktLookupTableSetDims3i(vktLookupTable lut, int32_t x, int32_t y, int32_t z) { lut->lut.setDims(x, y, z); }

void vktLookupTableGetDims3i(vktLookupTable lut, int32_t* x, int32_t* y, int32_t* z) { lut->lut.getDims(*x, *y, *z); }

void vktLookupTableSetDims3iv(vktLookupTable lut, vktVec3i_t d) { lut->lut.setDims(vkt::Vec3i{d.x, d.y, d.z}); }

vktVec3i_t vktLookupTableGetDims3iv(vktLookupTable lut)
{
    vkt::Vec3i d = lut->lut.getDims();
    return vktVec3i_t{d.x, d.y, d.z};
}

void vktLookupTableSetColorFormat(vktLookupTable lut, vktColorFormat f)
{
    lut->lut.setColorFormat(static_cast<vkt::ColorFormat>(f));
}

vktColorFormat vktLookupTableGetColorFormat(vktLookupTable lut)
{
    return static_cast<vktColorFormat>(lut->lut.getColorFormat());
}

void vktLookupTableSetData(vktLookupTable lut, uint8_t* data) { lut->lut.setData(data); }

uint8_t* vktLookupTableGetData(vktLookupTable lut) { return lut->lut.getData(); }

size_t vktLookupTableGetSizeInBytes(vktLookupTable lut) { return lut->lut.getSizeInBytes(); }

vktResourceHandle vktLookupTableGetResourceHandle(vktLookupTable lut) { return lut->lut.getResourceHandle(); }

void vktLookupTableMigrate(vktLookupTable lut) { lut->lut.migrate(); }

void vktRenderStateDefaultInit(vktRenderState_t* rs)
{
    vkt::RenderState d;
    std::memset(rs, 0, sizeof(*rs));
    rs->renderAlgo = vktRenderAlgoRayMarching;
    rs->dtRayMarching = d.dtRayMarching;
    rs->numIsoSurfaces = d.numIsoSurfaces;
    rs->isoSurfaces[0] = d.isoSurfaces[0];
    rs->dtImplicitIso = d.dtImplicitIso;
    rs->majorant = d.majorant;
    rs->animationFrame = 0;
    rs->rgbaLookupTable = d.rgbaLookupTable;
    rs->histogram = d.histogram;
    rs->viewportWidth = d.viewportWidth;
    rs->viewportHeight = d.viewportHeight;
    rs->sRGB = d.sRGB;
    toC(d, *rs);
    rs->snapshotTool.enabled = 0;
    rs->snapshotTool.fileName = "";
    rs->snapshotTool.takeOnClose = 0;
    rs->snapshotTool.key = 'p';
    rs->snapshotTool.message = "";
}

vktError vktRenderSV(vktStructuredVolume volume, vktRenderState_t renderState, vktRenderState_t* newRenderState)
{
    if (!volume)
        return vktInvalidValue;
    vkt::RenderState out;
    vkt::Error e = vkt::Render(volume->volume, toCpp(renderState), &out);
    if (e == vkt::NoError && newRenderState)
    {
        *newRenderState = renderState;
        toC(out, *newRenderState);
    }
    return static_cast<vktError>(e);
}

vktError vktHipRenderParamsFromState(vktRenderState_t const* renderState, vktVec3f_t bbox, vktHipRenderParams_t* params)
{
    if (!renderState || !params)
        return vkt::rt::fail("vktHipRenderParamsFromState: null pointer");
    vkt::RenderState rs = toCpp(*renderState);
    vkt::F3 box{bbox.x, bbox.y, bbox.z};
    *params = vkt::makeParams(rs, vkt::cameraFor(rs, box), box);
    return vktNoError;
}

vktError vktRenderSVToImage(vktStructuredVolume volume, vktRenderState_t renderState, uint32_t numFrames, float* rgba)
{
    if (!volume)
        return vktInvalidValue;
    return static_cast<vktError>(vkt::RenderToImage(volume->volume, toCpp(renderState), numFrames, rgba));
}

} // extern "C"
