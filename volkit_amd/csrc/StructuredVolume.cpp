// StructuredVolume.cpp -- the dense voxel container and its C handle layer.
//
// Reference: src/vkt/StructuredVolume.cpp:24-374 (C++ class and C Create/CreateCopy/
// Destroy), include/c/vkt/StructuredVolume.h:38-120 (accessors the reference declares but
// never defines -- all of them are defined here).
//
// Layout in memory (host or HBM): x-fastest, byte offset ((z*dimY + y)*dimX + x) * bpv with
// 64-bit arithmetic (the reference multiplies z*dimX in 32 bits).  Host accessors migrate
// first; under the GPU policy they move one voxel with a synchronous copy instead of
// dereferencing a device pointer on the host as the reference would.

#include "runtime/Runtime.hpp"
#include "volkit_codec.hpp"
#include "StructuredVolume_impl.hpp"

namespace vkt
{
    namespace
    {
        // where the bytes are (after migrate(): the thread's device, unless that migration failed
        // and left them where they were)
        bool residentOnGpu(ManagedBuffer<uint8_t> const& b)
        {
            ExecutionPolicy gpu;
            gpu.device = ExecutionPolicy::Device::GPU;
            return b.residentOn(gpu);
        }
    }

    StructuredVolume::StructuredVolume()
        : ManagedBuffer(0)
        , dims_{0, 0, 0}
        , dataFormat_(DataFormat::UInt8)
        , dist_{1.f, 1.f, 1.f}
        , voxelMapping_{0.f, 1.f}
        , haloSize_{.5f, .5f, .5f}
    {
    }

    StructuredVolume::StructuredVolume(int32_t dimX, int32_t dimY, int32_t dimZ, DataFormat dataFormat,
                                       float distX, float distY, float distZ, float mappingLo, float mappingHi)
        : ManagedBuffer(static_cast<std::size_t>(dimX) * static_cast<std::size_t>(dimY) *
                        static_cast<std::size_t>(dimZ) * codec::bytesPerVoxel(static_cast<int32_t>(dataFormat)))
        , dims_{dimX, dimY, dimZ}
        , dataFormat_(dataFormat)
        , dist_{distX, distY, distZ}
        , voxelMapping_{mappingLo, mappingHi}
        , haloSize_{.5f, .5f, .5f}
    {
    }

    void StructuredVolume::setDims(int32_t dimX, int32_t dimY, int32_t dimZ) { setDims(Vec3i{dimX, dimY, dimZ}); }

    void StructuredVolume::getDims(int32_t& dimX, int32_t& dimY, int32_t& dimZ)
    {
        dimX = dims_.x;
        dimY = dims_.y;
        dimZ = dims_.z;
    }

    void StructuredVolume::setDims(Vec3i dims)
    {
        dims_ = dims;
        resize(getSizeInBytes());
    }

    Vec3i StructuredVolume::getDims() const { return dims_; }

    void StructuredVolume::setDataFormat(DataFormat dataFormat)
    {
        dataFormat_ = dataFormat;
        resize(getSizeInBytes());
    }

    DataFormat StructuredVolume::getDataFormat() const { return dataFormat_; }

    void StructuredVolume::setDist(float distX, float distY, float distZ) { dist_ = {distX, distY, distZ}; }

    void StructuredVolume::getDist(float& distX, float& distY, float& distZ)
    {
        distX = dist_.x;
        distY = dist_.y;
        distZ = dist_.z;
    }

    void StructuredVolume::setDist(Vec3f dist) { dist_ = dist; }

    Vec3f StructuredVolume::getDist() const { return dist_; }

    void StructuredVolume::setVoxelMapping(float lo, float hi) { voxelMapping_ = {lo, hi}; }

    void StructuredVolume::getVoxelMapping(float& lo, float& hi)
    {
        lo = voxelMapping_.x;
        hi = voxelMapping_.y;
    }

    void StructuredVolume::setVoxelMapping(Vec2f mapping) { voxelMapping_ = mapping; }

    Vec2f StructuredVolume::getVoxelMapping() const { return voxelMapping_; }

    Box3f StructuredVolume::getDomainBounds() const
    {
        Box3f b = getObjectBounds();
        b.min = {b.min.x - haloSize_.x, b.min.y - haloSize_.y, b.min.z - haloSize_.z};
        b.max = {b.max.x + haloSize_.x, b.max.y + haloSize_.y, b.max.z + haloSize_.z};
        return b;
    }

    Box3f StructuredVolume::getObjectBounds() const
    {
        return {{0.f, 0.f, 0.f}, {dims_.x * dist_.x, dims_.y * dist_.y, dims_.z * dist_.z}};
    }

    uint8_t* StructuredVolume::getData()
    {
        migrate();
        return data_;
    }

    // One voxel's bytes between the buffer (wherever it lives) and host memory.
    void StructuredVolume::getBytes(int32_t x, int32_t y, int32_t z, uint8_t* out)
    {
        migrate();
        std::size_t off = linearIndex(x, y, z);
        uint8_t bpv = getBytesPerVoxel();
        if (residentOnGpu(*this))
            (void)detail::memcpyHip(out, data_ + off, bpv, CopyKind::DeviceToHost);
        else
            for (uint8_t i = 0; i < bpv; ++i)
                out[i] = data_[off + i];
    }

    void StructuredVolume::setBytes(int32_t x, int32_t y, int32_t z, uint8_t const* in)
    {
        migrate();
        std::size_t off = linearIndex(x, y, z);
        uint8_t bpv = getBytesPerVoxel();
        if (residentOnGpu(*this))
            (void)detail::memcpyHip(data_ + off, in, bpv, CopyKind::HostToDevice);
        else
            for (uint8_t i = 0; i < bpv; ++i)
                data_[off + i] = in[i];
    }

    void StructuredVolume::getBytes(Vec3i i, uint8_t* out) { getBytes(i.x, i.y, i.z, out); }

    void StructuredVolume::setBytes(Vec3i i, uint8_t const* in) { setBytes(i.x, i.y, i.z, in); }

    void StructuredVolume::setValue(int32_t x, int32_t y, int32_t z, float value)
    {
        int32_t fmt = static_cast<int32_t>(dataFormat_);
        bool write = false;
        uint32_t code = codec::encode(value, fmt, codec::makeMapParams(voxelMapping_.x, voxelMapping_.y), write);
        if (!write)
        {
            migrate();   // the reference still migrates, then writes nothing
            return;
        }
        uint8_t bytes[4] = {uint8_t(code), uint8_t(code >> 8), uint8_t(code >> 16), uint8_t(code >> 24)};
        setBytes(x, y, z, bytes);
    }

    void StructuredVolume::getValue(int32_t x, int32_t y, int32_t z, float& value)
    {
        int32_t fmt = static_cast<int32_t>(dataFormat_);
        uint8_t bytes[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (codec::bytesPerVoxel(fmt) <= 4)
            getBytes(x, y, z, bytes);
        else
            migrate();
        uint32_t code = uint32_t(bytes[0]) | uint32_t(bytes[1]) << 8 | uint32_t(bytes[2]) << 16 |
                        uint32_t(bytes[3]) << 24;
        value = codec::decode(code, fmt, voxelMapping_.x, voxelMapping_.y, value);
    }

    float StructuredVolume::getValue(int32_t x, int32_t y, int32_t z)
    {
        float value = 0.f;
        getValue(x, y, z, value);
        return value;
    }

    void StructuredVolume::setValue(Vec3i i, float value) { setValue(i.x, i.y, i.z, value); }

    void StructuredVolume::getValue(Vec3i i, float& value) { getValue(i.x, i.y, i.z, value); }

    float StructuredVolume::getValue(Vec3i i) { return getValue(i.x, i.y, i.z); }

    uint8_t StructuredVolume::getBytesPerVoxel() const
    {
        return static_cast<uint8_t>(codec::bytesPerVoxel(static_cast<int32_t>(dataFormat_)));
    }

    std::size_t StructuredVolume::getSizeInBytes() const
    {
        return static_cast<std::size_t>(dims_.x) * static_cast<std::size_t>(dims_.y) *
               static_cast<std::size_t>(dims_.z) * getBytesPerVoxel();
    }

    std::size_t StructuredVolume::linearIndex(int32_t x, int32_t y, int32_t z) const
    {
        std::size_t dx = static_cast<std::size_t>(dims_.x);
        std::size_t idx = (static_cast<std::size_t>(z) * static_cast<std::size_t>(dims_.y) +
                           static_cast<std::size_t>(y)) * dx + static_cast<std::size_t>(x);
        return idx * getBytesPerVoxel();
    }

    std::size_t StructuredVolume::linearIndex(Vec3i i) const { return linearIndex(i.x, i.y, i.z); }

    //--- Voxel codec API (reference src/vkt/Voxel.cpp:19-69) ----------------------------
    Error MapVoxel(uint8_t* dst, float value, DataFormat dataFormat, float mappingLo, float mappingHi)
    {
        int32_t fmt = static_cast<int32_t>(dataFormat);
        bool write = false;
        uint32_t code = codec::encode(value, fmt, codec::makeMapParams(mappingLo, mappingHi), write);
        if (write)
            for (uint32_t i = 0; i < codec::bytesPerVoxel(fmt); ++i)
                dst[i] = static_cast<uint8_t>(code >> (8 * i));
        return NoError;
    }

    Error UnmapVoxel(float& value, uint8_t const* src, DataFormat dataFormat, float mappingLo, float mappingHi)
    {
        int32_t fmt = static_cast<int32_t>(dataFormat);
        uint32_t code = 0;
        uint32_t n = codec::bytesPerVoxel(fmt);
        if (n <= 4)
            for (uint32_t i = 0; i < n; ++i)
                code |= static_cast<uint32_t>(src[i]) << (8 * i);
        value = codec::decode(code, fmt, mappingLo, mappingHi, value);
        return NoError;
    }
} // vkt

//--- C API -----------------------------------------------------------------------------
using vkt::StructuredVolume;

extern "C" {

uint8_t vktStructuredVolumeGetMaxBytesPerVoxel(void) { return StructuredVolume::GetMaxBytesPerVoxel(); }

void vktStructuredVolumeCreate(vktStructuredVolume* volume, int32_t dimX, int32_t dimY, int32_t dimZ,
                               vktDataFormat dataFormat, float distX, float distY, float distZ, float mappingLo,
                               float mappingHi)
{
    if (volume == nullptr)
        return;
    *volume = new vktStructuredVolume_impl(dimX, dimY, dimZ, static_cast<vkt::DataFormat>(dataFormat), distX, distY,
                                           distZ, mappingLo, mappingHi);
}

void vktStructuredVolumeCreateCopy(vktStructuredVolume* volume, vktStructuredVolume rhs)
{
    if (volume == nullptr || rhs == nullptr)
        return;
    *volume = new vktStructuredVolume_impl(rhs->volume);
}

void vktStructuredVolumeDestroy(vktStructuredVolume volume) { delete volume; }

void vktStructuredVolumeSetDims3i(vktStructuredVolume v, int32_t x, int32_t y, int32_t z) { v->volume.setDims(x, y, z); }

void vktStructuredVolumeGetDims3i(vktStructuredVolume v, int32_t* x, int32_t* y, int32_t* z)
{
    vkt::Vec3i d = v->volume.getDims();
    *x = d.x;
    *y = d.y;
    *z = d.z;
}

void vktStructuredVolumeSetDims3iv(vktStructuredVolume v, vktVec3i_t d) { v->volume.setDims(d.x, d.y, d.z); }

vktVec3i_t vktStructuredVolumeGetDims3iv(vktStructuredVolume v)
{
    vkt::Vec3i d = v->volume.getDims();
    return vktVec3i_t{d.x, d.y, d.z};
}

void vktStructuredVolumeSetDataFormat(vktStructuredVolume v, vktDataFormat f)
{
    v->volume.setDataFormat(static_cast<vkt::DataFormat>(f));
}

vktDataFormat vktStructuredVolumeGetDataFormat(vktStructuredVolume v)
{
    return static_cast<vktDataFormat>(v->volume.getDataFormat());
}

void vktStructuredVolumeSetDist3f(vktStructuredVolume v, float x, float y, float z) { v->volume.setDist(x, y, z); }

void vktStructuredVolumeGetDist3f(vktStructuredVolume v, float* x, float* y, float* z)
{
    vkt::Vec3f d = v->volume.getDist();
    *x = d.x;
    *y = d.y;
    *z = d.z;
}

void vktStructuredVolumeSetDist3fv(vktStructuredVolume v, vktVec3f_t d) { v->volume.setDist(d.x, d.y, d.z); }

vktVec3f_t vktStructuredVolumeGetDist3fv(vktStructuredVolume v)
{
    vkt::Vec3f d = v->volume.getDist();
    return vktVec3f_t{d.x, d.y, d.z};
}

void vktStructuredVolumeSetVoxelMapping2f(vktStructuredVolume v, float lo, float hi) { v->volume.setVoxelMapping(lo, hi); }

void vktStructuredVolumeGetVoxelMapping2f(vktStructuredVolume v, float* lo, float* hi)
{
    vkt::Vec2f m = v->volume.getVoxelMapping();
    *lo = m.x;
    *hi = m.y;
}

void vktStructuredVolumeSetVoxelMapping2fv(vktStructuredVolume v, vktVec2f_t m) { v->volume.setVoxelMapping(m.x, m.y); }

vktVec2f_t vktStructuredVolumeGetVoxelMapping2fv(vktStructuredVolume v)
{
    vkt::Vec2f m = v->volume.getVoxelMapping();
    return vktVec2f_t{m.x, m.y};
}

static vktBox3f_t toC(vkt::Box3f b) { return vktBox3f_t{{b.min.x, b.min.y, b.min.z}, {b.max.x, b.max.y, b.max.z}}; }

vktBox3f_t vktStructuredVolumeGetDomainBounds(vktStructuredVolume v) { return toC(v->volume.getDomainBounds()); }

vktBox3f_t vktStructuredVolumeGetObjectBounds(vktStructuredVolume v) { return toC(v->volume.getObjectBounds()); }

uint8_t* vktStructuredVolumeGetData(vktStructuredVolume v) { return v->volume.getData(); }

void vktStructuredVolumeSetValue(vktStructuredVolume v, int32_t x, int32_t y, int32_t z, float value)
{
    v->volume.setValue(x, y, z, value);
}

void vktStructuredVolumeGetValue(vktStructuredVolume v, int32_t x, int32_t y, int32_t z, float* value)
{
    v->volume.getValue(x, y, z, *value);
}

void vktStructuredVolumeSetBytes(vktStructuredVolume v, int32_t x, int32_t y, int32_t z, uint8_t const* data)
{
    v->volume.setBytes(x, y, z, data);
}

void vktStructuredVolumeGetBytes(vktStructuredVolume v, int32_t x, int32_t y, int32_t z, uint8_t* data)
{
    v->volume.getBytes(x, y, z, data);
}

size_t vktStructuredVolumeGetSizeInBytes(vktStructuredVolume v) { return v->volume.getSizeInBytes(); }

vktResourceHandle vktStructuredVolumeGetResourceHandle(vktStructuredVolume v) { return v->volume.getResourceHandle(); }

void vktStructuredVolumeMigrate(vktStructuredVolume v) { v->volume.migrate(); }

vktError vktStructuredVolumeMigrateChecked(vktStructuredVolume v)
{
    if (v == nullptr)
        return vkt::rt::fail("vktStructuredVolumeMigrateChecked: null volume");
    (void)vkt::rt::takeMigrationFailure();
    v->volume.migrate();
    std::string const m = vkt::rt::takeMigrationFailure();
    if (!v->volume.residentOn(vkt::GetThreadExecutionPolicy()))
        return vkt::rt::fail(m.empty() ? "vktStructuredVolumeMigrateChecked: migration failed" : m.c_str());
    return vktNoError;
}

vktError vktMapVoxel(uint8_t* dst, float value, vktDataFormat dataFormat, float mappingLo, float mappingHi)
{
    return static_cast<vktError>(vkt::MapVoxel(dst, value, static_cast<vkt::DataFormat>(dataFormat), mappingLo, mappingHi));
}

vktError vktUnmapVoxel(float* value, uint8_t const* src, vktDataFormat dataFormat, float mappingLo, float mappingHi)
{
    return static_cast<vktError>(
        vkt::UnmapVoxel(*value, src, static_cast<vkt::DataFormat>(dataFormat), mappingLo, mappingHi));
}

} // extern "C"
