// volkit.hpp -- C++ API of the MI355X-native volkit StructuredVolume core path.
//
// Source-compatible with the reference's include/cpp/vkt/*.hpp for the hot path:
// same namespace, class names, overload sets, default arguments and member order
// of ManagedBuffer / StructuredVolume (reference include/cpp/vkt/ManagedBuffer.hpp:50-56,
// include/cpp/vkt/StructuredVolume.hpp:118-128).  Per-name forwarding headers in
// include/cpp/vkt/ include this file, so `#include <vkt/StructuredVolume.hpp>` works.
//
// What differs by design (MI355X-first):
//  * ManagedBuffer::migrate() moves bytes with hipMemcpyAsync on a side copy stream,
//    ordered against the compute stream with events (volkit_amd/csrc/runtime/Memory.cpp).
//  * The per-thread policy is thread_local (race-free; same observable semantics as the
//    reference's unlocked global map, src/vkt/ExecutionPolicy.cpp:17).
//  * Algorithms dispatched under Device::GPU run hand-written gfx950 kernels and return
//    InvalidValue (instead of silently doing nothing) when a launch or allocation fails.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <memory>

#ifndef VKTAPI
#define VKTAPI __attribute__((visibility("default")))
#endif

namespace vkt
{
    //--- common.hpp (reference include/cpp/vkt/common.hpp:10-68) --------------------------
    typedef uint8_t Bool;
    static constexpr Bool False = 0;
    static constexpr Bool True = 1;

    enum Error
    {
        InvalidValue = -1,
        NoError = 0,
        InvalidDataSource = 1,
        ReadError = 2,
        WriteError = 3,
    };

    enum class ColorFormat
    {
        Unspecified, R8, RG8, RGB8, RGBA8, R16UI, RG16UI, RGB16UI, RGBA16UI,
        R32UI, RG32UI, RGB32UI, RGBA32UI, R32F, RG32F, RGB32F, RGBA32F, Count,
    };

    enum class DataFormat
    {
        Unspecified, Int8, Int16, Int32, UInt8, UInt16, UInt32, Float32, Count,
    };

    enum class OpenMode { Read, Write, ReadWrite };

    //--- DataSource (reference include/cpp/vkt/common.hpp:81-91) ---------------------------
    class DataSource
    {
    public:
        virtual ~DataSource() {}
        virtual std::size_t read(char* buf, std::size_t len) = 0;
        virtual std::size_t write(char const* buf, std::size_t len) = 0;
        virtual bool seek(std::size_t pos) = 0;
        virtual bool flush() = 0;
        virtual bool good() const = 0;
    };

    //--- linalg.hpp (reference include/cpp/vkt/linalg.hpp) -------------------------------
    struct Vec2f { float x, y; };
    struct Vec3f { float x, y, z; };
    struct Vec4f { float x, y, z, w; };
    struct Vec2i { int x, y; };
    struct Vec3i { int x, y, z; };
    struct Vec4i { int x, y, z, w; };
    struct Box2f { Vec2f min, max; };
    struct Box3f { Vec3f min, max; };
    struct Box2i { Vec2i min, max; };
    struct Box3i { Vec3i min, max; };
    struct Mat3f { Vec3f col0, col1, col2; };
    struct Mat4f { Vec4f col0, col1, col2, col3; };
    enum class Axis { X, Y, Z };

    inline bool operator==(Vec2f const& a, Vec2f const& b) { return a.x == b.x && a.y == b.y; }
    inline bool operator!=(Vec2f const& a, Vec2f const& b) { return !(a == b); }
    inline bool operator==(Vec3i const& a, Vec3i const& b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
    inline bool operator!=(Vec3i const& a, Vec3i const& b) { return !(a == b); }

    class StructuredVolume;

    //--- ExecutionPolicy.hpp (reference include/cpp/vkt/ExecutionPolicy.hpp:47-102) -------
    struct ExecutionPolicy
    {
        enum class Device { CPU, GPU, Unspecified };
        enum class HostAPI { Serial, OpenMP, Auto };
        // DeviceAPI::CUDA keeps value 0 for source/ABI compatibility and means "the GPU
        // backend", which is HIP on this build; HIP is an alias of the same value.
        enum class DeviceAPI { CUDA, Auto, HIP = CUDA };

        Device device = Device::CPU;
        HostAPI hostApi = HostAPI::Serial;
        DeviceAPI deviceApi = DeviceAPI::CUDA;
        Bool printPerformance = False;
    };

    VKTAPI void SetThreadExecutionPolicy(ExecutionPolicy policy);
    VKTAPI ExecutionPolicy GetThreadExecutionPolicy();

    //--- ManagedResource.hpp (reference include/cpp/vkt/ManagedResource.hpp:12-19) -------
    typedef void* ManagedResource;
    typedef uint32_t ResourceHandle;
    VKTAPI ResourceHandle RegisterManagedResource(ManagedResource resource);
    VKTAPI void UnregisterManagedResource(ResourceHandle handle);
    VKTAPI ManagedResource GetManagedResource(ResourceHandle handle);

    //--- Memory.hpp (reference include/cpp/vkt/Memory.hpp:15-30) -------------------------
    enum class CopyKind { HostToHost, HostToDevice, DeviceToHost, DeviceToDevice };
    VKTAPI void Allocate(void** ptr, std::size_t size);
    VKTAPI void Free(void* ptr);
    VKTAPI void Memcpy(void* dst, void const* src, std::size_t size, CopyKind ck);
    VKTAPI void MemsetRange(void* dst, void const* src, std::size_t dstSize, std::size_t srcSize);

    namespace detail
    {
        // Moves a buffer between address spaces when the thread's device differs from
        // `last`; returns the new pointer.  Implemented in csrc/runtime/Memory.cpp.
        VKTAPI void* MigrateBuffer(void* data, std::size_t bytes, ExecutionPolicy& last);
        // Frees `data` under `owner`'s device (host free or hipFree).
        VKTAPI void FreeOn(void* data, ExecutionPolicy const& owner);
        VKTAPI void* AllocateOn(std::size_t bytes, ExecutionPolicy const& owner);
        VKTAPI void CopyOn(void* dst, void const* src, std::size_t bytes, ExecutionPolicy const& owner);
        // Copies between buffers owned by (possibly) different devices -- a source whose
        // migration failed is still in its old address space.
        VKTAPI void CopyBetween(void* dst, ExecutionPolicy const& dstOwner, void const* src,
                                ExecutionPolicy const& srcOwner, std::size_t bytes);
        // MemsetRange where the bytes live (`owner`: the buffer's last allocation policy), not
        // where the thread's policy points -- a buffer whose migration failed is still in host
        // memory and gets the host pattern loop.
        VKTAPI void MemsetRangeOn(void* dst, void const* src, std::size_t dstSize, std::size_t srcSize,
                                  ExecutionPolicy const& owner);
    }

    //--- ManagedBuffer<T> (reference include/cpp/vkt/ManagedBuffer.hpp:21-276) -----------
    // Deferred migration: data lives where it was last allocated/migrated; the next access
    // under a different thread device moves it.  Moves copy-then-free like the reference
    // (ManagedBuffer.hpp:91-107) so a moved-from buffer is empty, not aliased.
    template <typename T>
    class ManagedBuffer
    {
    public:
        typedef T value_type;

        ManagedBuffer(std::size_t size = 0) : data_(nullptr), size_(size)
        {
            allocate(size);
            resourceHandle_ = RegisterManagedResource(this);
        }

        ManagedBuffer(ManagedBuffer& rhs)
            : data_(nullptr), size_(rhs.size_), lastAllocationPolicy_(rhs.lastAllocationPolicy_)
        {
            rhs.migrate();
            allocate(rhs.size_);
            copy(rhs);
            resourceHandle_ = RegisterManagedResource(this);
        }

        ManagedBuffer(ManagedBuffer&& rhs)
            : data_(nullptr), size_(rhs.size_), lastAllocationPolicy_(rhs.lastAllocationPolicy_)
        {
            rhs.migrate();
            allocate(rhs.size_);
            copy(rhs);
            resourceHandle_ = RegisterManagedResource(this);
            rhs.release();
        }

        virtual ~ManagedBuffer()
        {
            UnregisterManagedResource(resourceHandle_);
            deallocate();
        }

        ManagedBuffer& operator=(ManagedBuffer& rhs)
        {
            if (&rhs != this)
            {
                rhs.migrate();
                deallocate();
                size_ = rhs.size_;
                allocate(rhs.size_);
                copy(rhs);
            }
            return *this;
        }

        ManagedBuffer& operator=(ManagedBuffer&& rhs)
        {
            if (&rhs != this)
            {
                rhs.migrate();
                deallocate();
                size_ = rhs.size_;
                allocate(rhs.size_);
                copy(rhs);
                rhs.release();
            }
            return *this;
        }

        ResourceHandle getResourceHandle() const { return resourceHandle_; }

        //! True when the bytes already live on `ep`'s device (no migration pending for it).
        bool residentOn(ExecutionPolicy const& ep) const { return ep.device == lastAllocationPolicy_.device; }

        //! If the thread's device changed since the last allocation, move the bytes there.
        void migrate()
        {
            data_ = static_cast<T*>(detail::MigrateBuffer(data_, size_ * sizeof(T), lastAllocationPolicy_));
        }

    protected:
        void allocate(std::size_t size)
        {
            lastAllocationPolicy_ = GetThreadExecutionPolicy();
            size_ = size;
            data_ = static_cast<T*>(detail::AllocateOn(size_ * sizeof(T), lastAllocationPolicy_));
        }

        void deallocate()
        {
            detail::FreeOn(data_, lastAllocationPolicy_);
            data_ = nullptr;
            lastAllocationPolicy_ = GetThreadExecutionPolicy();
        }

        void resize(std::size_t size)
        {
            migrate();
            T* fresh = static_cast<T*>(detail::AllocateOn(size * sizeof(T), lastAllocationPolicy_));
            std::size_t keep = (size < size_ ? size : size_) * sizeof(T);
            if (keep > 0)
                detail::CopyOn(fresh, data_, keep, lastAllocationPolicy_);
            detail::FreeOn(data_, lastAllocationPolicy_);
            data_ = fresh;
            size_ = size;
        }

        void fill(T& value)
        {
            migrate();
            detail::MemsetRangeOn(data_, &value, size_ * sizeof(T), sizeof(T), lastAllocationPolicy_);
        }

        void fill(T const& value) { fill(const_cast<T&>(value)); }

        void copy(ManagedBuffer& rhs)
        {
            rhs.migrate();
            std::size_t n = (size_ < rhs.size_ ? size_ : rhs.size_) * sizeof(T);
            if (n > 0)
                detail::CopyBetween(data_, lastAllocationPolicy_, rhs.data_, rhs.lastAllocationPolicy_, n);
        }

        T* data_ = nullptr;
        std::size_t size_ = 0;

    private:
        void release()
        {
            detail::FreeOn(data_, lastAllocationPolicy_);
            data_ = nullptr;
            size_ = 0;
        }

        ExecutionPolicy lastAllocationPolicy_ = {};
        ResourceHandle resourceHandle_ = ResourceHandle(-1);
    };

    //--- StructuredVolume (reference include/cpp/vkt/StructuredVolume.hpp:34-132) ---------
    // Dense x-fastest voxel array: byte offset of (x,y,z) = ((z*dimY + y)*dimX + x) * bpv.
    class VKTAPI StructuredVolume : public ManagedBuffer<uint8_t>
    {
    public:
        constexpr static uint8_t GetMaxBytesPerVoxel() { return 8; }

        StructuredVolume();
        StructuredVolume(int32_t dimX, int32_t dimY, int32_t dimZ, DataFormat dataFormat,
                         float distX = 1.f, float distY = 1.f, float distZ = 1.f,
                         float mappingLo = 0.f, float mappingHi = 1.f);
        StructuredVolume(StructuredVolume& rhs) = default;
        StructuredVolume(StructuredVolume&& rhs) = default;
        StructuredVolume& operator=(StructuredVolume& rhs) = default;
        StructuredVolume& operator=(StructuredVolume&& rhs) = default;

        void setDims(int32_t dimX, int32_t dimY, int32_t dimZ);
        void getDims(int32_t& dimX, int32_t& dimY, int32_t& dimZ);
        void setDims(Vec3i dims);
        Vec3i getDims() const;

        void setDataFormat(DataFormat dataFormat);
        DataFormat getDataFormat() const;

        void setDist(float distX, float distY, float distZ);
        void getDist(float& distX, float& distY, float& distZ);
        void setDist(Vec3f dist);
        Vec3f getDist() const;

        void setVoxelMapping(float lo, float hi);
        void getVoxelMapping(float& lo, float& hi);
        void setVoxelMapping(Vec2f mapping);
        Vec2f getVoxelMapping() const;

        //! getData() for a caller that runs under `ep` (its thread's policy), without looking the
        //! policy up when the bytes already live there (per-brick walks of BrickDecompose).
        //! nullptr when the bytes could not be migrated there (they stay where they were).
        uint8_t* getDataFor(ExecutionPolicy const& ep)
        {
            if (!residentOn(ep))
                (void)getData();
            return residentOn(ep) ? data_ : nullptr;
        }

        Box3f getDomainBounds() const;
        Box3f getObjectBounds() const;

        //! Raw pointer in the address space of the calling thread's device (migrates first)
        uint8_t* getData();

        // Host accessors.  Under the GPU policy the reference dereferences a device
        // pointer on the host; here they move the single voxel with a synchronous copy.
        void setValue(int32_t x, int32_t y, int32_t z, float value);
        void getValue(int32_t x, int32_t y, int32_t z, float& value);
        float getValue(int32_t x, int32_t y, int32_t z);
        void setValue(Vec3i index, float value);
        void getValue(Vec3i index, float& value);
        float getValue(Vec3i index);
        void setBytes(int32_t x, int32_t y, int32_t z, uint8_t const* data);
        void getBytes(int32_t x, int32_t y, int32_t z, uint8_t* data);
        void setBytes(Vec3i index, uint8_t const* data);
        void getBytes(Vec3i index, uint8_t* data);

        uint8_t getBytesPerVoxel() const;
        std::size_t getSizeInBytes() const;

    private:
        Vec3i dims_;
        DataFormat dataFormat_;
        Vec3f dist_;
        Vec2f voxelMapping_;
        Vec3f haloSize_;

        std::size_t linearIndex(int32_t x, int32_t y, int32_t z) const;
        std::size_t linearIndex(Vec3i index) const;
    };

    //--- Voxel.hpp (reference include/cpp/vkt/Voxel.hpp:15-39) ---------------------------
    struct VoxelView
    {
        uint8_t* bytes;
        DataFormat dataFormat;
        float mappingLo;
        float mappingHi;
    };
    VKTAPI Error MapVoxel(uint8_t* dst, float value, DataFormat dataFormat, float mappingLo, float mappingHi);
    VKTAPI Error UnmapVoxel(float& value, uint8_t const* src, DataFormat dataFormat, float mappingLo, float mappingHi);

    //--- Fill.hpp (reference include/cpp/vkt/Fill.hpp:16-50, SV overloads) ---------------
    VKTAPI Error Fill(StructuredVolume& volume, float value);
    VKTAPI Error FillRange(StructuredVolume& volume, int32_t firstX, int32_t firstY, int32_t firstZ,
                           int32_t lastX, int32_t lastY, int32_t lastZ, float value);
    VKTAPI Error FillRange(StructuredVolume& volume, Vec3i first, Vec3i last, float value);

    //--- Copy.hpp (reference include/cpp/vkt/Copy.hpp:14-37) ------------------------------
    VKTAPI Error Copy(StructuredVolume& dst, StructuredVolume& src);
    VKTAPI Error CopyRange(StructuredVolume& dst, StructuredVolume& src, int32_t firstX, int32_t firstY,
                           int32_t firstZ, int32_t lastX, int32_t lastY, int32_t lastZ,
                           int32_t dstOffsetX = 0, int32_t dstOffsetY = 0, int32_t dstOffsetZ = 0);
    VKTAPI Error CopyRange(StructuredVolume& dst, StructuredVolume& src, Vec3i first, Vec3i last,
                           Vec3i dstOffset = {0, 0, 0});

    //--- Arithmetic.hpp (reference include/cpp/vkt/Arithmetic.hpp:31-299) ----------------
#define VKT_DECLARE_ARITHMETIC_CPP_(NAME)                                                          \
    VKTAPI Error NAME(StructuredVolume& dest, StructuredVolume& source1, StructuredVolume& source2); \
    VKTAPI Error NAME##Range(StructuredVolume& dest, StructuredVolume& source1,                    \
                             StructuredVolume& source2, int32_t firstX, int32_t firstY,            \
                             int32_t firstZ, int32_t lastX, int32_t lastY, int32_t lastZ,          \
                             int32_t dstOffsetX = 0, int32_t dstOffsetY = 0,                       \
                             int32_t dstOffsetZ = 0);                                              \
    VKTAPI Error NAME##Range(StructuredVolume& dest, StructuredVolume& source1,                    \
                             StructuredVolume& source2, Vec3i first, Vec3i last,                   \
                             Vec3i dstOffset = {0, 0, 0});
    VKT_DECLARE_ARITHMETIC_CPP_(Sum)
    VKT_DECLARE_ARITHMETIC_CPP_(Diff)
    VKT_DECLARE_ARITHMETIC_CPP_(Prod)
    VKT_DECLARE_ARITHMETIC_CPP_(Quot)
    VKT_DECLARE_ARITHMETIC_CPP_(AbsDiff)
    VKT_DECLARE_ARITHMETIC_CPP_(SafeSum)
    VKT_DECLARE_ARITHMETIC_CPP_(SafeDiff)
    VKT_DECLARE_ARITHMETIC_CPP_(SafeProd)
    VKT_DECLARE_ARITHMETIC_CPP_(SafeQuot)
    VKT_DECLARE_ARITHMETIC_CPP_(SafeAbsDiff)
#undef VKT_DECLARE_ARITHMETIC_CPP_

    //--- Transform.hpp (reference include/cpp/vkt/Transform.hpp:16-62) --------------------
    typedef void (*TransformUnaryOp)(int32_t x, int32_t y, int32_t z, VoxelView voxel);
    typedef void (*TransformBinaryOp)(int32_t x1, int32_t y1, int32_t z1, VoxelView voxel1, VoxelView voxel2);
    VKTAPI Error Transform(StructuredVolume& volume, TransformUnaryOp unaryOp);
    VKTAPI Error Transform(StructuredVolume& volume1, StructuredVolume& volume2, TransformBinaryOp binaryOp);
    VKTAPI Error TransformRange(StructuredVolume& volume, int32_t firstX, int32_t firstY, int32_t firstZ,
                                int32_t lastX, int32_t lastY, int32_t lastZ, TransformUnaryOp unaryOp);
    VKTAPI Error TransformRange(StructuredVolume& volume, Vec3i first, Vec3i last, TransformUnaryOp unaryOp);
    VKTAPI Error TransformRange(StructuredVolume& volume1, StructuredVolume& volume2, int32_t firstX,
                                int32_t firstY, int32_t firstZ, int32_t lastX, int32_t lastY, int32_t lastZ,
                                TransformBinaryOp binaryOp);
    VKTAPI Error TransformRange(StructuredVolume& volume1, StructuredVolume& volume2, Vec3i first, Vec3i last,
                                TransformBinaryOp binaryOp);

    //--- Resample.hpp (reference include/cpp/vkt/Resample.hpp:14-31, SV->SV) ------------
    enum class FilterMode { Nearest, Linear };
    VKTAPI Error Resample(StructuredVolume& dst, StructuredVolume& src, FilterMode fm);

    //--- Array3D<T> (reference include/cpp/vkt/Array3D.hpp:14-143) -------------------------
    // Dense x-fastest 3-D array with the reference's interface.  Deviation by design: the
    // element array itself lives on the HOST (it holds handles / small metadata), elements
    // are constructed and destroyed properly, and copies are deep.  The reference derives it
    // from ManagedBuffer<T>, which migrates the raw bytes of the elements -- for
    // Array3D<StructuredVolume> that would move host objects to device memory and then
    // dereference them on the host.  Each StructuredVolume element migrates its own voxels.
    template <typename T>
    class Array3D
    {
    public:
        typedef T value_type;
        typedef T* iterator;
        typedef T const* const_iterator;

        Array3D() = default;
        explicit Array3D(Vec3i const& dims) { resize(dims); }
        Array3D(Array3D& rhs) { *this = rhs; }
        Array3D(Array3D&& rhs) noexcept : elems_(std::move(rhs.elems_)), dims_(rhs.dims_) { rhs.dims_ = {0, 0, 0}; }
        ~Array3D() = default;

        Array3D& operator=(Array3D& rhs)
        {
            if (&rhs != this)
            {
                resize(rhs.dims_);
                for (std::size_t i = 0; i < numElements(); ++i)
                    elems_[i] = rhs.elems_[i];
            }
            return *this;
        }

        Array3D& operator=(Array3D&& rhs) noexcept
        {
            if (&rhs != this)
            {
                elems_ = std::move(rhs.elems_);
                dims_ = rhs.dims_;
                rhs.dims_ = {0, 0, 0};
            }
            return *this;
        }

        //! Re-shape; existing elements are dropped (reference: ManagedBuffer::resize of raw bytes)
        void resize(Vec3i const& dims)
        {
            std::size_t n = count(dims);
            elems_.reset(n ? new T[n] : nullptr);
            dims_ = dims;
        }

        void fill(T& value)
        {
            for (std::size_t i = 0; i < numElements(); ++i)
                elems_[i] = value;
        }
        void fill(T const& value) { fill(const_cast<T&>(value)); }

        iterator begin() { return data(); }
        const_iterator begin() const { return data(); }
        const_iterator cbegin() { return data(); }
        iterator end() { return data() + numElements(); }
        const_iterator end() const { return data() + numElements(); }
        const_iterator cend() { return data() + numElements(); }

        T& operator[](Vec3i const& index) { return elems_[linear(index)]; }
        T const& operator[](Vec3i const& index) const { return elems_[linear(index)]; }

        bool empty() const { return numElements() == 0; }
        T* data() { return elems_.get(); }
        T const* data() const { return elems_.get(); }
        Vec3i dims() const { return dims_; }
        std::size_t numElements() const { return count(dims_); }

    private:
        static std::size_t count(Vec3i const& d)
        {
            return d.x > 0 && d.y > 0 && d.z > 0
                       ? static_cast<std::size_t>(d.x) * static_cast<std::size_t>(d.y) * static_cast<std::size_t>(d.z)
                       : 0;
        }
        std::size_t linear(Vec3i const& i) const
        {
            return (static_cast<std::size_t>(i.z) * static_cast<std::size_t>(dims_.y) + static_cast<std::size_t>(i.y)) *
                       static_cast<std::size_t>(dims_.x) +
                   static_cast<std::size_t>(i.x);
        }

        std::unique_ptr<T[]> elems_;
        Vec3i dims_ = {0, 0, 0};
    };

    //--- Decompose.hpp (reference include/cpp/vkt/Decompose.hpp:16-50) -------------------
    // BrickDecomposeResize allocates the bricks (on the calling thread's device, like any
    // StructuredVolume); BrickDecompose copies source ranges with halos into them -- one
    // batched gfx950 launch for all bricks under the GPU policy.
    VKTAPI Error BrickDecompose(Array3D<StructuredVolume>& dest, StructuredVolume& source, int32_t brickSizeX,
                                int32_t brickSizeY, int32_t brickSizeZ, int32_t haloSizeNegX = 0,
                                int32_t haloSizeNegY = 0, int32_t haloSizeNegZ = 0, int32_t haloSizePosX = 0,
                                int32_t haloSizePosY = 0, int32_t haloSizePosZ = 0);
    VKTAPI Error BrickDecompose(Array3D<StructuredVolume>& dest, StructuredVolume& source, Vec3i brickSize,
                                Vec3i haloSizeNeg = {0, 0, 0}, Vec3i haloSizePos = {0, 0, 0});
    VKTAPI Error BrickDecomposeResize(Array3D<StructuredVolume>& dest, StructuredVolume& source, int32_t brickSizeX,
                                      int32_t brickSizeY, int32_t brickSizeZ, int32_t haloSizeNegX = 0,
                                      int32_t haloSizeNegY = 0, int32_t haloSizeNegZ = 0, int32_t haloSizePosX = 0,
                                      int32_t haloSizePosY = 0, int32_t haloSizePosZ = 0);
    VKTAPI Error BrickDecomposeResize(Array3D<StructuredVolume>& dest, StructuredVolume& source, Vec3i brickSize,
                                      Vec3i haloSizeNeg = {0, 0, 0}, Vec3i haloSizePos = {0, 0, 0});

    //--- Aggregates.hpp (reference include/cpp/vkt/Aggregates.hpp:14-42) -------------------
    struct Aggregates
    {
        float min;
        float max;
        float mean;
        float stddev;
        float var;
        float sum;
        float prod;
        Vec3i argmin;
        Vec3i argmax;
    };

    VKTAPI Error ComputeAggregates(StructuredVolume& volume, Aggregates& aggregates);
    VKTAPI Error ComputeAggregatesRange(StructuredVolume& volume, Aggregates& aggregates, int32_t firstX,
                                        int32_t firstY, int32_t firstZ, int32_t lastX, int32_t lastY, int32_t lastZ);
    VKTAPI Error ComputeAggregatesRange(StructuredVolume& volume, Aggregates& aggregates, Vec3i first, Vec3i last);

    //--- Histogram.hpp (reference include/cpp/vkt/Histogram.hpp:14-42) --------------------
    class VKTAPI Histogram : public ManagedBuffer<std::size_t>
    {
    public:
        Histogram(std::size_t numBins);

        std::size_t getNumBins() const;

        //! Bin counts in the calling thread's address space (migrates first)
        std::size_t* getBinCounts();
    };

    VKTAPI Error ComputeHistogram(StructuredVolume& volume, Histogram& histogram);
    VKTAPI Error ComputeHistogramRange(StructuredVolume& volume, Histogram& histogram, int32_t firstX, int32_t firstY,
                                       int32_t firstZ, int32_t lastX, int32_t lastY, int32_t lastZ);
    VKTAPI Error ComputeHistogramRange(StructuredVolume& volume, Histogram& histogram, Vec3i first, Vec3i last);

    //--- RawFile.hpp (reference include/cpp/vkt/RawFile.hpp:15-60) --------------------------
    // Dims and format are parsed from the file name ("<X>x<Y>x<Z>" and "[u]int<bits>" tokens
    // separated by '_', src/vkt/RawFile.cpp:36-106).  Deviations (documented fixes):
    // read()/write() return BYTES (the reference returns fread's item count, so every
    // InputStream::read reported ReadError on success); RawFile(FILE*) uses the given stream
    // and does not close it (the reference fopen()s a null name).
    class VKTAPI RawFile : public DataSource
    {
    public:
        RawFile(char const* fileName, char const* mode);
        RawFile(FILE* file);
        ~RawFile();

        virtual std::size_t read(char* buf, std::size_t len);
        virtual std::size_t write(char const* buf, std::size_t len);
        virtual bool seek(std::size_t pos);
        virtual bool flush();
        virtual bool good() const;

        //! read(), with large reads split over the library's host threads (pread at the
        //! stream's position, which then advances as read() would advance it)
        std::size_t readParallel(char* buf, std::size_t len);

        void setDims(Vec3i dims);
        Vec3i getDims() const;
        void setDataFormat(DataFormat dataFormat);
        DataFormat getDataFormat() const;

    private:
        char const* fileName_ = 0;
        char const* mode_ = 0;
        FILE* file_ = 0;
        bool owned_ = false;
        Vec3i dims_ = {0, 0, 0};
        DataFormat dataFormat_ = DataFormat::UInt8;
    };

    //--- InputStream.hpp / OutputStream.hpp (reference include/cpp/vkt/InputStream.hpp:14-40,
    //    OutputStream.hpp:14-42).  A volume resident in HBM (GPU policy) streams through
    //    pinned double buffers on the side copy stream -- the file read of chunk i+1 overlaps
    //    the DMA of chunk i; the reference would fread() into a device pointer.
    class VKTAPI InputStream
    {
    public:
        InputStream(DataSource& source);

        Error read(StructuredVolume& volume);
        Error readRange(StructuredVolume& dst, int32_t firstX, int32_t firstY, int32_t firstZ, int32_t lastX,
                        int32_t lastY, int32_t lastZ);
        Error readRange(StructuredVolume& dst, Vec3i first, Vec3i last);
        Error seek(std::size_t pos);

    private:
        DataSource& dataSource_;
    };

    class VKTAPI OutputStream
    {
    public:
        OutputStream(DataSource& source);

        Error write(StructuredVolume& volume);
        Error writeRange(StructuredVolume& dst, int32_t firstX, int32_t firstY, int32_t firstZ, int32_t lastX,
                         int32_t lastY, int32_t lastZ);
        Error writeRange(StructuredVolume& dst, Vec3i first, Vec3i last);
        Error seek(std::size_t pos);
        Error flush();

    private:
        DataSource& dataSource_;
    };

    //--- StructuredVolume stream format of the reference CLI (src/cli/main.cpp:32-88):
    // u32 magic 0x1, u32 asset type 0x0 (SV), Vec3i dims, u32 format, Vec3f dist, Vec2f mapping,
    // then the voxel bytes.  ReadSVStream builds the volume with dims.z (the CLI passes dims.x
    // for z, main.cpp:65).
    VKTAPI Error ReadSVStream(DataSource& source, StructuredVolume& volume);
    VKTAPI Error WriteSVStream(DataSource& source, StructuredVolume& volume);

    //--- LookupTable.hpp (reference include/cpp/vkt/LookupTable.hpp:14-70) ------------------
    // RGBA32F transfer function for the renderers (a managed buffer like the volumes).
    class VKTAPI LookupTable : public ManagedBuffer<uint8_t>
    {
    public:
        LookupTable();
        LookupTable(int32_t dimX, int32_t dimY, int32_t dimZ, ColorFormat format);

        void setDims(int32_t dimX, int32_t dimY, int32_t dimZ);
        void getDims(int32_t& dimX, int32_t& dimY, int32_t& dimZ);
        void setDims(Vec3i dims);
        Vec3i getDims() const;

        void setColorFormat(ColorFormat cf);
        ColorFormat getColorFormat() const;

        //! Copy getSizeInBytes() bytes from host memory into the table
        void setData(uint8_t* data);
        uint8_t* getData();
        std::size_t getSizeInBytes() const;

    private:
        Vec3i dims_ = {0, 0, 0};
        ColorFormat format_ = ColorFormat::Unspecified;
    };

    //--- Render.hpp (reference include/cpp/vkt/Render.hpp:16-179, structured volumes) ------
    enum class RenderAlgo
    {
        RayMarching,
        ImplicitIso,
        MultiScattering,
    };

    struct RenderState
    {
        RenderAlgo renderAlgo = RenderAlgo::RayMarching;
        float dtRayMarching = 1.f;
        uint16_t numIsoSurfaces = 1;
        enum { MaxIsoSurfaces = 10 };
        float isoSurfaces[MaxIsoSurfaces] = {.5f};
        float dtImplicitIso = 1.f;
        float majorant = 1.f;
        unsigned animationFrame = 0;
        ResourceHandle rgbaLookupTable = ResourceHandle(-1);
        ResourceHandle histogram = ResourceHandle(-1);
        int viewportWidth = 512;
        int viewportHeight = 512;
        Bool sRGB = 1;
        struct
        {
            Bool isSet = 0;
            Vec3f eye = {0.f, 0.f, 0.f};
            Vec3f center = {0.f, 0.f, -1.f};
            Vec3f up = {0.f, 1.f, 0.f};
            float fovy = 45.f;
            float lensRadius = .001f;
            float focalDistance = 10.f;
        } initialCamera;
        struct
        {
            Bool enabled = 0;
            char const* fileName = "";
            Bool takeOnClose = 0;
            char key = 'p';
            char const* message = "";
        } snapshotTool;
    };

    // The reference opens an interactive viewer.  This build renders headless: Render
    // accumulates VKT_RENDER_FRAMES frames (default 64) of renderState.animationFrame's
    // volume on the GPU, writes a PPM snapshot when snapshotTool.enabled, and returns the
    // camera it used in newRenderState->initialCamera.
    VKTAPI Error Render(StructuredVolume& volume, RenderState const& renderState = {},
                        RenderState* newRenderState = 0);
    VKTAPI Error RenderFrames(StructuredVolume* volumes, std::size_t numAnimationFrames,
                              RenderState const& renderState = {}, RenderState* newRenderState = 0);

    //! Headless extension: accumulate numFrames frames into `rgba` (host, width*height RGBA
    //! floats, row 0 = bottom, sRGB applied when renderState.sRGB).
    VKTAPI Error RenderToImage(StructuredVolume& volume, RenderState const& renderState, unsigned numFrames,
                               float* rgba);

} // vkt
