// transform_ops.hip -- TEST/BENCH FIXTURE: device functors run through the Transform
// templates of include/volkit_transform.hpp, and the same functors as host callbacks of the
// oracle's restatement of TransformRange_serial (oracle/vkt_oracle.c: vko_transform_range1/2),
// so a GPU test compares the two on identical inputs.  The functors are user code (the
// reference's own examples among them); what the comparison checks is the Transform
// machinery: coordinates, range, the zeroed 8-byte scratch, write-back of bytesPerVoxel
// bytes, volume1-then-volume2 stores, aliasing.
//
// Ops (unary):
//   0 Checkered<3>  reference src/examples/Arithmetic.cpp:8-21 (MakeCheckered<3>)
//   1 Checkered<2>  same, level 2
//   2 Diagonal      reference src/examples/CoreAlgorithms.c:14-18 (TransformOp1)
//   3 Rescale       unmap, value * 0.5 + (x + 2y + 3z) * 2^-10, map back (codec on the device)
//   4 ScratchProbe  checks the scratch bytes past bytesPerVoxel are zero, writes all 8 bytes
// Ops (binary):
//   0 Or            reference src/examples/CoreAlgorithms.c:20-24 (TransformOp2)
//   1 MixFormats    v1 = map(unmap(v1) + unmap(v2)); v2.bytes[0] ^= x + y + z (any formats)
#include "volkit_transform.hpp"

#include <cstdio>
#include <cstring>

namespace
{
    template <unsigned Level>
    struct Checkered
    {
        __host__ __device__ void operator()(int32_t x, int32_t y, int32_t z, vkt::VoxelView voxel) const
        {
            x >>= Level;
            y >>= Level;
            z >>= Level;
            std::size_t linearIndex = z * 32 * 32 + y * 32 + x;
            if ((y % 2 == z % 2 && linearIndex % 2 == 0) || (y % 2 != z % 2 && linearIndex % 2 == 1))
                voxel.bytes[0] = 128;
            else
                voxel.bytes[0] = 0;
        }
    };

    struct Diagonal
    {
        __host__ __device__ void operator()(int32_t x, int32_t y, int32_t z, vkt::VoxelView voxel) const
        {
            if (x == y && y == z)
                voxel.bytes[0] = 0xFF;
        }
    };

    struct Rescale
    {
        __host__ __device__ void operator()(int32_t x, int32_t y, int32_t z, vkt::VoxelView voxel) const
        {
            float v = 0.f;
            vkt::device::UnmapVoxel(v, voxel.bytes, voxel.dataFormat, voxel.mappingLo, voxel.mappingHi);
            float w = v * 0.5f;
            float t = static_cast<float>(x + 2 * y + 3 * z) * 0.0009765625f;
            vkt::device::MapVoxel(voxel.bytes, w + t, voxel.dataFormat, voxel.mappingLo, voxel.mappingHi);
        }
    };

    struct ScratchProbe
    {
        __host__ __device__ void operator()(int32_t x, int32_t, int32_t, vkt::VoxelView voxel) const
        {
            uint32_t bpv = vkt::codec::bytesPerVoxel(static_cast<int32_t>(voxel.dataFormat));
            uint8_t dirty = 0;
            for (uint32_t i = bpv; i < 8; ++i)
                dirty |= voxel.bytes[i];
            uint8_t b0 = dirty ? 0x5A : static_cast<uint8_t>(voxel.bytes[0] + 1 + (x & 3));
            for (int i = 0; i < 8; ++i)
                voxel.bytes[i] = static_cast<uint8_t>(0xA0 + i);
            voxel.bytes[0] = b0;
        }
    };

    struct Or
    {
        __host__ __device__ void operator()(int32_t, int32_t, int32_t, vkt::VoxelView voxel1,
                                            vkt::VoxelView voxel2) const
        {
            voxel1.bytes[0] |= voxel2.bytes[0];
            voxel2.bytes[0] = voxel1.bytes[0];
        }
    };

    struct MixFormats
    {
        __host__ __device__ void operator()(int32_t x, int32_t y, int32_t z, vkt::VoxelView voxel1,
                                            vkt::VoxelView voxel2) const
        {
            float a = 0.f, b = 0.f;
            vkt::device::UnmapVoxel(a, voxel1.bytes, voxel1.dataFormat, voxel1.mappingLo, voxel1.mappingHi);
            vkt::device::UnmapVoxel(b, voxel2.bytes, voxel2.dataFormat, voxel2.mappingLo, voxel2.mappingHi);
            vkt::device::MapVoxel(voxel1.bytes, a + b, voxel1.dataFormat, voxel1.mappingLo, voxel1.mappingHi);
            voxel2.bytes[0] ^= static_cast<uint8_t>(x + y + z);
        }
    };

    // oracle callback signature (oracle/vkt_oracle.h: vko_unary_op / vko_binary_op)
    typedef void (*HostUnary)(int32_t, int32_t, int32_t, uint8_t*, int32_t, float, float);
    typedef void (*HostBinary)(int32_t, int32_t, int32_t, uint8_t*, int32_t, float, float, uint8_t*, int32_t, float,
                               float);

    template <class Op>
    void hostUnary(int32_t x, int32_t y, int32_t z, uint8_t* b, int32_t f, float lo, float hi)
    {
        Op{}(x, y, z, vkt::VoxelView{b, static_cast<vkt::DataFormat>(f), lo, hi});
    }

    template <class Op>
    void hostBinary(int32_t x, int32_t y, int32_t z, uint8_t* b1, int32_t f1, float lo1, float hi1, uint8_t* b2,
                    int32_t f2, float lo2, float hi2)
    {
        Op{}(x, y, z, vkt::VoxelView{b1, static_cast<vkt::DataFormat>(f1), lo1, hi1},
             vkt::VoxelView{b2, static_cast<vkt::DataFormat>(f2), lo2, hi2});
    }

    template <class F>
    int withUnary(int op, F&& f)
    {
        switch (op)
        {
        case 0: return f(Checkered<3>{});
        case 1: return f(Checkered<2>{});
        case 2: return f(Diagonal{});
        case 3: return f(Rescale{});
        case 4: return f(ScratchProbe{});
        default: return -100;
        }
    }

    template <class F>
    int withBinary(int op, F&& f)
    {
        switch (op)
        {
        case 0: return f(Or{});
        case 1: return f(MixFormats{});
        default: return -100;
        }
    }

    struct GpuPolicy
    {
        vkt::ExecutionPolicy saved;
        GpuPolicy()
        {
            saved = vkt::GetThreadExecutionPolicy();
            vkt::ExecutionPolicy ep = saved;
            ep.device = vkt::ExecutionPolicy::Device::GPU;
            vkt::SetThreadExecutionPolicy(ep);
        }
        ~GpuPolicy() { vkt::SetThreadExecutionPolicy(saved); }
    };

    void upload(vkt::StructuredVolume& v, void const* host)
    {
        vkt::Memcpy(v.getData(), host, v.getSizeInBytes(), vkt::CopyKind::HostToDevice);
    }

    void download(void* host, vkt::StructuredVolume& v)
    {
        vkt::Memcpy(host, v.getData(), v.getSizeInBytes(), vkt::CopyKind::DeviceToHost);
    }
} // namespace

extern "C" {

// Unary TransformRange of op on a volume given by its host bytes (updated in place).
int vktt_run_unary(int op, void* data, int dx, int dy, int dz, int fmt, float lo, float hi, int fx, int fy, int fz,
                   int lx, int ly, int lz)
{
    GpuPolicy gpu;
    vkt::StructuredVolume v(dx, dy, dz, static_cast<vkt::DataFormat>(fmt), 1.f, 1.f, 1.f, lo, hi);
    upload(v, data);
    int rc = withUnary(op, [&](auto f) {
        return static_cast<int>(vkt::TransformRange(v, vkt::Vec3i{fx, fy, fz}, vkt::Vec3i{lx, ly, lz}, f));
    });
    download(data, v);
    return rc;
}

// Z-slab TransformRange: the global volume (host bytes, updated in place) is cut into nranks
// slabs of the ceil partition, each slab (its owned planes only) gets TransformRangeSlab.
int vktt_run_unary_slab(int op, void* data, int dx, int dy, int dz, int fmt, float lo, float hi, int nranks, int fx,
                        int fy, int fz, int lx, int ly, int lz)
{
    GpuPolicy gpu;
    size_t const plane = static_cast<size_t>(dx) * dy * vkt::codec::bytesPerVoxel(fmt);
    int const size = (dz + nranks - 1) / nranks;
    for (int r = 0; r < nranks; ++r)
    {
        int const z0 = std::min(r * size, dz), z1 = std::min(z0 + size, dz);
        if (z1 <= z0)
            continue;
        uint8_t* host = static_cast<uint8_t*>(data) + plane * z0;
        vkt::StructuredVolume v(dx, dy, z1 - z0, static_cast<vkt::DataFormat>(fmt), 1.f, 1.f, 1.f, lo, hi);
        upload(v, host);
        int rc = withUnary(op, [&](auto f) {
            return static_cast<int>(
                vkt::TransformRangeSlab(nranks, r, v, z0, dz, vkt::Vec3i{fx, fy, fz}, vkt::Vec3i{lx, ly, lz}, f));
        });
        download(host, v);
        if (rc != 0)
            return rc;
    }
    return 0;
}

// Whole-volume Transform of a volume created in HOST memory (CPU policy), run under the GPU
// policy so the bytes migrate to HBM first.  failAlloc > 0 makes that many device allocations
// fail (knob memory.fail_next_alloc): Transform must then return an error and leave the bytes,
// still in host memory, untouched.  data is updated in place either way.
int vktt_run_unary_migrating(int op, void* data, int dx, int dy, int dz, int fmt, int failAlloc)
{
    vkt::ExecutionPolicy const saved = vkt::GetThreadExecutionPolicy();
    vkt::ExecutionPolicy cpu = saved;
    cpu.device = vkt::ExecutionPolicy::Device::CPU;
    vkt::SetThreadExecutionPolicy(cpu);
    int rc = 0;
    {
        vkt::StructuredVolume v(dx, dy, dz, static_cast<vkt::DataFormat>(fmt));
        std::memcpy(v.getData(), data, v.getSizeInBytes());
        {
            GpuPolicy gpu;
            vktHipSetTuningKnob("memory.fail_next_alloc", failAlloc);
            rc = withUnary(op, [&](auto f) { return static_cast<int>(vkt::Transform(v, f)); });
            vktHipSetTuningKnob("memory.fail_next_alloc", 0);
            if (rc == 0)
                download(data, v);
        }
        if (rc != 0)   // CPU policy again: the host bytes, no migration
            std::memcpy(data, v.getData(), v.getSizeInBytes());
    }
    vkt::SetThreadExecutionPolicy(saved);
    return rc;
}

// Whole-volume Transform (the reference's vkt::Transform(volume, op) entry).
int vktt_run_unary_whole(int op, void* data, int dx, int dy, int dz, int fmt, float lo, float hi)
{
    GpuPolicy gpu;
    vkt::StructuredVolume v(dx, dy, dz, static_cast<vkt::DataFormat>(fmt), 1.f, 1.f, 1.f, lo, hi);
    upload(v, data);
    int rc = withUnary(op, [&](auto f) { return static_cast<int>(vkt::Transform(v, f)); });
    download(data, v);
    return rc;
}

// Binary TransformRange; alias != 0 passes ONE volume (data1's) as both operands.
int vktt_run_binary(int op, int alias, void* data1, int dx1, int dy1, int dz1, int fmt1, float lo1, float hi1,
                    void* data2, int dx2, int dy2, int dz2, int fmt2, float lo2, float hi2, int fx, int fy, int fz,
                    int lx, int ly, int lz)
{
    GpuPolicy gpu;
    vkt::StructuredVolume v1(dx1, dy1, dz1, static_cast<vkt::DataFormat>(fmt1), 1.f, 1.f, 1.f, lo1, hi1);
    upload(v1, data1);
    if (alias)
    {
        int rc = withBinary(op, [&](auto f) {
            return static_cast<int>(vkt::TransformRange(v1, v1, vkt::Vec3i{fx, fy, fz}, vkt::Vec3i{lx, ly, lz}, f));
        });
        download(data1, v1);
        return rc;
    }
    vkt::StructuredVolume v2(dx2, dy2, dz2, static_cast<vkt::DataFormat>(fmt2), 1.f, 1.f, 1.f, lo2, hi2);
    upload(v2, data2);
    int rc = withBinary(op, [&](auto f) {
        return static_cast<int>(vkt::TransformRange(v1, v2, vkt::Vec3i{fx, fy, fz}, vkt::Vec3i{lx, ly, lz}, f));
    });
    download(data1, v1);
    download(data2, v2);
    return rc;
}

// Binary Transform with a __device__ lambda (the form INTEGRATION.md §2 shows): OR of two
// UInt8 volumes of the same dims, both updated.
int vktt_lambda_or(void* data1, void* data2, int dx, int dy, int dz)
{
    GpuPolicy gpu;
    vkt::StructuredVolume v1(dx, dy, dz, vkt::DataFormat::UInt8), v2(dx, dy, dz, vkt::DataFormat::UInt8);
    upload(v1, data1);
    upload(v2, data2);
    int rc = static_cast<int>(vkt::Transform(v1, v2, [] __device__(int32_t, int32_t, int32_t, vkt::VoxelView a,
                                                                  vkt::VoxelView b) {
        a.bytes[0] |= b.bytes[0];
        b.bytes[0] = a.bytes[0];
    }));
    download(data1, v1);
    download(data2, v2);
    return rc;
}

// The same op as a host callback for the oracle.
void* vktt_host_unary(int op)
{
    void* out = nullptr;
    withUnary(op, [&](auto f) {
        out = reinterpret_cast<void*>(static_cast<HostUnary>(&hostUnary<decltype(f)>));
        return 0;
    });
    return out;
}

void* vktt_host_binary(int op)
{
    void* out = nullptr;
    withBinary(op, [&](auto f) {
        out = reinterpret_cast<void*>(static_cast<HostBinary>(&hostBinary<decltype(f)>));
        return 0;
    });
    return out;
}

// Device-resident timing: `reps` unary TransformRange calls over [first, last) (the whole
// volume when last.x <= 0), after 3 warm-up calls; *ms = average per call (HIP events on
// volkit's compute stream).
int vktt_bench_unary_range(int op, int dx, int dy, int dz, int fmt, int fx, int fy, int fz, int lx, int ly, int lz,
                           int reps, float* ms)
{
    GpuPolicy gpu;
    vkt::StructuredVolume v(dx, dy, dz, static_cast<vkt::DataFormat>(fmt));
    vktHipVolumeView_t view{v.getData(), dx, dy, dz, fmt, 0.f, 1.f};
    if (vktHipSynthesize(view, 0x5EED) != vktNoError)
        return -1;
    void* s = nullptr;
    vktHipGetComputeStream(&s);
    hipStream_t stream = static_cast<hipStream_t>(s);
    int rc = 0;
    auto call = [&] {
        int e = withUnary(op, [&](auto f) {
            return lx <= 0 ? static_cast<int>(vkt::Transform(v, f))
                           : static_cast<int>(vkt::TransformRange(v, vkt::Vec3i{fx, fy, fz}, vkt::Vec3i{lx, ly, lz}, f));
        });
        if (e != 0)
            rc = e;
    };
    for (int i = 0; i < 3; ++i)
        call();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, stream);
    for (int i = 0; i < reps; ++i)
        call();
    (void)hipEventRecord(e1, stream);
    (void)hipEventSynchronize(e1);
    float t = 0.f;
    (void)hipEventElapsedTime(&t, e0, e1);
    *ms = t / reps;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return rc;
}

int vktt_bench_unary(int op, int dx, int dy, int dz, int fmt, int reps, float* ms)
{
    return vktt_bench_unary_range(op, dx, dy, dz, fmt, 0, 0, 0, 0, 0, 0, reps, ms);
}

} // extern "C"
