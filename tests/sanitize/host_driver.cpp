// Host-side sanitizer driver (SURVEY.md §5 "Race detection / sanitizers"): exercises every
// host code path of libvolkit that runs without a GPU -- the CPU execution policy, the
// StructuredVolume / Array3D / LookupTable / Histogram handle layers, the codec, host memory,
// raw files and streams, the algorithms' CPU-policy error paths -- plus concurrent use of the
// per-thread ExecutionPolicy and the managed-resource registry.  Built twice by
// tests/sanitize/Makefile: AddressSanitizer + UBSan (host code of libvolkit instrumented with
// -Xarch_host -fsanitize=...) and ThreadSanitizer.  Exit status = number of failed checks.
#include "volkit_c.h"
#include "runtime/HostPool.hpp"

#include <atomic>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static int g_fails = 0;
#define CHECK(c)                                                                   \
    do {                                                                           \
        if (!(c))                                                                  \
        {                                                                          \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);      \
            ++g_fails;                                                             \
        }                                                                          \
    } while (0)

static vktDataFormat const kFormats[] = {vktDataFormatUInt8, vktDataFormatUInt16, vktDataFormatFloat32,
                                         vktDataFormatInt16, vktDataFormatUInt32, vktDataFormatInt8,
                                         vktDataFormatInt32};

static void cpuPolicy()
{
    vktExecutionPolicy_t ep = vktGetThreadExecutionPolicy();
    ep.device = vktExecutionPolicyDeviceCPU;
    vktSetThreadExecutionPolicy(ep);
}

static void volumes()
{
    uint8_t const maxBpv = vktStructuredVolumeGetMaxBytesPerVoxel();
    CHECK(maxBpv >= 4);
    for (vktDataFormat fmt : kFormats)
    {
        vktStructuredVolume v = nullptr;
        vktStructuredVolumeCreate(&v, 13, 7, 5, fmt, 1.f, 2.f, 3.f, -1.f, 3.f);
        int32_t x = 0, y = 0, z = 0;
        vktStructuredVolumeGetDims3i(v, &x, &y, &z);
        CHECK(x == 13 && y == 7 && z == 5);
        // every voxel through the value and byte accessors (first/last voxels are the edges)
        for (int32_t k = 0; k < 5; ++k)
            for (int32_t j = 0; j < 7; ++j)
                for (int32_t i = 0; i < 13; ++i)
                {
                    vktStructuredVolumeSetValue(v, i, j, k, 0.01f * static_cast<float>(i + j + k));
                    float f = -1.f;
                    vktStructuredVolumeGetValue(v, i, j, k, &f);
                    CHECK(std::isfinite(f));
                    uint8_t b[16] = {0};
                    vktStructuredVolumeGetBytes(v, i, j, k, b);
                    vktStructuredVolumeSetBytes(v, i, j, k, b);
                }
        size_t const bytes = vktStructuredVolumeGetSizeInBytes(v);
        vktStructuredVolume c = nullptr;
        vktStructuredVolumeCreateCopy(&c, v);
        CHECK(vktStructuredVolumeGetSizeInBytes(c) == bytes);
        CHECK(std::memcmp(vktStructuredVolumeGetData(c), vktStructuredVolumeGetData(v), bytes) == 0);
        vktStructuredVolumeSetDims3i(c, 3, 4, 2);   // resize keeps the leading bytes
        vktStructuredVolumeSetDims3iv(c, vktVec3i_t{17, 9, 6});
        vktStructuredVolumeSetVoxelMapping2f(c, 0.f, 1.f);
        vktStructuredVolumeSetDist3f(c, 0.5f, 0.5f, 0.5f);
        vktBox3f_t const db = vktStructuredVolumeGetDomainBounds(c);
        vktBox3f_t const ob = vktStructuredVolumeGetObjectBounds(c);
        CHECK(db.max.x > db.min.x && ob.max.z > ob.min.z);
        vktStructuredVolumeMigrate(c);   // CPU -> CPU: no-op
        CHECK(vktGetManagedResource(vktStructuredVolumeGetResourceHandle(c)) != nullptr);
        vktStructuredVolumeDestroy(c);
        vktStructuredVolumeDestroy(v);
    }
}

static void codec()
{
    float const maps[][2] = {{0.f, 1.f}, {-1.f, 3.f}, {-0.f, 1.f}, {2.f, -3.f}};
    for (auto const& m : maps)
    {
        for (uint32_t c = 0; c < 65536; ++c)
        {
            uint8_t in[8] = {static_cast<uint8_t>(c), static_cast<uint8_t>(c >> 8)}, out[8] = {0};
            float f = 0.f;
            for (vktDataFormat fmt : {vktDataFormatUInt8, vktDataFormatUInt16, vktDataFormatInt16})
            {
                CHECK(vktUnmapVoxel(&f, in, fmt, m[0], m[1]) == vktNoError);
                CHECK(vktMapVoxel(out, f, fmt, m[0], m[1]) == vktNoError);
            }
        }
        float const specials[] = {0.f, -0.f, 1.f, -1.f, INFINITY, -INFINITY, NAN, 1e-40f, 3e38f, -3e38f, 0.5f};
        for (float s : specials)
            for (vktDataFormat fmt : kFormats)
            {
                uint8_t out[8] = {0};
                float back = 0.f;
                vktMapVoxel(out, s, fmt, m[0], m[1]);
                vktUnmapVoxel(&back, out, fmt, m[0], m[1]);
            }
    }
}

static void memory()
{
    void* p = nullptr;
    vktAllocate(&p, 4096);
    CHECK(p != nullptr);
    std::vector<uint8_t> h(4096, 0x5A);
    vktMemcpy(p, h.data(), h.size(), vktCopyKindHostToHost);
    std::vector<uint8_t> back(4096, 0);
    vktMemcpy(back.data(), p, back.size(), vktCopyKindHostToHost);
    CHECK(back == h);
    vktFree(p);
}

static void handles()
{
    vktArray3D_vktStructuredVolume arr = nullptr;
    vktArray3D_vktStructuredVolume_Create(&arr, vktVec3i_t{3, 2, 2});
    CHECK(vktArray3D_vktStructuredVolume_NumElements(arr) == 12);
    for (int32_t k = 0; k < 2; ++k)
        for (int32_t j = 0; j < 2; ++j)
            for (int32_t i = 0; i < 3; ++i)
                vktStructuredVolumeCreate(vktArray3D_vktStructuredVolume_Access(arr, vktVec3i_t{i, j, k}), 4, 4, 4,
                                          vktDataFormatUInt16, 1.f, 1.f, 1.f, 0.f, 1.f);
    vktArray3D_vktStructuredVolume copy = nullptr;
    vktArray3D_vktStructuredVolume_CreateCopy(&copy, arr);   // shallow: same handles
    CHECK(vktArray3D_vktStructuredVolume_Empty(copy) == VKT_FALSE);
    vktArray3D_vktStructuredVolume_Resize(copy, vktVec3i_t{0, 0, 0});   // drop the shared handles
    vktArray3D_vktStructuredVolume_Destroy(copy);
    // BrickDecomposeResize allocates the bricks under the CPU policy (allocation is host-side)
    vktStructuredVolume src = nullptr;
    vktStructuredVolumeCreate(&src, 10, 9, 8, vktDataFormatUInt8, 1.f, 1.f, 1.f, 0.f, 1.f);
    CHECK(vktBrickDecomposeResizeSV(arr, src, 4, 4, 4, 1, 1, 1, 1, 1, 1) == vktNoError);
    CHECK(vktArray3D_vktStructuredVolume_NumElements(arr) == 18);
    CHECK(vktBrickDecomposeSV(arr, src, 4, 4, 4, 1, 1, 1, 1, 1, 1) == vktInvalidValue);   // CPU policy
    vktArray3D_vktStructuredVolume_Destroy(arr);

    vktLookupTable lut = nullptr;
    vktLookupTableCreate(&lut, 5, 1, 1, vktColorFormatRGBA32F);
    CHECK(vktLookupTableGetSizeInBytes(lut) == 5 * 16);
    std::vector<float> rgba(20, 0.25f);
    vktLookupTableSetData(lut, reinterpret_cast<uint8_t*>(rgba.data()));
    vktLookupTableSetDims3i(lut, 7, 1, 1);
    vktLookupTableMigrate(lut);
    vktLookupTableDestroy(lut);

    vktHistogram hist = nullptr;
    vktHistogramCreate(&hist, 256);
    CHECK(vktHistogramGetNumBins(hist) == 256);
    CHECK(vktHistogramGetBinCounts(hist) != nullptr);
    CHECK(vktComputeHistogramSV(src, hist) == vktInvalidValue);   // CPU policy: GPU backend only
    vktHistogramDestroy(hist);
    vktAggregates_t agg;
    CHECK(vktComputeAggregatesSV(src, &agg) == vktInvalidValue);
    vktStructuredVolumeDestroy(src);
}

static void algorithmsRefuseCpuPolicy()
{
    vktStructuredVolume a = nullptr, b = nullptr, d = nullptr;
    vktStructuredVolumeCreate(&a, 8, 8, 8, vktDataFormatUInt16, 1.f, 1.f, 1.f, 0.f, 1.f);
    vktStructuredVolumeCreate(&b, 8, 8, 8, vktDataFormatUInt16, 1.f, 1.f, 1.f, 0.f, 1.f);
    vktStructuredVolumeCreate(&d, 16, 16, 16, vktDataFormatUInt16, 1.f, 1.f, 1.f, 0.f, 1.f);
    CHECK(vktFillSV(a, 0.5f) == vktInvalidValue);
    CHECK(vktCopySV(b, a) == vktInvalidValue);
    CHECK(vktSumSV(d, a, b) == vktInvalidValue);
    CHECK(vktSafeDiffRangeSV(d, a, b, 0, 0, 0, 8, 8, 8, 0, 0, 0) == vktInvalidValue);
    CHECK(vktResampleSV(d, a, vktFilterModeLinear) == vktInvalidValue);
    vktStructuredVolumeDestroy(a);
    vktStructuredVolumeDestroy(b);
    vktStructuredVolumeDestroy(d);
}

static void streams(char const* dir)
{
    std::string const path = std::string(dir) + "/sanitize_sv.bin";
    vktStructuredVolume v = nullptr;
    vktStructuredVolumeCreate(&v, 11, 6, 4, vktDataFormatUInt16, 1.f, 1.f, 1.f, -1.f, 3.f);
    for (int32_t i = 0; i < 11; ++i)
        vktStructuredVolumeSetValue(v, i, 5, 3, 0.1f * static_cast<float>(i));
    {
        vktRawFile f = nullptr;
        vktRawFileCreateS(&f, path.c_str(), "wb");
        CHECK(vktWriteSVStream(vktRawFileGetBase(f), v) == vktNoError);
        vktRawFileDestroy(f);
    }
    {
        vktRawFile f = nullptr;
        vktRawFileCreateS(&f, path.c_str(), "rb");
        vktStructuredVolume r = nullptr;
        vktStructuredVolumeCreate(&r, 1, 1, 1, vktDataFormatUInt8, 1.f, 1.f, 1.f, 0.f, 1.f);
        CHECK(vktReadSVStream(vktRawFileGetBase(f), r) == vktNoError);
        CHECK(vktStructuredVolumeGetSizeInBytes(r) == vktStructuredVolumeGetSizeInBytes(v));
        CHECK(std::memcmp(vktStructuredVolumeGetData(r), vktStructuredVolumeGetData(v),
                          vktStructuredVolumeGetSizeInBytes(v)) == 0);
        vktStructuredVolumeDestroy(r);
        vktRawFileDestroy(f);
    }
    std::string const raw = std::string(dir) + "/sanitize_11x6x4_uint16.raw";
    {
        vktRawFile f = nullptr;
        vktRawFileCreateS(&f, raw.c_str(), "wb");
        vktOutputStream os = nullptr;
        vktOutputStreamCreate(&os, vktRawFileGetBase(f));
        CHECK(vktOutputStreamWriteSV(os, v) == vktNoError);
        CHECK(vktOutputStreamSeek(os, 0) == vktNoError);
        CHECK(vktOutputStreamWriteRangeSV(os, v, 1, 1, 1, 9, 5, 3) == vktNoError);
        CHECK(vktOutputStreamFlush(os) == vktNoError);
        vktOutputStreamDestroy(os);
        vktRawFileDestroy(f);
    }
    {
        vktRawFile f = nullptr;
        vktRawFileCreateS(&f, raw.c_str(), "rb");
        CHECK(vktRawFileGood(f) == VKT_TRUE);
        vktVec3i_t const dims = vktRawFileGetDims3iv(f);
        CHECK(dims.x == 11 && dims.y == 6 && dims.z == 4);
        vktInputStream is = nullptr;
        vktInputStreamCreate(&is, vktRawFileGetBase(f));
        vktStructuredVolume r = nullptr;
        vktStructuredVolumeCreate(&r, 11, 6, 4, vktDataFormatUInt16, 1.f, 1.f, 1.f, -1.f, 3.f);
        CHECK(vktInputStreamReadSV(is, r) == vktNoError);
        CHECK(vktInputStreamSeek(is, 0) == vktNoError);
        CHECK(vktInputStreamReadRangeSV(is, r, 2, 1, 0, 10, 6, 4) == vktNoError);
        vktStructuredVolumeDestroy(r);
        vktInputStreamDestroy(is);
        vktRawFileDestroy(f);
    }
    std::remove(path.c_str());
    std::remove(raw.c_str());
    vktStructuredVolumeDestroy(v);
}

// Concurrent policy changes, resource registration and volume lifetimes (TSan build).
static void threads()
{
    std::vector<std::thread> pool;
    for (int t = 0; t < 8; ++t)
        pool.emplace_back([t] {
            for (int i = 0; i < 2000; ++i)
            {
                vktExecutionPolicy_t ep = vktGetThreadExecutionPolicy();
                ep.device = (i + t) % 2 ? vktExecutionPolicyDeviceGPU : vktExecutionPolicyDeviceCPU;
                ep.printPerformance = static_cast<uint8_t>(i & 1);
                vktSetThreadExecutionPolicy(ep);
                vktExecutionPolicy_t back = vktGetThreadExecutionPolicy();
                CHECK(back.device == ep.device && back.printPerformance == ep.printPerformance);
            }
            cpuPolicy();
            for (int i = 0; i < 200; ++i)
            {
                int dummy = i;
                vktResourceHandle h = vktRegisterManagedResource(&dummy);
                CHECK(vktGetManagedResource(h) == &dummy);
                vktUnregisterManagedResource(h);
                vktStructuredVolume v = nullptr;
                vktStructuredVolumeCreate(&v, 4 + t, 3, 2, vktDataFormatUInt8, 1.f, 1.f, 1.f, 0.f, 1.f);
                vktStructuredVolumeSetValue(v, 1, 1, 1, 0.5f);
                vktStructuredVolumeDestroy(v);
            }
        });
    for (auto& th : pool)
        th.join();
}

// rt::parallelFor (BrickDecompose's host planning): every item visited exactly once, many jobs
// back to back (no worker may straddle two), concurrent callers (one runs on the pool, the
// others serially) and a nested call from inside a job.
static void hostPool()
{
    for (int job = 0; job < 200; ++job)
    {
        size_t const n = 1000 + 997 * static_cast<size_t>(job);
        std::vector<int> hits(n, 0);
        vkt::rt::parallelFor(n, 64, [&](size_t b, size_t e) {
            for (size_t i = b; i < e; ++i)
                hits[i] += 1;
        });
        bool once = true;
        for (int h : hits)
            once = once && h == 1;
        CHECK(once);
    }
    std::vector<std::thread> callers;
    std::atomic<long> total{0};
    for (int t = 0; t < 4; ++t)
        callers.emplace_back([&] {
            for (int r = 0; r < 20; ++r)
                vkt::rt::parallelFor(50000, 256, [&](size_t b, size_t e) {
                    long local = 0;
                    for (size_t i = b; i < e; ++i)
                        local += static_cast<long>(i);
                    vkt::rt::parallelFor(4, 1, [&](size_t, size_t) {});   // nested: serial
                    total += local;
                });
        });
    for (auto& th : callers)
        th.join();
    CHECK(total.load() == 4L * 20L * (50000L * 49999L / 2));
}

int main(int argc, char** argv)
{
    char const* dir = argc > 1 ? argv[1] : "/tmp";
    cpuPolicy();
    volumes();
    codec();
    memory();
    handles();
    algorithmsRefuseCpuPolicy();
    streams(dir);
    threads();
    hostPool();
    std::printf("host_driver: %d failed checks\n", g_fails);
    return g_fails;
}
