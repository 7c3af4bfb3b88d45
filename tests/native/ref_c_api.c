/* ref_c_api.c -- TEST FIXTURE: a C99 program written against the REFERENCE's own public C
 * declarations (the reference include/c/vkt headers, compiled here with those headers only) and
 * linked to libvolkit.so, i.e. an unmodified reference C user switched to this library.  It
 * runs the config-1 flow of src/examples/CoreAlgorithms.c (Fill, CopyRange, TransformRange,
 * CreateCopy, binary Transform) and UInt16 arithmetic on volumes whose voxels were set on the
 * host under the CPU policy (deferred migration on first GPU use), then writes every volume's
 * raw bytes to <outdir>/<name>.raw for tests/test_reference_boundary.py to compare with the
 * oracle.  Usage: ref_c_api <outdir>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vkt/Arithmetic.h>
#include <vkt/Copy.h>
#include <vkt/ExecutionPolicy.h>
#include <vkt/Fill.h>
#include <vkt/Memory.h>
#include <vkt/StructuredVolume.h>
#include <vkt/Transform.h>
#include <vkt/Voxel.h>

static int failures = 0;

#define CHECK(EXPR)                                                              \
    do {                                                                         \
        if ((EXPR) != vktNoError) {                                              \
            fprintf(stderr, "%s:%d: %s failed\n", __FILE__, __LINE__, #EXPR);    \
            ++failures;                                                          \
        }                                                                        \
    } while (0)

static void set_device(vktExecutionPolicyDevice dev)
{
    vktExecutionPolicy_t ep = vktGetThreadExecutionPolicy();
    ep.device = dev;
    vktSetThreadExecutionPolicy(ep);
}

static void mark_diagonal(int32_t x, int32_t y, int32_t z, vktVoxelView_t voxel)
{
    if (x == y && y == z)
        voxel.bytes[0] = 0xFF;
}

static void or_both(int32_t x, int32_t y, int32_t z, vktVoxelView_t v1, vktVoxelView_t v2)
{
    (void)x; (void)y; (void)z;
    v1.bytes[0] |= v2.bytes[0];
    v2.bytes[0] = v1.bytes[0];
}

/* host pattern (tests/test_reference_boundary.py reproduces it): code = x*7 + y*13 + z*29 + k*101 */
static void set_pattern_u16(vktStructuredVolume v, int k)
{
    int32_t dx, dy, dz, x, y, z;
    vktStructuredVolumeGetDims3i(v, &dx, &dy, &dz);
    for (z = 0; z < dz; ++z)
        for (y = 0; y < dy; ++y)
            for (x = 0; x < dx; ++x) {
                unsigned code = (unsigned)(x * 7 + y * 13 + z * 29 + k * 101) & 0xFFFFu;
                uint8_t b[2];
                b[0] = (uint8_t)(code & 0xFF);
                b[1] = (uint8_t)(code >> 8);
                vktStructuredVolumeSetBytes(v, x, y, z, b);
            }
}

static void dump(vktStructuredVolume v, const char* dir, const char* name)
{
    char path[4096];
    size_t n;
    uint8_t const* data;
    FILE* f;
    set_device(vktExecutionPolicyDeviceCPU);
    vktStructuredVolumeMigrate(v);            /* back to host memory */
    data = vktStructuredVolumeGetData(v);
    n = vktStructuredVolumeGetSizeInBytes(v);
    snprintf(path, sizeof(path), "%s/%s.raw", dir, name);
    f = fopen(path, "wb");
    if (!f || fwrite(data, 1, n, f) != n) {
        fprintf(stderr, "cannot write %s\n", path);
        ++failures;
    }
    if (f)
        fclose(f);
    set_device(vktExecutionPolicyDeviceGPU);
}

int main(int argc, char** argv)
{
    vktStructuredVolume v1, v2, v3, a, b, d, e;
    uint8_t code[8];
    float value = 0.f;
    if (argc < 2) {
        fprintf(stderr, "usage: %s <outdir>\n", argv[0]);
        return 2;
    }

    /* UInt16 inputs are created and filled on the host (CPU policy) */
    vktStructuredVolumeCreate(&a, 37, 23, 11, vktDataFormatUInt16, 1.f, 1.f, 1.f, 0.f, 1.f);
    vktStructuredVolumeCreate(&b, 37, 23, 11, vktDataFormatUInt16, 1.f, 1.f, 1.f, 0.f, 1.f);
    set_pattern_u16(a, 1);
    set_pattern_u16(b, 2);

    set_device(vktExecutionPolicyDeviceGPU);

    /* config 1 (CoreAlgorithms.c:57-93) and the steps after it */
    vktStructuredVolumeCreate(&v1, 64, 64, 64, vktDataFormatUInt8, 1.f, 1.f, 1.f, 0.f, 1.f);
    CHECK(vktFillSV(v1, .1f));
    vktStructuredVolumeCreate(&v2, 24, 24, 24, vktDataFormatUInt8, 1.f, 1.f, 1.f, 0.f, 1.f);
    CHECK(vktCopyRangeSV(v2, v1, 10, 10, 10, 34, 34, 34, 0, 0, 0));
    CHECK(vktTransformRangeSV1(v2, 2, 2, 2, 22, 22, 22, mark_diagonal));
    vktStructuredVolumeCreateCopy(&v3, v2);
    CHECK(vktFillRangeSV(v3, 0, 0, 0, 24, 24, 1, .5f));
    CHECK(vktTransformSV2(v2, v3, or_both));

    /* arithmetic on the migrated UInt16 volumes (mapping [0,1] and [-1,3]) */
    vktStructuredVolumeCreate(&d, 37, 23, 11, vktDataFormatUInt16, 1.f, 1.f, 1.f, 0.f, 1.f);
    CHECK(vktSafeSumSV(d, a, b));
    vktStructuredVolumeCreate(&e, 37, 23, 11, vktDataFormatUInt16, 1.f, 1.f, 1.f, -1.f, 3.f);
    CHECK(vktFillSV(e, 0.25f));
    CHECK(vktDiffRangeSV(e, a, b, 3, 2, 1, 30, 20, 9, 2, 1, 1));

    /* codec through the C API */
    memset(code, 0, sizeof(code));
    CHECK(vktMapVoxel(code, 0.1f, vktDataFormatUInt16, 0.f, 1.f));
    CHECK(vktUnmapVoxel(&value, code, vktDataFormatUInt16, 0.f, 1.f));
    printf("map(0.1f, UInt16) = %u, unmap = %.9g\n", (unsigned)(code[0] | (code[1] << 8)), value);

    dump(v1, argv[1], "v1");
    dump(v2, argv[1], "v2");
    dump(v3, argv[1], "v3");
    dump(d, argv[1], "d");
    dump(e, argv[1], "e");

    vktStructuredVolumeDestroy(v1);
    vktStructuredVolumeDestroy(v2);
    vktStructuredVolumeDestroy(v3);
    vktStructuredVolumeDestroy(a);
    vktStructuredVolumeDestroy(b);
    vktStructuredVolumeDestroy(d);
    vktStructuredVolumeDestroy(e);
    printf("%s\n", failures ? "FAILED" : "ok");
    return failures ? 1 : 0;
}
