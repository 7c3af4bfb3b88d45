/*
 * volkit_c.h -- C99 API of the MI355X-native volkit StructuredVolume core path.
 *
 * This is the drop-in C surface: every symbol below is exported unmangled by
 * volkit_amd/lib/libvolkit.so with the reference's name, argument meaning,
 * enum values and struct layout.  The reference declares the same API across
 * include/c/vkt/{common,linalg,forward,ExecutionPolicy,ManagedResource,Memory,
 * Voxel,StructuredVolume,Fill,Copy,Arithmetic,Transform}.h; per-name forwarding
 * headers in include/c/vkt/ include this file so `#include <vkt/Fill.h>` keeps
 * working.
 *
 * Backend: when the calling thread's execution policy says GPU, each algorithm
 * runs as a hand-written HIP kernel for gfx950 (see include/volkit_hip.h).
 * With the CPU policy the host accessors, allocation and migration work as in
 * the reference, but the algorithms return vktInvalidValue and log an error:
 * this library is the GPU backend only, it never falls back to a CPU loop.
 */
#ifndef VOLKIT_C_H
#define VOLKIT_C_H

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#ifndef VKTAPI
#define VKTAPI __attribute__((visibility("default")))
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ---- common.h (reference include/c/vkt/common.h:16-74) ------------------ */
typedef uint8_t vktBool_t;
#define VKT_FALSE 0
#define VKT_TRUE 1

typedef enum {
    vktInvalidValue = -1, vktNoError = 0,
    vktInvalidDataSource = 1, vktReadError = 2, vktWriteError = 3,
} vktError;

typedef enum {
    vktColorFormatUnspecified, vktColorFormatR8, vktColorFormatRG8, vktColorFormatRGB8,
    vktColorFormatRGBA8, vktColorFormatR16UI, vktColorFormatRG16UI, vktColorFormatRGB16UI,
    vktColorFormatRGBA16UI, vktColorFormatR32UI, vktColorFormatRG32UI, vktColorFormatRGB32UI,
    vktColorFormatRGBA32UI, vktColorFormatR32F, vktColorFormatRG32F, vktColorFormatRGB32F,
    vktColorFormatRGBA32F, vktColorFormatCount,
} vktColorFormat;

/* Values are ABI: Unspecified=0, Int8, Int16, Int32, UInt8=4, UInt16=5, UInt32, Float32=7. */
typedef enum {
    vktDataFormatUnspecified, vktDataFormatInt8, vktDataFormatInt16, vktDataFormatInt32,
    vktDataFormatUInt8, vktDataFormatUInt16, vktDataFormatUInt32, vktDataFormatFloat32,
    vktVoxelFormatCount,
} vktDataFormat;

typedef enum { vktOpenModeRead, vktOpenModeWrite, vktOpenModeReadWrite } vktOpenMode;

/* ---- linalg.h (reference include/c/vkt/linalg.h) ------------------------ */
typedef struct { float x, y; } vktVec2f_t;
typedef struct { float x, y, z; } vktVec3f_t;
typedef struct { float x, y, z, w; } vktVec4f_t;
typedef struct { int x, y; } vktVec2i_t;
typedef struct { int x, y, z; } vktVec3i_t;
typedef struct { int x, y, z, w; } vktVec4i_t;
typedef struct { vktVec2f_t min, max; } vktBox2f_t;
typedef struct { vktVec3f_t min, max; } vktBox3f_t;
typedef struct { vktVec2i_t min, max; } vktBox2i_t;
typedef struct { vktVec3i_t min, max; } vktBox3i_t;
typedef struct { vktVec3f_t col0, col1, col2; } vktMat3f_t;
typedef struct { vktVec4f_t col0, col1, col2, col3; } vktMat4f_t;
typedef enum { vktAxisX, vktAxisY, vktAxisZ } vktAxis;

/* ---- forward.h: opaque handles (reference include/c/vkt/forward.h) ------ */
struct vktStructuredVolume_impl;
typedef struct vktStructuredVolume_impl* vktStructuredVolume;

/* ---- ExecutionPolicy.h (reference include/c/vkt/ExecutionPolicy.h:13-45) -
 * deviceApi value 0 ("CUDA" in the reference) selects the HIP backend here;
 * vktExecutionPolicyDeviceAPIHIP is an alias with the same value. */
typedef enum { vktExecutionPolicyDeviceCPU, vktExecutionPolicyDeviceGPU } vktExecutionPolicyDevice;
typedef enum {
    vktExecutionPolicyHostAPISerial, vktExecutionPolicyAPIOpenMP, vktExecutionPolicyAPIAuto,
} vktExecutionPolicyHostAPI;
typedef enum {
    vktExecutionPolicyDeviceAPICUDA, vktExecutionPolicyDeviceAPIAuto,
} vktExecutionPolicyDeviceAPI;
#define vktExecutionPolicyDeviceAPIHIP vktExecutionPolicyDeviceAPICUDA

typedef struct {
    vktExecutionPolicyDevice device;
    vktExecutionPolicyHostAPI hostApi;
    vktExecutionPolicyDeviceAPI deviceApi;
    vktBool_t printPerformance;
} vktExecutionPolicy_t;

VKTAPI void vktSetThreadExecutionPolicy(vktExecutionPolicy_t policy);
VKTAPI vktExecutionPolicy_t vktGetThreadExecutionPolicy(void);

/* ---- ManagedResource.h (reference include/c/vkt/ManagedResource.h:14-22) */
typedef void* vktManagedResource;
typedef uint32_t vktResourceHandle;
VKTAPI vktResourceHandle vktRegisterManagedResource(vktManagedResource resource);
VKTAPI void vktUnregisterManagedResource(vktResourceHandle handle);
VKTAPI vktManagedResource vktGetManagedResource(vktResourceHandle handle);

/* ---- Memory.h (reference include/c/vkt/Memory.h:13-30) ------------------ */
typedef enum {
    vktCopyKindHostToHost, vktCopyKindHostToDevice, vktCopyKindDeviceToHost, vktCopyKindDeviceToDevice,
} vktCopyKind;
VKTAPI void vktAllocate(void** ptr, size_t size);
VKTAPI void vktFree(void* ptr);
VKTAPI void vktMemcpy(void* dst, void const* src, size_t size, vktCopyKind ck);

/* ---- Voxel.h (reference include/c/vkt/Voxel.h:16-45) -------------------- */
typedef struct {
    uint8_t* bytes;
    vktDataFormat dataFormat;
    float mappingLo;
    float mappingHi;
} vktVoxelView_t;
VKTAPI vktError vktMapVoxel(uint8_t* dst, float value, vktDataFormat dataFormat,
                            float mappingLo, float mappingHi);
VKTAPI vktError vktUnmapVoxel(float* value, uint8_t const* src, vktDataFormat dataFormat,
                              float mappingLo, float mappingHi);

/* ---- StructuredVolume.h (reference include/c/vkt/StructuredVolume.h:19-120)
 * The reference declares but never defines the accessors below Destroy;
 * this library defines all of them. */
VKTAPI uint8_t vktStructuredVolumeGetMaxBytesPerVoxel(void);
VKTAPI void vktStructuredVolumeCreate(vktStructuredVolume* volume, int32_t dimX, int32_t dimY,
                                      int32_t dimZ, vktDataFormat dataFormat, float distX,
                                      float distY, float distZ, float mappingLo, float mappingHi);
VKTAPI void vktStructuredVolumeCreateCopy(vktStructuredVolume* volume, vktStructuredVolume rhs);
VKTAPI void vktStructuredVolumeDestroy(vktStructuredVolume volume);
VKTAPI void vktStructuredVolumeSetDims3i(vktStructuredVolume volume, int32_t dimX, int32_t dimY, int32_t dimZ);
VKTAPI void vktStructuredVolumeGetDims3i(vktStructuredVolume volume, int32_t* dimX, int32_t* dimY, int32_t* dimZ);
VKTAPI void vktStructuredVolumeSetDims3iv(vktStructuredVolume volume, vktVec3i_t dims);
VKTAPI vktVec3i_t vktStructuredVolumeGetDims3iv(vktStructuredVolume volume);
VKTAPI void vktStructuredVolumeSetDataFormat(vktStructuredVolume volume, vktDataFormat dataFormat);
VKTAPI vktDataFormat vktStructuredVolumeGetDataFormat(vktStructuredVolume volume);
VKTAPI void vktStructuredVolumeSetDist3f(vktStructuredVolume volume, float distX, float distY, float distZ);
VKTAPI void vktStructuredVolumeGetDist3f(vktStructuredVolume volume, float* distX, float* distY, float* distZ);
VKTAPI void vktStructuredVolumeSetDist3fv(vktStructuredVolume volume, vktVec3f_t dist);
VKTAPI vktVec3f_t vktStructuredVolumeGetDist3fv(vktStructuredVolume volume);
VKTAPI void vktStructuredVolumeSetVoxelMapping2f(vktStructuredVolume volume, float lo, float hi);
VKTAPI void vktStructuredVolumeGetVoxelMapping2f(vktStructuredVolume volume, float* lo, float* hi);
VKTAPI void vktStructuredVolumeSetVoxelMapping2fv(vktStructuredVolume volume, vktVec2f_t mapping);
VKTAPI vktVec2f_t vktStructuredVolumeGetVoxelMapping2fv(vktStructuredVolume volume);
VKTAPI vktBox3f_t vktStructuredVolumeGetDomainBounds(vktStructuredVolume volume);
VKTAPI vktBox3f_t vktStructuredVolumeGetObjectBounds(vktStructuredVolume volume);
VKTAPI uint8_t* vktStructuredVolumeGetData(vktStructuredVolume volume);
VKTAPI void vktStructuredVolumeSetValue(vktStructuredVolume volume, int32_t x, int32_t y, int32_t z, float value);
VKTAPI void vktStructuredVolumeGetValue(vktStructuredVolume volume, int32_t x, int32_t y, int32_t z, float* value);
VKTAPI void vktStructuredVolumeSetBytes(vktStructuredVolume volume, int32_t x, int32_t y, int32_t z, uint8_t const* data);
VKTAPI void vktStructuredVolumeGetBytes(vktStructuredVolume volume, int32_t x, int32_t y, int32_t z, uint8_t* data);
VKTAPI size_t vktStructuredVolumeGetSizeInBytes(vktStructuredVolume volume);
VKTAPI vktResourceHandle vktStructuredVolumeGetResourceHandle(vktStructuredVolume volume);
VKTAPI void vktStructuredVolumeMigrate(vktStructuredVolume volume);
/* extension: migrate() with its outcome -- vktInvalidValue when the bytes could not be moved to
 * the thread's device (allocation or copy failure; vktHipGetLastErrorString says which).  They
 * then stay where they were, intact, and the next access tries again. */
VKTAPI vktError vktStructuredVolumeMigrateChecked(vktStructuredVolume volume);

/* ---- Fill.h (reference include/c/vkt/Fill.h:16-43; HV overloads out of scope) */
VKTAPI vktError vktFillSV(vktStructuredVolume volume, float value);
VKTAPI vktError vktFillRangeSV(vktStructuredVolume volume, int32_t firstX, int32_t firstY,
                               int32_t firstZ, int32_t lastX, int32_t lastY, int32_t lastZ,
                               float value);

/* ---- Copy.h (reference include/c/vkt/Copy.h:16-41) ---------------------- */
VKTAPI vktError vktCopySV(vktStructuredVolume dst, vktStructuredVolume src);
VKTAPI vktError vktCopyRangeSV(vktStructuredVolume dst, vktStructuredVolume src,
                               int32_t firstX, int32_t firstY, int32_t firstZ,
                               int32_t lastX, int32_t lastY, int32_t lastZ,
                               int32_t dstOffsetX, int32_t dstOffsetY, int32_t dstOffsetZ);

/* ---- Arithmetic.h (reference include/c/vkt/Arithmetic.h:16-216) ---------
 * Ten ops, each as whole-volume (`vkt<Op>SV`) and range (`vkt<Op>RangeSV`). */
#define VKT_DECLARE_ARITHMETIC_C_(NAME)                                                    \
    VKTAPI vktError vkt##NAME##SV(vktStructuredVolume dest, vktStructuredVolume source1,   \
                                  vktStructuredVolume source2);                             \
    VKTAPI vktError vkt##NAME##RangeSV(vktStructuredVolume dest, vktStructuredVolume source1,\
                                       vktStructuredVolume source2, int32_t firstX,         \
                                       int32_t firstY, int32_t firstZ, int32_t lastX,       \
                                       int32_t lastY, int32_t lastZ, int32_t dstOffsetX,    \
                                       int32_t dstOffsetY, int32_t dstOffsetZ);
VKT_DECLARE_ARITHMETIC_C_(Sum)
VKT_DECLARE_ARITHMETIC_C_(Diff)
VKT_DECLARE_ARITHMETIC_C_(Prod)
VKT_DECLARE_ARITHMETIC_C_(Quot)
VKT_DECLARE_ARITHMETIC_C_(AbsDiff)
VKT_DECLARE_ARITHMETIC_C_(SafeSum)
VKT_DECLARE_ARITHMETIC_C_(SafeDiff)
VKT_DECLARE_ARITHMETIC_C_(SafeProd)
VKT_DECLARE_ARITHMETIC_C_(SafeQuot)
VKT_DECLARE_ARITHMETIC_C_(SafeAbsDiff)
#undef VKT_DECLARE_ARITHMETIC_C_

/* ---- Transform.h (reference include/c/vkt/Transform.h:16-76) ------------
 * vktTransformRangeSV2 follows the header's 12-argument form (the reference
 * defines a 9-argument function under this name, src/vkt/Transform.cpp:131). */
typedef void (*vktTransformUnaryOp)(int32_t x, int32_t y, int32_t z, vktVoxelView_t voxel);
typedef void (*vktTransformBinaryOp)(int32_t x1, int32_t y1, int32_t z1,
                                     vktVoxelView_t voxel1, vktVoxelView_t voxel2);
VKTAPI vktError vktTransformSV1(vktStructuredVolume volume, vktTransformUnaryOp unaryOp);
VKTAPI vktError vktTransformSV2(vktStructuredVolume volume1, vktStructuredVolume volume2,
                                vktTransformBinaryOp binaryOp);
VKTAPI vktError vktTransformRangeSV1(vktStructuredVolume volume, int32_t firstX, int32_t firstY,
                                     int32_t firstZ, int32_t lastX, int32_t lastY, int32_t lastZ,
                                     vktTransformUnaryOp unaryOp);
VKTAPI vktError vktTransformRangeSV2(vktStructuredVolume volume1, vktStructuredVolume volume2,
                                     int32_t firstX, int32_t firstY, int32_t firstZ,
                                     int32_t lastX, int32_t lastY, int32_t lastZ,
                                     int32_t volume2OffsetX, int32_t volume2OffsetY,
                                     int32_t volume2OffsetZ, vktTransformBinaryOp binaryOp);

/* ---- Resample (C++-only in the reference, include/cpp/vkt/Resample.hpp:14-31).
 * C entry point added so that C, ctypes and cgo callers reach the same path. */
typedef enum { vktFilterModeNearest, vktFilterModeLinear } vktFilterMode;
VKTAPI vktError vktResampleSV(vktStructuredVolume dst, vktStructuredVolume src, vktFilterMode fm);

/* ---- Array3D.h for vktStructuredVolume (reference include/c/vkt/Array3D.h:18-237) ----
 * The reference instantiates these as header-inline functions over a ManagedBuffer of
 * handles; here they are exported functions over a host-resident handle array (see
 * vkt::Array3D in volkit.hpp).  Ownership: Destroy also destroys every non-NULL volume
 * handle the array holds (the reference leaks the bricks its examples create). */
struct vktArray3D_vktStructuredVolume_impl;
typedef struct vktArray3D_vktStructuredVolume_impl* vktArray3D_vktStructuredVolume;
typedef vktStructuredVolume vktArray3D_vktStructuredVolume_ValueType;
typedef vktStructuredVolume* vktArray3D_vktStructuredVolume_Iterator;
typedef vktStructuredVolume const* vktArray3D_vktStructuredVolume_ConstIterator;
VKTAPI void vktArray3D_vktStructuredVolume_CreateEmpty(vktArray3D_vktStructuredVolume* arr);
VKTAPI void vktArray3D_vktStructuredVolume_Create(vktArray3D_vktStructuredVolume* arr, vktVec3i_t dims);
VKTAPI void vktArray3D_vktStructuredVolume_CreateCopy(vktArray3D_vktStructuredVolume* arr,
                                                      vktArray3D_vktStructuredVolume rhs);
VKTAPI void vktArray3D_vktStructuredVolume_Destroy(vktArray3D_vktStructuredVolume arr);
VKTAPI void vktArray3D_vktStructuredVolume_Resize(vktArray3D_vktStructuredVolume arr, vktVec3i_t dims);
VKTAPI void vktArray3D_vktStructuredVolume_Fill(vktArray3D_vktStructuredVolume arr, vktStructuredVolume value);
VKTAPI vktArray3D_vktStructuredVolume_Iterator vktArray3D_vktStructuredVolume_Begin(vktArray3D_vktStructuredVolume arr);
VKTAPI vktArray3D_vktStructuredVolume_ConstIterator vktArray3D_vktStructuredVolume_CBegin(vktArray3D_vktStructuredVolume arr);
VKTAPI vktArray3D_vktStructuredVolume_Iterator vktArray3D_vktStructuredVolume_End(vktArray3D_vktStructuredVolume arr);
VKTAPI vktArray3D_vktStructuredVolume_ConstIterator vktArray3D_vktStructuredVolume_CEnd(vktArray3D_vktStructuredVolume arr);
VKTAPI vktArray3D_vktStructuredVolume_ValueType* vktArray3D_vktStructuredVolume_Access(vktArray3D_vktStructuredVolume arr,
                                                                                       vktVec3i_t index);
VKTAPI vktArray3D_vktStructuredVolume_ValueType const* vktArray3D_vktStructuredVolume_CAccess(
    vktArray3D_vktStructuredVolume arr, vktVec3i_t index);
VKTAPI vktBool_t vktArray3D_vktStructuredVolume_Empty(vktArray3D_vktStructuredVolume arr);
VKTAPI vktStructuredVolume* vktArray3D_vktStructuredVolume_Data(vktArray3D_vktStructuredVolume arr);
VKTAPI vktStructuredVolume const* vktArray3D_vktStructuredVolume_CData(vktArray3D_vktStructuredVolume arr);
VKTAPI vktVec3i_t vktArray3D_vktStructuredVolume_Dims(vktArray3D_vktStructuredVolume arr);
VKTAPI size_t vktArray3D_vktStructuredVolume_NumElements(vktArray3D_vktStructuredVolume arr);

/* ---- Decompose.h (reference include/c/vkt/Decompose.h:18-44) ------------- */
VKTAPI vktError vktBrickDecomposeSV(vktArray3D_vktStructuredVolume decomp, vktStructuredVolume source,
                                    int32_t brickSizeX, int32_t brickSizeY, int32_t brickSizeZ,
                                    int32_t haloSizeNegX, int32_t haloSizeNegY, int32_t haloSizeNegZ,
                                    int32_t haloSizePosX, int32_t haloSizePosY, int32_t haloSizePosZ);
VKTAPI vktError vktBrickDecomposeResizeSV(vktArray3D_vktStructuredVolume decomp, vktStructuredVolume source,
                                          int32_t brickSizeX, int32_t brickSizeY, int32_t brickSizeZ,
                                          int32_t haloSizeNegX, int32_t haloSizeNegY, int32_t haloSizeNegZ,
                                          int32_t haloSizePosX, int32_t haloSizePosY, int32_t haloSizePosZ);

/* ---- RawFile.h / InputStream.h (reference include/c/vkt/RawFile.h:16-40,
 *      include/c/vkt/InputStream.h:14-34; handles of forward.h) ------------------------
 * vktRawFileRead returns bytes (the reference returns fread's item count).  OutputStream
 * and the SV stream format have no C API in the reference; added here. */
struct vktDataSource_impl;
typedef struct vktDataSource_impl* vktDataSource;
struct vktRawFile_impl;
typedef struct vktRawFile_impl* vktRawFile;
struct vktInputStream_impl;
typedef struct vktInputStream_impl* vktInputStream;
struct vktOutputStream_impl;
typedef struct vktOutputStream_impl* vktOutputStream;
VKTAPI void vktRawFileCreateS(vktRawFile* file, char const* fileName, char const* mode);
VKTAPI void vktRawFileCreateFD(vktRawFile* file, FILE* fd);
VKTAPI vktDataSource vktRawFileGetBase(vktRawFile file);
VKTAPI void vktRawFileDestroy(vktRawFile file);
VKTAPI size_t vktRawFileRead(vktRawFile file, char* buf, size_t len);
VKTAPI vktBool_t vktRawFileGood(vktRawFile file);
VKTAPI vktVec3i_t vktRawFileGetDims3iv(vktRawFile file);
VKTAPI vktDataFormat vktRawFileGetDataFormat(vktRawFile file);
VKTAPI void vktInputStreamCreate(vktInputStream* stream, vktDataSource source);
VKTAPI void vktInputStreamDestroy(vktInputStream stream);
VKTAPI vktError vktInputStreamReadSV(vktInputStream stream, vktStructuredVolume volume);
VKTAPI vktError vktInputStreamReadRangeSV(vktInputStream stream, vktStructuredVolume volume,
                                          int32_t firstX, int32_t firstY, int32_t firstZ,
                                          int32_t lastX, int32_t lastY, int32_t lastZ);
VKTAPI vktError vktInputStreamSeek(vktInputStream stream, size_t pos);
VKTAPI void vktOutputStreamCreate(vktOutputStream* stream, vktDataSource source);
VKTAPI void vktOutputStreamDestroy(vktOutputStream stream);
VKTAPI vktError vktOutputStreamWriteSV(vktOutputStream stream, vktStructuredVolume volume);
VKTAPI vktError vktOutputStreamWriteRangeSV(vktOutputStream stream, vktStructuredVolume volume,
                                            int32_t firstX, int32_t firstY, int32_t firstZ,
                                            int32_t lastX, int32_t lastY, int32_t lastZ);
VKTAPI vktError vktOutputStreamSeek(vktOutputStream stream, size_t pos);
VKTAPI vktError vktOutputStreamFlush(vktOutputStream stream);
/* the reference CLI's StructuredVolume stream (src/cli/main.cpp:32-88); ReadSVStream
 * re-creates *volume (a handle created before, e.g. with vktStructuredVolumeCreate). */
VKTAPI vktError vktReadSVStream(vktDataSource source, vktStructuredVolume volume);
VKTAPI vktError vktWriteSVStream(vktDataSource source, vktStructuredVolume volume);

/* ---- Aggregates.h (reference include/c/vkt/Aggregates.h:17-44) ---------- */
typedef struct {
    float min;
    float max;
    float mean;
    float stddev;
    float var;
    float sum;
    float prod;
    vktVec3i_t argmin;
    vktVec3i_t argmax;
} vktAggregates_t;
VKTAPI vktError vktComputeAggregatesSV(vktStructuredVolume volume, vktAggregates_t* aggregates);
VKTAPI vktError vktComputeAggregatesRangeSV(vktStructuredVolume volume, vktAggregates_t* aggregates,
                                            int32_t firstX, int32_t firstY, int32_t firstZ,
                                            int32_t lastX, int32_t lastY, int32_t lastZ);

/* ---- Histogram (C++-only in the reference, include/cpp/vkt/Histogram.hpp:14-42).
 * C entry points added so that C, ctypes and cgo callers reach the same path: the
 * handle wraps a vkt::Histogram (a ManagedBuffer of size_t bin counts, migrated with the
 * thread policy like every ManagedBuffer). */
struct vktHistogram_impl;
typedef struct vktHistogram_impl* vktHistogram;
VKTAPI void vktHistogramCreate(vktHistogram* histogram, size_t numBins);
VKTAPI void vktHistogramDestroy(vktHistogram histogram);
VKTAPI size_t vktHistogramGetNumBins(vktHistogram histogram);
/* bin counts in the address space of the calling thread's device (migrates first) */
VKTAPI size_t* vktHistogramGetBinCounts(vktHistogram histogram);
VKTAPI vktError vktComputeHistogramSV(vktStructuredVolume volume, vktHistogram histogram);
VKTAPI vktError vktComputeHistogramRangeSV(vktStructuredVolume volume, vktHistogram histogram,
                                           int32_t firstX, int32_t firstY, int32_t firstZ,
                                           int32_t lastX, int32_t lastY, int32_t lastZ);

/* ---- LookupTable.h (reference include/c/vkt/LookupTable.h:18-58) --------- */
struct vktLookupTable_impl;
typedef struct vktLookupTable_impl* vktLookupTable;
VKTAPI void vktLookupTableCreate(vktLookupTable* lut, int32_t dimX, int32_t dimY, int32_t dimZ,
                                 vktColorFormat format);
VKTAPI void vktLookupTableDestroy(vktLookupTable lut);
VKTAPI void vktLookupTableSetDims3i(vktLookupTable lut, int32_t dimX, int32_t dimY, int32_t dimZ);
VKTAPI void vktLookupTableGetDims3i(vktLookupTable lut, int32_t* dimX, int32_t* dimY, int32_t* dimZ);
VKTAPI void vktLookupTableSetDims3iv(vktLookupTable lut, vktVec3i_t dims);
VKTAPI vktVec3i_t vktLookupTableGetDims3iv(vktLookupTable lut);
VKTAPI void vktLookupTableSetColorFormat(vktLookupTable lut, vktColorFormat format);
VKTAPI vktColorFormat vktLookupTableGetColorFormat(vktLookupTable lut);
VKTAPI void vktLookupTableSetData(vktLookupTable lut, uint8_t* data);
VKTAPI uint8_t* vktLookupTableGetData(vktLookupTable lut);
VKTAPI size_t vktLookupTableGetSizeInBytes(vktLookupTable lut);
VKTAPI vktResourceHandle vktLookupTableGetResourceHandle(vktLookupTable lut);
VKTAPI void vktLookupTableMigrate(vktLookupTable lut);

/* ---- Render.h (reference include/c/vkt/Render.h:15-150, structured volumes) ---- */
typedef enum {
    vktRenderAlgoRayMarching,
    vktRenderAlgoImplicitIso,
    vktRenderAlgoMultiScattering,
} vktRenderAlgo;

typedef struct {
    vktRenderAlgo renderAlgo;
    float dtRayMarching;
    uint16_t numIsoSurfaces;
    float isoSurfaces[10];
    float dtImplicitIso;
    float majorant;
    unsigned animationFrame;
    vktResourceHandle rgbaLookupTable;
    vktResourceHandle histogram;
    int viewportWidth;
    int viewportHeight;
    vktBool_t sRGB;
    struct {
        vktBool_t isSet;
        vktVec3f_t eye;
        vktVec3f_t center;
        vktVec3f_t up;
        float fovy;
        float lensRadius;
        float focalDistance;
    } initialCamera;
    struct {
        vktBool_t enabled;
        char const* fileName;
        vktBool_t takeOnClose;
        char key;
        char const* message;
    } snapshotTool;
} vktRenderState_t;

/* header-inline in the reference; exported here */
VKTAPI void vktRenderStateDefaultInit(vktRenderState_t* renderState);
/* headless (see vkt::Render in volkit.hpp) */
VKTAPI vktError vktRenderSV(vktStructuredVolume volume, vktRenderState_t renderState,
                            vktRenderState_t* newRenderState);
/* extension: accumulate numFrames frames into host RGBA floats (width*height*4, row 0 = bottom) */
VKTAPI vktError vktRenderSVToImage(vktStructuredVolume volume, vktRenderState_t renderState,
                                   uint32_t numFrames, float* rgba);

#ifdef __cplusplus
}
#endif

#endif /* VOLKIT_C_H */
