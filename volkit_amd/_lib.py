"""ctypes binding of libvolkit.so (the C ABI declared in include/volkit_c.h and
include/volkit_hip.h).

The library is built in-tree (``python -c "import __graft_entry__ as g; g.build()"`` or
``make -C volkit_amd/csrc``) and loaded from ``volkit_amd/lib/libvolkit.so``.  There is no
fallback: if the shared library is missing, importing :mod:`volkit_amd` raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VOLKIT_LIB", os.path.join(_HERE, "lib", "libvolkit.so"))


class VolkitLibraryMissing(ImportError):
    pass


if not os.path.exists(LIB_PATH):
    raise VolkitLibraryMissing(
        f"libvolkit.so not found at {LIB_PATH}: build it with `make -C volkit_amd/csrc` "
        "(the HIP/gfx950 backend has no CPU fallback)")

lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)

# ---- C types -----------------------------------------------------------------------------
c_vol = C.c_void_p            # vktStructuredVolume (opaque handle)
c_err = C.c_int               # vktError
i32, u32, u64, f32 = C.c_int32, C.c_uint32, C.c_uint64, C.c_float
P = C.POINTER


class Vec3i_t(C.Structure):
    _fields_ = [("x", C.c_int), ("y", C.c_int), ("z", C.c_int)]


class Vec3f_t(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class Vec2f_t(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float)]


class Box3f_t(C.Structure):
    _fields_ = [("min", Vec3f_t), ("max", Vec3f_t)]


class ExecutionPolicy_t(C.Structure):
    _fields_ = [("device", C.c_int), ("hostApi", C.c_int), ("deviceApi", C.c_int),
                ("printPerformance", C.c_uint8)]


class VoxelView_t(C.Structure):
    _fields_ = [("bytes", P(C.c_uint8)), ("dataFormat", C.c_int), ("mappingLo", C.c_float),
                ("mappingHi", C.c_float)]


class HipVolumeView_t(C.Structure):
    _fields_ = [("data", C.c_void_p), ("dimX", i32), ("dimY", i32), ("dimZ", i32),
                ("dataFormat", i32), ("mappingLo", f32), ("mappingHi", f32)]


class HipBrickRange_t(C.Structure):
    _fields_ = [("brick", HipVolumeView_t), ("first", Vec3i_t), ("last", Vec3i_t)]


class HipBrickGrid_t(C.Structure):
    _fields_ = [("numBricks", Vec3i_t), ("brickSize", Vec3i_t), ("haloNeg", Vec3i_t), ("haloPos", Vec3i_t)]


class HipSlabTransfer_t(C.Structure):
    _fields_ = [("peer", i32), ("z0", i32), ("z1", i32), ("send", i32)]


class HipSlab_t(C.Structure):
    _fields_ = [("view", HipVolumeView_t), ("z0", i32), ("globalDimZ", i32)]


class HipSlabPiece_t(C.Structure):
    _fields_ = [("zBegin", i32), ("zEnd", i32), ("dstZ", i32), ("srcZ", i32 * 2), ("srcPlanes", i32 * 2),
                ("bufPlane", i32 * 2)]


class HipSlabMove_t(C.Structure):
    _fields_ = [("peer", i32), ("send", i32), ("source", i32), ("z0", i32), ("z1", i32), ("bufPlane", i32)]


class HipCommId_t(C.Structure):
    _fields_ = [("internal", C.c_char * 128)]


c_comm = C.c_void_p           # vktHipComm_t (opaque handle)
c_arr = C.c_void_p            # vktArray3D_vktStructuredVolume (opaque handle)
c_hist = C.c_void_p           # vktHistogram (opaque handle)


class Aggregates_t(C.Structure):
    _fields_ = [("min", f32), ("max", f32), ("mean", f32), ("stddev", f32), ("var", f32), ("sum", f32),
                ("prod", f32), ("argmin", Vec3i_t), ("argmax", Vec3i_t)]


class HipAggregatePartial_t(C.Structure):
    _fields_ = [("sum", C.c_double), ("prod", C.c_double), ("sumSq", C.c_double), ("minValue", f32),
                ("maxValue", f32), ("minIndex", u64), ("maxIndex", u64), ("count", u64)]

class HipMomentPartial_t(C.Structure):
    _fields_ = [("count", u64), ("codeSum", u64), ("codeSumSqLo", u64), ("codeSumSqHi", u64),
                ("mean", C.c_double), ("m2", C.c_double), ("sum", C.c_double), ("prod", C.c_double),
                ("minValue", f32), ("maxValue", f32), ("minIndex", u64), ("maxIndex", u64),
                ("form", i32), ("flags", C.c_uint32)]


class Vec3fC_t(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class _InitialCamera(C.Structure):
    _fields_ = [("isSet", C.c_uint8), ("eye", Vec3fC_t), ("center", Vec3fC_t), ("up", Vec3fC_t),
                ("fovy", C.c_float), ("lensRadius", C.c_float), ("focalDistance", C.c_float)]


class _SnapshotTool(C.Structure):
    _fields_ = [("enabled", C.c_uint8), ("fileName", C.c_char_p), ("takeOnClose", C.c_uint8),
                ("key", C.c_char), ("message", C.c_char_p)]


class RenderState_t(C.Structure):
    _fields_ = [("renderAlgo", C.c_int), ("dtRayMarching", C.c_float), ("numIsoSurfaces", C.c_uint16),
                ("isoSurfaces", C.c_float * 10), ("dtImplicitIso", C.c_float), ("majorant", C.c_float),
                ("animationFrame", C.c_uint), ("rgbaLookupTable", C.c_uint32), ("histogram", C.c_uint32),
                ("viewportWidth", C.c_int), ("viewportHeight", C.c_int), ("sRGB", C.c_uint8),
                ("initialCamera", _InitialCamera), ("snapshotTool", _SnapshotTool)]


class HipRenderParams_t(C.Structure):
    _fields_ = [("algo", i32), ("width", i32), ("height", i32), ("frameBegin", u32),
                ("eye", f32 * 3), ("U", f32 * 3), ("V", f32 * 3), ("W", f32 * 3), ("right", f32 * 3), ("up", f32 * 3),
                ("lensRadius", f32), ("focalDistance", f32), ("bbox", f32 * 3),
                ("dtRayMarching", f32), ("dtImplicitIso", f32), ("majorant", f32),
                ("numIsoSurfaces", i32), ("isoSurfaces", f32 * 10), ("sRGB", i32),
                ("lut", C.c_void_p), ("lutSize", i32)]


UnaryOp = C.CFUNCTYPE(None, i32, i32, i32, VoxelView_t)
BinaryOp = C.CFUNCTYPE(None, i32, i32, i32, VoxelView_t, VoxelView_t)

ARITH_OPS = ["Sum", "Diff", "Prod", "Quot", "AbsDiff",
             "SafeSum", "SafeDiff", "SafeProd", "SafeQuot", "SafeAbsDiff"]

_R9 = [i32] * 9

# name -> (restype, argtypes)
SIGNATURES = {
    # ExecutionPolicy.h
    "vktSetThreadExecutionPolicy": (None, [ExecutionPolicy_t]),
    "vktGetThreadExecutionPolicy": (ExecutionPolicy_t, []),
    # ManagedResource.h
    "vktRegisterManagedResource": (u32, [C.c_void_p]),
    "vktUnregisterManagedResource": (None, [u32]),
    "vktGetManagedResource": (C.c_void_p, [u32]),
    # Memory.h
    "vktAllocate": (None, [P(C.c_void_p), C.c_size_t]),
    "vktFree": (None, [C.c_void_p]),
    "vktMemcpy": (None, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]),
    # Voxel.h
    "vktMapVoxel": (c_err, [P(C.c_uint8), f32, C.c_int, f32, f32]),
    "vktUnmapVoxel": (c_err, [P(C.c_float), P(C.c_uint8), C.c_int, f32, f32]),
    # StructuredVolume.h
    "vktStructuredVolumeGetMaxBytesPerVoxel": (C.c_uint8, []),
    "vktStructuredVolumeCreate": (None, [P(c_vol), i32, i32, i32, C.c_int, f32, f32, f32, f32, f32]),
    "vktStructuredVolumeCreateCopy": (None, [P(c_vol), c_vol]),
    "vktStructuredVolumeDestroy": (None, [c_vol]),
    "vktStructuredVolumeSetDims3i": (None, [c_vol, i32, i32, i32]),
    "vktStructuredVolumeGetDims3i": (None, [c_vol, P(i32), P(i32), P(i32)]),
    "vktStructuredVolumeSetDims3iv": (None, [c_vol, Vec3i_t]),
    "vktStructuredVolumeGetDims3iv": (Vec3i_t, [c_vol]),
    "vktStructuredVolumeSetDataFormat": (None, [c_vol, C.c_int]),
    "vktStructuredVolumeGetDataFormat": (C.c_int, [c_vol]),
    "vktStructuredVolumeSetDist3f": (None, [c_vol, f32, f32, f32]),
    "vktStructuredVolumeGetDist3f": (None, [c_vol, P(f32), P(f32), P(f32)]),
    "vktStructuredVolumeSetDist3fv": (None, [c_vol, Vec3f_t]),
    "vktStructuredVolumeGetDist3fv": (Vec3f_t, [c_vol]),
    "vktStructuredVolumeSetVoxelMapping2f": (None, [c_vol, f32, f32]),
    "vktStructuredVolumeGetVoxelMapping2f": (None, [c_vol, P(f32), P(f32)]),
    "vktStructuredVolumeSetVoxelMapping2fv": (None, [c_vol, Vec2f_t]),
    "vktStructuredVolumeGetVoxelMapping2fv": (Vec2f_t, [c_vol]),
    "vktStructuredVolumeGetDomainBounds": (Box3f_t, [c_vol]),
    "vktStructuredVolumeGetObjectBounds": (Box3f_t, [c_vol]),
    "vktStructuredVolumeGetData": (C.c_void_p, [c_vol]),
    "vktStructuredVolumeSetValue": (None, [c_vol, i32, i32, i32, f32]),
    "vktStructuredVolumeGetValue": (None, [c_vol, i32, i32, i32, P(f32)]),
    "vktStructuredVolumeSetBytes": (None, [c_vol, i32, i32, i32, P(C.c_uint8)]),
    "vktStructuredVolumeGetBytes": (None, [c_vol, i32, i32, i32, P(C.c_uint8)]),
    "vktStructuredVolumeGetSizeInBytes": (C.c_size_t, [c_vol]),
    "vktStructuredVolumeGetResourceHandle": (u32, [c_vol]),
    "vktStructuredVolumeMigrate": (None, [c_vol]),
    "vktStructuredVolumeMigrateChecked": (c_err, [c_vol]),
    # Fill.h / Copy.h
    "vktFillSV": (c_err, [c_vol, f32]),
    "vktFillRangeSV": (c_err, [c_vol, i32, i32, i32, i32, i32, i32, f32]),
    "vktCopySV": (c_err, [c_vol, c_vol]),
    "vktCopyRangeSV": (c_err, [c_vol, c_vol] + _R9),
    # Transform.h
    "vktTransformSV1": (c_err, [c_vol, UnaryOp]),
    "vktTransformSV2": (c_err, [c_vol, c_vol, BinaryOp]),
    "vktTransformRangeSV1": (c_err, [c_vol, i32, i32, i32, i32, i32, i32, UnaryOp]),
    "vktTransformRangeSV2": (c_err, [c_vol, c_vol] + _R9 + [BinaryOp]),
    # Resample (C entry point added by this library)
    "vktResampleSV": (c_err, [c_vol, c_vol, C.c_int]),
    # volkit_hip.h runtime
    "vktHipSetDevice": (c_err, [i32]),
    "vktHipGetDevice": (c_err, [P(i32)]),
    "vktHipSetAsyncExecution": (c_err, [i32]),
    "vktHipGetAsyncExecution": (c_err, [P(i32)]),
    "vktHipSetComputeStream": (c_err, [C.c_void_p]),
    "vktHipGetComputeStream": (c_err, [P(C.c_void_p)]),
    "vktHipGetCopyStream": (c_err, [P(C.c_void_p)]),
    "vktHipSetCopyStream": (c_err, [C.c_void_p]),
    "vktHipContextCreate": (c_err, [P(C.c_void_p)]),
    "vktHipContextDestroy": (c_err, [C.c_void_p]),
    "vktHipContextMakeCurrent": (c_err, [C.c_void_p]),
    "vktHipContextSetAsyncExecution": (c_err, [C.c_void_p, i32]),
    "vktHipContextGetAsyncExecution": (c_err, [C.c_void_p, P(i32)]),
    "vktHipContextSetNumStreams": (c_err, [C.c_void_p, i32]),
    "vktHipContextGetNumStreams": (c_err, [C.c_void_p, P(i32)]),
    "vktHipContextSetStream": (c_err, [C.c_void_p, i32, C.c_void_p]),
    "vktHipContextGetStream": (c_err, [C.c_void_p, i32, P(C.c_void_p)]),
    "vktHipContextSetComputeStreamId": (c_err, [C.c_void_p, i32]),
    "vktHipContextGetComputeStreamId": (c_err, [C.c_void_p, P(i32)]),
    "vktHipContextSetCopyStreamId": (c_err, [C.c_void_p, i32]),
    "vktHipContextGetCopyStreamId": (c_err, [C.c_void_p, P(i32)]),
    "vktHipSynchronize": (c_err, []),
    "vktHipGetLastErrorString": (C.c_char_p, []),
    "vktHipSetKernelTiming": (c_err, [i32]),
    "vktHipGetLastKernelMs": (c_err, [P(f32)]),
    "vktHipKernelScopeBegin": (c_err, [C.c_char_p, P(C.c_void_p), P(C.c_void_p)]),
    "vktHipKernelScopeEnd": (c_err, [C.c_void_p]),
    "vktHipReportError": (c_err, [C.c_char_p]),
    "vktHipSetTuningKnob": (c_err, [C.c_char_p, C.c_int64]),
    "vktHipGetTuningKnob": (c_err, [C.c_char_p, C.POINTER(C.c_int64)]),
    "vktHipAllocate": (c_err, [P(C.c_void_p), C.c_size_t]),
    "vktHipFree": (c_err, [C.c_void_p]),
    "vktHipReleaseCachedMemory": (c_err, [P(C.c_size_t)]),
    "vktHipMemcpy": (c_err, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]),
    "vktHipMemsetRange": (c_err, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t]),
    "vktHipSetPinnedHostAllocation": (c_err, [i32]),
    # volkit_hip.h algorithms
    "vktHipFillRange": (c_err, [HipVolumeView_t, Vec3i_t, Vec3i_t, f32]),
    "vktHipCopyRange": (c_err, [HipVolumeView_t, HipVolumeView_t, Vec3i_t, Vec3i_t, Vec3i_t]),
    "vktHipArithmeticRange": (c_err, [C.c_int, HipVolumeView_t, HipVolumeView_t, HipVolumeView_t,
                                      Vec3i_t, Vec3i_t, Vec3i_t]),
    "vktHipResample": (c_err, [HipVolumeView_t, HipVolumeView_t, C.c_int]),
    "vktHipResampleSlab": (c_err, [HipVolumeView_t, HipVolumeView_t, C.c_int, i32, i32, i32, i32]),
    "vktHipResampleSlabSourceRange": (c_err, [i32, i32, i32, i32, C.c_int, i32, P(i32), P(i32)]),
    "vktHipSlabResamplePlan": (c_err, [i32, i32, i32, i32, C.c_int, i32, P(i32), P(i32), P(HipSlabTransfer_t),
                                       i32, P(i32)]),
    "vktHipCommGetUniqueId": (c_err, [P(HipCommId_t)]),
    "vktHipCommInitRank": (c_err, [P(c_comm), i32, HipCommId_t, i32]),
    "vktHipCommDestroy": (c_err, [c_comm]),
    "vktHipCommSetTimeout": (c_err, [c_comm, C.c_int64]),
    "vktHipCommSynchronize": (c_err, [c_comm]),
    "vktHipCommExchange": (c_err, [c_comm, i32, C.c_void_p, C.c_void_p, C.c_size_t]),
    "vktHipResampleSlabOverlapped": (c_err, [c_comm, HipVolumeView_t, HipVolumeView_t, i32, i32, i32, C.c_int, i32]),
    "vktHipResampleSlabsOverlappedLocal": (c_err, [i32, P(HipVolumeView_t), P(HipVolumeView_t), P(i32), i32, i32,
                                                   C.c_int, i32]),
    "vktHipSlabExchangeHalo": (c_err, [c_comm, HipVolumeView_t, i32, i32, i32, C.c_int, i32]),
    "vktHipSlabExchangeHaloLocal": (c_err, [i32, P(HipVolumeView_t), P(i32), i32, i32, C.c_int, i32]),
    "vktHipSlabExchangeHaloPeer": (c_err, [i32, P(HipVolumeView_t), P(i32), P(i32), i32, i32, C.c_int, i32]),
    "vktHipSlabRangePlan": (c_err, [C.c_int, i32, i32, i32, i32, i32, Vec3i_t, Vec3i_t, Vec3i_t, P(HipSlabPiece_t),
                                    i32, P(i32), P(HipSlabMove_t), i32, P(i32), P(i32)]),
    "vktHipSlabFillRange": (c_err, [c_comm, i32, P(HipSlab_t), Vec3i_t, Vec3i_t, f32]),
    "vktHipSlabCopyRange": (c_err, [c_comm, i32, P(HipSlab_t), P(HipSlab_t), Vec3i_t, Vec3i_t, Vec3i_t]),
    "vktHipSlabArithmeticRange": (c_err, [c_comm, C.c_int, i32, P(HipSlab_t), P(HipSlab_t), P(HipSlab_t), Vec3i_t,
                                          Vec3i_t, Vec3i_t]),
    "vktHipSlabTransformRange1": (c_err, [i32, i32, HipSlab_t, Vec3i_t, Vec3i_t, UnaryOp]),
    "vktHipSlabRangePieces": (c_err, [C.c_int, C.c_int, i32, i32, HipSlab_t, P(HipSlab_t), P(HipSlab_t), Vec3i_t,
                                      Vec3i_t, Vec3i_t, f32, C.c_void_p, C.c_void_p]),
    "vktHipTransformRange1": (c_err, [HipVolumeView_t, Vec3i_t, Vec3i_t, UnaryOp]),
    "vktHipTransformRange2": (c_err, [HipVolumeView_t, HipVolumeView_t, Vec3i_t, Vec3i_t, Vec3i_t, BinaryOp]),
    "vktHipSynthesize": (c_err, [HipVolumeView_t, u64]),
    "vktHipBrickDecompose": (c_err, [HipVolumeView_t, P(HipBrickRange_t), i32]),
    "vktHipBrickDecomposeGrid": (c_err, [HipVolumeView_t, HipBrickGrid_t, P(C.c_void_p)]),
    # Array3D.h (vktStructuredVolume instantiation) / Decompose.h
    "vktArray3D_vktStructuredVolume_CreateEmpty": (None, [P(c_arr)]),
    "vktArray3D_vktStructuredVolume_Create": (None, [P(c_arr), Vec3i_t]),
    "vktArray3D_vktStructuredVolume_CreateCopy": (None, [P(c_arr), c_arr]),
    "vktArray3D_vktStructuredVolume_Destroy": (None, [c_arr]),
    "vktArray3D_vktStructuredVolume_Resize": (None, [c_arr, Vec3i_t]),
    "vktArray3D_vktStructuredVolume_Fill": (None, [c_arr, c_vol]),
    "vktArray3D_vktStructuredVolume_Begin": (P(c_vol), [c_arr]),
    "vktArray3D_vktStructuredVolume_CBegin": (P(c_vol), [c_arr]),
    "vktArray3D_vktStructuredVolume_End": (P(c_vol), [c_arr]),
    "vktArray3D_vktStructuredVolume_CEnd": (P(c_vol), [c_arr]),
    "vktArray3D_vktStructuredVolume_Access": (P(c_vol), [c_arr, Vec3i_t]),
    "vktArray3D_vktStructuredVolume_CAccess": (P(c_vol), [c_arr, Vec3i_t]),
    "vktArray3D_vktStructuredVolume_Empty": (C.c_uint8, [c_arr]),
    "vktArray3D_vktStructuredVolume_Data": (P(c_vol), [c_arr]),
    "vktArray3D_vktStructuredVolume_CData": (P(c_vol), [c_arr]),
    "vktArray3D_vktStructuredVolume_Dims": (Vec3i_t, [c_arr]),
    "vktArray3D_vktStructuredVolume_NumElements": (C.c_size_t, [c_arr]),
    "vktBrickDecomposeSV": (c_err, [c_arr, c_vol] + _R9),
    # Aggregates.h / Histogram (C entry points added by this library)
    "vktComputeAggregatesSV": (c_err, [c_vol, P(Aggregates_t)]),
    "vktComputeAggregatesRangeSV": (c_err, [c_vol, P(Aggregates_t), i32, i32, i32, i32, i32, i32]),
    "vktHistogramCreate": (None, [P(c_hist), C.c_size_t]),
    "vktHistogramDestroy": (None, [c_hist]),
    "vktHistogramGetNumBins": (C.c_size_t, [c_hist]),
    "vktHistogramGetBinCounts": (C.c_void_p, [c_hist]),
    "vktComputeHistogramSV": (c_err, [c_vol, c_hist]),
    "vktComputeHistogramRangeSV": (c_err, [c_vol, c_hist, i32, i32, i32, i32, i32, i32]),
    "vktHipAggregatesRange": (c_err, [HipVolumeView_t, Vec3i_t, Vec3i_t, P(Aggregates_t)]),
    "vktHipAggregatePartialInit": (c_err, [P(HipAggregatePartial_t)]),
    "vktHipAggregateMomentsSupported": (i32, [HipVolumeView_t, Vec3i_t, Vec3i_t]),
    "vktHipAggregateMoments": (c_err, [HipVolumeView_t, Vec3i_t, Vec3i_t, i32, P(HipMomentPartial_t)]),
    "vktHipAggregatesFromMoments": (c_err, [P(HipMomentPartial_t), i32, u64, i32, i32, P(Aggregates_t), P(i32)]),
    "vktHipAggregatePartialCombine": (c_err, [P(HipAggregatePartial_t), P(HipAggregatePartial_t)]),
    "vktHipAggregatesMean": (f32, [P(HipAggregatePartial_t), u64]),
    "vktHipAggregatesPass": (c_err, [HipVolumeView_t, Vec3i_t, Vec3i_t, i32, i32, f32, P(HipAggregatePartial_t)]),
    "vktHipAggregateCodesSupported": (i32, [HipVolumeView_t, Vec3i_t, Vec3i_t]),
    "vktHipAggregateCodeCounts": (c_err, [HipVolumeView_t, Vec3i_t, Vec3i_t, C.c_void_p]),
    "vktHipAggregatesFromCodes": (c_err, [C.c_void_p, i32, f32, f32, u64, P(HipAggregatePartial_t),
                                          P(HipAggregatePartial_t), P(i32)]),
    "vktHipAggregateFirstCodes": (c_err, [HipVolumeView_t, Vec3i_t, Vec3i_t, i32, i32, i32, P(u64)]),
    "vktHipAggregatesFinish": (c_err, [P(HipAggregatePartial_t), P(HipAggregatePartial_t), u64, i32, i32,
                                       P(Aggregates_t)]),
    "vktHipHistogramRange": (c_err, [HipVolumeView_t, Vec3i_t, Vec3i_t, C.c_void_p, u64, i32]),
    # RawFile.h / InputStream.h (+ OutputStream / SV stream C entry points added here)
    "vktRawFileCreateS": (None, [P(C.c_void_p), C.c_char_p, C.c_char_p]),
    "vktRawFileCreateFD": (None, [P(C.c_void_p), C.c_void_p]),
    "vktRawFileGetBase": (C.c_void_p, [C.c_void_p]),
    "vktRawFileDestroy": (None, [C.c_void_p]),
    "vktRawFileRead": (C.c_size_t, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "vktRawFileGood": (C.c_uint8, [C.c_void_p]),
    "vktRawFileGetDims3iv": (Vec3i_t, [C.c_void_p]),
    "vktRawFileGetDataFormat": (C.c_int, [C.c_void_p]),
    "vktInputStreamCreate": (None, [P(C.c_void_p), C.c_void_p]),
    "vktInputStreamDestroy": (None, [C.c_void_p]),
    "vktInputStreamReadSV": (c_err, [C.c_void_p, c_vol]),
    "vktInputStreamReadRangeSV": (c_err, [C.c_void_p, c_vol, i32, i32, i32, i32, i32, i32]),
    "vktInputStreamSeek": (c_err, [C.c_void_p, C.c_size_t]),
    "vktOutputStreamCreate": (None, [P(C.c_void_p), C.c_void_p]),
    "vktOutputStreamDestroy": (None, [C.c_void_p]),
    "vktOutputStreamWriteSV": (c_err, [C.c_void_p, c_vol]),
    "vktOutputStreamWriteRangeSV": (c_err, [C.c_void_p, c_vol, i32, i32, i32, i32, i32, i32]),
    "vktOutputStreamSeek": (c_err, [C.c_void_p, C.c_size_t]),
    "vktOutputStreamFlush": (c_err, [C.c_void_p]),
    "vktReadSVStream": (c_err, [C.c_void_p, c_vol]),
    # LookupTable.h / Render.h (+ headless extensions)
    "vktLookupTableCreate": (None, [P(C.c_void_p), i32, i32, i32, C.c_int]),
    "vktLookupTableDestroy": (None, [C.c_void_p]),
    "vktLookupTableSetDims3i": (None, [C.c_void_p, i32, i32, i32]),
    "vktLookupTableGetDims3i": (None, [C.c_void_p, P(i32), P(i32), P(i32)]),
    "vktLookupTableSetDims3iv": (None, [C.c_void_p, Vec3i_t]),
    "vktLookupTableGetDims3iv": (Vec3i_t, [C.c_void_p]),
    "vktLookupTableSetColorFormat": (None, [C.c_void_p, C.c_int]),
    "vktLookupTableGetColorFormat": (C.c_int, [C.c_void_p]),
    "vktLookupTableSetData": (None, [C.c_void_p, C.c_void_p]),
    "vktLookupTableGetData": (C.c_void_p, [C.c_void_p]),
    "vktLookupTableGetSizeInBytes": (C.c_size_t, [C.c_void_p]),
    "vktLookupTableGetResourceHandle": (u32, [C.c_void_p]),
    "vktLookupTableMigrate": (None, [C.c_void_p]),
    "vktRenderStateDefaultInit": (None, [P(RenderState_t)]),
    "vktRenderSV": (c_err, [c_vol, RenderState_t, P(RenderState_t)]),
    "vktRenderSVToImage": (c_err, [c_vol, RenderState_t, u32, C.c_void_p]),
    "vktHipRender": (c_err, [HipVolumeView_t, P(HipRenderParams_t), C.c_void_p, C.c_void_p, i32]),
    "vktHipRenderParamsFromState": (c_err, [P(RenderState_t), Vec3fC_t, P(HipRenderParams_t)]),
    "vktWriteSVStream": (c_err, [C.c_void_p, c_vol]),
    "vktBrickDecomposeResizeSV": (c_err, [c_arr, c_vol] + _R9),
}
for _op in ARITH_OPS:
    SIGNATURES[f"vkt{_op}SV"] = (c_err, [c_vol, c_vol, c_vol])
    SIGNATURES[f"vkt{_op}RangeSV"] = (c_err, [c_vol, c_vol, c_vol] + _R9)

for _name, (_res, _args) in SIGNATURES.items():
    _fn = getattr(lib, _name)   # AttributeError here = a declared symbol is not exported
    _fn.restype = _res
    _fn.argtypes = _args


def last_error() -> str:
    return lib.vktHipGetLastErrorString().decode(errors="replace")
