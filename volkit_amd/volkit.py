"""Python API of the MI355X-native volkit StructuredVolume path.

Mirrors the names that the reference's SWIG module ``volkit`` exposes
(reference src/vkt/volkit.i:47-102; usage in src/examples/*.py): ``vkt.StructuredVolume``,
``vkt.DataFormat_UInt16``, ``vkt.Vec3i``, ``vkt.ExecutionPolicy`` with ``Device_GPU``,
``vkt.SetThreadExecutionPolicy``, ``vkt.Fill`` / ``vkt.FillRange``, ``vkt.Copy`` /
``vkt.CopyRange``, the ten arithmetic ops and their ``*Range`` forms, plus ``vkt.Resample``
and ``vkt.Transform`` (which the SWIG module leaves out).  Every call goes through the C ABI
of libvolkit.so; algorithms run as gfx950 HIP kernels under the GPU execution policy and
return ``InvalidValue`` under the CPU policy (this package is the GPU backend only).

Use as ``import volkit_amd.volkit as vkt``.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable

import numpy as np

from . import _lib
from ._lib import lib, Vec3i_t, ExecutionPolicy_t, VoxelView_t

# ---- common.hpp -----------------------------------------------------------------------------
InvalidValue, NoError, InvalidDataSource, ReadError, WriteError = -1, 0, 1, 2, 3
(DataFormat_Unspecified, DataFormat_Int8, DataFormat_Int16, DataFormat_Int32, DataFormat_UInt8,
 DataFormat_UInt16, DataFormat_UInt32, DataFormat_Float32, DataFormat_Count) = range(9)
FilterMode_Nearest, FilterMode_Linear = 0, 1
CopyKind_HostToHost, CopyKind_HostToDevice, CopyKind_DeviceToHost, CopyKind_DeviceToDevice = range(4)

BYTES_PER_VOXEL = {1: 1, 2: 2, 3: 4, 4: 1, 5: 2, 6: 4, 7: 4}
NUMPY_CODE_DTYPE = {1: np.uint8, 2: np.uint16, 3: np.uint32, 4: np.uint8, 5: np.uint16, 6: np.uint32,
                    7: np.uint32}


class Vec3i:
    """linalg.hpp Vec3i (SWIG: ``vkt.Vec3i()`` then set .x/.y/.z)."""

    __slots__ = ("x", "y", "z")

    def __init__(self, x: int = 0, y: int = 0, z: int = 0):
        self.x, self.y, self.z = int(x), int(y), int(z)

    def __iter__(self):
        return iter((self.x, self.y, self.z))

    def __eq__(self, other):
        return tuple(self) == tuple(other)

    def __repr__(self):
        return f"Vec3i({self.x}, {self.y}, {self.z})"


class Vec2f:
    __slots__ = ("x", "y")

    def __init__(self, x: float = 0.0, y: float = 0.0):
        self.x, self.y = float(x), float(y)


class ExecutionPolicy:
    """ExecutionPolicy.hpp:47-84 with SWIG's flattened nested enums."""

    Device_CPU, Device_GPU, Device_Unspecified = 0, 1, 2
    HostAPI_Serial, HostAPI_OpenMP, HostAPI_Auto = 0, 1, 2
    DeviceAPI_CUDA, DeviceAPI_Auto = 0, 1
    DeviceAPI_HIP = DeviceAPI_CUDA

    def __init__(self):
        self.device = ExecutionPolicy.Device_CPU
        self.hostApi = ExecutionPolicy.HostAPI_Serial
        self.deviceApi = ExecutionPolicy.DeviceAPI_CUDA
        self.printPerformance = 0


def SetThreadExecutionPolicy(ep: ExecutionPolicy) -> None:
    lib.vktSetThreadExecutionPolicy(
        ExecutionPolicy_t(ep.device, ep.hostApi, ep.deviceApi, 1 if ep.printPerformance else 0))


def GetThreadExecutionPolicy() -> ExecutionPolicy:
    c = lib.vktGetThreadExecutionPolicy()
    ep = ExecutionPolicy()
    ep.device, ep.hostApi, ep.deviceApi, ep.printPerformance = c.device, c.hostApi, c.deviceApi, c.printPerformance
    return ep


def _set_device(device: int) -> ExecutionPolicy:
    prev = GetThreadExecutionPolicy()
    ep = GetThreadExecutionPolicy()
    ep.device = device
    SetThreadExecutionPolicy(ep)
    return prev


def on_gpu() -> bool:
    return GetThreadExecutionPolicy().device == ExecutionPolicy.Device_GPU


# ---- StructuredVolume -----------------------------------------------------------------------
class StructuredVolume:
    """StructuredVolume.hpp:34-132 over the C handle (vktStructuredVolume)."""

    def __init__(self, dimX: int = 0, dimY: int = 0, dimZ: int = 0, dataFormat: int = DataFormat_UInt8,
                 distX: float = 1.0, distY: float = 1.0, distZ: float = 1.0,
                 mappingLo: float = 0.0, mappingHi: float = 1.0, *, _handle=None, _owner=None):
        # _owner: a container that owns the handle (bricks of an Array3D); kept alive, never destroyed here
        self._owner = _owner
        if _handle is not None:
            self._h = _handle
            return
        h = C.c_void_p()
        lib.vktStructuredVolumeCreate(C.byref(h), int(dimX), int(dimY), int(dimZ), int(dataFormat),
                                      distX, distY, distZ, mappingLo, mappingHi)
        self._h = h

    @classmethod
    def CreateCopy(cls, other: "StructuredVolume") -> "StructuredVolume":
        h = C.c_void_p()
        lib.vktStructuredVolumeCreateCopy(C.byref(h), other._h)
        return cls(_handle=h)

    def __del__(self, lib=lib):   # bound now: module globals are gone at interpreter exit
        h = getattr(self, "_h", None)
        if h is not None and h.value and getattr(self, "_owner", None) is None:
            lib.vktStructuredVolumeDestroy(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    # dims / format / dist / mapping
    def setDims(self, x, y=None, z=None):
        if y is None:
            x, y, z = x
        lib.vktStructuredVolumeSetDims3i(self._h, int(x), int(y), int(z))

    def getDims(self) -> Vec3i:
        d = lib.vktStructuredVolumeGetDims3iv(self._h)
        return Vec3i(d.x, d.y, d.z)

    def setDataFormat(self, fmt: int):
        lib.vktStructuredVolumeSetDataFormat(self._h, int(fmt))

    def getDataFormat(self) -> int:
        return lib.vktStructuredVolumeGetDataFormat(self._h)

    def setDist(self, x, y, z):
        lib.vktStructuredVolumeSetDist3f(self._h, x, y, z)

    def getDist(self):
        d = lib.vktStructuredVolumeGetDist3fv(self._h)
        return (d.x, d.y, d.z)

    def setVoxelMapping(self, lo, hi=None):
        if hi is None:
            lo, hi = lo.x, lo.y
        lib.vktStructuredVolumeSetVoxelMapping2f(self._h, lo, hi)

    def getVoxelMapping(self) -> Vec2f:
        m = lib.vktStructuredVolumeGetVoxelMapping2fv(self._h)
        return Vec2f(m.x, m.y)

    def getDomainBounds(self):
        b = lib.vktStructuredVolumeGetDomainBounds(self._h)
        return ((b.min.x, b.min.y, b.min.z), (b.max.x, b.max.y, b.max.z))

    def getObjectBounds(self):
        b = lib.vktStructuredVolumeGetObjectBounds(self._h)
        return ((b.min.x, b.min.y, b.min.z), (b.max.x, b.max.y, b.max.z))

    def getData(self) -> int:
        """Raw pointer (int) in the address space of the thread's device; migrates first."""
        return lib.vktStructuredVolumeGetData(self._h) or 0

    def migrate(self):
        lib.vktStructuredVolumeMigrate(self._h)

    def migrateChecked(self):
        """migrate() with its outcome (extension): InvalidValue when the bytes could not be moved
        to the thread's device -- they then stay where they were, intact."""
        return lib.vktStructuredVolumeMigrateChecked(self._h)

    def setValue(self, x, y, z, value):
        lib.vktStructuredVolumeSetValue(self._h, int(x), int(y), int(z), float(value))

    def getValue(self, x, y, z) -> float:
        v = C.c_float(0.0)
        lib.vktStructuredVolumeGetValue(self._h, int(x), int(y), int(z), C.byref(v))
        return v.value

    def setBytes(self, x, y, z, data: bytes):
        buf = (C.c_uint8 * 8)(*bytes(data)[:8])
        lib.vktStructuredVolumeSetBytes(self._h, int(x), int(y), int(z), buf)

    def getBytes(self, x, y, z) -> bytes:
        buf = (C.c_uint8 * 8)()
        lib.vktStructuredVolumeGetBytes(self._h, int(x), int(y), int(z), buf)
        return bytes(buf[: self.getBytesPerVoxel()])

    def getBytesPerVoxel(self) -> int:
        return BYTES_PER_VOXEL.get(self.getDataFormat(), 255)

    def getSizeInBytes(self) -> int:
        return lib.vktStructuredVolumeGetSizeInBytes(self._h)

    def getResourceHandle(self) -> int:
        return lib.vktStructuredVolumeGetResourceHandle(self._h)

    @staticmethod
    def GetMaxBytesPerVoxel() -> int:
        return lib.vktStructuredVolumeGetMaxBytesPerVoxel()

    # ---- numpy helpers (not in the reference; host <-> wherever the volume lives) --------
    def to_numpy(self) -> np.ndarray:
        """Copy the stored codes out as a (z, y, x) array of uint8/uint16/uint32."""
        d = self.getDims()
        fmt = self.getDataFormat()
        out = np.empty((d.z, d.y, d.x), dtype=NUMPY_CODE_DTYPE[fmt])
        n = out.nbytes
        if n == 0:
            return out
        ptr = self.getData()
        if on_gpu():
            err = lib.vktHipMemcpy(out.ctypes.data, ptr, n, CopyKind_DeviceToHost)
            if err != NoError:
                raise RuntimeError(_lib.last_error())
        else:
            C.memmove(out.ctypes.data, ptr, n)
        return out

    def from_numpy(self, codes: np.ndarray) -> None:
        """Store raw codes (any array with getSizeInBytes() bytes) into the volume."""
        arr = np.ascontiguousarray(codes)
        n = self.getSizeInBytes()
        if arr.nbytes != n:
            raise ValueError(f"expected {n} bytes, got {arr.nbytes}")
        if n == 0:
            return
        ptr = self.getData()
        if on_gpu():
            err = lib.vktHipMemcpy(ptr, arr.ctypes.data, n, CopyKind_HostToDevice)
            if err != NoError:
                raise RuntimeError(_lib.last_error())
        else:
            C.memmove(ptr, arr.ctypes.data, n)

    def hip_view(self) -> _lib.HipVolumeView_t:
        """Backend view (include/volkit_hip.h) of the volume in its current address space."""
        d = self.getDims()
        m = self.getVoxelMapping()
        return _lib.HipVolumeView_t(self.getData(), d.x, d.y, d.z, self.getDataFormat(), m.x, m.y)


# ---- Voxel.hpp ------------------------------------------------------------------------------
def MapVoxel(value: float, dataFormat: int, mappingLo: float = 0.0, mappingHi: float = 1.0) -> bytes:
    buf = (C.c_uint8 * 8)()
    lib.vktMapVoxel(buf, value, int(dataFormat), mappingLo, mappingHi)
    return bytes(buf[: BYTES_PER_VOXEL.get(dataFormat, 0)])


def UnmapVoxel(data: bytes, dataFormat: int, mappingLo: float = 0.0, mappingHi: float = 1.0) -> float:
    buf = (C.c_uint8 * 8)(*bytes(data)[:8])
    v = C.c_float(0.0)
    lib.vktUnmapVoxel(C.byref(v), buf, int(dataFormat), mappingLo, mappingHi)
    return v.value


# ---- argument helpers ---------------------------------------------------------------------
def _ints(args, n):
    """Accept either n ints or n//3 Vec3i-likes."""
    flat = []
    for a in args:
        if isinstance(a, (Vec3i, tuple, list)):
            flat.extend(int(v) for v in a)
        else:
            flat.append(int(a))
    if len(flat) != n:
        raise TypeError(f"expected {n} coordinates, got {len(flat)}")
    return flat


# ---- Fill.hpp / Copy.hpp ----------------------------------------------------------------------
def Fill(volume: StructuredVolume, value: float) -> int:
    return lib.vktFillSV(volume.handle, float(value))


def FillRange(volume: StructuredVolume, *args) -> int:
    *coords, value = args
    f = _ints(coords, 6)
    return lib.vktFillRangeSV(volume.handle, *f, float(value))


def Copy(dst: StructuredVolume, src: StructuredVolume) -> int:
    return lib.vktCopySV(dst.handle, src.handle)


def CopyRange(dst: StructuredVolume, src: StructuredVolume, *coords) -> int:
    f = [int(v) for v in _flatlen(coords)]
    if len(f) == 6:
        f += [0, 0, 0]
    if len(f) != 9:
        raise TypeError("CopyRange expects first, last[, dstOffset]")
    return lib.vktCopyRangeSV(dst.handle, src.handle, *f)


def _flatlen(coords):
    out = []
    for a in coords:
        if isinstance(a, (Vec3i, tuple, list)):
            out.extend(a)
        else:
            out.append(a)
    return out


# ---- Arithmetic.hpp -----------------------------------------------------------------------
def _make_arith(name):
    whole = getattr(lib, f"vkt{name}SV")
    ranged = getattr(lib, f"vkt{name}RangeSV")

    def op(dest, source1, source2):
        return whole(dest.handle, source1.handle, source2.handle)

    def op_range(dest, source1, source2, *coords):
        f = [int(v) for v in _flatlen(coords)]
        if len(f) == 6:
            f += [0, 0, 0]
        if len(f) != 9:
            raise TypeError(f"{name}Range expects first, last[, dstOffset]")
        return ranged(dest.handle, source1.handle, source2.handle, *f)

    op.__name__, op_range.__name__ = name, f"{name}Range"
    op.__doc__ = f"vkt::{name} (reference include/cpp/vkt/Arithmetic.hpp)"
    op_range.__doc__ = f"vkt::{name}Range: dest[x + dstOffset] = f(source1[x], source2[x]) for x in [first, last)"
    return op, op_range


for _name in _lib.ARITH_OPS:
    globals()[_name], globals()[f"{_name}Range"] = _make_arith(_name)


# ---- Resample.hpp -------------------------------------------------------------------------
def Resample(dst: StructuredVolume, src: StructuredVolume, fm: int = FilterMode_Nearest) -> int:
    return lib.vktResampleSV(dst.handle, src.handle, int(fm))


# ---- Transform.hpp ------------------------------------------------------------------------
class VoxelView:
    """Transform callbacks receive (x, y, z, VoxelView); .bytes is a mutable 8-byte buffer."""

    __slots__ = ("bytes", "dataFormat", "mappingLo", "mappingHi")

    def __init__(self, c: VoxelView_t):
        self.bytes = C.cast(c.bytes, C.POINTER(C.c_uint8 * 8)).contents
        self.dataFormat, self.mappingLo, self.mappingHi = c.dataFormat, c.mappingLo, c.mappingHi


def Transform(volume1: StructuredVolume, a, b=None) -> int:
    if b is None:
        fn: Callable = a
        cb = _lib.UnaryOp(lambda x, y, z, v: fn(x, y, z, VoxelView(v)))
        return lib.vktTransformSV1(volume1.handle, cb)
    volume2, fn = a, b
    cb = _lib.BinaryOp(lambda x, y, z, v1, v2: fn(x, y, z, VoxelView(v1), VoxelView(v2)))
    return lib.vktTransformSV2(volume1.handle, volume2.handle, cb)


def TransformRange(volume1: StructuredVolume, *args) -> int:
    fn = args[-1]
    rest = list(args[:-1])
    if rest and isinstance(rest[0], StructuredVolume):
        volume2 = rest.pop(0)
        f = [int(v) for v in _flatlen(rest)]
        if len(f) == 6:
            f += [0, 0, 0]
        cb = _lib.BinaryOp(lambda x, y, z, v1, v2: fn(x, y, z, VoxelView(v1), VoxelView(v2)))
        return lib.vktTransformRangeSV2(volume1.handle, volume2.handle, *f, cb)
    f = [int(v) for v in _flatlen(rest)]
    cb = _lib.UnaryOp(lambda x, y, z, v: fn(x, y, z, VoxelView(v)))
    return lib.vktTransformRangeSV1(volume1.handle, *f, cb)


# ---- Array3D.hpp / Decompose.hpp --------------------------------------------------------------
class Array3D_StructuredVolume:
    """SWIG's ``vkt.Array3D_StructuredVolume`` (reference src/vkt/volkit.i:88-100) over the C
    array of volume handles.  ``decomp[vkt.Vec3i(x, y, z)]`` returns the brick; the array owns
    the bricks that BrickDecomposeResize created."""

    def __init__(self, dims=None):
        h = C.c_void_p()
        if dims is None:
            lib.vktArray3D_vktStructuredVolume_CreateEmpty(C.byref(h))
        else:
            lib.vktArray3D_vktStructuredVolume_Create(C.byref(h), Vec3i_t(*_ints([dims], 3)))
        self._h = h

    def __del__(self, lib=lib):   # bound now: module globals are gone at interpreter exit
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.vktArray3D_vktStructuredVolume_Destroy(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def dims(self) -> Vec3i:
        d = lib.vktArray3D_vktStructuredVolume_Dims(self._h)
        return Vec3i(d.x, d.y, d.z)

    def numElements(self) -> int:
        return lib.vktArray3D_vktStructuredVolume_NumElements(self._h)

    def empty(self) -> bool:
        return bool(lib.vktArray3D_vktStructuredVolume_Empty(self._h))

    def __len__(self):
        return self.numElements()

    def __getitem__(self, index) -> StructuredVolume:
        x, y, z = _ints([index], 3)
        d = self.dims()
        if not (0 <= x < d.x and 0 <= y < d.y and 0 <= z < d.z):
            raise IndexError(f"brick index {(x, y, z)} outside {tuple(d)}")
        slot = lib.vktArray3D_vktStructuredVolume_Access(self._h, Vec3i_t(x, y, z))
        h = slot[0]
        if not h:
            raise IndexError("unallocated brick (call BrickDecomposeResize first)")
        return StructuredVolume(_handle=C.c_void_p(h), _owner=self)   # borrowed: the array owns it


def _decompose_args(fn, args):
    f = [int(v) for v in _flatlen(args)]
    if len(f) == 3:
        f += [0] * 6
    elif len(f) == 6:
        f += [0] * 3
    if len(f) != 9:
        raise TypeError(f"{fn} expects brickSize[, haloSizeNeg[, haloSizePos]]")
    return f


def BrickDecompose(decomp: Array3D_StructuredVolume, volume: StructuredVolume, *args) -> int:
    """vkt::BrickDecompose: one CopyRange per brick (with halos), one gfx950 launch."""
    return lib.vktBrickDecomposeSV(decomp.handle, volume.handle, *_decompose_args("BrickDecompose", args))


def BrickDecomposeResize(decomp: Array3D_StructuredVolume, volume: StructuredVolume, *args) -> int:
    return lib.vktBrickDecomposeResizeSV(decomp.handle, volume.handle,
                                         *_decompose_args("BrickDecomposeResize", args))


# ---- Aggregates.hpp / Histogram.hpp ---------------------------------------------------------
class Aggregates:
    """SWIG's ``vkt.Aggregates()`` (reference include/cpp/vkt/Aggregates.hpp:14-25)."""

    __slots__ = ("min", "max", "mean", "stddev", "var", "sum", "prod", "argmin", "argmax")

    def __init__(self):
        self.min = self.max = self.mean = self.stddev = self.var = self.sum = self.prod = 0.0
        self.argmin, self.argmax = Vec3i(), Vec3i()

    def _set(self, c: "_lib.Aggregates_t"):
        self.min, self.max, self.mean, self.stddev = c.min, c.max, c.mean, c.stddev
        self.var, self.sum, self.prod = c.var, c.sum, c.prod
        self.argmin = Vec3i(c.argmin.x, c.argmin.y, c.argmin.z)
        self.argmax = Vec3i(c.argmax.x, c.argmax.y, c.argmax.z)


def ComputeAggregates(volume: StructuredVolume, aggregates: Aggregates) -> int:
    c = _lib.Aggregates_t()
    err = lib.vktComputeAggregatesSV(volume.handle, C.byref(c))
    if err == NoError:
        aggregates._set(c)
    return err


def ComputeAggregatesRange(volume: StructuredVolume, aggregates: Aggregates, *coords) -> int:
    f = _ints(coords, 6)
    c = _lib.Aggregates_t()
    err = lib.vktComputeAggregatesRangeSV(volume.handle, C.byref(c), *f)
    if err == NoError:
        aggregates._set(c)
    return err


class Histogram:
    """vkt::Histogram (reference include/cpp/vkt/Histogram.hpp:14-25): numBins size_t counters
    in a ManagedBuffer (migrated with the thread policy)."""

    def __init__(self, numBins: int):
        h = C.c_void_p()
        lib.vktHistogramCreate(C.byref(h), int(numBins))
        self._h = h

    def __del__(self, lib=lib):   # bound now: module globals are gone at interpreter exit
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.vktHistogramDestroy(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def getNumBins(self) -> int:
        return lib.vktHistogramGetNumBins(self._h)

    def getBinCounts(self) -> np.ndarray:
        """Copy of the bin counts (uint64), read from wherever the policy puts them."""
        n = self.getNumBins()
        out = np.zeros(n, dtype=np.uint64)
        if n == 0:
            return out
        ptr = lib.vktHistogramGetBinCounts(self._h)
        if on_gpu():
            if lib.vktHipMemcpy(out.ctypes.data, ptr, out.nbytes, CopyKind_DeviceToHost) != NoError:
                raise RuntimeError(_lib.last_error())
        else:
            C.memmove(out.ctypes.data, ptr, out.nbytes)
        return out


def ComputeHistogram(volume: StructuredVolume, histogram: Histogram) -> int:
    return lib.vktComputeHistogramSV(volume.handle, histogram.handle)


def ComputeHistogramRange(volume: StructuredVolume, histogram: Histogram, *coords) -> int:
    return lib.vktComputeHistogramRangeSV(volume.handle, histogram.handle, *_ints(coords, 6))


# ---- RawFile.hpp / InputStream.hpp / OutputStream.hpp ------------------------------------------
class RawFile:
    """SWIG's ``vkt.RawFile(fileName, mode)`` (reference include/cpp/vkt/RawFile.hpp:15-60):
    dims and format parsed from names like ``foo_256x256x128_uint16.raw``."""

    def __init__(self, fileName: str, mode: str):
        h = C.c_void_p()
        self._name = fileName.encode()   # the C++ object keeps the pointer
        lib.vktRawFileCreateS(C.byref(h), self._name, mode.encode())
        self._h = h

    def __del__(self, lib=lib):   # bound now: module globals are gone at interpreter exit
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.vktRawFileDestroy(h)
            self._h = None

    def close(self):
        self.__del__()

    def base(self):
        return lib.vktRawFileGetBase(self._h)

    def good(self) -> bool:
        return bool(lib.vktRawFileGood(self._h))

    def getDims(self) -> Vec3i:
        d = lib.vktRawFileGetDims3iv(self._h)
        return Vec3i(d.x, d.y, d.z)

    def getDataFormat(self) -> int:
        return lib.vktRawFileGetDataFormat(self._h)

    def read(self, n: int) -> bytes:
        buf = (C.c_char * n)()
        got = lib.vktRawFileRead(self._h, buf, n)
        return bytes(buf[:got])


class InputStream:
    """``vkt.InputStream(file)``; ``read(volume)`` streams straight into HBM under the GPU
    policy (pinned double buffers on the copy stream)."""

    def __init__(self, source: RawFile):
        h = C.c_void_p()
        lib.vktInputStreamCreate(C.byref(h), source.base())
        self._h, self._source = h, source

    def __del__(self, lib=lib):   # bound now: module globals are gone at interpreter exit
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.vktInputStreamDestroy(h)
            self._h = None

    def read(self, volume: StructuredVolume) -> int:
        return lib.vktInputStreamReadSV(self._h, volume.handle)

    def readRange(self, volume: StructuredVolume, *coords) -> int:
        return lib.vktInputStreamReadRangeSV(self._h, volume.handle, *_ints(coords, 6))

    def seek(self, pos: int) -> int:
        return lib.vktInputStreamSeek(self._h, int(pos))


class OutputStream:
    def __init__(self, source: RawFile):
        h = C.c_void_p()
        lib.vktOutputStreamCreate(C.byref(h), source.base())
        self._h, self._source = h, source

    def __del__(self, lib=lib):   # bound now: module globals are gone at interpreter exit
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.vktOutputStreamDestroy(h)
            self._h = None

    def write(self, volume: StructuredVolume) -> int:
        return lib.vktOutputStreamWriteSV(self._h, volume.handle)

    def writeRange(self, volume: StructuredVolume, *coords) -> int:
        return lib.vktOutputStreamWriteRangeSV(self._h, volume.handle, *_ints(coords, 6))

    def seek(self, pos: int) -> int:
        return lib.vktOutputStreamSeek(self._h, int(pos))

    def flush(self) -> int:
        return lib.vktOutputStreamFlush(self._h)


def ReadSVStream(source: RawFile, volume: StructuredVolume) -> int:
    """The reference CLI's StructuredVolume stream (src/cli/main.cpp:32-69)."""
    return lib.vktReadSVStream(source.base(), volume.handle)


def WriteSVStream(source: RawFile, volume: StructuredVolume) -> int:
    return lib.vktWriteSVStream(source.base(), volume.handle)


# ---- LookupTable.hpp / Render.hpp ----------------------------------------------------------------
(ColorFormat_Unspecified, ColorFormat_R8, ColorFormat_RG8, ColorFormat_RGB8, ColorFormat_RGBA8, ColorFormat_R16UI,
 ColorFormat_RG16UI, ColorFormat_RGB16UI, ColorFormat_RGBA16UI, ColorFormat_R32UI, ColorFormat_RG32UI,
 ColorFormat_RGB32UI, ColorFormat_RGBA32UI, ColorFormat_R32F, ColorFormat_RG32F, ColorFormat_RGB32F,
 ColorFormat_RGBA32F) = range(17)
RenderAlgo_RayMarching, RenderAlgo_ImplicitIso, RenderAlgo_MultiScattering = 0, 1, 2


class LookupTable:
    """``vkt.LookupTable(5, 1, 1, vkt.ColorFormat_RGBA32F)`` with ``setData`` (reference
    include/cpp/vkt/LookupTable.hpp; src/examples/Histogram.cpp:48-56)."""

    def __init__(self, dimX: int, dimY: int, dimZ: int, colorFormat: int):
        h = C.c_void_p()
        lib.vktLookupTableCreate(C.byref(h), int(dimX), int(dimY), int(dimZ), int(colorFormat))
        self._h = h

    def __del__(self, lib=lib):   # bound now: module globals are gone at interpreter exit
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.vktLookupTableDestroy(h)
            self._h = None

    def setData(self, data) -> None:
        arr = np.ascontiguousarray(np.asarray(data, dtype=np.float32))
        if arr.nbytes != self.getSizeInBytes():
            raise ValueError(f"expected {self.getSizeInBytes()} bytes, got {arr.nbytes}")
        lib.vktLookupTableSetData(self._h, arr.ctypes.data)

    def getDims(self) -> Vec3i:
        d = lib.vktLookupTableGetDims3iv(self._h)
        return Vec3i(d.x, d.y, d.z)

    def getSizeInBytes(self) -> int:
        return lib.vktLookupTableGetSizeInBytes(self._h)

    def getResourceHandle(self) -> int:
        return lib.vktLookupTableGetResourceHandle(self._h)


class RenderState:
    """``vkt.RenderState()`` with the reference's fields and defaults (Render.hpp:23-130)."""

    def __init__(self):
        self._c = _lib.RenderState_t()
        lib.vktRenderStateDefaultInit(C.byref(self._c))
        self._keep = []

    def __getattr__(self, name):
        c = self.__dict__.get("_c")
        if c is not None and name in dict(c._fields_):
            return getattr(c, name)
        raise AttributeError(name)

    def __setattr__(self, name, value):
        if name.startswith("_"):
            object.__setattr__(self, name, value)
        elif name in dict(_lib.RenderState_t._fields_):
            setattr(self._c, name, value)
        else:
            raise AttributeError(name)

    def setSnapshot(self, fileName: str, message: str = "") -> None:
        b, m = fileName.encode(), message.encode()
        self._keep = [b, m]
        self._c.snapshotTool.enabled = 1
        self._c.snapshotTool.fileName = b
        self._c.snapshotTool.message = m


def Render(volume: StructuredVolume, renderState: RenderState = None, newRenderState: RenderState = None) -> int:
    """Headless render (VKT_RENDER_FRAMES frames), snapshot written if requested."""
    rs = renderState or RenderState()
    out = newRenderState._c if newRenderState is not None else None
    return lib.vktRenderSV(volume.handle, rs._c, C.byref(out) if out is not None else None)


def RenderToImage(volume: StructuredVolume, renderState: RenderState, numFrames: int) -> np.ndarray:
    """Extension: (height, width, 4) float32 image, row 0 = bottom, after numFrames frames."""
    img = np.zeros((renderState.viewportHeight, renderState.viewportWidth, 4), dtype=np.float32)
    err = lib.vktRenderSVToImage(volume.handle, renderState._c, int(numFrames), img.ctypes.data)
    if err != NoError:
        raise RuntimeError(_lib.last_error())
    return img


# ---- backend utilities (include/volkit_hip.h) ----------------------------------------------
def Synthesize(volume: StructuredVolume, seed: int) -> int:
    """Fill a GPU-resident volume with the counter-based synthetic codes (see volkit_hip.h)."""
    return lib.vktHipSynthesize(volume.hip_view(), C.c_uint64(seed))


def Synchronize() -> int:
    return lib.vktHipSynchronize()


def compute_stream() -> int:
    p = C.c_void_p()
    lib.vktHipGetComputeStream(C.byref(p))
    return p.value or 0


def last_error() -> str:
    return _lib.last_error()
