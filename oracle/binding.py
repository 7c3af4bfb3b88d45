"""TEST INFRASTRUCTURE ONLY -- numpy/ctypes binding of oracle/liboracle.so, the CPU
restatement of the reference serial path (oracle/vkt_oracle.c).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, always as
the checker / CPU baseline, never as the thing measured or shipped.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")

CODE_DTYPE = {1: np.uint8, 2: np.uint16, 3: np.uint32, 4: np.uint8, 5: np.uint16, 6: np.uint32, 7: np.uint32}
BPV = {1: 1, 2: 2, 3: 4, 4: 1, 5: 2, 6: 4, 7: 4}


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


if not os.path.exists(LIB_PATH):
    build()

_lib = C.CDLL(LIB_PATH)
_i3 = C.c_int32 * 3


class _Vol(C.Structure):
    _fields_ = [("data", C.POINTER(C.c_uint8)), ("dims", C.c_int32 * 3), ("fmt", C.c_int32),
                ("lo", C.c_float), ("hi", C.c_float), ("nbytes", C.c_size_t)]


_lib.vko_map.argtypes = [C.POINTER(C.c_uint8), C.c_float, C.c_int32, C.c_float, C.c_float]
_lib.vko_unmap.argtypes = [C.POINTER(C.c_float), C.POINTER(C.c_uint8), C.c_int32, C.c_float, C.c_float]
_lib.vko_fill_range.argtypes = [C.POINTER(_Vol), _i3, _i3, C.c_float]
_lib.vko_copy_range.argtypes = [C.POINTER(_Vol), C.POINTER(_Vol), _i3, _i3, _i3]
_lib.vko_arith_range.argtypes = [C.c_int32, C.POINTER(_Vol), C.POINTER(_Vol), C.POINTER(_Vol), _i3, _i3, _i3]
_lib.vko_resample.argtypes = [C.POINTER(_Vol), C.POINTER(_Vol), C.c_int32]
_lib.vko_resample_slab.argtypes = [C.POINTER(_Vol), C.POINTER(_Vol), C.c_int32, C.c_int32, C.c_int32,
                                   C.c_int32, C.c_int32]
_lib.vko_splitmix64.restype = C.c_uint64
_lib.vko_splitmix64.argtypes = [C.c_uint64]
_lib.vko_synth.argtypes = [C.POINTER(C.c_uint8), C.c_size_t, C.c_uint64]

class Aggregates(C.Structure):
    _fields_ = [("min", C.c_float), ("max", C.c_float), ("mean", C.c_float), ("stddev", C.c_float),
                ("var", C.c_float), ("sum", C.c_float), ("prod", C.c_float), ("argmin", C.c_int32 * 3),
                ("argmax", C.c_int32 * 3)]


_lib.vko_aggregates_range.argtypes = [C.POINTER(_Vol), _i3, _i3, C.POINTER(Aggregates)]
_lib.vko_histogram_range.restype = C.c_uint64
_lib.vko_histogram_range.argtypes = [C.POINTER(_Vol), _i3, _i3, C.POINTER(C.c_uint64), C.c_uint64]

UNARY = C.CFUNCTYPE(None, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_uint8), C.c_int32, C.c_float, C.c_float)
BINARY = C.CFUNCTYPE(None, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_uint8), C.c_int32, C.c_float, C.c_float,
                     C.POINTER(C.c_uint8), C.c_int32, C.c_float, C.c_float)
_lib.vko_transform_range1.argtypes = [C.POINTER(_Vol), _i3, _i3, UNARY]
_lib.vko_transform_range2.argtypes = [C.POINTER(_Vol), C.POINTER(_Vol), _i3, _i3, _i3, BINARY]

OPS = ["Sum", "Diff", "Prod", "Quot", "AbsDiff", "SafeSum", "SafeDiff", "SafeProd", "SafeQuot", "SafeAbsDiff"]


class Volume:
    """A host volume: `codes` is a (z, y, x) array of raw stored codes."""

    def __init__(self, codes: np.ndarray, fmt: int, lo: float = 0.0, hi: float = 1.0):
        self.fmt = int(fmt)
        self.codes = np.ascontiguousarray(codes, dtype=CODE_DTYPE[self.fmt])
        self.lo, self.hi = float(lo), float(hi)
        z, y, x = self.codes.shape
        self._s = _Vol(self.codes.ctypes.data_as(C.POINTER(C.c_uint8)), _i3(x, y, z), self.fmt, self.lo, self.hi,
                       self.codes.nbytes)

    @classmethod
    def zeros(cls, dims, fmt, lo=0.0, hi=1.0, fill_byte=0):
        x, y, z = dims
        codes = np.empty((z, y, x), dtype=CODE_DTYPE[fmt])
        codes.view(np.uint8)[...] = fill_byte
        return cls(codes, fmt, lo, hi)

    @property
    def dims(self):
        z, y, x = self.codes.shape
        return (x, y, z)

    @property
    def ref(self):
        return C.byref(self._s)


def map_voxel(value: float, fmt: int, lo: float = 0.0, hi: float = 1.0) -> bytes:
    buf = (C.c_uint8 * 8)()
    _lib.vko_map(buf, value, fmt, lo, hi)
    return bytes(buf[: BPV.get(fmt, 0)])


def unmap_voxel(data: bytes, fmt: int, lo: float = 0.0, hi: float = 1.0) -> float:
    buf = (C.c_uint8 * 8)(*bytes(data)[:8])
    v = C.c_float(0.0)
    _lib.vko_unmap(C.byref(v), buf, fmt, lo, hi)
    return v.value


def fill_range(v: Volume, first, last, value: float) -> None:
    _lib.vko_fill_range(v.ref, _i3(*first), _i3(*last), value)


def copy_range(dst: Volume, src: Volume, first, last, off=(0, 0, 0)) -> None:
    _lib.vko_copy_range(dst.ref, src.ref, _i3(*first), _i3(*last), _i3(*off))


def arith_range(op, dst: Volume, s1: Volume, s2: Volume, first, last, off=(0, 0, 0)) -> None:
    code = OPS.index(op) if isinstance(op, str) else int(op)
    _lib.vko_arith_range(code, dst.ref, s1.ref, s2.ref, _i3(*first), _i3(*last), _i3(*off))


def resample(dst: Volume, src: Volume, filter_mode: int) -> None:
    _lib.vko_resample(dst.ref, src.ref, filter_mode)


def resample_slab(dst: Volume, src: Volume, filter_mode: int, dst_gdz: int, dst_z0: int, src_gdz: int,
                  src_z0: int) -> None:
    _lib.vko_resample_slab(dst.ref, src.ref, filter_mode, dst_gdz, dst_z0, src_gdz, src_z0)


def transform_range1(v: Volume, first, last, fn) -> None:
    cb = UNARY(lambda x, y, z, b, f, lo, hi: fn(x, y, z, b, f, lo, hi))
    _lib.vko_transform_range1(v.ref, _i3(*first), _i3(*last), cb)


def transform_range2(v1: Volume, v2: Volume, first, last, off, fn) -> None:
    cb = BINARY(lambda x, y, z, b1, f1, lo1, hi1, b2, f2, lo2, hi2: fn(x, y, z, b1, b2))
    _lib.vko_transform_range2(v1.ref, v2.ref, _i3(*first), _i3(*last), _i3(*off), cb)


def synth(nbytes: int, seed: int) -> np.ndarray:
    """Same bytes as vktHipSynthesize: byte i = byte i%8 of splitmix64(seed + i//8)."""
    out = np.empty(nbytes, dtype=np.uint8)
    if nbytes:
        _lib.vko_synth(out.ctypes.data_as(C.POINTER(C.c_uint8)), nbytes, C.c_uint64(seed))
    return out


def synth_codes(dims, fmt, seed) -> np.ndarray:
    x, y, z = dims
    b = synth(x * y * z * BPV[fmt], seed)
    return b.view(CODE_DTYPE[fmt]).reshape(z, y, x)


# ---- BrickDecompose (reference src/vkt/Decompose.cpp:96-150 + Decompose_serial.hpp:15-46) ----
def _div_up(a, b):
    return (a + b - 1) // b


def brick_layout(dims, brick, neg=(0, 0, 0), pos=(0, 0, 0)):
    """BrickDecomposeResize (Decompose.cpp:103-147): {(x, y, z): brick dims incl. halos}."""
    nb = [_div_up(d, b) for d, b in zip(dims, brick)]
    ext = [n * b for n, b in zip(nb, brick)]
    border = [b if d % b == 0 else b - e + d for d, b, e in zip(dims, brick, ext)]
    out = {}
    for z in range(nb[2]):
        for y in range(nb[1]):
            for x in range(nb[0]):
                idx = (x, y, z)
                size = [brick[a] if idx[a] < nb[a] - 1 else border[a] for a in range(3)]
                out[idx] = tuple(neg[a] + size[a] + pos[a] for a in range(3))
    return tuple(nb), out


def brick_ranges(dims, num_bricks, brick, neg=(0, 0, 0), pos=(0, 0, 0)):
    """Decompose_serial.hpp:24-44: {(x, y, z): (first, last)} of each brick's CopyRange."""
    out = {}
    for z in range(num_bricks[2]):
        for y in range(num_bricks[1]):
            for x in range(num_bricks[0]):
                first = [x * brick[0], y * brick[1], z * brick[2]]
                last = [min(first[a] + brick[a], dims[a]) for a in range(3)]
                out[(x, y, z)] = (tuple(first[a] - neg[a] for a in range(3)),
                                  tuple(last[a] + pos[a] for a in range(3)))
    return out


def brick_decompose(src: Volume, brick, neg=(0, 0, 0), pos=(0, 0, 0), init_byte=0):
    """BrickDecomposeResize + BrickDecompose on the oracle: {(x, y, z): Volume}."""
    nb, layout = brick_layout(src.dims, brick, neg, pos)
    ranges = brick_ranges(src.dims, nb, brick, neg, pos)
    out = {}
    for idx, bdims in layout.items():
        v = Volume.zeros(bdims, src.fmt, src.lo, src.hi, fill_byte=init_byte)
        first, last = ranges[idx]
        copy_range(v, src, first, last)
        out[idx] = v
    return out


# ---- reductions (reference Aggregates_serial.hpp:20-83, Histogram_serial.hpp:20-50) ----------
def aggregates_range(v: Volume, first, last) -> Aggregates:
    out = Aggregates()
    _lib.vko_aggregates_range(v.ref, _i3(*first), _i3(*last), C.byref(out))
    return out


def histogram_range(v: Volume, first, last, num_bins: int):
    """-> (bins as uint64 array, number of voxels the reference would count out of bounds)"""
    bins = np.zeros(max(num_bins, 1), dtype=np.uint64)
    skipped = _lib.vko_histogram_range(v.ref, _i3(*first), _i3(*last),
                                       bins.ctypes.data_as(C.POINTER(C.c_uint64)), num_bins)
    return bins[:num_bins], int(skipped)


# ---- renderers (reference src/vkt/Render_kernel.hpp:80-418) ----------------------------------
class RenderParams(C.Structure):
    """Same layout as vktHipRenderParams_t / vko_render_params."""
    _fields_ = [("algo", C.c_int32), ("width", C.c_int32), ("height", C.c_int32), ("frameBegin", C.c_uint32),
                ("eye", C.c_float * 3), ("U", C.c_float * 3), ("V", C.c_float * 3), ("W", C.c_float * 3),
                ("right", C.c_float * 3), ("up", C.c_float * 3), ("lensRadius", C.c_float),
                ("focalDistance", C.c_float), ("bbox", C.c_float * 3), ("dtRayMarching", C.c_float),
                ("dtImplicitIso", C.c_float), ("majorant", C.c_float), ("numIsoSurfaces", C.c_int32),
                ("isoSurfaces", C.c_float * 10), ("sRGB", C.c_int32), ("lut", C.c_void_p), ("lutSize", C.c_int32)]


_lib.vko_render.argtypes = [C.POINTER(_Vol), C.POINTER(RenderParams), C.c_void_p, C.c_void_p, C.c_int32]
_lib.vko_render_window.argtypes = [C.POINTER(_Vol), C.POINTER(RenderParams), C.c_void_p, C.c_void_p, C.c_int32,
                                   C.c_int32, C.c_int32, C.c_int32, C.c_int32]


def render(v: Volume, params: RenderParams, frames: int, accum=None):
    """-> (accum, color) float32 arrays of shape (height, width, 4)."""
    h, w = params.height, params.width
    acc = np.zeros((h, w, 4), np.float32) if accum is None else np.ascontiguousarray(accum, np.float32).copy()
    col = np.zeros((h, w, 4), np.float32)
    _lib.vko_render(v.ref, C.byref(params), acc.ctypes.data, col.ctypes.data, frames)
    return acc, col


def render_window(v: Volume, params: RenderParams, frames: int, window):
    """Pixels x0 <= x < x1, y0 <= y < y1 of the frame (window = (x0, y0, x1, y1)) from a cleared
    accumulation -> (accum, color) float32 arrays of shape (y1 - y0, x1 - x0, 4)."""
    x0, y0, x1, y1 = window
    h, w = params.height, params.width
    acc = np.zeros((h, w, 4), np.float32)
    col = np.zeros((h, w, 4), np.float32)
    _lib.vko_render_window(v.ref, C.byref(params), acc.ctypes.data, col.ctypes.data, frames, x0, y0, x1, y1)
    return acc[y0:y1, x0:x1].copy(), col[y0:y1, x0:x1].copy()
