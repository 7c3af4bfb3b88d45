"""Two interchangeable executors for the same test vectors:

* ``OracleBackend`` -- the CPU restatement in oracle/ (the checker; CPU-only tests).
* ``GpuBackend``    -- libvolkit through its public C ABI (volkit_amd.volkit): volumes are
  created and filled on the host under the CPU policy, the policy is switched to GPU (the
  next access migrates them to HBM), the algorithm runs as a gfx950 kernel, and the result
  is read back after switching to CPU again -- the reference's deferred-migration flow
  (README example, SURVEY.md §3 call stack (5)).

Every array is a (z, y, x) array of raw stored codes.
"""
from __future__ import annotations

import numpy as np

from oracle import binding as ob

CODE_DTYPE = ob.CODE_DTYPE


def codes_of(values, fmt):
    """Float values -> raw codes for Float32 volumes (bit patterns); ints pass through."""
    arr = np.asarray(values)
    if fmt == 7:
        return np.asarray(arr, dtype=np.float32).view(np.uint32)
    return arr.astype(CODE_DTYPE[fmt])


class OracleBackend:
    name = "oracle"

    def map(self, value, fmt, lo=0.0, hi=1.0):
        b = ob.map_voxel(value, fmt, lo, hi)
        return int.from_bytes(b, "little") if b else None

    def fill_range(self, fmt, mapping, dims, init, first, last, value):
        v = ob.Volume(init.reshape(dims[2], dims[1], dims[0]), fmt, *mapping)
        ob.fill_range(v, first, last, value)
        return v.codes

    def copy_range(self, dst_fmt, dst_map, dst_dims, dst_init, src_fmt, src_map, src_codes, first, last, off):
        d = ob.Volume(dst_init, dst_fmt, *dst_map)
        s = ob.Volume(src_codes, src_fmt, *src_map)
        ob.copy_range(d, s, first, last, off)
        return d.codes

    def arith(self, name, fmts, maps, a, b, dst_init, first, last, off):
        d = ob.Volume(dst_init, fmts[0], *maps[0])
        s1 = ob.Volume(a, fmts[1], *maps[1])
        s2 = ob.Volume(b, fmts[2], *maps[2])
        ob.arith_range(name, d, s1, s2, first, last, off)
        return d.codes

    def resample(self, dst_fmt, dst_map, dst_dims, src_fmt, src_map, src_codes, filter_mode, dst_init=None):
        x, y, z = dst_dims
        init = dst_init if dst_init is not None else np.zeros((z, y, x), dtype=CODE_DTYPE[dst_fmt])
        d = ob.Volume(init, dst_fmt, *dst_map)
        s = ob.Volume(src_codes, src_fmt, *src_map)
        ob.resample(d, s, filter_mode)
        return d.codes


class GpuBackend:
    name = "gpu"

    def __init__(self):
        import volkit_amd.volkit as vkt
        self.vkt = vkt

    def _cpu(self):
        ep = self.vkt.GetThreadExecutionPolicy()
        ep.device = self.vkt.ExecutionPolicy.Device_CPU
        self.vkt.SetThreadExecutionPolicy(ep)

    def _gpu(self):
        ep = self.vkt.GetThreadExecutionPolicy()
        ep.device = self.vkt.ExecutionPolicy.Device_GPU
        self.vkt.SetThreadExecutionPolicy(ep)

    def volume(self, codes, fmt, mapping):
        vkt = self.vkt
        z, y, x = codes.shape
        self._cpu()
        v = vkt.StructuredVolume(x, y, z, fmt, 1.0, 1.0, 1.0, float(mapping[0]), float(mapping[1]))
        v.from_numpy(np.ascontiguousarray(codes, dtype=CODE_DTYPE[fmt]))
        return v

    def _run(self, fn):
        self._gpu()
        try:
            err = fn()
        finally:
            self._cpu()
        if err != self.vkt.NoError:
            raise RuntimeError(f"volkit call failed ({err}): {self.vkt.last_error()}")

    def map(self, value, fmt, lo=0.0, hi=1.0):
        b = self.vkt.MapVoxel(value, fmt, lo, hi)
        return int.from_bytes(b, "little") if b else None

    def fill_range(self, fmt, mapping, dims, init, first, last, value):
        v = self.volume(init.reshape(dims[2], dims[1], dims[0]), fmt, mapping)
        self._run(lambda: self.vkt.FillRange(v, *first, *last, value))
        return v.to_numpy()

    def copy_range(self, dst_fmt, dst_map, dst_dims, dst_init, src_fmt, src_map, src_codes, first, last, off):
        d = self.volume(dst_init, dst_fmt, dst_map)
        s = self.volume(src_codes, src_fmt, src_map)
        self._run(lambda: self.vkt.CopyRange(d, s, *first, *last, *off))
        return d.to_numpy()

    def arith(self, name, fmts, maps, a, b, dst_init, first, last, off):
        d = self.volume(dst_init, fmts[0], maps[0])
        s1 = self.volume(a, fmts[1], maps[1])
        s2 = self.volume(b, fmts[2], maps[2])
        fn = getattr(self.vkt, name + "Range")
        self._run(lambda: fn(d, s1, s2, *first, *last, *off))
        return d.to_numpy()

    def resample(self, dst_fmt, dst_map, dst_dims, src_fmt, src_map, src_codes, filter_mode, dst_init=None):
        x, y, z = dst_dims
        init = dst_init if dst_init is not None else np.zeros((z, y, x), dtype=CODE_DTYPE[dst_fmt])
        d = self.volume(init, dst_fmt, dst_map)
        s = self.volume(src_codes, src_fmt, src_map)
        self._run(lambda: self.vkt.Resample(d, s, filter_mode))
        return d.to_numpy()
