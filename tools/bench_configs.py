"""Secondary BASELINE.json configs on one GPU (development/reporting tool; bench.py is the
driver's contract).  Prints one JSON line per case with kernel time (HIP events on the
backend's compute stream, median of N) and algorithmic GB/s.

  python tools/bench_configs.py [--reps 10] [--big]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from volkit_amd import _lib  # noqa: E402
from volkit_amd._lib import lib, HipVolumeView_t, Vec3i_t  # noqa: E402

BPV = {4: 1, 5: 2, 7: 4, 2: 2, 6: 4, 1: 1, 3: 4}


def alloc(dims, fmt, lo=0.0, hi=1.0, seed=None):
    x, y, z = dims
    p = C.c_void_p()
    n = x * y * z * BPV[fmt]
    if lib.vktHipAllocate(C.byref(p), n) != 0:
        raise RuntimeError(_lib.last_error())
    v = HipVolumeView_t(p.value, x, y, z, fmt, lo, hi)
    if seed is not None:
        lib.vktHipSynthesize(v, C.c_uint64(seed))
    return v


def rng_fill(v, n):
    """Float32 source of BASELINE config 3: uniform in [0, 1) (torch on the same device)."""
    t = torch.rand(n, device="cuda", dtype=torch.float32)
    lib.vktHipMemcpy(C.c_void_p(v.data), C.c_void_p(t.data_ptr()), n * 4, 3)
    torch.cuda.synchronize()


def free(*vs):
    for v in vs:
        lib.vktHipFree(C.c_void_p(v.data))


def timed(fn, reps):
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        if fn() != 0:
            raise RuntimeError(_lib.last_error())
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    del s
    return ts[len(ts) // 2]


def pipelined(fn, reps):
    """Back-to-back calls (host planning of call n+1 overlaps the kernels of call n)."""
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        if fn() != 0:
            raise RuntimeError(_lib.last_error())
    torch.cuda.synchronize()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def table_image(d, s):
    """Distinct source indices the exact per-axis table s = (int32)((float)x / (float)d * (float)s)
    of Resample_serial.hpp:26-71 hits for x in [0, d) (float32 arithmetic, as the kernels)."""
    import numpy as np
    x = np.arange(d, dtype=np.float32)
    return int(np.unique((x / np.float32(d) * np.float32(s)).astype(np.int32)).size)


def resample_bytes(sdims, ddims, bs, bd, every_row=False):
    """Bytes a Resample moves: the source rows the dst rows read (whole rows: the gather kernel
    stages each read row in LDS; the replication kernel reads rows too) x their planes, or every
    source row when the kernel reads them all (Float32 Linear: unstaged rows are classified for
    the chain), plus the dst bytes.  Equals the §8(d) N_src*b_s + N_dst*b_d
    whenever every source row is read (upsampling, same dims)."""
    sx, sy, sz = sdims
    rows = sy * sz if every_row else table_image(ddims[1], sy) * table_image(ddims[2], sz)
    return bs * sx * rows + bd * ddims[0] * ddims[1] * ddims[2]


def two_float_passes(on):
    """ComputeAggregates in the reference's two passes (mean, then variance) for every format:
    no code counts (knob aggregates.codes) and no one-pass moments (knob aggregates.moments)."""
    for k in (b"aggregates.codes", b"aggregates.moments"):
        lib.vktHipSetTuningKnob(k, 0 if on else -1)


def report(name, ms, nbytes, voxels):
    # a row above the HBM peak means the bytes credited are not the bytes the call moved (e.g. a
    # knob that no longer selects the path the label names): fail instead of committing it
    if nbytes / ms / 1e6 / 8000 > 1.0:
        raise AssertionError(f"{name}: {nbytes / ms / 1e6:.0f} GB/s is above 8 TB/s -- bytes or label wrong")
    print(json.dumps({"case": name, "ms": round(ms, 4), "GB/s": round(nbytes / ms / 1e6, 1),
                      "frac_of_8TBs": round(nbytes / ms / 1e6 / 8000, 4),
                      "Gvox/s": round(voxels / ms / 1e6, 2)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--big", action="store_true", help="include 2048^3 cases (~50 GB of HBM)")
    ap.add_argument("--only", default="", help="run only cases whose group name contains this")
    args = ap.parse_args()
    for kv in filter(None, os.environ.get("VKT_KNOBS", "").split(",")):   # "name=value,..." for PMC runs
        k, v = kv.split("=")
        if lib.vktHipSetTuningKnob(k.encode(), int(v)) != 0:
            raise RuntimeError(_lib.last_error())
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    lib.vktHipSetComputeStream(C.c_void_p(stream.cuda_stream))
    o = Vec3i_t(0, 0, 0)
    R = args.reps

    want = lambda g: args.only in g   # noqa: E731

    # config 2: 512^3 UInt16 SafeSum / SafeDiff / SumRange
    n = 512
    if not want("config2"):
        n = 0
    if n:
        A, B, D = alloc((n,) * 3, 5, seed=1), alloc((n,) * 3, 5, seed=2), alloc((n,) * 3, 5)
        last = Vec3i_t(n, n, n)
        for name, op in (("SafeSum", 5), ("SafeDiff", 6), ("SumRange", 0)):
            ms = timed(lambda: lib.vktHipArithmeticRange(op, D, A, B, o, last, o), R)
            report(f"config2 {name} 512^3 UInt16", ms, 6 * n ** 3, n ** 3)
        free(A, B, D)
        # the same ops on UInt8 volumes (decode = lerp of code / 255.999f), 1024^3
        m = 1024
        A, B, D = alloc((m,) * 3, 4, seed=1), alloc((m,) * 3, 4, seed=2), alloc((m,) * 3, 4)
        last = Vec3i_t(m, m, m)
        for name, op in (("SafeSum", 5), ("SumRange", 0)):
            ms = timed(lambda: lib.vktHipArithmeticRange(op, D, A, B, o, last, o), R)
            report(f"config2-u8 {name} 1024^3 UInt8", ms, 3 * m ** 3, m ** 3)
        free(A, B, D)
    # config 3: 1024^3 Float32 -> 2048^3 Linear (lerp-chain kernel) and Nearest (replication)
    s, e = 1024, 2048
    if want("config3"):
        S = alloc((s,) * 3, 7)
        rng_fill(S, s ** 3)
        Rv = alloc((e,) * 3, 7)
        for fm, lab in ((1, "Linear"), (0, "Nearest")):
            ms = timed(lambda: lib.vktHipResample(Rv, S, fm), max(3, R // 3))
            report(f"config3 Resample 1024^3->2048^3 Float32 {lab}", ms, 4 * s ** 3 + 4 * e ** 3, e ** 3)
        free(S, Rv)
    if want("transform"):
        # device-functor Transform (include/volkit_transform.hpp) through the test fixture
        # tests/native/libfixtures.so; unary algorithmic bytes 2b per voxel
        t = C.CDLL(os.path.join(ROOT, "tests", "native", "libfixtures.so"))
        t.vktt_bench_unary.argtypes = [C.c_int] * 6 + [C.POINTER(C.c_float)]
        ms = C.c_float(0.0)
        m = 1024
        for op, lab, fmt, b, rw in ((2, "Diagonal", 4, 1, 2), (2, "Diagonal", 5, 2, 2), (2, "Diagonal", 7, 4, 2),
                                    (0, "Checkered<3> (write-only: loads are dead)", 4, 1, 1)):
            if t.vktt_bench_unary(op, m, m, m, fmt, R, C.byref(ms)) != 0:
                raise RuntimeError(_lib.last_error())
            report(f"Transform {lab} 1024^3 fmt={fmt}", ms.value, rw * b * m ** 3, m ** 3)
        # TransformRange over a sub-box whose rows start and end inside 16-B chunks (the shape of
        # CoreAlgorithms.c's TransformRange 2..22, scaled): padded vector path
        t.vktt_bench_unary_range.argtypes = [C.c_int] * 12 + [C.POINTER(C.c_float)]
        for fmt, b in ((4, 1), (5, 2), (7, 4)):
            if t.vktt_bench_unary_range(2, m, m, m, fmt, 2, 2, 2, m - 2, m - 2, m - 2, R, C.byref(ms)) != 0:
                raise RuntimeError(_lib.last_error())
            nv = (m - 4) ** 3
            report(f"TransformRange Diagonal 2..{m - 2} of 1024^3 fmt={fmt}", ms.value, 2 * b * nv, nv)
    if want("tshape"):
        # Transform vector-kernel workgroup shape A/B (knob transform.shape: 0 256x4, 1 64x2, 2 64x1)
        t = C.CDLL(os.path.join(ROOT, "tests", "native", "libfixtures.so"))
        t.vktt_bench_unary.argtypes = [C.c_int] * 6 + [C.POINTER(C.c_float)]
        t.vktt_bench_unary_range.argtypes = [C.c_int] * 12 + [C.POINTER(C.c_float)]
        ms = C.c_float(0.0)
        m = 1024
        try:
            for shape in (0, 1, 2):
                lib.vktHipSetTuningKnob(b"transform.shape", shape)
                for fmt, b in ((4, 1), (5, 2), (7, 4)):
                    if t.vktt_bench_unary(2, m, m, m, fmt, R, C.byref(ms)) != 0:
                        raise RuntimeError(_lib.last_error())
                    report(f"Transform Diagonal 1024^3 fmt={fmt} shape={shape}", ms.value, 2 * b * m ** 3, m ** 3)
                    if t.vktt_bench_unary_range(2, m, m, m, fmt, 2, 2, 2, m - 2, m - 2, m - 2, R, C.byref(ms)) != 0:
                        raise RuntimeError(_lib.last_error())
                    nv = (m - 4) ** 3
                    report(f"TransformRange Diagonal 2..{m - 2} fmt={fmt} shape={shape}", ms.value, 2 * b * nv, nv)
                    if t.vktt_bench_unary_range(2, m, m, m, fmt, 16, 3, 5, m - 16, m - 3, m - 5, R, C.byref(ms)) != 0:
                        raise RuntimeError(_lib.last_error())
                    nv = (m - 32) * (m - 6) * (m - 10)
                    report(f"TransformRange Diagonal x16..{m - 16} fmt={fmt} shape={shape}", ms.value, 2 * b * nv, nv)
                    if t.vktt_bench_unary_range(2, m, m, m, fmt, 0, 2, 2, m, m - 2, m - 2, R, C.byref(ms)) != 0:
                        raise RuntimeError(_lib.last_error())
                    nv = m * (m - 4) * (m - 4)
                    report(f"TransformRange Diagonal full rows y,z 2..{m - 2} fmt={fmt} shape={shape}", ms.value,
                           2 * b * nv, nv)
        finally:
            lib.vktHipSetTuningKnob(b"transform.shape", -1)
    if want("memset"):
        # MemsetRange / ManagedBuffer::fill at 1024^3-UInt16 scale (2 GiB), write-only bytes
        nb = 2 << 30
        p = C.c_void_p()
        if lib.vktHipAllocate(C.byref(p), nb + 64) != 0:
            raise RuntimeError(_lib.last_error())
        import numpy as np
        for psize, off in ((2, 0), (4, 1), (2, 16), (3, 0), (12, 0), (17, 0), (300, 0)):
            pat = np.arange(1, psize + 1, dtype=np.uint8)
            n = nb - off
            ms = timed(lambda: lib.vktHipMemsetRange(C.c_void_p(p.value + off), pat.ctypes.data_as(C.c_void_p), n,
                                                     psize), R)
            report(f"MemsetRange 2 GiB pattern {psize} B dst+{off}", ms, (n // psize) * psize, n // 2)
        lib.vktHipFree(p)
    if want("subbox"):
        # one case per kernel for PMC passes: the 800^3 sub-box of 1024^3 at x0 = 100
        m = 1024
        A, B, D = alloc((m,) * 3, 5, seed=1), alloc((m,) * 3, 5, seed=2), alloc((m,) * 3, 5)
        report("subbox SafeSumRange 800^3 sub-box of 1024^3 UInt16 x0=100",
               timed(lambda: lib.vktHipArithmeticRange(5, D, A, B, Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900), o),
                     R), 6 * 800 ** 3, 800 ** 3)
        free(A, B, D)
    if want("u8sub") or want("f32sub"):
        # multi-row sub-boxes of 1024^3: one launch per case, for PMC passes
        m = 1024
        for fmt, bpv, name, grp in ((4, 1, "UInt8", "u8sub"), (7, 4, "Float32", "f32sub")):
            if not want(grp):
                continue
            A, B, D = alloc((m,) * 3, fmt, seed=1), alloc((m,) * 3, fmt, seed=2), alloc((m,) * 3, fmt)
            for lab, f0, f1 in (("x0=100", Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900)),
                                ("x 0..800", Vec3i_t(0, 100, 100), Vec3i_t(800, 900, 900)),
                                ("x 0..1024 (planes)", Vec3i_t(0, 100, 100), Vec3i_t(1024, 900, 900))):
                nv = (f1.x - f0.x) * (f1.y - f0.y) * (f1.z - f0.z)
                report(f"{grp} CopyRange {lab} same offset {name}",
                       timed(lambda: lib.vktHipCopyRange(D, A, f0, f1, f0), R), 2 * bpv * nv, nv)
                report(f"{grp} CopyRange {lab} -> dst 0 {name}",
                       timed(lambda: lib.vktHipCopyRange(D, A, f0, f1, o), R), 2 * bpv * nv, nv)
                report(f"{grp} SumRange {lab} {name}",
                       timed(lambda: lib.vktHipArithmeticRange(0, D, A, B, f0, f1, o), R), 3 * bpv * nv, nv)
            free(A, B, D)
    if want("u8row"):
        # UInt8 whole-volume ops on the row kernel: items per lane (knob pointwise.u8_unroll) x
        # occupancy cap (pointwise.row_lds), against the general kernel (row_kernel 0)
        m = 1024
        A, B, D = alloc((m,) * 3, 4, seed=1), alloc((m,) * 3, 4, seed=2), alloc((m,) * 3, 4)
        last = Vec3i_t(m, m, m)
        settings = [(0, 4, 0), (1, 4, 8192), (1, 2, 8192), (1, 8, 8192), (1, 2, 0), (1, 8, 0), (1, 2, 10240)]
        for rep in range(2):
            for rk, un, lds in settings:
                for k, v in ((b"pointwise.row_kernel", rk), (b"pointwise.u8_unroll", un), (b"pointwise.row_lds_u8", lds)):
                    lib.vktHipSetTuningKnob(k, v)
                tag = f"[row_kernel={rk} unroll={un} lds={lds}]"
                report(f"u8row Copy 1024^3 UInt8 {tag}", timed(lambda: lib.vktHipCopyRange(D, A, o, last, o), R),
                       2 * m ** 3, m ** 3)
                report(f"u8row SumRange 1024^3 UInt8 {tag}",
                       timed(lambda: lib.vktHipArithmeticRange(0, D, A, B, o, last, o), R), 3 * m ** 3, m ** 3)
                report(f"u8row SafeSum 1024^3 UInt8 {tag}",
                       timed(lambda: lib.vktHipArithmeticRange(5, D, A, B, o, last, o), R), 3 * m ** 3, m ** 3)
        for k in (b"pointwise.row_kernel", b"pointwise.u8_unroll", b"pointwise.row_lds_u8"):
            lib.vktHipSetTuningKnob(k, -1)
        free(A, B, D)
    if want("u16row"):
        # UInt16 whole-volume ops: the row kernel (knob pointwise.row_kernel bit 1) at 1 or 2 KiB
        # per stream per workgroup (pointwise.u16_unroll) and occupancy caps (pointwise.row_lds),
        # against the general kernel; alternated on the same allocations
        m = 1024
        A, B, D = alloc((m,) * 3, 5, seed=1), alloc((m,) * 3, 5, seed=2), alloc((m,) * 3, 5)
        last = Vec3i_t(m, m, m)
        settings = [(1, 2, 0), (3, 1, 0), (3, 1, 5376), (3, 1, 5632), (3, 1, 5888), (3, 1, 6144), (3, 2, 5632)]
        for rep in range(3):
            for rk, un, lds in settings:
                for k, v in ((b"pointwise.row_kernel", rk), (b"pointwise.u16_unroll", un), (b"pointwise.row_lds", lds)):
                    lib.vktHipSetTuningKnob(k, v)
                tag = f"[row_kernel={rk} unroll={un} lds={lds}]"
                report(f"u16row Copy 1024^3 UInt16 {tag}", timed(lambda: lib.vktHipCopyRange(D, A, o, last, o), R),
                       4 * m ** 3, m ** 3)
                report(f"u16row SumRange 1024^3 UInt16 {tag}",
                       timed(lambda: lib.vktHipArithmeticRange(0, D, A, B, o, last, o), R), 6 * m ** 3, m ** 3)
                report(f"u16row SafeDiff 1024^3 UInt16 {tag}",
                       timed(lambda: lib.vktHipArithmeticRange(6, D, A, B, o, last, o), R), 6 * m ** 3, m ** 3)
        for k in (b"pointwise.row_kernel", b"pointwise.u16_unroll", b"pointwise.row_lds"):
            lib.vktHipSetTuningKnob(k, -1)
        free(A, B, D)
    if want("rowswz"):
        # XCD mapping of the row kernel's quanta (knob pointwise.row_swizzle: 0 every 8th quantum
        # per XCD, r > 0 runs of r consecutive quanta), UInt16 SumRange / UInt8 SumRange + Copy
        m = 1024
        for fmt, bpv, name in ((5, 2, "UInt16"), (4, 1, "UInt8")):
            A, B, D = alloc((m,) * 3, fmt, seed=1), alloc((m,) * 3, fmt, seed=2), alloc((m,) * 3, fmt)
            last = Vec3i_t(m, m, m)
            for rep in range(3):
                for r in (0, 2, 8, 64, 4096):
                    lib.vktHipSetTuningKnob(b"pointwise.row_swizzle", r)
                    report(f"rowswz SumRange 1024^3 {name} [row_swizzle={r}]",
                           timed(lambda: lib.vktHipArithmeticRange(0, D, A, B, o, last, o), R), 3 * bpv * m ** 3, m ** 3)
                    if fmt == 4:
                        report(f"rowswz Copy 1024^3 {name} [row_swizzle={r}]",
                               timed(lambda: lib.vktHipCopyRange(D, A, o, last, o), R), 2 * bpv * m ** 3, m ** 3)
            lib.vktHipSetTuningKnob(b"pointwise.row_swizzle", -1)
            free(A, B, D)
    if want("rowsk"):
        # multi-row sub-boxes of 1024^3 on the MODE-1-only kernel (knob pointwise.rows_kernel),
        # with 1 / 2 KiB per stream (u8_unroll / u16_unroll), against the general kernel
        m = 1024
        boxes = (("x0=100", Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900)),
                 ("x 0..800", Vec3i_t(0, 100, 100), Vec3i_t(800, 900, 900)))
        settings = ((0, 2, 1), (3, 2, 1))   # (u8_unroll / u16_unroll: the whole-volume kernel's)
        for fmt, bpv, name in ((4, 1, "UInt8"), (5, 2, "UInt16")):
            A, B, D = alloc((m,) * 3, fmt, seed=1), alloc((m,) * 3, fmt, seed=2), alloc((m,) * 3, fmt)
            for rep in range(2):
                for rk, u8, u16 in settings:
                    for k, v in ((b"pointwise.rows_kernel", rk), (b"pointwise.u8_unroll", u8),
                                 (b"pointwise.u16_unroll", u16)):
                        lib.vktHipSetTuningKnob(k, v)
                    tag = f"[rows_kernel={rk} u8_unroll={u8} u16_unroll={u16}]"
                    for lab, f0, f1 in boxes:
                        nv = (f1.x - f0.x) * (f1.y - f0.y) * (f1.z - f0.z)
                        if fmt == 4:
                            report(f"rowsk CopyRange {lab} same offset {name} {tag}",
                                   timed(lambda: lib.vktHipCopyRange(D, A, f0, f1, f0), R), 2 * bpv * nv, nv)
                        report(f"rowsk SumRange {lab} {name} {tag}",
                               timed(lambda: lib.vktHipArithmeticRange(0, D, A, B, f0, f1, o), R), 3 * bpv * nv, nv)
            for k in (b"pointwise.rows_kernel", b"pointwise.u8_unroll", b"pointwise.u16_unroll"):
                lib.vktHipSetTuningKnob(k, -1)
            free(A, B, D)
    if want("rowslds"):
        # occupancy cap (dynamic LDS per one-wave workgroup, knob pointwise.row_lds_u8) for the
        # UInt8 row / rows kernels: the x0 = 100 sub-boxes (MODE 1) and the whole volume (MODE 0)
        m = 1024
        A, B, D = alloc((m,) * 3, 4, seed=1), alloc((m,) * 3, 4, seed=2), alloc((m,) * 3, 4)
        f0, f1, last = Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900), Vec3i_t(m, m, m)
        nv = 800 ** 3
        try:
            for rep in range(2):
                for lds in (0, 4096, 5120, 5632, 6656, 8192):
                    lib.vktHipSetTuningKnob(b"pointwise.row_lds_u8", lds)
                    tag = f"[row_lds_u8={lds}]"
                    report(f"rowslds CopyRange x0=100 same offset UInt8 {tag}",
                           timed(lambda: lib.vktHipCopyRange(D, A, f0, f1, f0), R), 2 * nv, nv)
                    report(f"rowslds SumRange x0=100 UInt8 {tag}",
                           timed(lambda: lib.vktHipArithmeticRange(0, D, A, B, f0, f1, o), R), 3 * nv, nv)
                    report(f"rowslds Copy 1024^3 UInt8 {tag}",
                           timed(lambda: lib.vktHipCopyRange(D, A, o, last, o), R), 2 * m ** 3, m ** 3)
                    report(f"rowslds SumRange 1024^3 UInt8 {tag}",
                           timed(lambda: lib.vktHipArithmeticRange(0, D, A, B, o, last, o), R), 3 * m ** 3, m ** 3)
        finally:
            lib.vktHipSetTuningKnob(b"pointwise.row_lds_u8", -1)
            free(A, B, D)
    if want("u8cal"):
        # FETCH_SIZE calibration for the UInt8 access shapes and the
        # whole-volume UInt8 ops against UInt16 (item 4); one launch per case for PMC passes.
        # Known byte counts: whole volumes, whole planes (rows merged into one run per plane),
        # 768-B rows on 128-B lines (x 128..896); then the 800-B rows at x0 = 100 / 64 with and
        # without sector completion (knob pointwise.merge_sectors).
        m = 1024
        for fmt, bpv, name in ((4, 1, "UInt8"), (5, 2, "UInt16")):
            A, B, D = alloc((m,) * 3, fmt, seed=1), alloc((m,) * 3, fmt, seed=2), alloc((m,) * 3, fmt)
            last = Vec3i_t(m, m, m)
            report(f"u8cal Copy 1024^3 {name}", timed(lambda: lib.vktHipCopyRange(D, A, o, last, o), R),
                   2 * bpv * m ** 3, m ** 3)
            report(f"u8cal SumRange 1024^3 {name}", timed(lambda: lib.vktHipArithmeticRange(0, D, A, B, o, last, o), R),
                   3 * bpv * m ** 3, m ** 3)
            if fmt == 4:
                for lab, f0, f1, mg in (("planes x 0..1024", Vec3i_t(0, 100, 100), Vec3i_t(1024, 900, 900), 1),
                                        ("x 128..896 (128-B lines)", Vec3i_t(128, 100, 100), Vec3i_t(896, 900, 900), 1),
                                        ("x 100..900", Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900), 1),
                                        ("x 100..900 [merge 0]", Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900), 0),
                                        ("x 64..864", Vec3i_t(64, 100, 100), Vec3i_t(864, 900, 900), 1),
                                        ("x 64..864 [merge 0]", Vec3i_t(64, 100, 100), Vec3i_t(864, 900, 900), 0)):
                    lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", mg)
                    nv = (f1.x - f0.x) * (f1.y - f0.y) * (f1.z - f0.z)
                    report(f"u8cal CopyRange {lab} same offset UInt8",
                           timed(lambda: lib.vktHipCopyRange(D, A, f0, f1, f0), R), 2 * nv, nv)
                    report(f"u8cal SumRange {lab} UInt8",
                           timed(lambda: lib.vktHipArithmeticRange(0, D, A, B, f0, f1, o), R), 3 * nv, nv)
                lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", -1)
            free(A, B, D)
    if want("f32shift"):
        # one launch per case (PMC passes): the Float32 general path with a
        # phase shift, and UInt8 SumRange on the 800^3 sub-box at x0 = 100, default knobs
        m = 1024
        for fmt, bpv, name in ((7, 4, "Float32"), (4, 1, "UInt8")):
            A, B, D = alloc((m,) * 3, fmt, seed=1), alloc((m,) * 3, fmt, seed=2), alloc((m,) * 3, fmt)
            f0, f1 = Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900)
            nv = 800 ** 3
            if fmt == 7:
                report(f"f32shift CopyRange 800^3 x0=100 -> dst 0 {name}",
                       timed(lambda: lib.vktHipCopyRange(D, A, f0, f1, o), R), 2 * bpv * nv, nv)
                report(f"f32shift CopyRange 800^3 x0=100 -> dst x0=3 {name}",
                       timed(lambda: lib.vktHipCopyRange(D, A, f0, f1, Vec3i_t(3, 100, 100)), R), 2 * bpv * nv, nv)
                report(f"f32shift SumRange 800^3 x0=100 dstOffset x=-97 {name}",
                       timed(lambda: lib.vktHipArithmeticRange(0, D, A, B, f0, f1, Vec3i_t(-97, 0, 0)), R),
                       3 * bpv * nv, nv)
                report(f"f32shift CopyRange 800^3 x0=100 same offset {name}",
                       timed(lambda: lib.vktHipCopyRange(D, A, f0, f1, f0), R), 2 * bpv * nv, nv)
            else:
                report(f"f32shift SumRange 800^3 x0=100 {name}",
                       timed(lambda: lib.vktHipArithmeticRange(0, D, A, B, f0, f1, o), R), 3 * bpv * nv, nv)
                report(f"f32shift CopyRange 800^3 x0=100 same offset {name}",
                       timed(lambda: lib.vktHipCopyRange(D, A, f0, f1, f0), R), 2 * bpv * nv, nv)
            free(A, B, D)
    if want("f32s3"):
        # Float32 SumRange on the 800^3 sub-box at x0 = 100: same offset (aligned path) vs
        # dstOffset x = -97 (general path) with 8-voxel items (knob pointwise.f32_wide 2, the
        # default) and 16-B items (f32_wide 1); one launch per case for PMC passes
        m = 1024
        A, B, D = alloc((m,) * 3, 7, seed=1), alloc((m,) * 3, 7, seed=2), alloc((m,) * 3, 7)
        f0, f1 = Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900)
        nv = 800 ** 3
        report("f32s3 SumRange 800^3 x0=100 same offset Float32",
               timed(lambda: lib.vktHipArithmeticRange(0, D, A, B, f0, f1, o), R), 12 * nv, nv)
        for wide in (2, 1):
            lib.vktHipSetTuningKnob(b"pointwise.f32_wide", wide)
            report(f"f32s3 SumRange 800^3 x0=100 dstOffset x=-97 Float32 [f32_wide={wide}]",
                   timed(lambda: lib.vktHipArithmeticRange(0, D, A, B, f0, f1, Vec3i_t(-97, 0, 0)), R), 12 * nv, nv)
        lib.vktHipSetTuningKnob(b"pointwise.f32_wide", -1)
        free(A, B, D)
    if want("f32dw"):
        # in-process A/B: whole-dword window shifts (knob pointwise.dword_shift) x 16-B items
        # (pointwise.f32_wide) on the Float32 general path, 800^3 sub-box of 1024^3
        m = 1024
        A, B, D = alloc((m,) * 3, 7, seed=1), alloc((m,) * 3, 7, seed=2), alloc((m,) * 3, 7)
        f0, f1 = Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900)
        cases = (("CopyRange 800^3 x0=100 -> dst 0", lambda: lib.vktHipCopyRange(D, A, f0, f1, o), 2),
                 ("CopyRange 800^3 x0=100 -> dst x0=3", lambda: lib.vktHipCopyRange(D, A, f0, f1, Vec3i_t(3, 100, 100)), 2),
                 ("SumRange 800^3 x0=100 dstOffset x=-97",
                  lambda: lib.vktHipArithmeticRange(0, D, A, B, f0, f1, Vec3i_t(-97, 0, 0)), 3))
        kvs = ((1, 0), (0, 0), (1, 1), (0, 1))   # (dword_shift, f32_wide)
        ab = {}
        for rnd in range(3):
            for kv in kvs:
                lib.vktHipSetTuningKnob(b"pointwise.dword_shift", kv[0])
                lib.vktHipSetTuningKnob(b"pointwise.f32_wide", kv[1])
                for lab, fn, _ in cases:
                    ab.setdefault((lab, kv), []).append(timed(fn, R))
        lib.vktHipSetTuningKnob(b"pointwise.dword_shift", -1)
        lib.vktHipSetTuningKnob(b"pointwise.f32_wide", -1)
        for lab, fn, streams in cases:
            for kv in kvs:
                ts = sorted(ab[(lab, kv)])
                report(f"f32dw {lab} Float32 dword_shift={kv[0]} f32_wide={kv[1]} (median of 3 rounds, "
                       f"spread {ts[0]:.4f}-{ts[-1]:.4f})", ts[1], streams * 4 * 800 ** 3, 800 ** 3)
        free(A, B, D)
    if want("p16"):
        # the 65 536-bin UInt16 histogram (packed 16-bit LDS counters), one launch per case
        # (accumulate: no zeroing kernel) -- the code-count kernel of the UInt16 aggregates too
        n = 1024
        V = alloc((n,) * 3, 5, seed=11)
        hb = C.c_void_p()
        if lib.vktHipAllocate(C.byref(hb), 65536 * 8) != 0:
            raise RuntimeError(_lib.last_error())
        bins = C.c_void_p(hb.value)
        last = Vec3i_t(n, n, n)
        report("p16 Histogram 1024^3 UInt16 65536 bins (P16)",
               timed(lambda: lib.vktHipHistogramRange(V, o, last, bins, 65536, 1), R), 2 * n ** 3, n ** 3)
        report("p16 Histogram 1024^3 UInt16 256 bins (replicated counters)",
               timed(lambda: lib.vktHipHistogramRange(V, o, last, bins, 256, 1), R), 2 * n ** 3, n ** 3)
        lib.vktHipFree(hb)
        free(V)
    if want("u8ab"):
        # in-process A/B of the UInt8 16-voxel pair grid (knob pointwise.u8_pairs: 0 off, 1
        # default rule, 2 forced, 3 the general path's wide items), alternating on the same
        # allocations (VKT_U8AB_GEN=1: default vs general path only)
        m = 1024
        A, B, D = alloc((m,) * 3, 4, seed=1), alloc((m,) * 3, 4, seed=2), alloc((m,) * 3, 4)
        ab = {}
        boxes = (("x0=100", Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900)),
                 ("x 0..800", Vec3i_t(0, 100, 100), Vec3i_t(800, 900, 900)),
                 ("x 0..1024 (planes)", Vec3i_t(0, 100, 100), Vec3i_t(1024, 900, 900)))
        for rnd in range(3):
            for kv in ((1, -1), (3, -1), (3, 2)) if os.environ.get("VKT_U8AB_GEN") else \
                    ((0, -1), (1, 0), (1, 1), (1, 2), (2, -1)):   # (u8_pairs, merge_sectors)
                lib.vktHipSetTuningKnob(b"pointwise.u8_pairs", kv[0])
                lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", kv[1])
                for lab, f0, f1 in boxes:
                    ab.setdefault(("CopyRange", lab, kv), []).append(
                        timed(lambda: lib.vktHipCopyRange(D, A, f0, f1, f0), R))
                    ab.setdefault(("SumRange", lab, kv), []).append(
                        timed(lambda: lib.vktHipArithmeticRange(0, D, A, B, f0, f1, o), R))
        lib.vktHipSetTuningKnob(b"pointwise.u8_pairs", -1)
        lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", -1)
        for (op, lab, kv), ts in sorted(ab.items()):
            ts.sort()
            f0, f1 = [(b[1], b[2]) for b in boxes if b[0] == lab][0]
            nv = (f1.x - f0.x) * (f1.y - f0.y) * (f1.z - f0.z)
            report(f"u8ab {op} {lab} UInt8 u8_pairs={kv[0]} merge_sectors={kv[1]} (median of 3 rounds, "
                   f"spread {ts[0]:.4f}-{ts[-1]:.4f})",
                   ts[1], (2 if op == "CopyRange" else 3) * nv, nv)
        free(A, B, D)
    for gname, gfmt, gb, gknob in (("u8gen", 4, 1, b"pointwise.u8_wide"), ("f32gen", 7, 4, b"pointwise.f32_wide")):
        if not want(gname):
            continue
        # general path (source and destination at different phases, 800^3 sub-box of 1024^3):
        # in-process A/B of 16-B items (knob pointwise.u8_wide / f32_wide)
        m = 1024
        A, B, D = alloc((m,) * 3, gfmt, seed=1), alloc((m,) * 3, gfmt, seed=2), alloc((m,) * 3, gfmt)
        ab = {}
        cases = (("CopyRange x0=100 -> dst 0", lambda: lib.vktHipCopyRange(D, A, Vec3i_t(100, 100, 100),
                                                                          Vec3i_t(900, 900, 900), o), 2),
                 ("CopyRange x0=100 -> dst x0=3", lambda: lib.vktHipCopyRange(D, A, Vec3i_t(100, 100, 100),
                                                                             Vec3i_t(900, 900, 900),
                                                                             Vec3i_t(3, 100, 100)), 2),
                 ("CopyRange 1021x1024^2 x0=3 -> 0", lambda: lib.vktHipCopyRange(D, A, Vec3i_t(3, 0, 0),
                                                                                Vec3i_t(m, m, m), o), 2),
                 ("SumRange 800^3 x0=100 dstOffset x=-97", lambda: lib.vktHipArithmeticRange(
                     0, D, A, B, Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900), Vec3i_t(-97, 0, 0)), 3))
        kvs = ((0, -1), (1, -1), (1, 2))   # (wide, merge_sectors)
        for rnd in range(3):
            for kv in kvs:
                lib.vktHipSetTuningKnob(gknob, kv[0])
                lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", kv[1])
                for lab, fn, _ in cases:
                    ab.setdefault((lab, kv), []).append(timed(fn, R))
        lib.vktHipSetTuningKnob(gknob, -1)
        lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", -1)
        for lab, fn, streams in cases:
            nv = 1021 * m * m if "1021" in lab else 800 ** 3
            for kv in kvs:
                ts = sorted(ab[(lab, kv)])
                report(f"{gname} {lab} fmt={gfmt} wide={kv[0]} merge_sectors={kv[1]} (median of 3 rounds, "
                       f"spread {ts[0]:.4f}-{ts[-1]:.4f})", ts[1], streams * nv * gb, nv)
        free(A, B, D)
    if want("f32ab"):
        # Float32 padded multi-row boxes: contiguous-lane halves (knob pointwise.f32_halves) A/B
        m = 1024
        A, B, D = alloc((m,) * 3, 7, seed=1), alloc((m,) * 3, 7, seed=2), alloc((m,) * 3, 7)
        boxes = (("x0=100", Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900)),
                 ("x0=101", Vec3i_t(101, 100, 100), Vec3i_t(901, 900, 900)))
        ab = {}
        for rnd in range(3):
            for kv in (0, 1):
                lib.vktHipSetTuningKnob(b"pointwise.f32_halves", kv)
                for lab, f0, f1 in boxes:
                    ab.setdefault(("CopyRange", lab, kv), []).append(
                        timed(lambda: lib.vktHipCopyRange(D, A, f0, f1, f0), R))
                    ab.setdefault(("SumRange", lab, kv), []).append(
                        timed(lambda: lib.vktHipArithmeticRange(0, D, A, B, f0, f1, o), R))
        lib.vktHipSetTuningKnob(b"pointwise.f32_halves", -1)
        for (op, lab, kv), ts in sorted(ab.items()):
            ts.sort()
            report(f"f32ab {op} 800^3 sub-box {lab} Float32 f32_halves={kv} (median of 3 rounds, "
                   f"spread {ts[0]:.4f}-{ts[-1]:.4f})", ts[1], (8 if op == "CopyRange" else 12) * 800 ** 3, 800 ** 3)
        free(A, B, D)
    if want("u16merge"):
        # 3-stream UInt16 / Float32 ops on padded sub-boxes: sector completion (merge_sectors = 2)
        for fmt, bpv in ((5, 2), (7, 4)):
            m = 1024
            A, B, D = alloc((m,) * 3, fmt, seed=1), alloc((m,) * 3, fmt, seed=2), alloc((m,) * 3, fmt)
            ab = {}
            for rnd in range(3):
                for kv in (1, 2):
                    lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", kv)
                    for lab, f0, f1 in (("x0=100", Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900)),):
                        ab.setdefault((lab, kv, 5), []).append(
                            timed(lambda: lib.vktHipArithmeticRange(5, D, A, B, f0, f1, o), R))
                        ab.setdefault((lab, kv, 0), []).append(
                            timed(lambda: lib.vktHipArithmeticRange(0, D, A, B, f0, f1, o), R))
            lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", -1)
            for (lab, kv, op), ts in sorted(ab.items()):
                ts.sort()
                report(f"u16merge {'SafeSum' if op == 5 else 'Sum'}Range 800^3 sub-box {lab} fmt={fmt} merge_sectors={kv} "
                       f"(median of 3 rounds, spread {ts[0]:.4f}-{ts[-1]:.4f})", ts[1], 3 * bpv * 800 ** 3, 800 ** 3)
            free(A, B, D)
    if want("chunked"):
        # metric pipeline scheduled in plane chunks (Resample of dst planes [z0, z1), then SumRange
        # over the same planes): does the R chunk come back from the Infinity Cache?
        s_, e = 512, 1024
        S, Rv, B, D = alloc((s_,) * 3, 5, seed=4), alloc((e,) * 3, 5), alloc((e,) * 3, 5, seed=5), alloc((e,) * 3, 5)
        plane = e * e * 2

        def whole():
            lib.vktHipResample(Rv, S, 1)
            return lib.vktHipArithmeticRange(0, D, Rv, B, o, Vec3i_t(e, e, e), o)

        def chunked(n):
            def run():
                for z0 in range(0, e, n):
                    z1 = min(z0 + n, e)
                    rv = HipVolumeView_t(Rv.data + z0 * plane, e, e, z1 - z0, 5, 0.0, 1.0)
                    if lib.vktHipResampleSlab(rv, S, 1, e, z0, s_, 0):
                        return 1
                    if lib.vktHipArithmeticRange(0, D, Rv, B, Vec3i_t(0, 0, z0), Vec3i_t(e, e, z1), o):
                        return 1
                return 0
            return run
        for rnd in range(2):
            report(f"chunked whole calls (round {rnd})", timed(whole, R), 8858370048, e ** 3)
            for n in (8, 16, 32, 64, 128):
                report(f"chunked {n} planes per chunk (round {rnd})", timed(chunked(n), R), 8858370048, e ** 3)
        free(S, Rv, B, D)
    if want("weakspots"):
        # the kernels furthest below the roofline in round 1 (VERDICT r1 "What's weak" 5)
        m = 1024
        A, B, D = alloc((m,) * 3, 5, seed=1), alloc((m,) * 3, 5, seed=2), alloc((m,) * 3, 5)
        sub0, sub1 = Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900)
        a0, a1 = Vec3i_t(96, 100, 100), Vec3i_t(896, 900, 900)
        # in-process A/B of the 64-B sector completion (knob pointwise.merge_sectors) on the same
        # allocations, alternating: SafeSumRange and CopyRange over the sub-boxes
        ab = {}
        for rnd in range(4):
            for mg in (1, 0):
                lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", mg)
                for lab, f0, f1 in (("x0=100", sub0, sub1), ("x0=96", a0, a1)):
                    ab.setdefault(("SafeSumRange", lab, mg), []).append(
                        timed(lambda: lib.vktHipArithmeticRange(5, D, A, B, f0, f1, o), R))
                    ab.setdefault(("CopyRange", lab, mg), []).append(
                        timed(lambda: lib.vktHipCopyRange(D, A, f0, f1, f0), R))
        lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", -1)
        for (op, lab, mg), ts in sorted(ab.items()):
            ts.sort()
            nb = (6 if op == "SafeSumRange" else 4) * 800 ** 3
            report(f"weak {op} 800^3 sub-box of 1024^3 UInt16 {lab} merge={mg} "
                   f"(median of 4 rounds, spread {ts[0]:.4f}-{ts[-1]:.4f})", ts[len(ts) // 2], nb, 800 ** 3)
        # what the multi-row boxes lose: line-aligned row starts, long rows (whole x lines)
        for lab, f0, f1 in (("x 64..864 (rows start on a 128-B line)", Vec3i_t(64, 100, 100), Vec3i_t(864, 900, 900)),
                            ("x 0..800", Vec3i_t(0, 100, 100), Vec3i_t(800, 900, 900)),
                            ("x 0..1024 y,z 100..900 (plane-contiguous rows)", Vec3i_t(0, 100, 100),
                             Vec3i_t(1024, 900, 900)),
                            ("x,y 0..1024 z 100..900 (one contiguous run)", Vec3i_t(0, 0, 100),
                             Vec3i_t(1024, 1024, 900)),
                            ("whole 1024^3 (one contiguous run)", Vec3i_t(0, 0, 0), Vec3i_t(1024, 1024, 1024))):
            nv = (f1.x - f0.x) * (f1.y - f0.y) * (f1.z - f0.z)
            report(f"weak SafeSumRange sub-box {lab}", timed(lambda: lib.vktHipArithmeticRange(5, D, A, B, f0, f1, o),
                                                           R), 6 * nv, nv)
        free(A, B, D)
        n = 512
        A, B, D = alloc((n,) * 3, 5, seed=1), alloc((n,) * 3, 5, seed=2), alloc((n,) * 3, 5)
        report("weak config2 SafeSum 512^3 UInt16",
               timed(lambda: lib.vktHipArithmeticRange(5, D, A, B, o, Vec3i_t(n, n, n), o), R), 6 * n ** 3, n ** 3)
        free(A, B, D)
        S = alloc((1024,) * 3, 7)
        rng_fill(S, 1024 ** 3)
        Rv = alloc((768,) * 3, 7)
        report("weak Resample 1024^3->768^3 Float32 Linear (gather)", timed(lambda: lib.vktHipResample(Rv, S, 1), R),
               resample_bytes((1024,) * 3, (768,) * 3, 4, 4, every_row=True), 768 ** 3)
        free(S, Rv)
    if want("general"):
        # boxes the aligned vector path cannot take: operands at different 8-voxel phases,
        # clamped (halo) CopyRange sources, mixed formats
        m = 1024
        A, B, D = alloc((m,) * 3, 5, seed=1), alloc((m,) * 3, 5, seed=2), alloc((m,) * 3, 5)
        nv = (m - 3) * m * m
        report("general CopyRange 1021x1024x1024 UInt16 src x0=3 -> dst x0=0 (phase shift)",
               timed(lambda: lib.vktHipCopyRange(D, A, Vec3i_t(3, 0, 0), Vec3i_t(m, m, m), o), R), 4 * nv, nv)
        nv = 1000 * 1000 * 1000
        report("general CopyRange 1000^3 of 1024^3 UInt16 src (5,7,9) -> dst (1,2,3)",
               timed(lambda: lib.vktHipCopyRange(D, A, Vec3i_t(5, 7, 9), Vec3i_t(1005, 1007, 1009), Vec3i_t(1, 2, 3)),
                     R), 4 * nv, nv)
        nv = (m - 3) * m * m
        report("general SumRange 1021x1024x1024 UInt16 dstOffset x=3 (phase shift)",
               timed(lambda: lib.vktHipArithmeticRange(0, D, A, B, o, Vec3i_t(m - 3, m, m), Vec3i_t(3, 0, 0)), R),
               6 * nv, nv)
        # references: the aligned path on a multi-row box of the same shape (x0 = 8 -> 0), and the
        # general path on one collapsed row (whole volume, source view one voxel off)
        nv = (m - 8) * m * m
        report("general-ref CopyRange 1016x1024x1024 UInt16 src x0=8 -> dst x0=0 (aligned path, rows)",
               timed(lambda: lib.vktHipCopyRange(D, A, Vec3i_t(8, 0, 0), Vec3i_t(m, m, m), o), R), 4 * nv, nv)
        # partial 128-B lines at the row ends: x 64..960 covers whole lines, 64..959 / 63..959 not
        # in-process A/B of the 64-B sector completion (knob pointwise.merge_sectors), alternating
        cases = ((64, 960), (64, 959), (63, 959), (64, 952), (64, 944), (64, 928), (100, 900))
        ab = {}
        for rnd in range(3):
            for mg in (1, 0):
                lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", mg)
                for x0, x1 in cases:
                    ab.setdefault((x0, x1, mg), []).append(timed(
                        lambda: lib.vktHipCopyRange(D, A, Vec3i_t(x0, 0, 0), Vec3i_t(x1, m, m), Vec3i_t(x0, 0, 0)), R))
        lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", -1)
        for (x0, x1, mg), ts in sorted(ab.items()):
            ts.sort()
            nv = (x1 - x0) * m * m
            report(f"general-ref CopyRange rows x {x0}..{x1} of 1024^3 UInt16 (same x in src and dst) merge={mg} "
                   f"(median of 3 rounds, spread {ts[0]:.4f}-{ts[-1]:.4f})", ts[1], 4 * nv, nv)
        A1 = HipVolumeView_t(A.data + 2, m, m, m - 1, 5, 0.0, 1.0)
        nv = m * m * (m - 1)
        report("general-ref CopyRange 1024x1024x1023 UInt16, source view +1 voxel (one collapsed row, shifted)",
               timed(lambda: lib.vktHipCopyRange(D, A1, o, Vec3i_t(m, m, m - 1), o), R), 4 * nv, nv)
        free(D)
        H = alloc((m - 2,) * 3, 5)   # halo copy: (m-2)^3 dst from first=-1 .. m-1 (clamped border)
        h = m - 2
        report(f"general CopyRange clamped halo: {h}^3 from first=(-1,-1,-1) of {h - 2}^3-box UInt16",
               timed(lambda: lib.vktHipCopyRange(H, A, Vec3i_t(-1, -1, -1), Vec3i_t(h - 1, h - 1, h - 1), o), R),
               4 * h ** 3, h ** 3)
        free(H)
        F = alloc((m,) * 3, 7)
        report("general CopyRange 1024^3 UInt16 -> Float32 (convert)",
               timed(lambda: lib.vktHipCopyRange(F, A, o, Vec3i_t(m, m, m), o), R), 6 * m ** 3, m ** 3)
        free(A, B, F)
    if want("gather"):
        # non-integer ratios (gather path): up/down-sampling 768^3 <-> 1024^3, all dst formats
        cases = [(768, 1024, 5, 1), (1024, 768, 5, 1), (768, 1024, 4, 1), (768, 1024, 7, 0), (768, 1024, 7, 1),
                 (1024, 768, 7, 1), (1000, 1024, 5, 1)]
        for se, de, fmt, fm in cases:
            b = {4: 1, 5: 2, 7: 4}[fmt]
            S = alloc((se,) * 3, fmt, seed=21)
            if fmt == 7:
                rng_fill(S, se ** 3)
            Rv = alloc((de,) * 3, fmt)
            ms = timed(lambda: lib.vktHipResample(Rv, S, fm), max(3, R // 2))
            report(f"gather Resample {se}^3->{de}^3 fmt{fmt} {'Linear' if fm else 'Nearest'}", ms,
                   resample_bytes((se,) * 3, (de,) * 3, b, b, every_row=fmt == 7 and fm == 1), de ** 3)
            free(S, Rv)
    if want("gatherp"):
        # in-process A/B of the LDS gather's next-row prefetch (knob resample.prefetch), alternated
        cases = [(768, 1024, 4, 1), (1000, 1024, 4, 1), (1024, 768, 4, 1), (768, 1024, 5, 1), (1024, 768, 5, 1)]
        try:
            for se, de, fmt, fm in cases:
                b = {4: 1, 5: 2, 7: 4}[fmt]
                S = alloc((se,) * 3, fmt, seed=21)
                Rv = alloc((de,) * 3, fmt)
                for rep in range(2):
                    for k in (0, 2):
                        lib.vktHipSetTuningKnob(b"resample.prefetch", k)
                        ms = timed(lambda: lib.vktHipResample(Rv, S, fm), max(3, R // 2))
                        report(f"gatherp Resample {se}^3->{de}^3 fmt{fmt} {'Linear' if fm else 'Nearest'} "
                               f"[prefetch={k}]", ms, resample_bytes((se,) * 3, (de,) * 3, b, b), de ** 3)
                free(S, Rv)
        finally:
            lib.vktHipSetTuningKnob(b"resample.prefetch", -1)
    if want("gathera"):
        # in-process A/B: source rows that are not 16-B multiples staged in LDS (knob
        # resample.any_rows 1) vs the per-voxel gather (0)
        cases = [(1000, 1024, 4, 1), (1000, 768, 4, 1), (1000, 1024, 7, 0), (1001, 1024, 5, 1)]
        try:
            for se, de, fmt, fm in cases:
                b = {4: 1, 5: 2, 7: 4}[fmt]
                S = alloc((se,) * 3, fmt, seed=21)
                if fmt == 7:
                    rng_fill(S, se ** 3)
                Rv = alloc((de,) * 3, fmt)
                for rep in range(2):
                    for k in (0, 1):
                        lib.vktHipSetTuningKnob(b"resample.any_rows", k)
                        ms = timed(lambda: lib.vktHipResample(Rv, S, fm), max(3, R // 2))
                        report(f"gathera Resample {se}^3->{de}^3 fmt{fmt} {'Linear' if fm else 'Nearest'} "
                               f"[any_rows={k}]", ms, resample_bytes((se,) * 3, (de,) * 3, b, b), de ** 3)
                free(S, Rv)
        finally:
            lib.vktHipSetTuningKnob(b"resample.any_rows", -1)
    if want("u8gather"):
        # the UInt8 LDS gather beside UInt16 on the same ratios (Linear = Nearest
        # for integer formats), one case per launch group for the counter passes
        cases = [(1024, 768, 4), (768, 1024, 4), (1000, 1024, 4), (1024, 768, 5), (768, 1024, 5), (1000, 1024, 5)]
        for se, de, fmt in cases:
            b = {4: 1, 5: 2}[fmt]
            S = alloc((se,) * 3, fmt, seed=21)
            Rv = alloc((de,) * 3, fmt)
            ms = timed(lambda: lib.vktHipResample(Rv, S, 1), R)
            report(f"u8gather Resample {se}^3->{de}^3 fmt{fmt} Linear", ms,
                   resample_bytes((se,) * 3, (de,) * 3, b, b), de ** 3)
            free(S, Rv)
    if want("padab"):
        # in-process A/B: padded LDS rows (knob resample.lds_pad 0 / 2) on the gather shapes
        try:
            for se, de, fmt in ((1024, 768, 4), (768, 1024, 4), (1000, 1024, 4), (1024, 768, 5), (768, 1024, 5),
                                (768, 1024, 7), (1024, 768, 7)):
                b = {4: 1, 5: 2, 7: 4}[fmt]
                S = alloc((se,) * 3, fmt, seed=21)
                Rv = alloc((de,) * 3, fmt)
                for rep in range(2):
                    for pad in (0, 2):
                        lib.vktHipSetTuningKnob(b"resample.lds_pad", pad)
                        ms = timed(lambda: lib.vktHipResample(Rv, S, 0), R)
                        report(f"padab Resample {se}^3->{de}^3 fmt{fmt} Nearest [pad={pad}]", ms,
                               resample_bytes((se,) * 3, (de,) * 3, b, b), de ** 3)
                free(S, Rv)
        finally:
            lib.vktHipSetTuningKnob(b"resample.lds_pad", -1)
    if want("dstab"):
        # in-process A/B: destination-row gather (knob resample.dst_rows = grid cap in 1024s of
        # workgroups; 0 = the source-row LDS gather)
        caps = [int(c) for c in os.environ.get("VKT_DST_CAPS", "0,4,16,64,1024").split(",")]
        try:
            for se, de, fmt in ((768, 1024, 4), (1000, 1024, 4), (1024, 768, 4), (768, 1024, 5), (1024, 768, 5),
                                (1000, 1024, 5)):
                b = {4: 1, 5: 2}[fmt]
                S = alloc((se,) * 3, fmt, seed=21)
                Rv = alloc((de,) * 3, fmt)
                for rep in range(2):
                    for cap in caps:
                        lib.vktHipSetTuningKnob(b"resample.dst_rows", cap)
                        ms = timed(lambda: lib.vktHipResample(Rv, S, 1), R)
                        report(f"dstab Resample {se}^3->{de}^3 fmt{fmt} Linear [dst_rows={cap}]", ms,
                               resample_bytes((se,) * 3, (de,) * 3, b, b), de ** 3)
                free(S, Rv)
        finally:
            lib.vktHipSetTuningKnob(b"resample.dst_rows", -1)
    if want("f32lin"):
        # Float32 "Linear" (optimistic gather + fix-up) against Nearest on the
        # gather ratios; Linear's bytes: every source row (the chain's neighbours are classified)
        for se, de in ((768, 1024), (1024, 768)):
            S = alloc((se,) * 3, 7)
            rng_fill(S, se ** 3)
            Rv = alloc((de,) * 3, 7)
            for fm, lab in ((0, "Nearest"), (1, "Linear")):
                ms = timed(lambda: lib.vktHipResample(Rv, S, fm), R)
                report(f"f32lin Resample {se}^3->{de}^3 Float32 {lab}", ms,
                       resample_bytes((se,) * 3, (de,) * 3, 4, 4, every_row=fm == 1), de ** 3)
            free(S, Rv)
    if want("gpmc"):
        # one launch per case for FETCH / WRITE passes: the downsampling gathers whose bytes the
        # table image decides (UInt16: staged rows only; Float32 Linear: every source row)
        for fmt, b, fm in ((5, 2, 1), (7, 4, 1)):
            S = alloc((1024,) * 3, fmt, seed=21)
            if fmt == 7:
                rng_fill(S, 1024 ** 3)
            Rv = alloc((768,) * 3, fmt)
            ms = timed(lambda: lib.vktHipResample(Rv, S, fm), R)
            report(f"gpmc Resample 1024^3->768^3 fmt{fmt} Linear", ms,
                   resample_bytes((1024,) * 3, (768,) * 3, b, b, every_row=fmt == 7), 768 ** 3)
            free(S, Rv)
    if want("decrow"):
        # in-process A/B of the row-image BrickDecompose (knob decompose.row_image), back-to-back
        import volkit_amd.volkit as vkt
        ep = vkt.GetThreadExecutionPolicy()
        ep.device = vkt.ExecutionPolicy.Device_GPU
        vkt.SetThreadExecutionPolicy(ep)
        n = 1024
        try:
            for fmt, bs in ((vkt.DataFormat_UInt16, 16), (vkt.DataFormat_UInt8, 16), (vkt.DataFormat_UInt16, 8)):
                V = vkt.StructuredVolume(n, n, n, fmt)
                vkt.Synthesize(V, 77)
                arr = vkt.Array3D_StructuredVolume()
                b3, h3 = vkt.Vec3i(bs, bs, bs), vkt.Vec3i(1, 1, 1)
                vkt.BrickDecomposeResize(arr, V, b3, h3, h3)
                bpv = 1 if fmt == vkt.DataFormat_UInt8 else 2
                vox = (bs + 2) ** 3 * (n // bs) ** 3
                for rep in range(2):
                    for k in (0, 1):
                        lib.vktHipSetTuningKnob(b"decompose.row_image", 1 if k else 0)
                        ms = pipelined(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R)
                        report(f"decrow BrickDecompose 1024^3 bpv{bpv} -> {bs}^3 bricks halo 1 back-to-back "
                               f"[row_image={k}]", ms, 2 * bpv * vox, vox)
                del arr, V
        finally:
            lib.vktHipSetTuningKnob(b"decompose.row_image", -1)
    if want("decompose"):
        # BrickDecompose: 1024^3 UInt16 into 64^3 bricks with a 1-voxel halo
        import volkit_amd.volkit as vkt
        ep = vkt.GetThreadExecutionPolicy()
        ep.device = vkt.ExecutionPolicy.Device_GPU
        vkt.SetThreadExecutionPolicy(ep)
        n = 1024
        cases = [(64, (1, 1, 1)), (128, (0, 0, 0)), (32, (1, 1, 1)), (16, (1, 1, 1))]
        if os.environ.get("VKT_DECOMP_CASES"):   # "bs:hx,hy,hz;..."
            cases = [(int(c.split(":")[0]), tuple(int(h) for h in c.split(":")[1].split(",")))
                     for c in os.environ["VKT_DECOMP_CASES"].split(";")]
        for bs, halo in cases:
            V = vkt.StructuredVolume(n, n, n, vkt.DataFormat_UInt16)
            vkt.Synthesize(V, 77)
            arr = vkt.Array3D_StructuredVolume()
            b3, h3 = vkt.Vec3i(bs, bs, bs), vkt.Vec3i(*halo)
            vkt.BrickDecomposeResize(arr, V, b3, h3, h3)
            vox = sum(arr[(i, j, k)].getSizeInBytes() // 2 for k in range(arr.dims().z)
                      for j in range(arr.dims().y) for i in range(arr.dims().x))
            ms = timed(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R)
            report(f"decompose BrickDecompose 1024^3 UInt16 -> {bs}^3 bricks halo {halo} (incl. host planning)",
                   ms, 4 * vox, vox)
            ms = pipelined(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R)
            report(f"decompose BrickDecompose 1024^3 UInt16 -> {bs}^3 bricks halo {halo} (back-to-back calls)",
                   ms, 4 * vox, vox)
            del arr, V
        ep.device = vkt.ExecutionPolicy.Device_CPU
        vkt.SetThreadExecutionPolicy(ep)
    if want("decblk"):
        # in-process A/B of the threads per BrickDecompose workgroup (knob decompose.block: 256, 128
        # -- the same 16-KiB chunk, twice the items and staged words per thread with 128)
        import volkit_amd.volkit as vkt
        ep = vkt.GetThreadExecutionPolicy()
        ep.device = vkt.ExecutionPolicy.Device_GPU
        vkt.SetThreadExecutionPolicy(ep)
        n = 1024
        V = vkt.StructuredVolume(n, n, n, vkt.DataFormat_UInt16)
        vkt.Synthesize(V, 77)
        ab = {}
        for bs, halo in ((16, (1, 1, 1)), (32, (1, 1, 1)), (64, (1, 1, 1))):
            arr = vkt.Array3D_StructuredVolume()
            b3, h3 = vkt.Vec3i(bs, bs, bs), vkt.Vec3i(*halo)
            vkt.BrickDecomposeResize(arr, V, b3, h3, h3)
            vox = sum(arr[(i, j, k)].getSizeInBytes() // 2 for k in range(arr.dims().z)
                      for j in range(arr.dims().y) for i in range(arr.dims().x))
            for rnd in range(3):
                for kv in (256, 128):
                    lib.vktHipSetTuningKnob(b"decompose.block", kv)
                    ab.setdefault((bs, halo, kv, vox, "back-to-back"), []).append(
                        pipelined(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R))
                    ab.setdefault((bs, halo, kv, vox, "incl. host planning"), []).append(
                        timed(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R))
            del arr
        lib.vktHipSetTuningKnob(b"decompose.block", -1)
        for (bs, halo, kv, vox, how), ts in sorted(ab.items()):
            ts.sort()
            report(f"decblk BrickDecompose 1024^3 UInt16 -> {bs}^3 bricks halo {halo} block={kv} ({how}; median of 3 "
                   f"rounds, spread {ts[0]:.4f}-{ts[-1]:.4f})", ts[1], 4 * vox, vox)
        del V
        ep.device = vkt.ExecutionPolicy.Device_CPU
        vkt.SetThreadExecutionPolicy(ep)
    if want("decab"):
        # in-process A/B of the staged copy's LDS writes (knob decompose.aligned_lds: 0 unaligned
        # 16-B words + per-voxel row ends, 1 row-end words as aligned pieces, 2 every word)
        import volkit_amd.volkit as vkt
        ep = vkt.GetThreadExecutionPolicy()
        ep.device = vkt.ExecutionPolicy.Device_GPU
        vkt.SetThreadExecutionPolicy(ep)
        n = 1024
        V = vkt.StructuredVolume(n, n, n, vkt.DataFormat_UInt16)
        vkt.Synthesize(V, 77)
        ab = {}
        cases = ((16, (1, 1, 1)), (32, (1, 1, 1)), (64, (1, 1, 1)), (128, (0, 0, 0)), (256, (1, 1, 1)))
        if os.environ.get("VKT_DECAB_SIZES"):   # e.g. "16,32"
            keep = {int(x) for x in os.environ["VKT_DECAB_SIZES"].split(",")}
            cases = tuple(c for c in cases if c[0] in keep)
        for bs, halo in cases:
            arr = vkt.Array3D_StructuredVolume()
            b3, h3 = vkt.Vec3i(bs, bs, bs), vkt.Vec3i(*halo)
            vkt.BrickDecomposeResize(arr, V, b3, h3, h3)
            vox = sum(arr[(i, j, k)].getSizeInBytes() // 2 for k in range(arr.dims().z)
                      for j in range(arr.dims().y) for i in range(arr.dims().x))
            for rnd in range(3):
                for kv in ((0, 5), (1, 5), (0, 6), (1, 6), (2, 6), (0, 8)):   # (aligned_lds, stage_words)
                    lib.vktHipSetTuningKnob(b"decompose.aligned_lds", kv[0])
                    lib.vktHipSetTuningKnob(b"decompose.stage_words", kv[1])
                    ab.setdefault((bs, halo, kv, vox), []).append(
                        pipelined(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R))
            del arr
        lib.vktHipSetTuningKnob(b"decompose.aligned_lds", -1)
        lib.vktHipSetTuningKnob(b"decompose.stage_words", -1)
        for (bs, halo, kv, vox), ts in sorted(ab.items()):
            ts.sort()
            report(f"decab BrickDecompose 1024^3 UInt16 -> {bs}^3 bricks halo {halo} aligned_lds={kv[0]} "
                   f"stage_words={kv[1]} "
                   f"(back-to-back, median of 3 rounds, spread {ts[0]:.4f}-{ts[-1]:.4f})", ts[1], 4 * vox, vox)
        del V
        ep.device = vkt.ExecutionPolicy.Device_CPU
        vkt.SetThreadExecutionPolicy(ep)
    if want("decgrid"):
        # in-process A/B of grid-derived brick descriptors (knob decompose.grid): back-to-back and
        # single synchronised calls, median of 3 rounds
        import volkit_amd.volkit as vkt
        ep = vkt.GetThreadExecutionPolicy()
        ep.device = vkt.ExecutionPolicy.Device_GPU
        vkt.SetThreadExecutionPolicy(ep)
        n = 1024
        V = vkt.StructuredVolume(n, n, n, vkt.DataFormat_UInt16)
        vkt.Synthesize(V, 77)
        ab = {}
        for bs, halo in ((16, (1, 1, 1)), (32, (1, 1, 1)), (64, (1, 1, 1)), (128, (0, 0, 0))):
            arr = vkt.Array3D_StructuredVolume()
            b3, h3 = vkt.Vec3i(bs, bs, bs), vkt.Vec3i(*halo)
            vkt.BrickDecomposeResize(arr, V, b3, h3, h3)
            vox = sum(arr[(i, j, k)].getSizeInBytes() // 2 for k in range(arr.dims().z)
                      for j in range(arr.dims().y) for i in range(arr.dims().x))
            for rnd in range(3):
                for k in (1, 0):
                    lib.vktHipSetTuningKnob(b"decompose.grid", k)
                    ab.setdefault((bs, halo, k, "back-to-back", vox), []).append(
                        pipelined(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R))
                    ab.setdefault((bs, halo, k, "incl. host planning", vox), []).append(
                        timed(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R))
            del arr
        lib.vktHipSetTuningKnob(b"decompose.grid", -1)
        for (bs, halo, k, how, vox), ts in sorted(ab.items()):
            ts.sort()
            report(f"decgrid BrickDecompose 1024^3 UInt16 -> {bs}^3 bricks halo {halo} grid={k} ({how}, median of 3 "
                   f"rounds, spread {ts[0]:.4f}-{ts[-1]:.4f})", ts[1], 4 * vox, vox)
        del V
        ep.device = vkt.ExecutionPolicy.Device_CPU
        vkt.SetThreadExecutionPolicy(ep)
    if want("memresize"):
        # BrickDecomposeResize (one StructuredVolume per brick, allocated on the device) with the
        # small-buffer pool on / off (knob memory.pool): host wall time of the resize, and of a
        # second resize over the same array (the first one's bricks freed, their blocks reused)
        import time
        import volkit_amd.volkit as vkt
        ep = vkt.GetThreadExecutionPolicy()
        ep.device = vkt.ExecutionPolicy.Device_GPU
        vkt.SetThreadExecutionPolicy(ep)
        n = 1024
        V = vkt.StructuredVolume(n, n, n, vkt.DataFormat_UInt16)
        vkt.Synthesize(V, 77)
        arrs = {}
        for bs in (32, 16):
            for k in (1, 0):
                lib.vktHipSetTuningKnob(b"memory.pool", k)
                arr = vkt.Array3D_StructuredVolume()
                b3, h3 = vkt.Vec3i(bs, bs, bs), vkt.Vec3i(1, 1, 1)
                t0 = time.perf_counter()
                vkt.BrickDecomposeResize(arr, V, b3, h3, h3)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                vkt.BrickDecomposeResize(arr, V, b3, h3, h3)
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                nb = arr.dims().x * arr.dims().y * arr.dims().z
                print(json.dumps({"case": f"memresize BrickDecomposeResize 1024^3 -> {bs}^3 bricks halo 1 pool={k}",
                                  "bricks": nb, "first_ms": round((t1 - t0) * 1e3, 2),
                                  "again_ms": round((t2 - t1) * 1e3, 2)}), flush=True)
                arrs[(bs, k)] = arr
            # the decomposition into bricks from the pool vs from one hipMalloc each, alternating
            b3, h3 = vkt.Vec3i(bs, bs, bs), vkt.Vec3i(1, 1, 1)
            ts = {}
            for rnd in range(3):
                for k in (1, 0):
                    ts.setdefault(k, []).append(pipelined(lambda: vkt.BrickDecompose(arrs[(bs, k)], V, b3, h3, h3), R))
            for k, v in ts.items():
                v.sort()
                print(json.dumps({"case": f"memresize BrickDecompose into {bs}^3 bricks halo 1 pool={k} (back-to-back, "
                                  f"median of 3 rounds, spread {v[0]:.4f}-{v[-1]:.4f})", "ms": round(v[1], 4)}), flush=True)
            arrs.clear()
        lib.vktHipSetTuningKnob(b"memory.pool", -1)
        del V
        ep.device = vkt.ExecutionPolicy.Device_CPU
        vkt.SetThreadExecutionPolicy(ep)
    if want("decpmc"):
        # one case for PMC passes (VKT_KNOBS picks the variant): 32^3 bricks + halo 1
        import volkit_amd.volkit as vkt
        ep = vkt.GetThreadExecutionPolicy()
        ep.device = vkt.ExecutionPolicy.Device_GPU
        vkt.SetThreadExecutionPolicy(ep)
        V = vkt.StructuredVolume(1024, 1024, 1024, vkt.DataFormat_UInt16)
        vkt.Synthesize(V, 77)
        arr = vkt.Array3D_StructuredVolume()
        b3, h3 = vkt.Vec3i(32, 32, 32), vkt.Vec3i(1, 1, 1)
        vkt.BrickDecomposeResize(arr, V, b3, h3, h3)
        vox = sum(arr[(i, j, k)].getSizeInBytes() // 2 for k in range(arr.dims().z)
                  for j in range(arr.dims().y) for i in range(arr.dims().x))
        report("decpmc BrickDecompose 1024^3 UInt16 -> 32^3 bricks halo 1", timed(
            lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R), 4 * vox, vox)
        del arr, V
        ep.device = vkt.ExecutionPolicy.Device_CPU
        vkt.SetThreadExecutionPolicy(ep)
    if want("fmts"):
        # every data format through each hot-path call at 512^3 (per-format fall-backs show up as
        # outliers): Fill, Copy, SumRange, SafeSum, Resample up (integer ratio) / down (gather),
        # Aggregates, Histogram 256 bins
        m = 512
        lastm = Vec3i_t(m, m, m)
        bins = C.c_void_p()
        lib.vktHipAllocate(C.byref(bins), 256 * 8)
        names = {1: "Int8", 2: "Int16", 3: "Int32", 4: "UInt8", 5: "UInt16", 6: "UInt32", 7: "Float32"}
        try:
            for fmt in (4, 5, 7, 2, 6):   # (Int8 / Int32: the reference's codec leaves them untouched)
                b = BPV[fmt]
                A, B2, D = alloc((m,) * 3, fmt, seed=1), alloc((m,) * 3, fmt, seed=2), alloc((m,) * 3, fmt)
                if fmt == 7:
                    rng_fill(A, m ** 3)
                    rng_fill(B2, m ** 3)
                nv = m ** 3
                nm = names[fmt]
                report(f"fmts FillRange 512^3 {nm}", timed(lambda: lib.vktHipFillRange(D, o, lastm, C.c_float(0.3)), R),
                       b * nv, nv)
                report(f"fmts CopyRange 512^3 {nm}", timed(lambda: lib.vktHipCopyRange(D, A, o, lastm, o), R), 2 * b * nv, nv)
                report(f"fmts SumRange 512^3 {nm}", timed(lambda: lib.vktHipArithmeticRange(0, D, A, B2, o, lastm, o), R),
                       3 * b * nv, nv)
                report(f"fmts SafeSumRange 512^3 {nm}",
                       timed(lambda: lib.vktHipArithmeticRange(5, D, A, B2, o, lastm, o), R), 3 * b * nv, nv)
                S = alloc((256,) * 3, fmt, seed=3)
                report(f"fmts Resample 256^3->512^3 {nm} Linear", timed(lambda: lib.vktHipResample(D, S, 1), R),
                       b * 256 ** 3 + b * nv, nv)
                Rd = alloc((384,) * 3, fmt)
                report(f"fmts Resample 512^3->384^3 {nm} Nearest", timed(lambda: lib.vktHipResample(Rd, A, 0), R),
                       resample_bytes((m,) * 3, (384,) * 3, b, b), 384 ** 3)
                agg = _lib.Aggregates_t()
                report(f"fmts Aggregates 512^3 {nm}", timed(lambda: lib.vktHipAggregatesRange(A, o, lastm, C.byref(agg)), R),
                       b * nv, nv)
                report(f"fmts Histogram 512^3 {nm} 256 bins",
                       timed(lambda: lib.vktHipHistogramRange(A, o, lastm, bins, 256, 0), R), b * nv, nv)
                free(A, B2, D, S, Rd)
        finally:
            lib.vktHipFree(bins)
    if want("f32small"):
        # Float32 Linear Resample at small sizes (fixed cost vs voxels)
        for se, de in ((256, 512), (512, 1024), (384, 512)):
            S = alloc((se,) * 3, 7)
            rng_fill(S, se ** 3)
            Rv = alloc((de,) * 3, 7)
            report(f"f32small Resample {se}^3->{de}^3 Float32 Linear", timed(lambda: lib.vktHipResample(Rv, S, 1), R),
                   4 * se ** 3 + 4 * de ** 3, de ** 3)
            free(S, Rv)
    if want("aggfix"):
        # ComputeAggregates per call at 256^3 / 512^3 for every format (fixed cost vs voxels)
        names = {2: "Int16", 4: "UInt8", 5: "UInt16", 6: "UInt32", 7: "Float32"}
        for m in (256, 512, 1024):
            lastm = Vec3i_t(m, m, m)
            for fmt in (4, 5, 7, 2, 6):
                A = alloc((m,) * 3, fmt, seed=1)
                if fmt == 7:
                    rng_fill(A, m ** 3)
                agg = _lib.Aggregates_t()
                for k in ((3, 7) if fmt in (2, 6) else (-1,)):
                    lib.vktHipSetTuningKnob(b"aggregates.moments", k)
                    report(f"aggfix Aggregates {m}^3 {names[fmt]} [moments={k}]",
                           timed(lambda: lib.vktHipAggregatesRange(A, o, lastm, C.byref(agg)), R), BPV[fmt] * m ** 3,
                           m ** 3)
                lib.vktHipSetTuningKnob(b"aggregates.moments", -1)
                free(A)
    if want("p16size"):
        # the packed-16 histogram (UInt16, 65 536 integer bins) over volume sizes: time vs voxels
        bins = C.c_void_p()
        lib.vktHipAllocate(C.byref(bins), 65536 * 8)
        try:
            for n in (256, 512, 768, 1024):
                last = Vec3i_t(n, n, n)
                V = alloc((n,) * 3, 5, seed=11)
                ms = timed(lambda: lib.vktHipHistogramRange(V, o, last, bins, 65536, 0), R)
                report(f"p16size Histogram {n}^3 UInt16 65536 bins", ms, 2 * n ** 3, n ** 3)
                free(V)
        finally:
            lib.vktHipFree(bins)
    if want("p16tiles"):
        # knob histogram.packed16 = 2: more bins than one packed-16 launch holds (Float32; UInt16
        # with the code counts off) in packed-16 tiles, one pass per tile, vs PAIR / 32-bit tiles (1)
        n = 1024
        last = Vec3i_t(n, n, n)
        bins = C.c_void_p()
        lib.vktHipAllocate(C.byref(bins), 300000 * 8)
        lib.vktHipSetTuningKnob(b"histogram.u16_codes", 0)
        try:
            for fmt, b in ((7, 4), (5, 2)):
                V = alloc((n,) * 3, fmt, -1.0, 3.0, seed=11 if fmt == 5 else None)
                if fmt == 7:
                    rng_fill(V, n ** 3)
                for nb in (100000, 150000, 300000):
                    for rep in range(2):
                        for k in (1, 2):
                            lib.vktHipSetTuningKnob(b"histogram.packed16", k)
                            ms = timed(lambda: lib.vktHipHistogramRange(V, o, last, bins, nb, 0), R)
                            report(f"p16tiles Histogram 1024^3 fmt={fmt} {nb} bins [packed16={k}]", ms, b * n ** 3,
                                   n ** 3)
                free(V)
        finally:
            lib.vktHipSetTuningKnob(b"histogram.packed16", -1)
            lib.vktHipSetTuningKnob(b"histogram.u16_codes", -1)
            lib.vktHipFree(bins)
    if want("partials"):
        # knob histogram.partials: tiled histogram launches store per-workgroup counts summed by
        # one kernel (1) vs global 64-bit atomics per counter (0)
        bins = C.c_void_p()
        lib.vktHipAllocate(C.byref(bins), 200000 * 8)
        try:
            for n in (1024, 512):
                last = Vec3i_t(n, n, n)
                for fmt, lo, hi, nbs in ((5, 0.0, 1.0, (65536, 100000)), (5, -1.0, 3.0, (20000, 65536)),
                                         (7, 0.0, 1.0, (20000, 65536, 150000)), (2, 0.0, 1.0, (256,))):
                    b = BPV[fmt]
                    V = alloc((n,) * 3, fmt, lo, hi, seed=11 if fmt != 7 else None)
                    if fmt == 7:
                        rng_fill(V, n ** 3)
                    for nb in nbs:
                        for rep in range(2):
                            for k in (0, 1, 2):
                                lib.vktHipSetTuningKnob(b"histogram.partials", k)
                                ms = timed(lambda: lib.vktHipHistogramRange(V, o, last, bins, nb, 0), R)
                                report(f"partials Histogram {n}^3 fmt={fmt} map=({lo},{hi}) {nb} bins [partials={k}]",
                                       ms, b * n ** 3, n ** 3)
                    free(V)
        finally:
            lib.vktHipSetTuningKnob(b"histogram.partials", -1)
            lib.vktHipFree(bins)
    if want("u16codes"):
        # knob histogram.u16_codes: UInt16 float-formula bins through one pass of code counts and a
        # fold (1: beyond one LDS tile, 2: also single-tile bins) vs the per-voxel kernels (0)
        n = 1024
        bins = C.c_void_p()
        lib.vktHipAllocate(C.byref(bins), 1000000 * 8)
        last = Vec3i_t(n, n, n)
        try:
            for lo, hi in ((0.0, 1.0), (-1.0, 3.0)):
                V = alloc((n,) * 3, 5, lo, hi, seed=11)
                cases = (20000, 100000, 150000, 1000000) if lo == 0.0 else (20000, 50000, 65536)
                for nb in cases:
                    for rep in range(2):
                        for k in (0, 1, 2):
                            lib.vktHipSetTuningKnob(b"histogram.u16_codes", k)
                            ms = timed(lambda: lib.vktHipHistogramRange(V, o, last, bins, nb, 0), R)
                            report(f"u16codes Histogram 1024^3 UInt16 map=({lo},{hi}) {nb} bins [u16_codes={k}]", ms,
                                   2 * n ** 3, n ** 3)
                u0, u1 = Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900)
                for k in (0, 1):
                    lib.vktHipSetTuningKnob(b"histogram.u16_codes", k)
                    ms = timed(lambda: lib.vktHipHistogramRange(V, u0, u1, bins, 100000, 0), R)
                    report(f"u16codes Histogram 800^3 at x0=100 UInt16 map=({lo},{hi}) 100000 bins [u16_codes={k}]",
                           ms, 2 * 800 ** 3, 800 ** 3)
                free(V)
            V = alloc((n,) * 3, 2, seed=11)   # Int16: the per-row kernel (0) vs the code counts (1)
            for nb in (256, 100000):
                for rep in range(2):
                    for k in (0, 1):
                        lib.vktHipSetTuningKnob(b"histogram.u16_codes", k)
                        ms = timed(lambda: lib.vktHipHistogramRange(V, o, last, bins, nb, 0), R)
                        report(f"u16codes Histogram 1024^3 Int16 {nb} bins [u16_codes={k}]", ms, 2 * n ** 3, n ** 3)
            free(V)
        finally:
            lib.vktHipSetTuningKnob(b"histogram.u16_codes", -1)
            lib.vktHipFree(bins)
    if want("pairtiles"):
        # knob histogram.pair_tiles: the tiles of a > 40 704-bin histogram side by side in one
        # launch (XCD-grouped workgroups) vs P16 (65 536 bins) / one pass per tile (more bins)
        n = 1024
        bins = C.c_void_p()
        lib.vktHipAllocate(C.byref(bins), 150000 * 8)
        last = Vec3i_t(n, n, n)
        lib.vktHipSetTuningKnob(b"histogram.u16_codes", 0)   # (the tiled kernels, not the code counts)
        lib.vktHipSetTuningKnob(b"histogram.packed16", 1)    # (PAIR, not packed-16 tiles)
        try:
            for fmt, b in ((5, 2), (7, 4)):
                V = alloc((n,) * 3, fmt, seed=11 if fmt == 5 else None)
                if fmt == 7:
                    rng_fill(V, n ** 3)
                for nb in ((65536, 50000, 100000, 150000) if fmt == 5 else (65536, 100000)):
                    for rep in range(2):
                        for k in (0, 2):
                            lib.vktHipSetTuningKnob(b"histogram.pair_tiles", k)
                            ms = timed(lambda: lib.vktHipHistogramRange(V, o, last, bins, nb, 0), R)
                            report(f"pairtiles Histogram 1024^3 fmt={fmt} {nb} bins [pair_tiles={k}]", ms,
                                   b * n ** 3, n ** 3)
                u0, u1 = Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900)
                for k in (0, 2):
                    lib.vktHipSetTuningKnob(b"histogram.pair_tiles", k)
                    ms = timed(lambda: lib.vktHipHistogramRange(V, u0, u1, bins, 65536, 0), R)
                    report(f"pairtiles Histogram 800^3 at x0=100 fmt={fmt} 65536 bins [pair_tiles={k}]", ms,
                           b * 800 ** 3, 800 ** 3)
                free(V)
        finally:
            lib.vktHipSetTuningKnob(b"histogram.pair_tiles", -1)
            lib.vktHipSetTuningKnob(b"histogram.u16_codes", -1)
            lib.vktHipSetTuningKnob(b"histogram.packed16", -1)
            lib.vktHipFree(bins)
    if want("reduce"):
        # ComputeHistogram / ComputeAggregates on a device-resident 1024^3 UInt16
        n = 1024
        V = alloc((n,) * 3, 5, seed=11)
        last = Vec3i_t(n, n, n)
        bins = C.c_void_p()
        lib.vktHipAllocate(C.byref(bins), 65536 * 8)
        for nb in (256, 1024, 4096, 10240, 65536):
            ms = timed(lambda: lib.vktHipHistogramRange(V, o, last, bins, nb, 0), R)
            report(f"reduce Histogram 1024^3 UInt16 {nb} bins", ms, 2 * n ** 3, n ** 3)
        # one pass over packed 16-bit counters vs one pass per LDS tile (knob histogram.packed16),
        # integer bins (unit mapping) and float bins (mapping [-1, 3] on the same codes: 50 000 bins)
        lib.vktHipSetTuningKnob(b"histogram.packed16", 0)
        ms = timed(lambda: lib.vktHipHistogramRange(V, o, last, bins, 65536, 0), R)
        report("reduce Histogram 1024^3 UInt16 65536 bins [one pass per tile]", ms, 2 * n ** 3, n ** 3)
        lib.vktHipSetTuningKnob(b"histogram.packed16", -1)
        # mul-shift bins ((code * numBins) >> 16, host-verified) vs the float formula
        for nb in (10240, 40960, 65535):
            for k in (1, 0):
                lib.vktHipSetTuningKnob(b"histogram.mulshift", k)
                ms = timed(lambda: lib.vktHipHistogramRange(V, o, last, bins, nb, 0), R)
                report(f"reduce Histogram 1024^3 UInt16 {nb} bins [mulshift={k}]", ms, 2 * n ** 3, n ** 3)
            lib.vktHipSetTuningKnob(b"histogram.mulshift", -1)
        # P16 threshold tests once per wave-step vs after every item
        for k in (1, 0):
            lib.vktHipSetTuningKnob(b"histogram.p16_step", k)
            ms = timed(lambda: lib.vktHipHistogramRange(V, o, last, bins, 65536, 0), R)
            report(f"reduce Histogram 1024^3 UInt16 65536 bins [p16_step={k}]", ms, 2 * n ** 3, n ** 3)
        lib.vktHipSetTuningKnob(b"histogram.p16_step", -1)
        sub0, sub1 = Vec3i_t(64, 64, 64), Vec3i_t(960, 960, 960)
        ms = timed(lambda: lib.vktHipHistogramRange(V, sub0, sub1, bins, 256, 0), R)
        report("reduce Histogram UInt16 896^3 sub-box of 1024^3, 256 bins", ms, 2 * 896 ** 3, 896 ** 3)
        # rows that start and end off the 8-voxel grid (x 100..900)
        u0, u1 = Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900)
        ms = timed(lambda: lib.vktHipHistogramRange(V, u0, u1, bins, 256, 0), R)
        report("reduce Histogram UInt16 800^3 sub-box of 1024^3 at x0=100, 256 bins", ms, 2 * 800 ** 3, 800 ** 3)
        agg0 = _lib.Aggregates_t()
        two_float_passes(True)   # UInt16: the two float passes
        ms = timed(lambda: lib.vktHipAggregatesRange(V, u0, u1, C.byref(agg0)), R)
        two_float_passes(False)
        report("reduce Aggregates UInt16 800^3 sub-box of 1024^3 at x0=100 (2 passes)", ms, 2 * 2 * 800 ** 3, 800 ** 3)
        for fmt, bpv, name in ((4, 1, "UInt8"), (7, 4, "Float32")):
            W = alloc((n,) * 3, fmt, seed=12 if fmt != 7 else None)
            if fmt == 7:
                rng_fill(W, n ** 3)   # uniform [0, 1): every voxel lands in a bin
            ms = timed(lambda: lib.vktHipHistogramRange(W, o, last, bins, 256, 0), R)
            report(f"reduce Histogram 1024^3 {name} 256 bins", ms, bpv * n ** 3, n ** 3)
            aggW = _lib.Aggregates_t()
            ms = timed(lambda: lib.vktHipAggregatesRange(W, o, last, C.byref(aggW)), R)
            if fmt == 4:   # one pass of code counts (knob aggregates.codes)
                report(f"reduce Aggregates 1024^3 {name} (1 pass of code counts, incl. D2H of the result)", ms,
                       bpv * n ** 3, n ** 3)
            else:          # one pass of float moments (knob aggregates.moments bit 1)
                report(f"reduce Aggregates 1024^3 {name} (1 pass of float moments, incl. D2H of the result)", ms,
                       bpv * n ** 3, n ** 3)
                two_float_passes(True)
                ms = timed(lambda: lib.vktHipAggregatesRange(W, o, last, C.byref(aggW)), R)
                two_float_passes(False)
                report(f"reduce Aggregates 1024^3 {name} (2 passes, incl. D2H of the result)", ms, 2 * bpv * n ** 3,
                       n ** 3)
            free(W)
        Vc = alloc((n,) * 3, 5)
        lib.vktHipFillRange(Vc, o, last, C.c_float(0.5))
        ms = timed(lambda: lib.vktHipHistogramRange(Vc, o, last, bins, 256, 0), R)
        report("reduce Histogram 1024^3 UInt16 256 bins, constant volume", ms, 2 * n ** 3, n ** 3)
        for nb in (20000, 65536):   # the tiled / packed-16 paths (no counter replicas)
            ms = timed(lambda: lib.vktHipHistogramRange(Vc, o, last, bins, nb, 0), R)
            report(f"reduce Histogram 1024^3 UInt16 {nb} bins, constant volume", ms, 2 * n ** 3, n ** 3)
        agg = _lib.Aggregates_t()
        two_float_passes(True)   # UInt16: the two float passes
        ms = timed(lambda: lib.vktHipAggregatesRange(V, o, last, C.byref(agg)), R)
        two_float_passes(False)
        report("reduce Aggregates 1024^3 UInt16 (2 passes, incl. D2H of the result)", ms, 2 * 2 * n ** 3, n ** 3)
        free(V, Vc)
        lib.vktHipFree(bins)
    if want("aggcodes"):
        # UInt8 ComputeAggregates: one pass of code counts vs the two float passes (knob
        # aggregates.codes), whole volume and the 800^3 sub-box at x0 = 100 (padded rows)
        n = 1024
        W = alloc((n,) * 3, 4, seed=12)
        last = Vec3i_t(n, n, n)
        u0, u1 = Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900)
        agg = _lib.Aggregates_t()
        for k in (1, 0):
            lib.vktHipSetTuningKnob(b"aggregates.codes", k)
            passes = 1 if k else 2
            ms = timed(lambda: lib.vktHipAggregatesRange(W, o, last, C.byref(agg)), R)
            report(f"aggcodes Aggregates 1024^3 UInt8 [codes={k}, {passes} pass(es)]", ms, passes * n ** 3, n ** 3)
            ms = timed(lambda: lib.vktHipAggregatesRange(W, u0, u1, C.byref(agg)), R)
            report(f"aggcodes Aggregates UInt8 800^3 sub-box at x0=100 [codes={k}, {passes} pass(es)]", ms,
                   passes * 800 ** 3, 800 ** 3)
        lib.vktHipSetTuningKnob(b"aggregates.codes", -1)
        # the code-count walk over range rows: 16-voxel items + row-end subtraction vs 8-voxel items
        hb = C.c_void_p()
        if lib.vktHipAllocate(C.byref(hb), 256 * 8) != 0:
            raise RuntimeError(_lib.last_error())
        hbins = C.c_void_p(hb.value)
        for k in (1, 2, 0):
            lib.vktHipSetTuningKnob(b"reduce.u8_rows16", k)
            for (a0, a1, what) in ((u0, u1, "800^3 sub-box at x0=100"),
                                   (Vec3i_t(0, 100, 100), Vec3i_t(800, 900, 900), "800^3 sub-box x 0..800"),
                                   (Vec3i_t(3, 0, 0), Vec3i_t(1021, n, n), "1018x1024^2 x 3..1021"),
                                   (Vec3i_t(3, 0, 0), Vec3i_t(67, 64, 64), "64^3 box (fixed cost)")):
                nv = (a1.x - a0.x) * (a1.y - a0.y) * (a1.z - a0.z)
                ms = timed(lambda: lib.vktHipAggregatesRange(W, a0, a1, C.byref(agg)), R)
                report(f"aggcodes Aggregates UInt8 {what} [rows16={k}]", ms, nv, nv)
                ms = timed(lambda: lib.vktHipHistogramRange(W, a0, a1, hbins, 256, 0), R)
                report(f"aggcodes Histogram UInt8 {what}, 256 bins [rows16={k}]", ms, nv, nv)
        lib.vktHipSetTuningKnob(b"reduce.u8_rows16", -1)
        lib.vktHipFree(hb)
        free(W)
        V = alloc((n,) * 3, 5, seed=11)
        lib.vktHipSetTuningKnob(b"aggregates.moments", 0)   # (moments would take both cases)
        for k in (3, 1):
            lib.vktHipSetTuningKnob(b"aggregates.codes", k)
            passes = 1 if k & 2 else 2
            ms = timed(lambda: lib.vktHipAggregatesRange(V, o, last, C.byref(agg)), R)
            report(f"aggcodes Aggregates 1024^3 UInt16 [codes={k}, {passes} pass(es)]", ms, passes * 2 * n ** 3, n ** 3)
            ms = timed(lambda: lib.vktHipAggregatesRange(V, u0, u1, C.byref(agg)), R)
            report(f"aggcodes Aggregates UInt16 800^3 sub-box at x0=100 [codes={k}, {passes} pass(es)]", ms,
                   passes * 2 * 800 ** 3, 800 ** 3)
            a0, a1 = Vec3i_t(0, 100, 100), Vec3i_t(800, 900, 900)
            ms = timed(lambda: lib.vktHipAggregatesRange(V, a0, a1, C.byref(agg)), R)
            report(f"aggcodes Aggregates UInt16 800^3 sub-box x 0..800 [codes={k}, {passes} pass(es)]", ms,
                   passes * 2 * 800 ** 3, 800 ** 3)
        lib.vktHipSetTuningKnob(b"aggregates.codes", -1)
        lib.vktHipSetTuningKnob(b"aggregates.moments", -1)
        free(V)
    if want("moments"):
        # UInt16 ComputeAggregates under the unit mapping: one pass of integer moments (knob
        # aggregates.moments) vs the packed-16 code counts vs the two float passes; per call,
        # incl. the D2H of the result.  Bytes: one read of the range.
        n = 1024
        V = alloc((n,) * 3, 5, seed=11)
        last = Vec3i_t(n, n, n)
        agg = _lib.Aggregates_t()
        boxes = ((o, last, "1024^3"), (Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900), "800^3 sub-box at x0=100"),
                 (Vec3i_t(0, 100, 100), Vec3i_t(800, 900, 900), "800^3 sub-box x 0..800"),
                 (Vec3i_t(3, 0, 0), Vec3i_t(67, 64, 64), "64^3 box (fixed cost)"))
        for mom, codes, what in ((1, 3, "moments"), (0, 3, "code counts"), (0, 1, "2 float passes")):
            lib.vktHipSetTuningKnob(b"aggregates.moments", mom)
            lib.vktHipSetTuningKnob(b"aggregates.codes", codes)
            for a0, a1, box in boxes:
                nv = (a1.x - a0.x) * (a1.y - a0.y) * (a1.z - a0.z)
                ms = timed(lambda: lib.vktHipAggregatesRange(V, a0, a1, C.byref(agg)), R)
                report(f"moments Aggregates UInt16 {box} [{what}]", ms, 2 * nv, nv)
        lib.vktHipSetTuningKnob(b"aggregates.moments", -1)
        lib.vktHipSetTuningKnob(b"aggregates.codes", -1)
        free(V)
    if want("mompipe"):
        # in-process A/B of the integer-moments kernel variants (knob aggregates.moments_pipe: 0
        # one buffer x 4 items, 1 two buffers x 4 items, 3 one buffer x 8, 4 two x 2, 5 as 1 at 7 waves
        # per SIMD), per call incl.
        # the D2H of the result, median of 3 rounds
        n = 1024
        V = alloc((n,) * 3, 5, seed=11)
        agg = _lib.Aggregates_t()
        boxes = ((o, Vec3i_t(n, n, n), "1024^3"), (Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900), "800^3 sub-box at x0=100"),
                 (Vec3i_t(0, 100, 100), Vec3i_t(800, 900, 900), "800^3 sub-box x 0..800"))
        ab = {}
        for rnd in range(3):
            for pv in (0, 1, 3, 4, 5):
                lib.vktHipSetTuningKnob(b"aggregates.moments_pipe", pv)
                for a0, a1, box in boxes:
                    ab.setdefault((box, pv), []).append(
                        timed(lambda: lib.vktHipAggregatesRange(V, a0, a1, C.byref(agg)), R))
        lib.vktHipSetTuningKnob(b"aggregates.moments_pipe", -1)
        for a0, a1, box in boxes:
            nv = (a1.x - a0.x) * (a1.y - a0.y) * (a1.z - a0.z)
            for pv in (0, 1, 3, 4, 5):
                ts = sorted(ab[(box, pv)])
                report(f"mompipe Aggregates UInt16 {box} moments_pipe={pv} (median of 3 rounds, spread "
                       f"{ts[0]:.4f}-{ts[-1]:.4f})", ts[1], 2 * nv, nv)
        free(V)
    if want("mom1"):
        # integer-moments variants, one ComputeAggregates per case (PMC passes:
        # PMC_KERNEL=aggregatesMomentsU16Kernel scripts/gpu_pmc_groups.sh)
        n = 1024
        V = alloc((n,) * 3, 5, seed=11)
        agg = _lib.Aggregates_t()
        for pv in (0, 1, 3, 4):
            lib.vktHipSetTuningKnob(b"aggregates.moments_pipe", pv)
            for a0, a1, box in ((o, Vec3i_t(n, n, n), "1024^3"),
                                (Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900), "800^3 sub-box at x0=100")):
                nv = (a1.x - a0.x) * (a1.y - a0.y) * (a1.z - a0.z)
                report(f"mom1 Aggregates UInt16 {box} moments_pipe={pv}",
                       timed(lambda: lib.vktHipAggregatesRange(V, a0, a1, C.byref(agg)), R), 2 * nv, nv)
        lib.vktHipSetTuningKnob(b"aggregates.moments_pipe", -1)
        free(V)
    if want("momf"):
        # float moments (knob aggregates.moments bit 1: UInt16 under another mapping, Float32) vs
        # the two float passes, per call incl. the D2H of the result
        n = 1024
        agg = _lib.Aggregates_t()
        for fmt, bpv, lo, hi, name in ((7, 4, 0.0, 1.0, "Float32"), (5, 2, -1.0, 3.0, "UInt16 mapping [-1,3]")):
            V = alloc((n,) * 3, fmt, lo, hi, seed=12)
            if fmt == 7:   # finite values (random bits would hold NaNs: the moments fall back)
                rng_fill(V, n ** 3)
            for mom, what in ((3, "moments"), (1, "2 float passes")):
                lib.vktHipSetTuningKnob(b"aggregates.moments", mom)
                for a0, a1, box in ((o, Vec3i_t(n, n, n), "1024^3"),
                                    (Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900), "800^3 sub-box at x0=100")):
                    nv = (a1.x - a0.x) * (a1.y - a0.y) * (a1.z - a0.z)
                    report(f"momf Aggregates {name} {box} [{what}]",
                           timed(lambda: lib.vktHipAggregatesRange(V, a0, a1, C.byref(agg)), R), bpv * nv, nv)
            lib.vktHipSetTuningKnob(b"aggregates.moments", -1)
            free(V)
    if want("dec16"):
        # BrickDecompose of 1024^3 UInt16 into small bricks, one call per case (PMC passes)
        import volkit_amd.volkit as vkt
        ep = vkt.GetThreadExecutionPolicy()
        ep.device = vkt.ExecutionPolicy.Device_GPU
        vkt.SetThreadExecutionPolicy(ep)
        n = 1024
        V = vkt.StructuredVolume(n, n, n, vkt.DataFormat_UInt16)
        vkt.Synthesize(V, 77)
        for bs, halo in ((16, (1, 1, 1)), (16, (0, 0, 0)), (32, (1, 1, 1))):
            arr = vkt.Array3D_StructuredVolume()
            b3, h3 = vkt.Vec3i(bs, bs, bs), vkt.Vec3i(*halo)
            vkt.BrickDecomposeResize(arr, V, b3, h3, h3)
            vox = (n // bs) ** 3 * (bs + halo[0] + halo[0]) ** 3
            report(f"dec16 BrickDecompose 1024^3 UInt16 -> {bs}^3 bricks halo {halo}",
                   timed(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R), 4 * vox, vox)
            del arr
        del V
        ep.device = vkt.ExecutionPolicy.Device_CPU
        vkt.SetThreadExecutionPolicy(ep)
    if want("decdirect"):
        # in-process A/B of the direct halo-free brick copy (knob decompose.direct: 1 one load +
        # one store per 16-B word, 0 the LDS-staged kernel), alternated, on the same bricks
        import volkit_amd.volkit as vkt
        ep = vkt.GetThreadExecutionPolicy()
        ep.device = vkt.ExecutionPolicy.Device_GPU
        vkt.SetThreadExecutionPolicy(ep)
        n = 1024
        for fmt, b in ((vkt.DataFormat_UInt16, 2), (vkt.DataFormat_UInt8, 1)):
            V = vkt.StructuredVolume(n, n, n, fmt)
            vkt.Synthesize(V, 77)
            ab = {}
            for bs in ((16, 32, 64) if b == 2 else (16, 32)):
                arr = vkt.Array3D_StructuredVolume()
                b3, h3 = vkt.Vec3i(bs, bs, bs), vkt.Vec3i(0, 0, 0)
                vkt.BrickDecomposeResize(arr, V, b3, h3, h3)
                for rnd in range(3):
                    for kv in (1, 2, 0):
                        lib.vktHipSetTuningKnob(b"decompose.direct", kv)
                        ab.setdefault((b, bs, kv, "back-to-back"), []).append(
                            pipelined(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R))
                        ab.setdefault((b, bs, kv, "incl. host planning"), []).append(
                            timed(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R))
                del arr
            lib.vktHipSetTuningKnob(b"decompose.direct", -1)
            for (bb, bs, kv, how), ts in sorted(ab.items()):
                ts.sort()
                report(f"decdirect BrickDecompose 1024^3 {'UInt16' if bb == 2 else 'UInt8'} -> {bs}^3 bricks halo 0 "
                       f"direct={kv} ({how}; median of 3 rounds, spread {ts[0]:.4f}-{ts[-1]:.4f})", ts[1],
                       2 * bb * n ** 3, n ** 3)
            del V
        ep.device = vkt.ExecutionPolicy.Device_CPU
        vkt.SetThreadExecutionPolicy(ep)
    if want("decedge"):
        # in-process A/B of the staged copy's row-end handling for UInt8 / UInt16 bricks with halos
        # (knob decompose.aligned_lds: 0 per-voxel branches, 4 the row-end voxels in a loop of their
        # own, 3 branch-free with dump bytes), back-to-back calls, alternated
        import volkit_amd.volkit as vkt
        ep = vkt.GetThreadExecutionPolicy()
        ep.device = vkt.ExecutionPolicy.Device_GPU
        vkt.SetThreadExecutionPolicy(ep)
        n = 1024
        for fmt, b, name in ((vkt.DataFormat_UInt8, 1, "UInt8"), (vkt.DataFormat_UInt16, 2, "UInt16")):
            V = vkt.StructuredVolume(n, n, n, fmt)
            vkt.Synthesize(V, 77)
            arr = vkt.Array3D_StructuredVolume()
            b3, h3 = vkt.Vec3i(16, 16, 16), vkt.Vec3i(1, 1, 1)
            vkt.BrickDecomposeResize(arr, V, b3, h3, h3)
            vox = (n // 16) ** 3 * 18 ** 3
            for rep in range(3):
                for k in (0, 4, 3):
                    lib.vktHipSetTuningKnob(b"decompose.aligned_lds", k)
                    report(f"decedge BrickDecompose 1024^3 {name} -> 16^3 bricks halo 1 [aligned_lds={k}] (back-to-back)",
                           pipelined(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R), 2 * b * vox, vox)
            lib.vktHipSetTuningKnob(b"decompose.aligned_lds", -1)
            del arr, V
        ep.device = vkt.ExecutionPolicy.Device_CPU
        vkt.SetThreadExecutionPolicy(ep)
    if want("decdump"):
        # in-process A/B of the staged copy's partial-word writes (knob decompose.aligned_lds:
        # 0 per-voxel branches, 3 branch-free with dump bytes), alternated, on the same bricks
        import volkit_amd.volkit as vkt
        ep = vkt.GetThreadExecutionPolicy()
        ep.device = vkt.ExecutionPolicy.Device_GPU
        vkt.SetThreadExecutionPolicy(ep)
        n = 1024
        V = vkt.StructuredVolume(n, n, n, vkt.DataFormat_UInt16)
        vkt.Synthesize(V, 77)
        for bs, halo in ((16, (1, 1, 1)), (32, (1, 1, 1))):
            arr = vkt.Array3D_StructuredVolume()
            b3, h3 = vkt.Vec3i(bs, bs, bs), vkt.Vec3i(*halo)
            vkt.BrickDecomposeResize(arr, V, b3, h3, h3)
            vox = (n // bs) ** 3 * (bs + halo[0] + halo[0]) ** 3
            for rep in range(3):
                for k in (0, 3):
                    lib.vktHipSetTuningKnob(b"decompose.aligned_lds", k)
                    report(f"decdump BrickDecompose 1024^3 UInt16 -> {bs}^3 bricks halo {halo} [aligned_lds={k}]",
                           timed(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R), 4 * vox, vox)
            lib.vktHipSetTuningKnob(b"decompose.aligned_lds", -1)
            del arr
        del V
        ep.device = vkt.ExecutionPolicy.Device_CPU
        vkt.SetThreadExecutionPolicy(ep)
    if want("decpipe"):
        # in-process A/B of the uniform-grid copy kernels (knob decompose.pipe: 1 resident grid
        # loading chunk k + 1 while storing chunk k, 0 one workgroup per chunk; the gather form,
        # knob decompose.gather, measured no faster: profiles/r04/decgather.jsonl)
        import volkit_amd.volkit as vkt
        ep = vkt.GetThreadExecutionPolicy()
        ep.device = vkt.ExecutionPolicy.Device_GPU
        vkt.SetThreadExecutionPolicy(ep)
        n = 1024
        V = vkt.StructuredVolume(n, n, n, vkt.DataFormat_UInt16)
        vkt.Synthesize(V, 77)
        ab = {}
        for bs, halo in ((16, (1, 1, 1)), (16, (0, 0, 0)), (32, (1, 1, 1)), (64, (1, 1, 1)), (256, (1, 1, 1))):
            arr = vkt.Array3D_StructuredVolume()
            b3, h3 = vkt.Vec3i(bs, bs, bs), vkt.Vec3i(*halo)
            vkt.BrickDecomposeResize(arr, V, b3, h3, h3)
            vox = (n // bs) ** 3 * (bs + 2 * halo[0]) ** 3
            for rnd in range(3):
                for kv in (1, 0):
                    lib.vktHipSetTuningKnob(b"decompose.pipe", kv)
                    ab.setdefault((bs, halo, kv, vox, "back-to-back"), []).append(
                        pipelined(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R))
                    ab.setdefault((bs, halo, kv, vox, "incl. host planning"), []).append(
                        timed(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R))
            del arr
        lib.vktHipSetTuningKnob(b"decompose.pipe", -1)
        for (bs, halo, kv, vox, how), ts in sorted(ab.items()):
            ts.sort()
            report(f"decpipe BrickDecompose 1024^3 UInt16 -> {bs}^3 bricks halo {halo} pipe={kv} ({how}; median of "
                   f"3 rounds, spread {ts[0]:.4f}-{ts[-1]:.4f})", ts[1], 4 * vox, vox)
        del V
        ep.device = vkt.ExecutionPolicy.Device_CPU
        vkt.SetThreadExecutionPolicy(ep)
    if want("decpair"):
        # in-process A/B: two x-neighbour small bricks per workgroup (knob decompose.pair)
        import volkit_amd.volkit as vkt
        ep = vkt.GetThreadExecutionPolicy()
        ep.device = vkt.ExecutionPolicy.Device_GPU
        vkt.SetThreadExecutionPolicy(ep)
        n = 1024
        V = vkt.StructuredVolume(n, n, n, vkt.DataFormat_UInt16)
        vkt.Synthesize(V, 77)
        ab = {}
        for bs, halo in ((16, (1, 1, 1)), (16, (0, 0, 0)), (32, (1, 1, 1)), (64, (1, 1, 1)), (256, (1, 1, 1))):
            arr = vkt.Array3D_StructuredVolume()
            b3, h3 = vkt.Vec3i(bs, bs, bs), vkt.Vec3i(*halo)
            vkt.BrickDecomposeResize(arr, V, b3, h3, h3)
            vox = (n // bs) ** 3 * (bs + 2 * halo[0]) ** 3
            for rnd in range(3):
                for kv in (1, 0):
                    lib.vktHipSetTuningKnob(b"decompose.pair", kv)
                    ab.setdefault((bs, halo, kv, vox, "back-to-back"), []).append(
                        pipelined(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R))
                    ab.setdefault((bs, halo, kv, vox, "incl. host planning"), []).append(
                        timed(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R))
            del arr
        lib.vktHipSetTuningKnob(b"decompose.pair", -1)
        for (bs, halo, kv, vox, how), ts in sorted(ab.items()):
            ts.sort()
            report(f"decpair BrickDecompose 1024^3 UInt16 -> {bs}^3 bricks halo {halo} pair={kv} ({how}; median of "
                   f"3 rounds, spread {ts[0]:.4f}-{ts[-1]:.4f})", ts[1], 4 * vox, vox)
        del V
        ep.device = vkt.ExecutionPolicy.Device_CPU
        vkt.SetThreadExecutionPolicy(ep)
    if want("u8ab"):
        # in-process A/B of the UInt8 row-edge knobs on the 800^3 sub-box at x0 = 100 (SumRange and
        # CopyRange, same offsets): pointwise.u8_pairs x pointwise.merge_sectors x pointwise.u8_wide
        m = 1024
        A, B, D = alloc((m,) * 3, 4, seed=1), alloc((m,) * 3, 4, seed=2), alloc((m,) * 3, 4)
        f0, f1 = Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900)
        nv = 800 ** 3
        cases = (("SumRange", lambda: lib.vktHipArithmeticRange(0, D, A, B, f0, f1, o), 3),
                 ("CopyRange same offset", lambda: lib.vktHipCopyRange(D, A, f0, f1, f0), 2))
        kvs = [(p_, mg, w) for p_ in (1, 2, 0) for mg in (1, 2, 0) for w in (1, 0)]
        ab = {}
        for rnd in range(3):
            for kv in kvs:
                lib.vktHipSetTuningKnob(b"pointwise.u8_pairs", kv[0])
                lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", kv[1])
                lib.vktHipSetTuningKnob(b"pointwise.u8_wide", kv[2])
                for lab, fn, _ in cases:
                    ab.setdefault((lab, kv), []).append(timed(fn, R))
        for k in (b"pointwise.u8_pairs", b"pointwise.merge_sectors", b"pointwise.u8_wide"):
            lib.vktHipSetTuningKnob(k, -1)
        for lab, fn, streams in cases:
            for kv in kvs:
                ts = sorted(ab[(lab, kv)])
                report(f"u8ab {lab} 800^3 x0=100 UInt8 u8_pairs={kv[0]} merge_sectors={kv[1]} u8_wide={kv[2]} "
                       f"(median of 3, spread {ts[0]:.4f}-{ts[-1]:.4f})", ts[1], streams * nv, nv)
        free(A, B, D)
    if want("f32m3"):
        # in-process A/B: 64-B sector completion for 3-stream Float32 ops on the general path
        # (knob pointwise.merge_sectors = 2) on the 800^3 sub-box at x0 = 100
        m = 1024
        A, B, D = alloc((m,) * 3, 7, seed=1), alloc((m,) * 3, 7, seed=2), alloc((m,) * 3, 7)
        f0, f1 = Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900)
        cases = (("SumRange dstOffset x=-97", lambda: lib.vktHipArithmeticRange(0, D, A, B, f0, f1, Vec3i_t(-97, 0, 0))),
                 ("SumRange dstOffset x=-100 (aligned dst)", lambda: lib.vktHipArithmeticRange(0, D, A, B, f0, f1, Vec3i_t(-100, -100, -100))))
        ab = {}
        for rnd in range(3):
            for kv in (1, 2):
                lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", kv)
                for lab, fn in cases:
                    ab.setdefault((lab, kv), []).append(timed(fn, R))
        lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", -1)
        for lab, fn in cases:
            for kv in (1, 2):
                ts = sorted(ab[(lab, kv)])
                report(f"f32m3 {lab} 800^3 x0=100 Float32 merge_sectors={kv} (median of 3, spread {ts[0]:.4f}-{ts[-1]:.4f})",
                       ts[1], 3 * 4 * 800 ** 3, 800 ** 3)
        free(A, B, D)
    if want("m3ab"):
        # in-process A/B: sector completion for 3-stream UInt16 / UInt8 ops (knob
        # pointwise.merge_sectors = 2) on the 800^3 sub-box at x0 = 100, same offsets (aligned
        # path) and shifted (general path)
        m = 1024
        res = {}
        for fmt, name in ((5, "UInt16"), (4, "UInt8")):
            A, B, D = alloc((m,) * 3, fmt, seed=1), alloc((m,) * 3, fmt, seed=2), alloc((m,) * 3, fmt)
            bpv = BPV[fmt]
            f0, f1 = Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900)
            cases = (("SumRange same offsets", lambda: lib.vktHipArithmeticRange(0, D, A, B, f0, f1, o)),
                     ("SumRange dstOffset x=-97", lambda: lib.vktHipArithmeticRange(0, D, A, B, f0, f1, Vec3i_t(-97, 0, 0))))
            ab = {}
            for rnd in range(3):
                for kv in (1, 2):
                    lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", kv)
                    for lab, fn in cases:
                        ab.setdefault((lab, kv), []).append(timed(fn, R))
            lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", -1)
            for lab, fn in cases:
                for kv in (1, 2):
                    ts = sorted(ab[(lab, kv)])
                    report(f"m3ab {lab} 800^3 x0=100 {name} merge_sectors={kv} (median of 3, spread {ts[0]:.4f}-{ts[-1]:.4f})",
                           ts[1], 3 * bpv * 800 ** 3, 800 ** 3)
            free(A, B, D)
    if want("decbatch"):
        # in-process A/B of BrickDecompose's batched planning (knob decompose.batch: 1 up to 8
        # batches of brick planes, planning batch k + 1 while the GPU copies batch k; 0 one batch)
        import volkit_amd.volkit as vkt
        ep = vkt.GetThreadExecutionPolicy()
        ep.device = vkt.ExecutionPolicy.Device_GPU
        vkt.SetThreadExecutionPolicy(ep)
        n = 1024
        V = vkt.StructuredVolume(n, n, n, vkt.DataFormat_UInt16)
        vkt.Synthesize(V, 77)
        ab = {}
        for bs, halo in ((16, (1, 1, 1)), (16, (0, 0, 0)), (32, (1, 1, 1))):
            arr = vkt.Array3D_StructuredVolume()
            b3, h3 = vkt.Vec3i(bs, bs, bs), vkt.Vec3i(*halo)
            vkt.BrickDecomposeResize(arr, V, b3, h3, h3)
            vox = sum(arr[(i, j, k)].getSizeInBytes() // 2 for k in range(arr.dims().z)
                      for j in range(arr.dims().y) for i in range(arr.dims().x))
            for rnd in range(3):
                for kv in (1, 0):
                    lib.vktHipSetTuningKnob(b"decompose.batch", kv)
                    ab.setdefault((bs, halo, kv, vox, "back-to-back"), []).append(
                        pipelined(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R))
                    ab.setdefault((bs, halo, kv, vox, "incl. host planning"), []).append(
                        timed(lambda: vkt.BrickDecompose(arr, V, b3, h3, h3), R))
            del arr
        lib.vktHipSetTuningKnob(b"decompose.batch", -1)
        for (bs, halo, kv, vox, how), ts in sorted(ab.items()):
            ts.sort()
            report(f"decbatch BrickDecompose 1024^3 UInt16 -> {bs}^3 bricks halo {halo} batch={kv} ({how}; median of "
                   f"3 rounds, spread {ts[0]:.4f}-{ts[-1]:.4f})", ts[1], 4 * vox, vox)
        del V
        ep.device = vkt.ExecutionPolicy.Device_CPU
        vkt.SetThreadExecutionPolicy(ep)
    if want("config5"):
        # BASELINE config 5: 1024^3 UInt8 multi-scattering, 1024^2 viewport (headless frames)
        import volkit_amd.volkit as vkt
        n = 1024
        V = alloc((n,) * 3, 4)
        # smooth procedural density (a soft ball with a low-density halo and ripples), built
        # plane by plane on the device: long Woodcock paths, unlike white noise
        zz = torch.arange(n, device="cuda", dtype=torch.float32)
        yy, xx = torch.meshgrid(zz, zz, indexing="ij")
        vol = torch.empty((n, n, n), dtype=torch.uint8, device="cuda")
        for z in range(n):
            r = torch.sqrt((xx - n / 2) ** 2 + (yy - n / 2) ** 2 + (z - n / 2) ** 2) / (0.45 * n)
            d = torch.clamp(1.0 - r, 0, 1) * (0.15 + 0.1 * torch.sin(xx * 0.05) * torch.cos(yy * 0.03))
            vol[z] = torch.clamp(d * 255, 0, 255).to(torch.uint8)
        lib.vktHipMemcpy(C.c_void_p(V.data), C.c_void_p(vol.data_ptr()), n ** 3, 3)
        torch.cuda.synchronize()
        del vol
        for algo, lab, frames in ((2, "MultiScattering", 8), (0, "RayMarching", 4), (1, "ImplicitIso", 4)):
            rs = vkt.RenderState()
            rs.viewportWidth = rs.viewportHeight = 1024
            rs.renderAlgo = algo
            rs.dtRayMarching = rs.dtImplicitIso = 1.0
            rs.isoSurfaces[0] = 0.1
            p = _lib.HipRenderParams_t()
            lib.vktHipRenderParamsFromState(C.byref(rs._c), _lib.Vec3fC_t(n, n, n), C.byref(p))
            acc = torch.empty(1024 * 1024 * 4, dtype=torch.float32, device="cuda")
            col = torch.empty_like(acc)
            ms = timed(lambda: lib.vktHipRender(V, C.byref(p), acc.data_ptr(), col.data_ptr(), frames), 3) / frames
            print(json.dumps({"case": f"config5 Render {lab} 1024^3 UInt8, 1024^2 viewport", "ms_per_frame": round(ms, 3),
                              "Mpaths/s": round(1024 * 1024 / ms / 1e3, 1)}), flush=True)
        free(V)
    if want("io"):
        # InputStream / OutputStream into / out of HBM: 1 GiB UInt16 file in
        # the page cache; staged double-buffered path vs host read + migrate()
        import time
        import numpy as np
        import volkit_amd.volkit as vkt
        path = "/tmp/vkt_io_1024x1024x512_uint16.raw"
        nbytes = 1024 * 1024 * 512 * 2
        np.random.default_rng(0).integers(0, 65535, nbytes // 2, dtype=np.uint16).tofile(path)
        ep = vkt.GetThreadExecutionPolicy()

        def dev(d):
            ep.device = d
            vkt.SetThreadExecutionPolicy(ep)

        def wall(fn, reps=3):
            ts = []
            for _ in range(reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            return sorted(ts)[len(ts) // 2] * 1e3

        dev(vkt.ExecutionPolicy.Device_GPU)
        V = vkt.StructuredVolume(1024, 1024, 512, vkt.DataFormat_UInt16)

        def staged():
            f = vkt.RawFile(path, "rb")
            assert vkt.InputStream(f).read(V) == 0
            f.close()
        report("io InputStream.read 1 GiB -> HBM (pinned double buffers, copy stream)", wall(staged), nbytes, nbytes // 2)

        def naive():
            dev(vkt.ExecutionPolicy.Device_CPU)
            H = vkt.StructuredVolume(1024, 1024, 512, vkt.DataFormat_UInt16)
            f = vkt.RawFile(path, "rb")
            assert vkt.InputStream(f).read(H) == 0
            f.close()
            dev(vkt.ExecutionPolicy.Device_GPU)
            H.migrate()
        report("io host read + migrate() 1 GiB (reference flow)", wall(naive), nbytes, nbytes // 2)

        def out():
            f = vkt.RawFile("/tmp/vkt_io_out.raw", "wb")
            assert vkt.OutputStream(f).write(V) == 0
            f.close()
        report("io OutputStream.write HBM -> 1 GiB file", wall(out), nbytes, nbytes // 2)
        dev(vkt.ExecutionPolicy.Device_CPU)
        del V
        os.remove(path)
        os.remove("/tmp/vkt_io_out.raw")
    if not want("metric"):
        return

    # metric kernels at 1024^3 and some extra ops
    s, e = 512, 1024
    S, Rv, B, D = alloc((s,) * 3, 5, seed=4), alloc((e,) * 3, 5), alloc((e,) * 3, 5, seed=5), alloc((e,) * 3, 5)
    lastE = Vec3i_t(e, e, e)
    report("metric Resample 512^3->1024^3 UInt16 Linear",
           timed(lambda: lib.vktHipResample(Rv, S, 1), R), 2 * s ** 3 + 2 * e ** 3, e ** 3)
    report("metric SumRange 1024^3 UInt16", timed(lambda: lib.vktHipArithmeticRange(0, D, Rv, B, o, lastE, o), R),
           6 * e ** 3, e ** 3)
    report("FillRange 1024^3 UInt16", timed(lambda: lib.vktHipFillRange(D, o, lastE, C.c_float(0.3)), R), 2 * e ** 3,
           e ** 3)
    report("Copy 1024^3 UInt16", timed(lambda: lib.vktHipCopyRange(D, B, o, lastE, o), R), 4 * e ** 3, e ** 3)
    Dm = HipVolumeView_t(D.data, e, e, e, 5, -1.0, 3.0)
    report("Copy 1024^3 UInt16 remap [0,1]->[-1,3]", timed(lambda: lib.vktHipCopyRange(Dm, B, o, lastE, o), R),
           4 * e ** 3, e ** 3)
    sub0, sub1 = Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900)
    report("SafeSumRange 800^3 sub-box of 1024^3", timed(lambda: lib.vktHipArithmeticRange(5, D, Rv, B, sub0, sub1, o),
                                                          R), 6 * 800 ** 3, 800 ** 3)
    D1000 = alloc((1000, 1000, 1000), 5)
    report("Resample 1024^3->1000^3 UInt16 Nearest (gather)", timed(lambda: lib.vktHipResample(D1000, Rv, 0), R),
           resample_bytes((e,) * 3, (1000,) * 3, 2, 2), 1000 ** 3)
    free(S, Rv, B, D, D1000)
    # per-format streaming rates of the pointwise engine (8-voxel items: 8 B / 16 B / 32 B per lane)
    for fmt, bpv, name in ((4, 1, "UInt8"), (7, 4, "Float32")):
        A8, B8, D8 = alloc((e,) * 3, fmt, seed=8), alloc((e,) * 3, fmt, seed=9), alloc((e,) * 3, fmt)
        report(f"Copy 1024^3 {name}", timed(lambda: lib.vktHipCopyRange(D8, A8, o, lastE, o), R),
               2 * bpv * e ** 3, e ** 3)
        report(f"SumRange 1024^3 {name}", timed(lambda: lib.vktHipArithmeticRange(0, D8, A8, B8, o, lastE, o), R),
               3 * bpv * e ** 3, e ** 3)
        # multi-row boxes (rows 8-voxel aligned: no padded edges; and x0 = 100)
        for lab, f0, f1 in (("x 0..800", Vec3i_t(0, 100, 100), Vec3i_t(800, 900, 900)),
                            ("x0=100", Vec3i_t(100, 100, 100), Vec3i_t(900, 900, 900))):
            report(f"Copy 800^3 sub-box {lab} of 1024^3 {name}",
                   timed(lambda: lib.vktHipCopyRange(D8, A8, f0, f1, o), R), 2 * bpv * 800 ** 3, 800 ** 3)
            report(f"SumRange 800^3 sub-box {lab} of 1024^3 {name}",
                   timed(lambda: lib.vktHipArithmeticRange(0, D8, A8, B8, f0, f1, o), R), 3 * bpv * 800 ** 3, 800 ** 3)
        free(A8, B8, D8)

    if args.big:
        s, e = 1024, 2048
        S, Rv, B, D = alloc((s,) * 3, 5, seed=6), alloc((e,) * 3, 5), alloc((e,) * 3, 5, seed=7), alloc((e,) * 3, 5)
        lastE = Vec3i_t(e, e, e)
        ms_r = timed(lambda: lib.vktHipResample(Rv, S, 1), 3)
        ms_s = timed(lambda: lib.vktHipArithmeticRange(0, D, Rv, B, o, lastE, o), 3)
        report("config4 (1 GPU, strong) Resample 1024^3->2048^3 UInt16", ms_r, 2 * s ** 3 + 2 * e ** 3, e ** 3)
        report("config4 (1 GPU, strong) SumRange 2048^3 UInt16", ms_s, 6 * e ** 3, e ** 3)
        report("config4 (1 GPU, strong) pipeline", ms_r + ms_s, 2 * s ** 3 + 8 * e ** 3, e ** 3)
        free(S, Rv, B, D)


if __name__ == "__main__":
    main()
