"""Transform with device functors (include/volkit_transform.hpp) vs the oracle's restatement of
TransformRange_serial (reference src/vkt/Transform_serial.hpp:15-101, oracle/vkt_oracle.c:
vko_transform_range1/2).  The functors live in tests/native/transform_ops.hip: each is run on
the GPU through the template API and, compiled for the host, as the oracle's callback -- the
same user operation on both sides, so the comparison checks the Transform machinery (visit
coordinates, range, zeroed 8-byte scratch, write-back of bytesPerVoxel bytes, volume1-then-
volume2 stores, aliasing).  Bit-exact; Float32 NaNs match any NaN."""
import ctypes as C
import os

import numpy as np
import pytest

from backends import CODE_DTYPE
from oracle import binding as ob
from test_gpu_parity import assert_codes_equal, rand_codes

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "native", "libfixtures.so")

UNARY_OPS = {0: "Checkered<3>", 1: "Checkered<2>", 2: "Diagonal", 3: "Rescale", 4: "ScratchProbe"}
BINARY_OPS = {0: "Or", 1: "MixFormats"}
FMTS = [4, 5, 2, 6, 7]    # UInt8, UInt16, Int16, UInt32, Float32


@pytest.fixture(scope="module")
def t():
    import volkit_amd  # noqa: F401  (loads libvolkit.so first)
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} missing: run __graft_entry__.build()")
    lib = C.CDLL(LIB)
    i, f, p = C.c_int, C.c_float, C.c_void_p
    lib.vktt_run_unary.argtypes = [i, p, i, i, i, i, f, f, i, i, i, i, i, i]
    lib.vktt_run_unary_whole.argtypes = [i, p, i, i, i, i, f, f]
    lib.vktt_run_unary_slab.argtypes = [i, p, i, i, i, i, f, f, i, i, i, i, i, i, i]
    lib.vktt_run_binary.argtypes = [i, i, p, i, i, i, i, f, f, p, i, i, i, i, f, f, i, i, i, i, i, i]
    lib.vktt_host_unary.restype = p
    lib.vktt_host_unary.argtypes = [i]
    lib.vktt_host_binary.restype = p
    lib.vktt_host_binary.argtypes = [i]
    lib.vktt_bench_unary.argtypes = [i, i, i, i, i, i, C.POINTER(f)]
    lib.vktt_lambda_or.argtypes = [p, p, i, i, i]
    lib.vktt_run_unary_migrating.argtypes = [i, p, i, i, i, i, i]
    return lib


def gpu_unary(t, op, codes, fmt, mapping, first, last, whole=False):
    out = np.ascontiguousarray(codes.copy())
    z, y, x = out.shape
    if whole:
        rc = t.vktt_run_unary_whole(op, out.ctypes.data, x, y, z, fmt, *mapping)
    else:
        rc = t.vktt_run_unary(op, out.ctypes.data, x, y, z, fmt, *mapping, *first, *last)
    assert rc == 0, rc
    return out


def oracle_unary(t, op, codes, fmt, mapping, first, last):
    v = ob.Volume(codes.copy(), fmt, *mapping)
    ob._lib.vko_transform_range1(v.ref, ob._i3(*first), ob._i3(*last), ob.UNARY(t.vktt_host_unary(op)))
    return v.codes


def gpu_binary(t, op, c1, f1, m1, c2, f2, m2, first, last, alias=False):
    o1 = np.ascontiguousarray(c1.copy())
    o2 = np.ascontiguousarray(c2.copy())
    z1, y1, x1 = o1.shape
    z2, y2, x2 = o2.shape
    rc = t.vktt_run_binary(op, int(alias), o1.ctypes.data, x1, y1, z1, f1, *m1, o2.ctypes.data, x2, y2, z2, f2, *m2,
                           *first, *last)
    assert rc == 0, rc
    return o1, o2


def oracle_binary(t, op, c1, f1, m1, c2, f2, m2, first, last, alias=False):
    v1 = ob.Volume(c1.copy(), f1, *m1)
    v2 = v1 if alias else ob.Volume(c2.copy(), f2, *m2)
    ob._lib.vko_transform_range2(v1.ref, v2.ref, ob._i3(*first), ob._i3(*last), ob._i3(0, 0, 0),
                                 ob.BINARY(t.vktt_host_binary(op)))
    return v1.codes, v2.codes


# (dims xyz, first, last): 16-byte rows (vector kernels), partial rows, ragged dims (row kernel),
# one voxel, and an empty range
RANGES = [
    ((64, 16, 8), (0, 0, 0), (64, 16, 8)),
    ((64, 16, 8), (16, 3, 2), (48, 13, 7)),
    ((37, 23, 11), (0, 0, 0), (37, 23, 11)),
    ((37, 23, 11), (3, 2, 1), (30, 20, 9)),
    ((40, 9, 5), (1, 0, 0), (33, 9, 5)),
    ((24, 24, 24), (2, 2, 2), (22, 22, 22)),
    ((16, 16, 16), (5, 5, 5), (6, 6, 6)),
    ((16, 16, 16), (4, 4, 4), (4, 9, 9)),
    ((64, 16, 8), (3, 1, 1), (61, 15, 7)),      # rows on 64-B boundaries: padded to sectors
    ((128, 4, 3), (17, 0, 0), (100, 4, 3)),
]


@pytest.mark.parametrize("op", sorted(UNARY_OPS))
@pytest.mark.parametrize("fmt", FMTS)
def test_unary_functor_vs_oracle(t, op, fmt):
    rng = np.random.default_rng(100 * op + fmt)
    for mapping in ((0.0, 1.0), (-1.0, 3.0)):
        for dims, first, last in RANGES:
            codes = rand_codes(rng, fmt, dims[::-1])
            out = gpu_unary(t, op, codes, fmt, mapping, first, last)
            ref = oracle_unary(t, op, codes, fmt, mapping, first, last)
            assert_codes_equal(out, ref, fmt, f"{UNARY_OPS[op]} fmt={fmt} map={mapping} {dims} {first}->{last}")


@pytest.mark.parametrize("nranks", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("fmt", [4, 5, 7])
def test_unary_functor_slabs(t, nranks, fmt):
    """vkt::TransformRangeSlab: the volume cut into nranks Z-slabs (ceil partition, empty
    trailing slabs for 8 ranks over 5..11 planes), each slab transforms the owned planes of the
    GLOBAL range with the functor seeing global z: the slabs put together equal one
    whole-volume oracle call.  Checkered<3> and Diagonal read z, so a missed shift shows."""
    rng = np.random.default_rng(31 * nranks + fmt)
    for op in (0, 2, 4):
        for dims, first, last in RANGES[2:6] + [((40, 9, 5), (0, 0, 0), (40, 9, 5))]:
            codes = rand_codes(rng, fmt, dims[::-1])
            out = np.ascontiguousarray(codes.copy())
            z, y, x = out.shape
            rc = t.vktt_run_unary_slab(op, out.ctypes.data, x, y, z, fmt, 0.0, 1.0, nranks, *first, *last)
            assert rc == 0, rc
            ref = oracle_unary(t, op, codes, fmt, (0.0, 1.0), first, last)
            assert_codes_equal(out, ref, fmt, f"slabs={nranks} {UNARY_OPS[op]} fmt={fmt} {dims} {first}->{last}")


@pytest.mark.parametrize("op", [0, 2, 3])
def test_unary_functor_whole_volume(t, op):
    """vkt::Transform(volume, op): the whole volume, incl. a multi-workgroup vector launch with
    a guarded tail (dims not a multiple of the 16 KiB workgroup quantum)."""
    rng = np.random.default_rng(op)
    for fmt, dims in ((4, (96, 70, 9)), (5, (64, 40, 33)), (7, (32, 33, 17)), (4, (33, 7, 5))):
        codes = rand_codes(rng, fmt, dims[::-1])
        out = gpu_unary(t, op, codes, fmt, (0.0, 1.0), None, None, whole=True)
        ref = oracle_unary(t, op, codes, fmt, (0.0, 1.0), (0, 0, 0), dims)
        assert_codes_equal(out, ref, fmt, f"whole {UNARY_OPS[op]} fmt={fmt} {dims}")


def test_reference_checkerboard_example(t):
    """src/examples/Arithmetic.cpp: Transform(volume1, MakeCheckered<3>) on 32^3 UInt8."""
    codes = np.zeros((32, 32, 32), np.uint8)
    out = gpu_unary(t, 0, codes, 4, (0.0, 1.0), None, None, whole=True)
    ref = oracle_unary(t, 0, codes, 4, (0.0, 1.0), (0, 0, 0), (32, 32, 32))
    np.testing.assert_array_equal(out, ref)
    assert set(np.unique(out)) == {0, 128}


@pytest.mark.parametrize("op", sorted(BINARY_OPS))
@pytest.mark.parametrize("f1,f2", [(4, 4), (5, 5), (7, 7), (5, 4), (4, 7), (2, 6)])
def test_binary_functor_vs_oracle(t, op, f1, f2):
    rng = np.random.default_rng(1000 + 10 * f1 + f2 + 7 * op)
    for m1, m2 in (((0.0, 1.0), (0.0, 1.0)), ((-1.0, 3.0), (0.25, 7.5))):
        for dims, first, last in RANGES:
            c1 = rand_codes(rng, f1, dims[::-1])
            c2 = rand_codes(rng, f2, dims[::-1])
            o1, o2 = gpu_binary(t, op, c1, f1, m1, c2, f2, m2, first, last)
            r1, r2 = oracle_binary(t, op, c1, f1, m1, c2, f2, m2, first, last)
            what = f"{BINARY_OPS[op]} {f1}/{f2} {dims} {first}->{last}"
            assert_codes_equal(o1, r1, f1, what + " volume1")
            assert_codes_equal(o2, r2, f2, what + " volume2")


def test_binary_volume2_larger(t):
    """volume2 may be larger than the range (the reference reads it at the same x, y, z)."""
    rng = np.random.default_rng(5)
    c1 = rand_codes(rng, 4, (8, 16, 32))
    c2 = rand_codes(rng, 4, (9, 20, 48))
    o1, o2 = gpu_binary(t, 0, c1, 4, (0.0, 1.0), c2, 4, (0.0, 1.0), (0, 0, 0), (32, 16, 8))
    r1, r2 = oracle_binary(t, 0, c1, 4, (0.0, 1.0), c2, 4, (0.0, 1.0), (0, 0, 0), (32, 16, 8))
    np.testing.assert_array_equal(o1, r1)
    np.testing.assert_array_equal(o2, r2)


@pytest.mark.parametrize("op", sorted(BINARY_OPS))
@pytest.mark.parametrize("fmt", [4, 5, 7])
def test_binary_functor_aliased(t, op, fmt):
    """Transform(v, v, op): both views read the same voxel; the serial loop stores volume1's
    bytes, then volume2's, to the same address, so volume2's win."""
    rng = np.random.default_rng(77 + fmt + op)
    for dims, first, last in RANGES[:5]:
        c = rand_codes(rng, fmt, dims[::-1])
        o1, _ = gpu_binary(t, op, c, fmt, (0.0, 1.0), c, fmt, (0.0, 1.0), first, last, alias=True)
        r1, _ = oracle_binary(t, op, c, fmt, (0.0, 1.0), c, fmt, (0.0, 1.0), first, last, alias=True)
        assert_codes_equal(o1, r1, fmt, f"aliased {BINARY_OPS[op]} fmt={fmt} {dims} {first}->{last}")


def test_out_of_range_is_rejected(t):
    codes = np.zeros((4, 4, 4), np.uint8)
    out = codes.copy()
    rc = t.vktt_run_unary(2, out.ctypes.data, 4, 4, 4, 4, 0.0, 1.0, 0, 0, 0, 5, 4, 4)
    assert rc == -1
    np.testing.assert_array_equal(out, codes)


def test_unary_1024_uint8_full_size(t):
    """1024^3 UInt8 Diagonal through the vector kernel (multi-launch-free, 65 536 workgroups):
    the diagonal is set, nothing else moves (size-independent property; the oracle pins the
    same op on the small cases above)."""
    n = 1024
    codes = np.full((n, n, n), 7, np.uint8)
    out = gpu_unary(t, 2, codes, 4, (0.0, 1.0), None, None, whole=True)
    d = np.arange(n)
    assert np.all(out[d, d, d] == 0xFF)
    out[d, d, d] = 7
    assert np.all(out == 7)


def test_bench_entry_runs(t):
    ms = C.c_float(0.0)
    assert t.vktt_bench_unary(2, 256, 256, 256, 4, 3, C.byref(ms)) == 0
    assert ms.value > 0.0


def test_device_lambda(t):
    """vkt::Transform(v1, v2, [] __device__ (...) {...}) -- a device lambda as the binary op."""
    rng = np.random.default_rng(4)
    a = rng.integers(0, 256, (9, 17, 48), dtype=np.uint8)
    b = rng.integers(0, 256, (9, 17, 48), dtype=np.uint8)
    ga, gb = a.copy(), b.copy()
    assert t.vktt_lambda_or(ga.ctypes.data, gb.ctypes.data, 48, 17, 9) == 0
    r1, r2 = oracle_binary(t, 0, a, 4, (0.0, 1.0), b, 4, (0.0, 1.0), (0, 0, 0), (48, 17, 9))
    np.testing.assert_array_equal(ga, r1)
    np.testing.assert_array_equal(gb, r2)


@pytest.fixture
def shape_knob():
    """Set the vector kernels' workgroup shape (knob transform.shape) for one test."""
    from volkit_amd._lib import lib
    shapes = []

    def set_shape(k):
        assert lib.vktHipSetTuningKnob(b"transform.shape", k) == 0
        got = C.c_int64(-1)
        assert lib.vktHipGetTuningKnob(b"transform.shape", C.byref(got)) == 0 and got.value == k
        shapes.append(k)

    yield set_shape
    lib.vktHipSetTuningKnob(b"transform.shape", -1)


@pytest.mark.parametrize("shape", [0, 1, 2])
def test_vector_kernel_shapes(t, shape_knob, shape):
    """Every workgroup shape of the 16-B vector kernels (256x4, one wave x 2, one wave x 1
    items per lane): unguarded whole workgroups plus the guarded tail, padded sector rows,
    unary and binary (incl. aliased) functors, against the oracle."""
    shape_knob(shape)
    rng = np.random.default_rng(900 + shape)
    for fmt in (4, 5, 7):
        for dims, first, last in RANGES:
            codes = rand_codes(rng, fmt, dims[::-1])
            for op in (0, 3):
                out = gpu_unary(t, op, codes, fmt, (-1.0, 3.0), first, last)
                ref = oracle_unary(t, op, codes, fmt, (-1.0, 3.0), first, last)
                assert_codes_equal(out, ref, fmt, f"shape={shape} {UNARY_OPS[op]} fmt={fmt} {dims} {first}->{last}")
            c2 = rand_codes(rng, 4, dims[::-1])
            o1, o2 = gpu_binary(t, 1, codes, fmt, (0.0, 1.0), c2, 4, (0.0, 1.0), first, last)
            r1, r2 = oracle_binary(t, 1, codes, fmt, (0.0, 1.0), c2, 4, (0.0, 1.0), first, last)
            assert_codes_equal(o1, r1, fmt, f"shape={shape} MixFormats {dims} volume1")
            assert_codes_equal(o2, r2, 4, f"shape={shape} MixFormats {dims} volume2")
            o1, _ = gpu_binary(t, 0, codes, fmt, (0.0, 1.0), codes, fmt, (0.0, 1.0), first, last, alias=True)
            r1, _ = oracle_binary(t, 0, codes, fmt, (0.0, 1.0), codes, fmt, (0.0, 1.0), first, last, alias=True)
            assert_codes_equal(o1, r1, fmt, f"shape={shape} aliased Or fmt={fmt} {dims}")
    for fmt, dims in ((4, (96, 70, 9)), (5, (64, 40, 33)), (7, (32, 33, 17)), (4, (256, 129, 7))):
        codes = rand_codes(rng, fmt, dims[::-1])
        out = gpu_unary(t, 2, codes, fmt, (0.0, 1.0), None, None, whole=True)
        ref = oracle_unary(t, 2, codes, fmt, (0.0, 1.0), (0, 0, 0), dims)
        assert_codes_equal(out, ref, fmt, f"shape={shape} whole Diagonal fmt={fmt} {dims}")


def test_failed_migration_is_an_error(t):
    """Transform of a host-resident volume whose migration to HBM fails: an error, the bytes
    (still in host memory) untouched; with the allocation allowed the same call migrates and
    matches the oracle."""
    from volkit_amd._lib import lib
    rng = np.random.default_rng(12)
    codes = rand_codes(rng, 5, (33, 40, 64))
    out = np.ascontiguousarray(codes.copy())
    z, y, x = out.shape
    assert t.vktt_run_unary_migrating(2, out.ctypes.data, x, y, z, 5, 1) != 0
    assert b"migration failed" in lib.vktHipGetLastErrorString()
    np.testing.assert_array_equal(out, codes)
    assert t.vktt_run_unary_migrating(2, out.ctypes.data, x, y, z, 5, 0) == 0
    ref = oracle_unary(t, 2, codes, 5, (0.0, 1.0), (0, 0, 0), (x, y, z))
    assert_codes_equal(out, ref, 5, "migrated Diagonal")
