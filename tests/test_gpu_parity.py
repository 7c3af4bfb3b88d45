"""Parity of the HIP/gfx950 path (through the public C ABI) with the CPU oracle on seeded
inputs: every op, data format and mapping of the hot path, ragged dims, ranges that need
clamping, offsets, and the reference's numeric traps.  Integer outputs must be bit-exact;
Float32 outputs are bit-exact too except that any NaN matches any NaN (payload bits of NaNs
produced by x86 SSE and gfx950 VALU arithmetic are not compared -- see DESIGN.md §3).
"""
import numpy as np
import pytest

from backends import CODE_DTYPE, GpuBackend, OracleBackend, codes_of

pytestmark = pytest.mark.gpu

MAPPINGS = [(0.0, 1.0), (-1.0, 3.0), (0.25, 7.5)]
INT_FMTS = [4, 5, 2, 6]        # UInt8, UInt16, Int16, UInt32
ALL_FMTS = INT_FMTS + [7, 1, 3]  # + Float32, Int8, Int32 (no-write/zero-read formats)
OPS = ["Sum", "Diff", "Prod", "Quot", "AbsDiff", "SafeSum", "SafeDiff", "SafeProd", "SafeQuot", "SafeAbsDiff"]


@pytest.fixture(scope="module")
def g():
    return GpuBackend()


@pytest.fixture(scope="module")
def o():
    return OracleBackend()


def rand_codes(rng, fmt, shape, floats="mixed"):
    dt = CODE_DTYPE[fmt]
    if fmt == 7:
        if floats == "bits":
            return rng.integers(0, 2**32, size=shape, dtype=np.uint64).astype(np.uint32)
        vals = rng.uniform(-0.5, 1.5, size=shape).astype(np.float32)
        flat = vals.reshape(-1)
        specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-40, -1e-40, 3e38, 1.0], dtype=np.float32)
        idx = rng.choice(flat.size, size=min(flat.size, 2 * len(specials)), replace=False)
        flat[idx] = np.resize(specials, idx.size)
        return vals.view(np.uint32)
    info = np.iinfo(dt)
    return rng.integers(0, int(info.max) + 1, size=shape, dtype=np.uint64).astype(dt)


def assert_codes_equal(out, ref, fmt, what=""):
    if fmt == 7:
        fo, fr = out.view(np.float32), ref.view(np.float32)
        nan_o, nan_r = np.isnan(fo), np.isnan(fr)
        bad = (nan_o != nan_r) | (~nan_r & (out != ref))
    else:
        bad = out != ref
    n = int(np.count_nonzero(bad))
    if n:
        i = tuple(np.argwhere(bad)[0])
        raise AssertionError(f"{what}: {n} mismatching voxels, first at zyx={i}: gpu={out[i]!r} ref={ref[i]!r}")


# ---- Fill -----------------------------------------------------------------------------
@pytest.mark.parametrize("fmt", ALL_FMTS)
@pytest.mark.parametrize("mapping", MAPPINGS[:2])
def test_fill_range(g, o, fmt, mapping):
    rng = np.random.default_rng(fmt)
    dims = (37, 23, 11)
    init = rand_codes(rng, fmt, (11, 23, 37))
    for value in (0.0, 0.1, 0.5, 1.0, 1.5, -0.25):
        for first, last in (((0, 0, 0), dims), ((3, 2, 1), (30, 20, 9)), ((5, 5, 5), (6, 6, 6)), ((4, 4, 4), (4, 9, 9))):
            out = g.fill_range(fmt, mapping, dims, init.copy(), first, last, value)
            ref = o.fill_range(fmt, mapping, dims, init.copy(), first, last, value)
            assert_codes_equal(out, ref, fmt, f"fill fmt={fmt} v={value} {first}->{last}")


# ---- Copy -----------------------------------------------------------------------------
@pytest.mark.parametrize("sfmt,dfmt", [(4, 4), (5, 5), (7, 7), (5, 4), (4, 7), (7, 5), (2, 6)])
def test_copy_range(g, o, sfmt, dfmt):
    rng = np.random.default_rng(11 * sfmt + dfmt)
    src = rand_codes(rng, sfmt, (20, 24, 32))      # dims (32, 24, 20)
    for smap, dmap in (((0.0, 1.0), (0.0, 1.0)), ((0.0, 1.0), (-1.0, 3.0))):
        for first, last, off in (((0, 0, 0), (32, 24, 20), (0, 0, 0)),        # whole, vector path
                                 ((10, 10, 10), (34, 34, 34), (0, 0, 0)),     # CoreAlgorithms.c: clamps
                                 ((-3, -2, -1), (8, 9, 5), (2, 1, 3)),        # negative first: clamps
                                 ((8, 0, 4), (24, 24, 12), (0, 0, 0))):       # partial rows, aligned
            n = [l - f for f, l in zip(first, last)]
            dd = (max(n[0] + off[0], 24), max(n[1] + off[1], 24), max(n[2] + off[2], 24))
            init = rand_codes(rng, dfmt, (dd[2], dd[1], dd[0]))
            out = g.copy_range(dfmt, dmap, dd, init.copy(), sfmt, smap, src, first, last, off)
            ref = o.copy_range(dfmt, dmap, dd, init.copy(), sfmt, smap, src, first, last, off)
            assert_codes_equal(out, ref, dfmt, f"copy {sfmt}->{dfmt} {smap}->{dmap} {first}->{last}+{off}")


# ---- Arithmetic -------------------------------------------------------------------------
@pytest.mark.parametrize("op", OPS)
@pytest.mark.parametrize("fmt", [4, 5, 7, 2, 6])
def test_arithmetic_same_format(g, o, op, fmt):
    rng = np.random.default_rng(hash((op, fmt)) % 2**32)
    for mapping in MAPPINGS:
        maps = [mapping] * 3
        a = rand_codes(rng, fmt, (16, 16, 16))
        b = rand_codes(rng, fmt, (16, 16, 16))
        # whole volume (vector path)
        d0 = rand_codes(rng, fmt, (16, 16, 16))
        out = g.arith(op, [fmt] * 3, maps, a, b, d0.copy(), (0, 0, 0), (16, 16, 16), (0, 0, 0))
        ref = o.arith(op, [fmt] * 3, maps, a, b, d0.copy(), (0, 0, 0), (16, 16, 16), (0, 0, 0))
        assert_codes_equal(out, ref, fmt, f"{op} fmt={fmt} map={mapping} whole")
        # SURVEY Appendix C range case: first=(3,2,1) last=(13,11,9) off=(1,0,2) into a 20^3 dst of 0x5A
        dinit = np.empty((20, 20, 20), dtype=CODE_DTYPE[fmt])
        dinit.view(np.uint8)[...] = 0x5A
        out = g.arith(op, [fmt] * 3, maps, a, b, dinit.copy(), (3, 2, 1), (13, 11, 9), (1, 0, 2))
        ref = o.arith(op, [fmt] * 3, maps, a, b, dinit.copy(), (3, 2, 1), (13, 11, 9), (1, 0, 2))
        assert_codes_equal(out, ref, fmt, f"{op} fmt={fmt} map={mapping} range")


@pytest.mark.parametrize("op", ["Sum", "SafeDiff", "Quot"])
def test_arithmetic_mixed_formats(g, o, op):
    rng = np.random.default_rng(99)
    for fd, f1, f2 in ((4, 5, 7), (7, 4, 5), (5, 2, 4), (6, 7, 5), (1, 5, 5), (5, 3, 4)):
        maps = [(-1.0, 3.0), (0.0, 1.0), (0.25, 7.5)]
        a = rand_codes(rng, f1, (9, 10, 17))
        b = rand_codes(rng, f2, (9, 10, 17))
        d = rand_codes(rng, fd, (9, 10, 17))
        out = g.arith(op, [fd, f1, f2], maps, a, b, d.copy(), (1, 2, 0), (17, 10, 9), (0, 0, 0))
        ref = o.arith(op, [fd, f1, f2], maps, a, b, d.copy(), (1, 2, 0), (17, 10, 9), (0, 0, 0))
        assert_codes_equal(out, ref, fd, f"{op} {f1},{f2}->{fd}")


def test_arithmetic_ragged_whole_volume(g, o):
    # odd dims: collapsed single row with a scalar tail
    rng = np.random.default_rng(5)
    for fmt in (4, 5, 7):
        a = rand_codes(rng, fmt, (11, 23, 37))
        b = rand_codes(rng, fmt, (11, 23, 37))
        d = rand_codes(rng, fmt, (11, 23, 37))
        out = g.arith("SafeSum", [fmt] * 3, [(0.0, 1.0)] * 3, a, b, d.copy(), (0, 0, 0), (37, 23, 11), (0, 0, 0))
        ref = o.arith("SafeSum", [fmt] * 3, [(0.0, 1.0)] * 3, a, b, d.copy(), (0, 0, 0), (37, 23, 11), (0, 0, 0))
        assert_codes_equal(out, ref, fmt, f"ragged fmt={fmt}")


@pytest.mark.parametrize("op", OPS)
def test_arithmetic_unit_mapping_all_code_pairs(g, o, op):
    """The unit mapping (+0, 1) takes a compile-time path without the codec's lerp and
    normalisation (codec::decodeUnit / normalise<3>): every UInt8 code pair, a UInt16 sweep
    that covers every code as either operand, and the look-alike mappings -0 / 1.0 - ulp that
    must NOT take it."""
    a8 = np.repeat(np.arange(256, dtype=np.uint8), 256).reshape(16, 16, 256)
    b8 = np.tile(np.arange(256, dtype=np.uint8), 256).reshape(16, 16, 256)
    c16 = np.arange(65536, dtype=np.uint16)
    a16 = np.concatenate([c16, np.random.default_rng(3).permutation(c16)]).reshape(8, 64, 256)
    b16 = np.concatenate([np.random.default_rng(4).permutation(c16), c16]).reshape(8, 64, 256)
    near1 = float(np.nextafter(np.float32(1.0), np.float32(0.0)))
    for mapping in ((0.0, 1.0), (-0.0, 1.0), (0.0, near1)):
        for fmt, a, b in ((4, a8, b8), (5, a16, b16)):
            d = np.zeros_like(a)
            last = (a.shape[2], a.shape[1], a.shape[0])
            out = g.arith(op, [fmt] * 3, [mapping] * 3, a, b, d.copy(), (0, 0, 0), last, (0, 0, 0))
            ref = o.arith(op, [fmt] * 3, [mapping] * 3, a, b, d.copy(), (0, 0, 0), last, (0, 0, 0))
            assert_codes_equal(out, ref, fmt, f"{op} fmt={fmt} map={mapping} all code pairs")


@pytest.mark.parametrize("op", ["Sum", "Diff", "SafeSum", "SafeDiff", "AbsDiff", "SafeAbsDiff"])
def test_arithmetic_unit_mapping_code_pairs_strided_subbox(g, o, op):
    """The unit-mapping integer paths (IntArithU16F, UnitArithU8F) on a strided sub-box: odd
    first.x, an extent that is not a multiple of 8, several rows -- the padded row items that
    straddle the row ends (masked stores), the multi-row addressing, every UInt8 code pair and
    every UInt16 code as either operand."""
    # dims x multiple of 8 (vector path with several rows); box x 3..(3+253), odd start
    a8 = np.zeros((18, 16, 264), np.uint8)
    b8 = np.zeros_like(a8)
    a8[1:17, :, 3:259] = np.repeat(np.arange(256, dtype=np.uint8), 256).reshape(16, 16, 256)
    b8[1:17, :, 3:259] = np.tile(np.arange(256, dtype=np.uint8), 256).reshape(16, 16, 256)
    c16 = np.arange(65536, dtype=np.uint16)
    a16 = np.zeros((10, 64, 264), np.uint16)
    b16 = np.zeros_like(a16)
    a16[1:9, :, 3:259] = np.concatenate([c16, np.random.default_rng(5).permutation(c16)]).reshape(8, 64, 256)
    b16[1:9, :, 3:259] = np.concatenate([np.random.default_rng(6).permutation(c16), c16]).reshape(8, 64, 256)
    for fmt, a, b in ((4, a8, b8), (5, a16, b16)):
        nz, ny = a.shape[0], a.shape[1]
        for first, last in (((3, 0, 1), (259, ny, nz - 1)), ((3, 1, 1), (256, ny - 1, nz - 1)),
                            ((5, 0, 0), (262, ny, nz))):
            d = np.full_like(a, 7)
            out = g.arith(op, [fmt] * 3, [(0.0, 1.0)] * 3, a, b, d.copy(), first, last, (0, 0, 0))
            ref = o.arith(op, [fmt] * 3, [(0.0, 1.0)] * 3, a, b, d.copy(), first, last, (0, 0, 0))
            assert_codes_equal(out, ref, fmt, f"{op} fmt={fmt} sub-box {first}->{last}")


@pytest.mark.parametrize("max_quanta", [1, 2, 3])
def test_pointwise_multi_launch_split(g, o, max_quanta):
    """Lower the launch split (knob pointwise.max_quanta_per_launch) so small ops need several
    launches: one collapsed row with a scalar head and tail (edges only in the first launch)
    and padded multi-row boxes, vs the oracle."""
    from volkit_amd._lib import lib
    rng = np.random.default_rng(max_quanta)
    assert lib.vktHipSetTuningKnob(b"pointwise.max_quanta_per_launch", max_quanta) == 0
    try:
        for fmt in (5, 4, 7):
            for dims, first, last in (((37, 23, 11), (0, 0, 1), (37, 23, 11)),    # one row, head 5
                                      ((40, 23, 11), (3, 2, 1), (37, 21, 10)),    # padded rows
                                      ((64, 31, 9), (0, 0, 0), (64, 31, 9))):     # whole volume
                a = rand_codes(rng, fmt, dims[::-1])
                b = rand_codes(rng, fmt, dims[::-1])
                d = rand_codes(rng, fmt, dims[::-1])
                for op in ("Sum", "SafeDiff"):
                    for mapping in ((0.0, 1.0), (-1.0, 3.0)):
                        out = g.arith(op, [fmt] * 3, [mapping] * 3, a, b, d.copy(), first, last, (0, 0, 0))
                        ref = o.arith(op, [fmt] * 3, [mapping] * 3, a, b, d.copy(), first, last, (0, 0, 0))
                        assert_codes_equal(out, ref, fmt, f"{op} fmt={fmt} {dims} {first}->{last} q={max_quanta}")
                v = 0.3
                out = g.fill_range(fmt, (0.0, 1.0), dims, d.copy(), first, last, v)
                ref = o.fill_range(fmt, (0.0, 1.0), dims, d.copy(), first, last, v)
                assert_codes_equal(out, ref, fmt, f"fill fmt={fmt} {dims} {first}->{last}")
    finally:
        lib.vktHipSetTuningKnob(b"pointwise.max_quanta_per_launch", -1)


@pytest.mark.parametrize("padded", [0, 1])
def test_pointwise_padded_rows_knob(g, o, padded):
    """Multi-row boxes with and without padded row items (the scalar-edge pass they replace)."""
    from volkit_amd._lib import lib
    rng = np.random.default_rng(40 + padded)
    assert lib.vktHipSetTuningKnob(b"pointwise.padded_rows", padded) == 0
    try:
        for fmt in (4, 5, 7):
            a = rand_codes(rng, fmt, (9, 21, 1200))
            b = rand_codes(rng, fmt, (9, 21, 1200))
            d = rand_codes(rng, fmt, (9, 21, 1200))
            for first, last, off in (((1, 1, 1), (1199, 20, 8), (0, 0, 0)), ((7, 0, 0), (9, 21, 9), (0, 0, 0)),
                                     ((2, 3, 1), (1030, 15, 7), (8, 2, 1)), ((0, 0, 0), (1200, 21, 9), (0, 0, 0)),
                                     ((3, 2, 2), (1027, 19, 8), (0, 0, 0))):
                for op in ("SafeSum", "AbsDiff", "Quot"):
                    out = g.arith(op, [fmt] * 3, [(0.0, 1.0)] * 3, a, b, d.copy(), first, last, off)
                    ref = o.arith(op, [fmt] * 3, [(0.0, 1.0)] * 3, a, b, d.copy(), first, last, off)
                    assert_codes_equal(out, ref, fmt, f"{op} fmt={fmt} {first}->{last} off={off} padded={padded}")
    finally:
        lib.vktHipSetTuningKnob(b"pointwise.padded_rows", -1)


def test_arithmetic_float_bit_patterns(g, o):
    # every float bit pattern class, including NaN payloads, denormals and infinities
    rng = np.random.default_rng(17)
    a = rand_codes(rng, 7, (8, 16, 64), floats="bits")
    b = rand_codes(rng, 7, (8, 16, 64), floats="bits")
    for op in OPS:
        for mapping in ((0.0, 1.0), (-1.0, 3.0)):
            d = np.zeros((8, 16, 64), np.uint32)
            out = g.arith(op, [7] * 3, [mapping] * 3, a, b, d.copy(), (0, 0, 0), (64, 16, 8), (0, 0, 0))
            ref = o.arith(op, [7] * 3, [mapping] * 3, a, b, d.copy(), (0, 0, 0), (64, 16, 8), (0, 0, 0))
            assert_codes_equal(out, ref, 7, f"{op} f32 bits {mapping}")


# ---- Resample -------------------------------------------------------------------------
RESAMPLE_PAIRS = [((10, 1, 1), (7, 1, 1)), ((4, 4, 4), (8, 8, 8)), ((16, 16, 16), (32, 32, 32)),
                  ((37, 23, 11), (64, 40, 19)), ((64, 37, 9), (37, 64, 5)), ((22, 22, 22), (22, 22, 22)),
                  ((33, 33, 33), (16, 16, 16)), ((32, 16, 8), (64, 32, 16)), ((24, 8, 8), (96, 8, 4)),
                  ((10, 9, 8), (7, 6, 5)), ((5, 7, 3), (13, 19, 11))]
FORMAT_PAIRS = [(4, 4), (5, 5), (7, 7), (4, 7), (7, 5), (5, 4), (2, 2)]


@pytest.mark.parametrize("src_dims,dst_dims", RESAMPLE_PAIRS)
@pytest.mark.parametrize("sfmt,dfmt", FORMAT_PAIRS)
def test_resample(g, o, src_dims, dst_dims, sfmt, dfmt):
    rng = np.random.default_rng(abs(hash((src_dims, dst_dims, sfmt, dfmt))) % 2**32)
    src = rand_codes(rng, sfmt, src_dims[::-1])
    for smap, dmap in (((0.0, 1.0), (0.0, 1.0)), ((-1.0, 3.0), (0.0, 1.0))):
        for fm in (0, 1):
            out = g.resample(dfmt, dmap, dst_dims, sfmt, smap, src, fm)
            ref = o.resample(dfmt, dmap, dst_dims, sfmt, smap, src, fm)
            assert_codes_equal(out, ref, dfmt, f"resample {src_dims}->{dst_dims} {sfmt}->{dfmt} fm={fm} {smap}")


def test_resample_float_bit_patterns(g, o):
    rng = np.random.default_rng(23)
    src = rand_codes(rng, 7, (6, 10, 16), floats="bits")
    for fm in (0, 1):
        out = g.resample(7, (0.0, 1.0), (32, 20, 12), 7, (0.0, 1.0), src, fm)
        ref = o.resample(7, (0.0, 1.0), (32, 20, 12), 7, (0.0, 1.0), src, fm)
        assert_codes_equal(out, ref, 7, f"f32 bits fm={fm}")


# ---- Transform -------------------------------------------------------------------------
class _View:
    def __init__(self, b):
        self.bytes = b


def _oracle_transform1(codes, fmt, first, last, op):
    from oracle import binding as ob
    v = ob.Volume(codes.copy(), fmt)
    ob.transform_range1(v, first, last, lambda x, y, z, b, f, lo, hi: op(x, y, z, _View(b)))
    return v.codes


def _oracle_transform2(c1, c2, fmt, first, last, op):
    from oracle import binding as ob
    v1, v2 = ob.Volume(c1.copy(), fmt), ob.Volume(c2.copy(), fmt)
    ob.transform_range2(v1, v2, first, last, (0, 0, 0), lambda x, y, z, b1, b2: op(x, y, z, _View(b1), _View(b2)))
    return v1.codes, v2.codes


def test_transform_examples(g):
    """Host-callback Transform (the reference's function-pointer API, staged through host
    memory under the GPU policy) vs the oracle's TransformRange_serial restatement: unary
    checkerboard of reference src/examples/Arithmetic.cpp:8-21, binary OR of
    src/examples/CoreAlgorithms.c:20-24, and the range form's diagonal marker
    (CoreAlgorithms.c:14-18)."""
    vkt = g.vkt
    n = 32

    def checker(level):
        def op(x, y, z, v):
            x, y, z = x >> level, y >> level, z >> level
            li = z * 32 * 32 + y * 32 + x
            v.bytes[0] = 128 if ((y % 2 == z % 2 and li % 2 == 0) or (y % 2 != z % 2 and li % 2 == 1)) else 0
        return op

    for level in (3, 2):
        v1 = g.volume(np.zeros((n, n, n), np.uint8), 4, (0.0, 1.0))
        g._run(lambda: vkt.Transform(v1, checker(level)))
        ref = _oracle_transform1(np.zeros((n, n, n), np.uint8), 4, (0, 0, 0), (n, n, n), checker(level))
        np.testing.assert_array_equal(v1.to_numpy(), ref)

    ca = np.random.default_rng(1).integers(0, 256, (8, 8, 8), dtype=np.uint8)
    cb = np.random.default_rng(2).integers(0, 256, (8, 8, 8), dtype=np.uint8)
    a = g.volume(ca, 4, (0.0, 1.0))
    b = g.volume(cb, 4, (0.0, 1.0))

    def orop(x, y, z, v1, v2):
        v1.bytes[0] |= v2.bytes[0]
        v2.bytes[0] = v1.bytes[0]

    g._run(lambda: vkt.Transform(a, b, orop))
    ra, rb = _oracle_transform2(ca, cb, 4, (0, 0, 0), (8, 8, 8), orop)
    np.testing.assert_array_equal(a.to_numpy(), ra)
    np.testing.assert_array_equal(b.to_numpy(), rb)

    c = g.volume(np.zeros((24, 24, 24), np.uint8), 4, (0.0, 1.0))

    def diag(x, y, z, v):
        if x == y and y == z:
            v.bytes[0] = 0xFF

    g._run(lambda: vkt.TransformRange(c, 2, 2, 2, 22, 22, 22, diag))
    ref = _oracle_transform1(np.zeros((24, 24, 24), np.uint8), 4, (2, 2, 2), (22, 22, 22), diag)
    np.testing.assert_array_equal(c.to_numpy(), ref)


# ---- runtime semantics -------------------------------------------------------------------
def test_deferred_migration_roundtrip(g):
    """README flow: data written on the CPU, op on the GPU, read back on the CPU."""
    vkt = g.vkt
    v = g.volume(np.zeros((4, 5, 6), np.uint16), 5, (0.0, 1.0))
    v.setValue(1, 2, 3, 0.5)                      # host accessor, CPU policy
    g._gpu()
    assert v.getValue(1, 2, 3) == 0.5             # host accessor under GPU policy (1-voxel copy)
    v.setValue(0, 0, 0, 0.25)
    assert vkt.FillRange(v, 2, 0, 0, 4, 1, 1, 0.75) == vkt.NoError
    g._cpu()
    arr = v.to_numpy()
    assert arr[3, 2, 1] == 32768 and arr[0, 0, 0] == 16384
    assert arr[0, 0, 2] == arr[0, 0, 3] == int(0.75 * 65536)


def test_errors_are_returned_not_ignored(g):
    vkt = g.vkt
    v = g.volume(np.zeros((4, 4, 4), np.uint8), 4, (0.0, 1.0))
    g._gpu()
    try:
        assert vkt.FillRange(v, 0, 0, 0, 5, 4, 4, 0.5) == vkt.InvalidValue   # out of bounds
        assert "outside" in vkt.last_error()
        assert vkt.FillRange(v, 2, 2, 2, 1, 1, 1, 0.5) == vkt.NoError        # empty range
    finally:
        g._cpu()


def test_copy_constructor_on_gpu(g):
    vkt = g.vkt
    v = g.volume(np.arange(64, dtype=np.uint8).reshape(4, 4, 4), 4, (0.0, 1.0))
    g._gpu()
    v.migrate()
    w = vkt.StructuredVolume.CreateCopy(v)
    g._cpu()
    np.testing.assert_array_equal(w.to_numpy(), np.arange(64, dtype=np.uint8).reshape(4, 4, 4))


# ---- paths added for performance: common-phase heads, vector gather, row chain ---------
@pytest.mark.parametrize("fmt", [4, 5, 7])
def test_arithmetic_subbox_phases(g, o, fmt):
    """Sub-boxes whose rows start off an 8-voxel boundary: same phase in every operand
    (vector middle + scalar head/tail) and different phases (scalar path)."""
    rng = np.random.default_rng(fmt + 40)
    a = rand_codes(rng, fmt, (40, 50, 96))
    b = rand_codes(rng, fmt, (40, 50, 96))
    d = rand_codes(rng, fmt, (40, 50, 96))
    for first, last, off in (((5, 3, 2), (91, 47, 39), (0, 0, 0)), ((1, 0, 0), (96, 50, 40), (0, 0, 0)),
                             ((13, 7, 3), (80, 40, 30), (3, 2, 1)), ((8, 1, 1), (16, 49, 39), (0, 0, 0)),
                             ((7, 0, 0), (9, 50, 40), (0, 0, 0))):
        for op in ("SafeSum", "Diff"):
            out = g.arith(op, [fmt] * 3, [(0.0, 1.0)] * 3, a, b, d.copy(), first, last, off)
            ref = o.arith(op, [fmt] * 3, [(0.0, 1.0)] * 3, a, b, d.copy(), first, last, off)
            assert_codes_equal(out, ref, fmt, f"{op} fmt={fmt} {first}->{last}+{off}")


@pytest.mark.parametrize("sfmt,dfmt", [(5, 5), (4, 4), (7, 7), (7, 5), (5, 7), (4, 7), (7, 4)])
def test_resample_vector_gather_and_row_chain(g, o, sfmt, dfmt):
    rng = np.random.default_rng(sfmt * 10 + dfmt)
    for sd, dd in (((96, 20, 12), (64, 24, 16)), ((40, 24, 10), (128, 16, 20)), ((64, 32, 8), (256, 64, 16)),
                   ((256, 8, 4), (512, 16, 8)), ((100, 10, 5), (400, 20, 10)),
                   # LDS-staged gather: 16-byte-multiple source rows, non-integer ratios
                   ((48, 20, 12), (80, 24, 16)), ((256, 12, 6), (144, 20, 9)), ((64, 9, 7), (208, 13, 11))):
        src = rand_codes(rng, sfmt, sd[::-1])
        for smap, dmap in (((0.0, 1.0), (0.0, 1.0)), ((0.0, 1.0), (-1.0, 3.0))):
            for fm in (0, 1):
                out = g.resample(dfmt, dmap, dd, sfmt, smap, src, fm)
                ref = o.resample(dfmt, dmap, dd, sfmt, smap, src, fm)
                assert_codes_equal(out, ref, dfmt, f"resample {sd}->{dd} {sfmt}->{dfmt} fm={fm} {smap}->{dmap}")


@pytest.mark.parametrize("sfmt", [4, 5, 2])
def test_resample_integer_source_to_float_linear(g, o, sfmt):
    """Integer codes -> Float32 "Linear": the chain equals v000 unless the source mapping can
    unmap to -0 (lo = hi = -0 side), which a Float32 destination would store as +0 after the
    chain.  Mappings that can / cannot produce -0, integer and non-integer ratios."""
    rng = np.random.default_rng(sfmt + 7)
    for sd, dd in (((32, 16, 8), (64, 32, 16)), ((30, 17, 9), (64, 40, 16)), ((64, 16, 8), (40, 10, 5))):
        src = rand_codes(rng, sfmt, sd[::-1])
        src.reshape(-1)[:7] = 0   # code 0 -> lo (-0 for lo = -0)
        for smap in ((0.0, 1.0), (-0.0, 1.0), (-0.0, -1.0), (-0.0, -0.0), (-1.0, -0.0), (2.0, -3.0)):
            for dmap in ((0.0, 1.0), (-1.0, 3.0)):
                out = g.resample(7, dmap, dd, sfmt, smap, src, 1)
                ref = o.resample(7, dmap, dd, sfmt, smap, src, 1)
                assert_codes_equal(out, ref, 7, f"resample {sd}->{dd} {sfmt}->7 Linear {smap}->{dmap}")


@pytest.mark.parametrize("dfmt", [7, 5])
def test_resample_chain_sparse_specials(g, o, dfmt):
    """Float32 "Linear" with mostly finite data: clean source rows take the conversion path
    (no neighbour reads), rows near a non-finite value or a -0 take the lerp chain.  Specials
    sit where the chain's neighbourhood crosses rows: a row's first voxel (hi.x of the row
    before), the y+1 / z+1 neighbour rows, the last voxel of the buffer (clamped hi.x)."""
    rng = np.random.default_rng(99 + dfmt)
    for sd, dd in (((64, 32, 8), (128, 64, 16)), ((64, 16, 6), (64, 32, 12)), ((32, 8, 4), (128, 32, 16)),
                   # non-integer ratios: flagged gather (rowDirty + rowChain pre-pass)
                   ((60, 30, 9), (128, 64, 16)), ((64, 16, 6), (48, 20, 5)), ((33, 8, 4), (100, 30, 9))):
        sx, sy, sz = sd
        vals = rng.uniform(0.0, 1.0, size=(sz, sy, sx)).astype(np.float32)
        cases = [
            [],                                            # all clean
            [((1, 3, 0), np.inf)],                         # first voxel of a row: hi.x of row (2,1)
            [((2, 5, 7), -0.0)],                           # -0 as v000
            [((sz - 1, sy - 1, sx - 1), np.nan)],          # last voxel: clamped hi.x read
            [((0, 0, 5), -np.inf), ((sz - 1, 0, 0), np.nan), ((3, sy - 1, sx - 1), -0.0)],
        ]
        for specials in cases:
            v = vals.copy()
            for (z, y, x), val in specials:
                v[z, y, x] = val
            src = v.view(np.uint32)
            for dmap in ((0.0, 1.0), (-1.0, 3.0)):
                out = g.resample(dfmt, dmap, dd, 7, (0.0, 1.0), src, 1)
                ref = o.resample(dfmt, dmap, dd, 7, (0.0, 1.0), src, 1)
                assert_codes_equal(out, ref, dfmt, f"chain {sd}->{dd} specials={specials} dmap={dmap}")


@pytest.mark.parametrize("dfmt", [7, 5])
def test_resample_chain_downsampling_unstaged_rows(g, o, dfmt):
    """Float32 "Linear" when downsampling: the optimistic LDS gather flags only the source rows
    it stages, and rowDirtyUnstagedKernel classifies the rows no task stages.  16 -> 12 per axis
    stages y, z in {0,1,2,4,5,6,8,9,10,12,13,14}: specials in the skipped rows 3, 7, 11, 15 are
    only reachable through the y+1 / z+1 neighbours of a staged row."""
    rng = np.random.default_rng(7 + dfmt)
    for sd, dd in (((16, 16, 16), (12, 12, 12)), ((64, 24, 20), (48, 18, 15)), ((32, 16, 16), (16, 12, 12))):
        sx, sy, sz = sd
        vals = rng.uniform(0.0, 1.0, size=(sz, sy, sx)).astype(np.float32)
        cases = [
            [((1, 3, 5), np.nan)],                          # skipped y row of a staged plane
            [((7, 5, 0), np.inf)],                          # skipped plane, first voxel of a row
            [((3, 3, sx - 1), -np.inf)],                    # skipped row and plane, row end
            [((sz - 1, sy - 1, sx - 1), -0.0)],             # last voxel (clamped neighbours)
            [((2, 2, 3), np.nan), ((11, 7, 1), -0.0)],      # staged row + skipped row
        ]
        for specials in cases:
            v = vals.copy()
            for (z, y, x), val in specials:
                v[z, y, x] = val
            src = v.view(np.uint32)
            for dmap in ((0.0, 1.0), (-1.0, 3.0)):
                out = g.resample(dfmt, dmap, dd, 7, (0.0, 1.0), src, 1)
                ref = o.resample(dfmt, dmap, dd, 7, (0.0, 1.0), src, 1)
                assert_codes_equal(out, ref, dfmt, f"down {sd}->{dd} specials={specials} dmap={dmap}")


@pytest.mark.parametrize("pinned", [0, 1])
def test_large_migrations_keep_the_data(g, pinned):
    """Buffers of >= 64 MiB take the migration fast paths (runtime/Memory.cpp MigrateBuffer): a
    pageable buffer released by the H2D copy kept (pages resident) as the destination of the next
    D2H of the same size, pinned buffers kept for reuse by the next migration of the same size.
    Three round trips of a 128 MiB UInt16 volume with a GPU op in between: the data arrives intact
    each way (a reused destination still holds the previous round's bytes until the copy);
    vktHipReleaseCachedMemory then returns the cached pinned buffer, or the pageable one a last
    H2D released."""
    import ctypes as C
    from volkit_amd._lib import lib
    vkt = g.vkt
    assert lib.vktHipSetPinnedHostAllocation(pinned) == 0
    try:
        rng = np.random.default_rng(31 + pinned)
        codes = rng.integers(0, 60000, (256, 512, 512), dtype=np.uint16)
        v = g.volume(codes, 5, (0.0, 1.0))
        for r in range(3):
            g._gpu()
            v.migrate()
            assert vkt.FillRange(v, 7, 3 + r, 2, 9, 5 + r, 4, 1.0 - 1.0 / 65536) == vkt.NoError
            g._cpu()
            got = v.to_numpy()
            codes[2:4, 3 + r:5 + r, 7:9] = 65535
            np.testing.assert_array_equal(got, codes, err_msg=f"round {r}")
        if not pinned:
            g._gpu()
            v.migrate()   # its pageable host buffer goes to the cache
        del v
        released = C.c_size_t(0)
        assert lib.vktHipReleaseCachedMemory(C.byref(released)) == 0
        assert released.value >= codes.nbytes
    finally:
        lib.vktHipSetPinnedHostAllocation(0)


@pytest.mark.parametrize("shape", [(16, 24, 40), (256, 512, 512)])
def test_failed_migration_keeps_the_data(g, shape):
    """A host -> HBM migration whose device allocation fails (test knob memory.fail_next_alloc)
    keeps the only copy of the data: the buffer stays in host memory (same pointer), the
    migration and the algorithm that asked for it return InvalidValue naming the failure, and
    after the knob is spent the next migration succeeds and the op runs bit-exactly.  The
    128 MiB case takes the large-buffer path whose source the reference-style migrate freed
    (runtime/Memory.cpp MigrateBuffer; reference include/cpp/vkt/ManagedBuffer.hpp:168-198)."""
    from volkit_amd._lib import lib
    vkt = g.vkt
    rng = np.random.default_rng(41 + shape[0])
    codes = rng.integers(0, 65536, shape, dtype=np.uint16)
    v = g.volume(codes, 5, (0.0, 1.0))
    host_ptr = v.getData()
    try:
        assert lib.vktHipSetTuningKnob(b"memory.fail_next_alloc", 2) == 0
        g._gpu()
        assert v.migrateChecked() == vkt.InvalidValue
        assert "allocation failed" in vkt.last_error()
        assert v.getData() == host_ptr          # (retries and fails again) still the host buffer
        assert lib.vktHipSetTuningKnob(b"memory.fail_next_alloc", 1) == 0
        assert vkt.FillRange(v, 1, 1, 1, 3, 3, 3, 1.0) == vkt.InvalidValue
        assert "FillRange_hip" in vkt.last_error() and "allocation failed" in vkt.last_error()
        g._cpu()
        assert v.getData() == host_ptr
        np.testing.assert_array_equal(v.to_numpy(), codes)
        # knob spent: the next migration and op succeed
        g._gpu()
        assert v.migrateChecked() == vkt.NoError
        assert v.getData() != host_ptr
        assert vkt.FillRange(v, 1, 1, 1, 3, 3, 3, 1.0 - 1.0 / 65536) == vkt.NoError
        g._cpu()
        codes[1:3, 1:3, 1:3] = 65535
        np.testing.assert_array_equal(v.to_numpy(), codes)
    finally:
        lib.vktHipSetTuningKnob(b"memory.fail_next_alloc", 0)
        g._cpu()


def test_failed_migration_in_a_copy_constructor(g):
    """CreateCopy under the GPU policy of a host volume whose migration fails: the copy still
    gets the source's bytes (copied across address spaces, detail::CopyBetween), the source keeps
    them."""
    from volkit_amd._lib import lib
    vkt = g.vkt
    codes = np.arange(4 * 6 * 10, dtype=np.uint8).reshape(4, 6, 10)
    v = g.volume(codes, 4, (0.0, 1.0))
    try:
        assert lib.vktHipSetTuningKnob(b"memory.fail_next_alloc", 1) == 0
        g._gpu()
        w = vkt.StructuredVolume.CreateCopy(v)   # v's migration fails, w's allocation succeeds
        g._cpu()
        np.testing.assert_array_equal(v.to_numpy(), codes)
        np.testing.assert_array_equal(w.to_numpy(), codes)
    finally:
        lib.vktHipSetTuningKnob(b"memory.fail_next_alloc", 0)
        g._cpu()
