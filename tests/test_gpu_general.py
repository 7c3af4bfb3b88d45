"""The general vector path of the pointwise engine (kernels/Pointwise.hpp, pointwiseGenKernel)
vs the oracle: boxes the aligned path cannot take -- operands at different 8-voxel phases
(CopyRange x0 = 3 -> 0, arithmetic dstOffset), row pitches that are not multiples of 8,
clamped CopyRange sources (halo copies past every border, reference Copy_serial.hpp:38-40),
format conversion between voxel sizes, view pointers that are not 16-B aligned.  Volumes live
in plain device buffers and the backend is called through the C ABI (include/volkit_hip.h),
so one case costs a kernel launch, not a volume migration.  Bit-exact (NaN matches NaN)."""
import ctypes as C

import numpy as np
import pytest

from backends import CODE_DTYPE, OracleBackend
from test_gpu_parity import assert_codes_equal, rand_codes

pytestmark = pytest.mark.gpu

BPV = {1: 1, 2: 2, 3: 4, 4: 1, 5: 2, 6: 4, 7: 4}
OPS = ["Sum", "Diff", "Prod", "Quot", "AbsDiff", "SafeSum", "SafeDiff", "SafeProd", "SafeQuot", "SafeAbsDiff"]


@pytest.fixture(scope="module")
def o():
    return OracleBackend()


@pytest.fixture(scope="module")
def lib():
    import torch
    from volkit_amd._lib import lib as L
    torch.cuda.set_device(0)
    return L


class Dev:
    """A volume's codes in a device buffer at byte offset `pad` (view pointer pad bytes past a
    256-B aligned allocation)."""

    def __init__(self, codes, fmt, mapping=(0.0, 1.0), pad=0):
        import torch
        from volkit_amd._lib import HipVolumeView_t
        self.codes = np.ascontiguousarray(codes)
        self.fmt, self.pad = fmt, pad
        z, y, x = codes.shape
        raw = self.codes.view(np.uint8).reshape(-1)
        self.buf = torch.zeros(raw.size + pad + 64, dtype=torch.uint8, device="cuda")
        self.buf[pad:pad + raw.size].copy_(torch.from_numpy(raw.copy()))
        self.view = HipVolumeView_t(self.buf.data_ptr() + pad, x, y, z, fmt, float(mapping[0]), float(mapping[1]))

    def read(self):
        import torch
        torch.cuda.synchronize()
        raw = self.buf[self.pad:self.pad + self.codes.nbytes].cpu().numpy()
        return raw.view(CODE_DTYPE[self.fmt]).reshape(self.codes.shape)


def vec(x):
    from volkit_amd._lib import Vec3i_t
    return Vec3i_t(*x)


def last_error():
    from volkit_amd import _lib
    return _lib.last_error()


def knob(lib, on):
    assert lib.vktHipSetTuningKnob(b"pointwise.general", 1 if on else 0) == 0


def copy_case(lib, o, sfmt, dfmt, smap, dmap, src, dst_init, first, last, off, spad=0, dpad=0, what=""):
    s = Dev(src, sfmt, smap, spad)
    d = Dev(dst_init, dfmt, dmap, dpad)
    err = lib.vktHipCopyRange(d.view, s.view, vec(first), vec(last), vec(off))
    assert err == 0, f"{what}: {last_error()}"
    ref = o.copy_range(dfmt, dmap, None, dst_init.copy(), sfmt, smap, src, first, last, off)
    assert_codes_equal(d.read(), ref, dfmt, what)


@pytest.mark.parametrize("sfmt,dfmt", [(4, 4), (5, 5), (7, 7), (2, 2), (6, 6)])
def test_copy_phase_sweep_bytewise(lib, o, sfmt, dfmt):
    """Every source x phase against several destination phases, rows not multiples of 8,
    ranges clamped on every side."""
    rng = np.random.default_rng(7 * sfmt + dfmt)
    src = rand_codes(rng, sfmt, (5, 7, 29))          # dims (29, 7, 5)
    dinit = rand_codes(rng, dfmt, (6, 6, 43))        # dims (43, 6, 6)
    for sx in range(9):
        for dx in (0, 1, 3, 5, 7, 8):
            # interior box, then a box clamped at x/y/z on both sides
            for first, last in (((sx, 1, 1), (sx + 19, 6, 4)), ((sx - 5, -2, -1), (sx + 30, 4, 5))):
                n = [l - f for f, l in zip(first, last)]
                off = (dx, 0, 0) if n[0] + dx <= 43 else (43 - n[0], 0, 0)
                copy_case(lib, o, sfmt, dfmt, (0.0, 1.0), (0.0, 1.0), src, dinit, first, last, off,
                          what=f"copy {sfmt} sx={sx} dx={dx} {first}->{last}+{off}")


@pytest.mark.parametrize("sfmt,dfmt", [(5, 4), (4, 5), (4, 7), (7, 4), (5, 7), (7, 5), (2, 6), (6, 2), (1, 5), (5, 3)])
@pytest.mark.parametrize("maps", [((0.0, 1.0), (0.0, 1.0)), ((0.0, 1.0), (-1.0, 3.0)), ((0.25, 7.5), (0.0, 1.0))])
def test_copy_convert_phases(lib, o, sfmt, dfmt, maps):
    """CopyRange with unmap -> map between voxel sizes (general path with mixed sizes)."""
    rng = np.random.default_rng(13 * sfmt + dfmt)
    src = rand_codes(rng, sfmt, (4, 9, 37))
    dinit = rand_codes(rng, dfmt, (7, 12, 43))
    for first, last, off in (((0, 0, 0), (37, 9, 4), (0, 0, 0)), ((3, 1, 0), (30, 8, 4), (1, 0, 1)),
                             ((-2, -1, -1), (39, 10, 5), (0, 0, 0)), ((5, 2, 1), (12, 3, 2), (7, 5, 3))):
        copy_case(lib, o, sfmt, dfmt, maps[0], maps[1], src, dinit, first, last, off,
                  what=f"convert {sfmt}->{dfmt} {maps} {first}->{last}+{off}")


@pytest.mark.parametrize("fmt", [4, 5, 7])
def test_copy_unaligned_view_pointers(lib, o, fmt):
    """View pointers one voxel (not 16 B) past an aligned address, source and destination."""
    b = BPV[fmt]
    rng = np.random.default_rng(fmt)
    src = rand_codes(rng, fmt, (3, 5, 64))
    dinit = rand_codes(rng, fmt, (3, 5, 64))
    for spad, dpad in ((b, 0), (0, b), (3 * b, 5 * b), (8 * b, 8 * b)):
        for first, last, off in (((0, 0, 0), (64, 5, 3), (0, 0, 0)), ((1, 0, 0), (60, 5, 3), (2, 0, 0)),
                                 ((-1, 0, 0), (63, 5, 3), (0, 0, 0))):
            copy_case(lib, o, fmt, fmt, (0.0, 1.0), (0.0, 1.0), src, dinit, first, last, off, spad, dpad,
                      what=f"copy pads {spad},{dpad} {first}->{last}+{off}")


def test_copy_narrow_rows(lib, o):
    """Boxes 1..9 voxels wide: every item straddles a row end or a clamped border."""
    rng = np.random.default_rng(3)
    for fmt in (4, 5, 7):
        src = rand_codes(rng, fmt, (4, 5, 11))
        dinit = rand_codes(rng, fmt, (4, 6, 13))
        for w in range(1, 10):
            for fx in (-3, 0, 1, 6):
                copy_case(lib, o, fmt, fmt, (0.0, 1.0), (0.0, 1.0), src, dinit, (fx, -1, 0), (fx + w, 5, 4), (2, 0, 0),
                          what=f"narrow fmt={fmt} w={w} fx={fx}")


@pytest.mark.parametrize("fmt", [4, 5, 7])
@pytest.mark.parametrize("mapping", [(0.0, 1.0), (-1.0, 3.0)])
def test_arith_dst_offset_phases(lib, o, fmt, mapping):
    """Arithmetic with an x dstOffset of every phase: destination and sources at different
    phases (the packed UInt16 / UInt8 unit-mapping functors and the float codec)."""
    rng = np.random.default_rng(fmt)
    a = rand_codes(rng, fmt, (4, 6, 45))
    b = rand_codes(rng, fmt, (4, 6, 45))
    dinit = rand_codes(rng, fmt, (5, 7, 53))
    from volkit_amd._lib import lib as L
    for op in OPS:
        idx = OPS.index(op)
        for dx in range(8):
            for first, last in (((0, 0, 0), (45, 6, 4)), ((3, 1, 1), (40, 5, 3))):
                da, db, dd = Dev(a, fmt, mapping), Dev(b, fmt, mapping, 2 * BPV[fmt]), Dev(dinit, fmt, mapping)
                assert L.vktHipArithmeticRange(idx, dd.view, da.view, db.view, vec(first), vec(last),
                                               vec((dx, 1, 1))) == 0
                ref = o.arith(op, [fmt] * 3, [mapping] * 3, a, b, dinit.copy(), first, last, (dx, 1, 1))
                assert_codes_equal(dd.read(), ref, fmt, f"{op} fmt={fmt} {mapping} dx={dx} {first}->{last}")


@pytest.mark.parametrize("fmt", [4, 7, 3, 6])
@pytest.mark.parametrize("pad", [0, 16, 8])
def test_collapsed_row_contiguous_lanes(lib, o, fmt, pad):
    """Whole-volume (one collapsed row) Fill, Copy and arithmetic on 1- and 4-byte formats:
    full quanta with 16-B aligned operands take the contiguous-lane loop (UInt8 item pairs in
    one 16-B access, Float32 items as two 4-voxel halves 1 KiB apart), the partial last
    quantum and 8-B aligned views (pad 8) the per-item loop.  Every voxel vs the oracle."""
    rng = np.random.default_rng(fmt * 10 + pad)
    dims = (3, 7, 613)                       # 12 873 voxels: several full quanta + a partial one
    a = rand_codes(rng, fmt, dims)
    b = rand_codes(rng, fmt, dims)
    dinit = rand_codes(rng, fmt, dims)
    first, last = (0, 0, 0), (dims[2], dims[1], dims[0])
    from volkit_amd._lib import lib as L
    for op in ("Sum", "SafeDiff", "Prod"):
        da, db, dd = Dev(a, fmt, pad=pad), Dev(b, fmt, pad=pad), Dev(dinit, fmt, pad=pad)
        assert L.vktHipArithmeticRange(OPS.index(op), dd.view, da.view, db.view, vec(first), vec(last),
                                       vec((0, 0, 0))) == 0, last_error()
        ref = o.arith(op, [fmt] * 3, [(0.0, 1.0)] * 3, a, b, dinit.copy(), first, last, (0, 0, 0))
        assert_codes_equal(dd.read(), ref, fmt, f"{op} fmt={fmt} pad={pad}")
    copy_case(lib, o, fmt, fmt, (0.0, 1.0), (0.0, 1.0), a, dinit, first, last, (0, 0, 0), pad, pad,
              f"copy fmt={fmt} pad={pad}")
    d = Dev(dinit, fmt, pad=pad)
    assert L.vktHipFillRange(d.view, vec(first), vec(last), C.c_float(0.375)) == 0, last_error()
    ref = o.fill_range(fmt, (0.0, 1.0), (dims[2], dims[1], dims[0]), dinit.copy(), first, last, 0.375)
    assert_codes_equal(d.read(), ref, fmt, f"fill fmt={fmt} pad={pad}")


@pytest.mark.parametrize("fmt", [4, 5, 7])
@pytest.mark.parametrize("knobs", [(1, 4, 8192), (1, 2, 0), (1, 8, 6656), (0, 4, 0), (3, 1, 0), (3, 2, 5632)])
def test_row_kernel(lib, o, fmt, knobs):
    """The MODE-0-only kernel for one collapsed row (pointwiseRowKernel: UInt8 / UInt16 copies and
    arithmetic, knob pointwise.row_kernel bits 0 / 1, with the items per lane of
    pointwise.u8_unroll / u16_unroll and the occupancy cap pointwise.row_lds; Float32 keeps the
    general kernel): voxel counts
    that are whole 8-voxel items (no scalar edges -- the condition for the kernel), full and
    partial quanta, 16-B and 8-B aligned views.  Sum / SafeDiff / Prod, Copy and Fill vs the
    oracle."""
    from volkit_amd._lib import lib as L
    rk, unroll, lds = knobs
    rng = np.random.default_rng(fmt * 100 + unroll)
    try:
        for k, v in ((b"pointwise.row_kernel", rk), (b"pointwise.u8_unroll", unroll if fmt == 4 else 2),
                     (b"pointwise.u16_unroll", unroll if fmt == 5 and unroll <= 2 else 2), (b"pointwise.row_lds", lds),
                     (b"pointwise.row_lds_u8", lds)):
            assert L.vktHipSetTuningKnob(k, v) == 0
        for dims in ((3, 7, 616), (1, 1, 4096), (2, 5, 1032)):
            a, b, dinit = (rand_codes(rng, fmt, dims) for _ in range(3))
            first, last = (0, 0, 0), (dims[2], dims[1], dims[0])
            for pad in (0, 8):
                for op in ("Sum", "SafeDiff", "Prod"):
                    da, db, dd = Dev(a, fmt, pad=pad), Dev(b, fmt, pad=pad), Dev(dinit, fmt, pad=pad)
                    assert L.vktHipArithmeticRange(OPS.index(op), dd.view, da.view, db.view, vec(first), vec(last),
                                                   vec((0, 0, 0))) == 0, last_error()
                    ref = o.arith(op, [fmt] * 3, [(0.0, 1.0)] * 3, a, b, dinit.copy(), first, last, (0, 0, 0))
                    assert_codes_equal(dd.read(), ref, fmt, f"{op} fmt={fmt} dims={dims} pad={pad} knobs={knobs}")
                copy_case(lib, o, fmt, fmt, (0.0, 1.0), (0.0, 1.0), a, dinit, first, last, (0, 0, 0), pad, pad,
                          f"copy fmt={fmt} dims={dims} pad={pad} knobs={knobs}")
                d = Dev(dinit, fmt, pad=pad)
                assert L.vktHipFillRange(d.view, vec(first), vec(last), C.c_float(0.375)) == 0, last_error()
                ref = o.fill_range(fmt, (0.0, 1.0), (dims[2], dims[1], dims[0]), dinit.copy(), first, last, 0.375)
                assert_codes_equal(d.read(), ref, fmt, f"fill fmt={fmt} dims={dims} pad={pad} knobs={knobs}")
    finally:
        for k in (b"pointwise.row_kernel", b"pointwise.u8_unroll", b"pointwise.u16_unroll", b"pointwise.row_lds",
                  b"pointwise.row_lds_u8"):
            L.vktHipSetTuningKnob(k, -1)


@pytest.mark.parametrize("fmt", [4, 5])
@pytest.mark.parametrize("rk", [3, 0])
def test_rows_kernel(lib, o, fmt, rk):
    """Multi-row boxes on the MODE-1-only kernel (knob pointwise.rows_kernel 3, the default: UInt8
    copies at 1 KiB per stream, UInt8 / UInt16 arithmetic at 2 KiB; 32-bit row math, no scalar
    edges: padded rows, with and without sector completion, or rows of whole items) and on the
    general kernel (0): Copy, SumRange, SafeSum vs the oracle."""
    from volkit_amd._lib import lib as L
    rng = np.random.default_rng(fmt * 7 + rk)
    dims = (9, 40, 272)
    a, b, dinit = (rand_codes(rng, fmt, dims) for _ in range(3))
    try:
        for k, v in ((b"pointwise.rows_kernel", rk),):
            assert L.vktHipSetTuningKnob(k, v) == 0
        for merge in (1, 0):
            assert L.vktHipSetTuningKnob(b"pointwise.merge_sectors", merge) == 0
            for first, last in (((100, 3, 1), (200, 37, 8)), ((0, 1, 1), (256, 39, 9)), ((16, 2, 0), (144, 40, 9)),
                                ((3, 0, 2), (269, 40, 7))):
                for op in ("Sum", "SafeSum"):
                    da, db, dd = Dev(a, fmt), Dev(b, fmt), Dev(dinit, fmt)
                    assert L.vktHipArithmeticRange(OPS.index(op), dd.view, da.view, db.view, vec(first), vec(last),
                                                   vec((0, 0, 0))) == 0, last_error()
                    ref = o.arith(op, [fmt] * 3, [(0.0, 1.0)] * 3, a, b, dinit.copy(), first, last, (0, 0, 0))
                    assert_codes_equal(dd.read(), ref, fmt, f"{op} fmt={fmt} rk={rk} {first}->{last} merge={merge}")
                copy_case(lib, o, fmt, fmt, (0.0, 1.0), (0.0, 1.0), a, dinit, first, last, first, 0, 0,
                          f"copy fmt={fmt} rk={rk} {first}->{last} merge={merge}")
    finally:
        for k in (b"pointwise.rows_kernel", b"pointwise.merge_sectors"):
            L.vktHipSetTuningKnob(k, -1)


@pytest.mark.parametrize("fmt", [4, 7, 6])
@pytest.mark.parametrize("box", [((0, 1, 1), (256, 30, 6)),      # rows of 32 items (even)
                                 ((16, 2, 0), (136, 29, 7)),     # 15 items per row
                                 ((8, 0, 1), (264, 31, 5)),      # 32 items, rows start 8 voxels in
                                 ((3, 1, 1), (253, 30, 6))])     # padded rows: per-item loop
def test_multirow_contiguous_lanes(lib, o, fmt, box):
    """Multi-row boxes through the contiguous-lane loop (4-byte formats; rows without padded
    edges, 16-B aligned rows in every operand) and the cases that stay on the per-item loop
    (UInt8, padded rows).  Copy and SafeSum vs the oracle."""
    rng = np.random.default_rng(fmt + box[0][0])
    dims = (8, 32, 272)
    a = rand_codes(rng, fmt, dims)
    b = rand_codes(rng, fmt, dims)
    dinit = rand_codes(rng, fmt, dims)
    first, last = box
    from volkit_amd._lib import lib as L
    da, db, dd = Dev(a, fmt), Dev(b, fmt), Dev(dinit, fmt)
    assert L.vktHipArithmeticRange(OPS.index("SafeSum"), dd.view, da.view, db.view, vec(first), vec(last),
                                   vec((0, 0, 0))) == 0, last_error()
    ref = o.arith("SafeSum", [fmt] * 3, [(0.0, 1.0)] * 3, a, b, dinit.copy(), first, last, (0, 0, 0))
    assert_codes_equal(dd.read(), ref, fmt, f"SafeSum fmt={fmt} box={box}")
    copy_case(lib, o, fmt, fmt, (0.0, 1.0), (0.0, 1.0), a, dinit, first, last, (0, 0, 0), 0, 0,
              f"copy fmt={fmt} box={box}")


@pytest.mark.parametrize("x0", list(range(16)) + [37, 50, 63])
@pytest.mark.parametrize("dims", [(6, 48, 96), (5, 40, 192)], ids=["rows96", "rows192-merge"])
def test_uint8_pair16_rows(lib, o, x0, dims):
    """UInt8 multi-row boxes on the 16-voxel grid (pair16: one 16-B access per lane for two
    items, byte-range stores at the row ends, kernels/KernelCommon.hpp storeByteRange16): every
    row-start phase x0 mod 16 times row lengths covering every tail length 1..16 and rows shorter
    than one access, for Copy (same offset: the aligned path) and SafeSum / Sum vs the oracle,
    with the knob pointwise.u8_pairs on and off.  On 192-voxel rows (64-B aligned pitches) boxes
    with >= 64-B gaps take 64-B sector completion (pairs in the end sectors merged with the
    destination's own bytes; knob pointwise.merge_sectors = 2 extends it to the arithmetic ops).
    The destination's bytes outside the box must survive."""
    rng = np.random.default_rng(100 + x0)
    if x0 >= 16 and dims[2] == 96:
        pytest.skip("phases past 16 only on the wide rows")
    a = rand_codes(rng, 4, dims)
    b = rand_codes(rng, 4, dims)
    dinit = rand_codes(rng, 4, dims)
    X = dims[2]
    from volkit_amd._lib import lib as L
    try:
        for on, mk in ((1, -1), (1, 2), (0, -1)):
            assert L.vktHipSetTuningKnob(b"pointwise.u8_pairs", on) == 0
            assert L.vktHipSetTuningKnob(b"pointwise.merge_sectors", mk) == 0
            for w in (1, 3, 8, 15, 16, 17, 24, 31, 32, 33, 45, 64, 65, 100, 127, X - x0):
                if x0 + w > X:
                    continue
                first, last = (x0, 1, 0), (x0 + w, dims[1] - 1, dims[0])
                for op in ("SafeSum", "Sum"):
                    da, db, dd = Dev(a, 4), Dev(b, 4), Dev(dinit, 4)
                    assert L.vktHipArithmeticRange(OPS.index(op), dd.view, da.view, db.view, vec(first), vec(last),
                                                   vec((0, 0, 0))) == 0, last_error()
                    ref = o.arith(op, [4] * 3, [(0.0, 1.0)] * 3, a, b, dinit.copy(), first, last, (0, 0, 0))
                    assert_codes_equal(dd.read(), ref, 4, f"{op} pairs={on} merge={mk} x0={x0} w={w}")
                copy_case(lib, o, 4, 4, (0.0, 1.0), (0.0, 1.0), a, dinit, first, last, first, 0, 0,
                          f"copy pairs={on} merge={mk} x0={x0} w={w}")
    finally:
        assert L.vktHipSetTuningKnob(b"pointwise.u8_pairs", -1) == 0
        assert L.vktHipSetTuningKnob(b"pointwise.merge_sectors", -1) == 0


@pytest.mark.parametrize("x0", [0, 3, 4, 13, 37])
def test_three_stream_sector_completion(lib, o, x0):
    """pointwise.merge_sectors = 2: 64-B sector completion for the 3-stream ops on the aligned
    path (UInt16 packed functor, Float32 halves, UInt8 pairs): SafeSum / Sum over padded rows
    with >= 64-B gaps vs the oracle; bytes outside the box keep their values."""
    from volkit_amd._lib import lib as L
    try:
        assert L.vktHipSetTuningKnob(b"pointwise.merge_sectors", 2) == 0
        for fmt, X in ((5, 128), (7, 64), (4, 256)):
            rng = np.random.default_rng(500 + x0 + fmt)
            dims = (4, 20, X)
            a, b, dinit = rand_codes(rng, fmt, dims), rand_codes(rng, fmt, dims), rand_codes(rng, fmt, dims)
            for w in (1, 5, 17, X // 2, X - x0 - 40):
                if w <= 0 or x0 + w > X:
                    continue
                first, last = (x0, 1, 0), (x0 + w, 19, 4)
                for op in ("SafeSum", "Sum"):
                    da, db, dd = Dev(a, fmt), Dev(b, fmt), Dev(dinit, fmt)
                    assert L.vktHipArithmeticRange(OPS.index(op), dd.view, da.view, db.view, vec(first), vec(last),
                                                   vec((0, 0, 0))) == 0, last_error()
                    ref = o.arith(op, [fmt] * 3, [(0.0, 1.0)] * 3, a, b, dinit.copy(), first, last, (0, 0, 0))
                    assert_codes_equal(dd.read(), ref, fmt, f"{op} fmt={fmt} x0={x0} w={w}")
    finally:
        assert L.vktHipSetTuningKnob(b"pointwise.merge_sectors", -1) == 0


@pytest.mark.parametrize("fmt", [7, 6])
@pytest.mark.parametrize("x0", [0, 1, 3, 4, 7, 9, 13, 16])
def test_float32_padded_rows_halves(lib, o, fmt, x0):
    """4-byte multi-row boxes with padded rows through the contiguous-lane shape
    (Geom::f32halves: every 16-B half of an item stored whole, as its row's dwords, or merged
    with the destination's own dwords under 64-B sector completion): row phases x0 mod 8 and
    widths covering every tail, on 64-voxel rows (256-B pitches: completion where the gaps
    allow) -- Copy / SafeSum / Diff, knobs pointwise.f32_halves and merge_sectors on and off."""
    rng = np.random.default_rng(400 + x0 + fmt)
    dims = (5, 36, 64)
    a = rand_codes(rng, fmt, dims)
    b = rand_codes(rng, fmt, dims)
    dinit = rand_codes(rng, fmt, dims)
    from volkit_amd._lib import lib as L
    try:
        for on, mk in ((1, -1), (1, 0), (0, -1)):
            assert L.vktHipSetTuningKnob(b"pointwise.f32_halves", on) == 0
            assert L.vktHipSetTuningKnob(b"pointwise.merge_sectors", mk) == 0
            for w in (1, 2, 3, 4, 5, 8, 11, 16, 17, 29, 33, 48, 64 - x0):
                if x0 + w > 64:
                    continue
                first, last = (x0, 1, 0), (x0 + w, 35, 5)
                for op in ("SafeSum", "Diff"):
                    da, db, dd = Dev(a, fmt), Dev(b, fmt), Dev(dinit, fmt)
                    assert L.vktHipArithmeticRange(OPS.index(op), dd.view, da.view, db.view, vec(first), vec(last),
                                                   vec((0, 0, 0))) == 0, last_error()
                    ref = o.arith(op, [fmt] * 3, [(0.0, 1.0)] * 3, a, b, dinit.copy(), first, last, (0, 0, 0))
                    assert_codes_equal(dd.read(), ref, fmt, f"{op} halves={on} merge={mk} x0={x0} w={w}")
                copy_case(lib, o, fmt, fmt, (0.0, 1.0), (0.0, 1.0), a, dinit, first, last, first, 0, 0,
                          f"copy halves={on} merge={mk} x0={x0} w={w}")
    finally:
        assert L.vktHipSetTuningKnob(b"pointwise.f32_halves", -1) == 0
        assert L.vktHipSetTuningKnob(b"pointwise.merge_sectors", -1) == 0


@pytest.mark.parametrize("fmt", [4, 7, 6])
@pytest.mark.parametrize("sx", [0, 1, 5, 8, 15, 16, 37, 63])
def test_uint8_wide_general_path(lib, o, sx, fmt):
    """1- and 4-byte boxes on the general path with 16-B items (GenGeom::wide: 16 UInt8 / 4
    Float32 voxels, one 16-B store per lane, byte-range or sector-merged row ends): source x
    phases against destination x phases, widths around the item and 64-B units, gaps that allow /
    forbid sector completion (192-voxel rows), clamped sources past x = 0 / dimX - 1, and SafeSum /
    Diff with an x dstOffset -- knob pointwise.u8_wide / f32_wide on and off, vs the oracle."""
    rng = np.random.default_rng(300 + sx + fmt)
    dims = (5, 24, 192)
    src = rand_codes(rng, fmt, dims)
    src2 = rand_codes(rng, fmt, dims)
    dinit = rand_codes(rng, fmt, dims)
    knob_name = b"pointwise.u8_wide" if fmt == 4 else b"pointwise.f32_wide"
    from volkit_amd._lib import lib as L
    try:
        # f32_wide 2 (the default): 16-B items for the copies only, 8-voxel items for SafeSum / Diff
        for on, mk in ((1, -1), (1, 2), (2, -1), (0, -1)):
            assert L.vktHipSetTuningKnob(knob_name, on) == 0
            assert L.vktHipSetTuningKnob(b"pointwise.merge_sectors", mk) == 0
            for dx in (0, 3, 16, 17, 64):
                for w in (1, 7, 16, 17, 33, 64, 100, 128, 150):
                    if dx + w > 192:
                        continue
                    first, last = (sx, 2, 1), (sx + w, 22, 5)
                    if sx + w <= 192:
                        copy_case(lib, o, fmt, fmt, (0.0, 1.0), (0.0, 1.0), src, dinit, first, last, (dx, 1, 0),
                                  what=f"copy wide={on} sx={sx} dx={dx} w={w}")
                    # clamped source: starts left of x = 0
                    copy_case(lib, o, fmt, fmt, (0.0, 1.0), (0.0, 1.0), src, dinit, (sx - 20, -1, 0),
                              (sx - 20 + w, 22, 4), (dx, 0, 1), what=f"clamped copy wide={on} sx={sx} dx={dx} w={w}")
                    if sx + w <= 192 and dx + w <= 192:
                        off = (dx - sx, 1, 0)
                        for op in ("SafeSum", "Diff"):
                            da, db, dd = Dev(src, fmt), Dev(src2, fmt), Dev(dinit, fmt)
                            assert L.vktHipArithmeticRange(OPS.index(op), dd.view, da.view, db.view, vec(first),
                                                           vec(last), vec(off)) == 0, last_error()
                            ref = o.arith(op, [fmt] * 3, [(0.0, 1.0)] * 3, src, src2, dinit.copy(), first, last, off)
                            assert_codes_equal(dd.read(), ref, fmt, f"{op} wide={on} sx={sx} dx={dx} w={w}")
    finally:
        assert L.vktHipSetTuningKnob(knob_name, -1) == 0
        assert L.vktHipSetTuningKnob(b"pointwise.merge_sectors", -1) == 0


def test_general_knob_matches_scalar_kernel(lib, o):
    """The same phase-shifted and clamped cases through the general path and, with the knob
    off, through the per-voxel kernel: both equal the oracle."""
    rng = np.random.default_rng(11)
    src = rand_codes(rng, 5, (6, 10, 70))
    dinit = rand_codes(rng, 5, (6, 10, 70))
    try:
        for on in (True, False):
            knob(lib, on)
            for first, last, off in (((3, 0, 0), (70, 10, 6), (0, 0, 0)), ((-4, -3, -2), (66, 12, 7), (0, 0, 0)),
                                     ((1, 2, 3), (69, 9, 5), (0, 1, 0))):
                n = [l - f for f, l in zip(first, last)]
                if n[0] > 70 or n[1] > 10 or n[2] > 6:
                    continue
                copy_case(lib, o, 5, 5, (0.0, 1.0), (0.0, 1.0), src, dinit, first, last, off,
                          what=f"knob={on} {first}->{last}+{off}")
    finally:
        knob(lib, True)
        assert lib.vktHipSetTuningKnob(b"pointwise.general", -1) == 0


@pytest.mark.parametrize("fmt", [4, 5, 7])
def test_general_path_kernels(lib, o, fmt):
    """The general vector path's kernels -- one per span path for 1- and 4-byte destinations
    (wide 16-B items, 32-bit addressing, and with knob pointwise.general_32bit 0 the 64-bit row
    paths), the combined kernel for 2-byte ones: phase-shifted copies, clamped halos and a shifted
    SafeSum, every one vs the oracle."""
    rng = np.random.default_rng(fmt + 77)
    src = rand_codes(rng, fmt, (7, 12, 150))
    src2 = rand_codes(rng, fmt, (7, 12, 150))
    dinit = rand_codes(rng, fmt, (7, 12, 150))
    from volkit_amd._lib import lib as L
    try:
        for g32 in (1, 0):
            assert L.vktHipSetTuningKnob(b"pointwise.general_32bit", g32) == 0
            for first, last, off in (((3, 0, 0), (150, 12, 7), (0, 0, 0)), ((-4, -3, -2), (146, 9, 5), (0, 0, 0)),
                                     ((5, 2, 1), (141, 11, 6), (2, 1, 0))):
                copy_case(lib, o, fmt, fmt, (0.0, 1.0), (0.0, 1.0), src, dinit, first, last, off,
                          what=f"g32={g32} {first}->{last}+{off}")
            first, last, off = (9, 1, 1), (140, 11, 6), (-7, 1, 0)
            da, db, dd = Dev(src, fmt), Dev(src2, fmt), Dev(dinit, fmt)
            assert L.vktHipArithmeticRange(OPS.index("SafeSum"), dd.view, da.view, db.view, vec(first), vec(last),
                                           vec(off)) == 0, last_error()
            ref = o.arith("SafeSum", [fmt] * 3, [(0.0, 1.0)] * 3, src, src2, dinit.copy(), first, last, off)
            assert_codes_equal(dd.read(), ref, fmt, f"SafeSum g32={g32}")
    finally:
        L.vktHipSetTuningKnob(b"pointwise.general_32bit", -1)


def test_general_multi_launch(lib, o):
    """Launch split of the general path (knob pointwise.max_quanta_per_launch = 1)."""
    rng = np.random.default_rng(12)
    src = rand_codes(rng, 5, (5, 9, 300))
    dinit = rand_codes(rng, 5, (6, 11, 301))
    assert lib.vktHipSetTuningKnob(b"pointwise.max_quanta_per_launch", 1) == 0
    try:
        copy_case(lib, o, 5, 5, (0.0, 1.0), (0.0, 1.0), src, dinit, (3, -1, 0), (300, 10, 5), (1, 0, 0),
                  what="multi-launch")
    finally:
        assert lib.vktHipSetTuningKnob(b"pointwise.max_quanta_per_launch", -1) == 0


def test_copy_halo_large(lib, o):
    """A clamped halo copy at a size with many workgroups: 258 x 130 x 9 UInt16 from first =
    (-1, -1, -1) of a 256 x 128 x 7 volume, oracle on the whole result."""
    rng = np.random.default_rng(21)
    src = rand_codes(rng, 5, (7, 128, 256))
    dinit = np.zeros((9, 130, 258), np.uint16)
    copy_case(lib, o, 5, 5, (0.0, 1.0), (0.0, 1.0), src, dinit, (-1, -1, -1), (257, 129, 8), (0, 0, 0),
              what="halo 258x130x9")


@pytest.mark.parametrize("fmt", [4, 5, 7])
def test_sector_completion(lib, o, fmt):
    """64-B sector completion at the row ends (pointwise.merge_sectors): destinations whose size
    and start are 64-B aligned, box rows with >= 64-B gaps -- the bytes around each box row in
    its end sectors are rewritten with their own values; everything outside the box must stay
    as it was.  Copies (same and shifted phases, clamped), arithmetic, fill; knob on and off."""
    b = BPV[fmt]
    sv = 64 // b                      # voxels per sector
    X = 3 * sv                        # row = 3 sectors
    rng = np.random.default_rng(50 + fmt)
    src = rand_codes(rng, fmt, (5, 7, X))
    src2 = rand_codes(rng, fmt, (5, 7, X))
    dinit = rand_codes(rng, fmt, (6, 8, X))
    boxes = [((1, 0, 0), (1 + sv, 7, 5), (0, 0, 0)),            # one sector wide, starts mid-sector
             ((sv - 1, 1, 1), (2 * sv, 6, 4), (3, 1, 1)),       # shifted destination
             ((0, 0, 0), (2 * sv, 7, 5), (sv // 2, 1, 1)),      # gap of exactly one sector
             ((-2, -1, 0), (sv + 3, 6, 5), (5, 0, 1)),          # clamped source
             ((7, 2, 2), (9, 3, 3), (sv - 1, 4, 4))]            # tiny box straddling a sector end
    try:
        for on in (True, False):
            assert lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", 1 if on else 0) == 0
            for first, last, off in boxes:
                copy_case(lib, o, fmt, fmt, (0.0, 1.0), (0.0, 1.0), src, dinit, first, last, off,
                          what=f"merge={on} copy {first}->{last}+{off}")
                inside = min(first) >= 0 and last[0] <= X and last[1] <= 7 and last[2] <= 5
                inside = inside and last[0] + off[0] <= X and last[1] + off[1] <= 8 and last[2] + off[2] <= 6
                if inside:   # arithmetic writes dst[first + off .. last + off)
                    for op in ("Sum", "SafeDiff", "Quot"):
                        da, db, dd = Dev(src, fmt), Dev(src2, fmt), Dev(dinit, fmt)
                        from volkit_amd._lib import lib as L
                        assert L.vktHipArithmeticRange(OPS.index(op), dd.view, da.view, db.view, vec(first),
                                                       vec(last), vec(off)) == 0
                        ref = o.arith(op, [fmt] * 3, [(0.0, 1.0)] * 3, src, src2, dinit.copy(), first, last, off)
                        assert_codes_equal(dd.read(), ref, fmt, f"merge={on} {op} {first}->{last}+{off}")
    finally:
        assert lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", -1) == 0


def test_sector_completion_fill_and_subbox(lib, o):
    """FillRange and the aligned-phase sub-box (routed to the general path when its rows end
    inside a sector) on a 64-B aligned destination."""
    from volkit_amd._lib import lib as L
    rng = np.random.default_rng(77)
    for fmt in (4, 5, 7):
        X = 192 // BPV[fmt] * 2
        a = rand_codes(rng, fmt, (6, 9, X))
        bb = rand_codes(rng, fmt, (6, 9, X))
        dinit = rand_codes(rng, fmt, (6, 9, X))
        for first, last in (((8, 1, 1), (X - 40, 8, 5)), ((3, 0, 0), (X // 2 + 1, 9, 6)), ((0, 2, 1), (X - 33, 3, 2))):
            dd = Dev(dinit, fmt)
            assert L.vktHipFillRange(dd.view, vec(first), vec(last), C.c_float(0.3)) == 0
            ref = o.fill_range(fmt, (0.0, 1.0), (X, 9, 6), dinit.copy(), first, last, 0.3)
            assert_codes_equal(dd.read(), ref, fmt, f"fill fmt={fmt} {first}->{last}")
            da, db, dd = Dev(a, fmt), Dev(bb, fmt), Dev(dinit, fmt)
            assert L.vktHipArithmeticRange(5, dd.view, da.view, db.view, vec(first), vec(last), vec((0, 0, 0))) == 0
            ref = o.arith("SafeSum", [fmt] * 3, [(0.0, 1.0)] * 3, a, bb, dinit.copy(), first, last, (0, 0, 0))
            assert_codes_equal(dd.read(), ref, fmt, f"SafeSum fmt={fmt} {first}->{last}")


@pytest.mark.parametrize("fmt", [4, 5, 7])
def test_sector_close_rows(lib, o, fmt):
    """Box rows closer than 64 B in a 64-B aligned destination (no sector completion there: a
    sector holds voxels of two rows): near-full-width boxes at several gap sizes, 8-voxel items
    spanning two rows, clamped halo copies into a whole destination, phase shifts,
    conversions; knob on and off.  (A mode that walked each plane's rows and gaps as one run,
    rewriting the gap bytes, measured slower -- 1000^3 of 1024^3 copy 0.81 -> 1.17 ms: the items
    spanning two rows went voxel by voxel after the streamed items.)"""
    b = BPV[fmt]
    sv = 64 // b
    X = 2 * sv + 8                     # rows not a multiple of a sector; 64-B aligned volume below
    Y, Z = 7, 8 if fmt == 4 else (4 if fmt == 5 else 2)
    rng = np.random.default_rng(90 + fmt)
    src = rand_codes(rng, fmt, (5, 9, X + 3))
    dinit = rand_codes(rng, fmt, (Z * 2, Y, X))        # Z*2 planes: total size a multiple of 64 B
    assert dinit.nbytes % 64 == 0
    cases = [((0, 0, 0), (X, Y, 2), (0, 0, 0)),                 # whole rows, planes contiguous (uniform)
             ((3, 0, 0), (X + 3, Y, 3), (0, 0, 1)),             # phase shift, whole dst rows
             ((-1, -1, -1), (X - 1, Y - 1, 3), (0, 0, 0)),      # clamped halo into whole rows
             ((1, 0, 0), (X - 2, Y, 2), (1, 0, 0)),             # gap of 3 voxels, uniform planes
             ((2, 1, 0), (X - 1, 6, 3), (0, 1, 1)),             # gaps in x and y (plane gap >= 64 B)
             ((0, 0, 0), (X - sv // 2, Y, 2), (sv // 4, 0, 0))]  # gap of half a sector
    try:
        for on in (True, False):
            assert lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", 1 if on else 0) == 0
            for first, last, off in cases:
                copy_case(lib, o, fmt, fmt, (0.0, 1.0), (0.0, 1.0), src, dinit, first, last, off,
                          what=f"close merge={on} copy {first}->{last}+{off}")
                other = {4: 5, 5: 7, 7: 4}[fmt]
                copy_case(lib, o, other, fmt, (0.0, 1.0), (-1.0, 3.0), rand_codes(rng, other, src.shape), dinit,
                          first, last, off, what=f"close merge={on} convert {other}->{fmt} {first}->{last}+{off}")
    finally:
        assert lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", -1) == 0


def test_close_rows_large(lib, o):
    """Close rows at a size with many workgroups: a 1000 x 96 x 5 UInt16 box (gap 48 B) shifted by
    (5, 7, 9) -> (1, 2, 3) in 1024 x 128 x 16 volumes, and a halo copy into a whole volume."""
    rng = np.random.default_rng(91)
    src = rand_codes(rng, 5, (16, 128, 1024))
    dinit = rand_codes(rng, 5, (16, 128, 1024))
    copy_case(lib, o, 5, 5, (0.0, 1.0), (0.0, 1.0), src, dinit, (5, 7, 9), (1005, 103, 14), (1, 2, 3),
              what="span 1000x96x5")
    h = rand_codes(rng, 5, (8, 32, 1022))
    hsrc = rand_codes(rng, 5, (6, 30, 1020))
    copy_case(lib, o, 5, 5, (0.0, 1.0), (0.0, 1.0), hsrc, h, (-1, -1, -1), (1021, 31, 7), (0, 0, 0),
              what="span halo 1022x32x8")


@pytest.mark.parametrize("fmt", [4, 5, 7])
def test_sector_completion_aligned_path(lib, o, fmt):
    """The aligned vector path's sector completion (padded rows, same phase in source and
    destination, rows ending inside 64-B sectors): CopyRange and FillRange, knob on and off."""
    from volkit_amd._lib import lib as L
    b = BPV[fmt]
    X = 256 // b                                   # 256-B rows: 64-B multiples, room for gaps
    rng = np.random.default_rng(60 + fmt)
    src = rand_codes(rng, fmt, (6, 9, X))
    dinit = rand_codes(rng, fmt, (6, 9, X))
    cases = [((8, 1, 1), (X - 40, 8, 5)), ((24, 0, 0), (X // 2 + 8, 9, 6)), ((0, 2, 1), (X - 40, 3, 2)),
             ((40, 1, 0), (48, 8, 6))]
    try:
        for on in (True, False):
            assert lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", 1 if on else 0) == 0
            for first, last in cases:
                copy_case(lib, o, fmt, fmt, (0.0, 1.0), (0.0, 1.0), src, dinit, first, last, first,
                          what=f"aligned merge={on} copy {first}->{last}")
                dd = Dev(dinit, fmt)
                assert L.vktHipFillRange(dd.view, vec(first), vec(last), C.c_float(0.7)) == 0
                ref = o.fill_range(fmt, (0.0, 1.0), (X, 9, 6), dinit.copy(), first, last, 0.7)
                assert_codes_equal(dd.read(), ref, fmt, f"aligned merge={on} fill {first}->{last}")
    finally:
        assert lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", -1) == 0


def test_general_64bit_addressing(lib, o):
    """The general path's 64-bit addressing (taken for operands of 4 GiB and more, so never by
    the small cases above): knob pointwise.general_32bit = 0 forces it on phase shifts, clamped
    halos, narrow rows, conversions and shifted arithmetic."""
    from volkit_amd._lib import lib as L
    rng = np.random.default_rng(123)
    assert lib.vktHipSetTuningKnob(b"pointwise.general_32bit", 0) == 0
    try:
        for fmt in (4, 5, 7):
            src = rand_codes(rng, fmt, (5, 7, 29))
            dinit = rand_codes(rng, fmt, (6, 8, 43))
            for first, last, off in (((3, 1, 1), (22, 6, 4), (0, 0, 0)), ((-5, -2, -1), (24, 6, 5), (7, 0, 0)),
                                     ((2, 0, 0), (5, 7, 5), (1, 1, 1))):
                copy_case(lib, o, fmt, fmt, (0.0, 1.0), (0.0, 1.0), src, dinit, first, last, off,
                          what=f"64-bit copy fmt={fmt} {first}->{last}+{off}")
                other = {4: 7, 5: 4, 7: 5}[fmt]
                copy_case(lib, o, other, fmt, (0.0, 1.0), (-1.0, 3.0), rand_codes(rng, other, src.shape), dinit,
                          first, last, off, what=f"64-bit convert {other}->{fmt} {first}->{last}+{off}")
            a = rand_codes(rng, fmt, (4, 6, 45))
            b = rand_codes(rng, fmt, (4, 6, 45))
            d0 = rand_codes(rng, fmt, (5, 7, 53))
            for op in ("Sum", "SafeDiff", "Quot"):
                da, db, dd = Dev(a, fmt), Dev(b, fmt, pad=2 * BPV[fmt]), Dev(d0, fmt)
                assert L.vktHipArithmeticRange(OPS.index(op), dd.view, da.view, db.view, vec((3, 1, 1)), vec((40, 5, 3)),
                                               vec((3, 1, 1))) == 0
                ref = o.arith(op, [fmt] * 3, [(0.0, 1.0)] * 3, a, b, d0.copy(), (3, 1, 1), (40, 5, 3), (3, 1, 1))
                assert_codes_equal(dd.read(), ref, fmt, f"64-bit {op} fmt={fmt}")
    finally:
        assert lib.vktHipSetTuningKnob(b"pointwise.general_32bit", -1) == 0


@pytest.mark.parametrize("seed", range(4))
def test_random_geometry_fuzz(lib, o, seed):
    """Random dims, boxes (clamped or not), offsets, view paddings, formats and mappings through
    CopyRange, FillRange and arithmetic vs the oracle, with the sector completion and the
    general path's 32-bit addressing on and off: every planning branch of the pointwise engine
    (aligned rows, padded rows with and without sector completion, general path with and
    without it, per-voxel kernel for mixed-format arithmetic)."""
    from volkit_amd._lib import lib as L
    rng = np.random.default_rng(1000 + seed)
    fmts = [4, 5, 7, 2, 6]
    knobs = [(b"pointwise.merge_sectors", 1), (b"pointwise.merge_sectors", 0), (b"pointwise.general_32bit", 0)]
    try:
        for case in range(40):
            kname, kval = knobs[case % len(knobs)]
            assert lib.vktHipSetTuningKnob(kname, kval) == 0
            sf = int(rng.choice(fmts))
            df = sf if rng.random() < 0.7 else int(rng.choice(fmts))
            b = BPV[df]
            # destination rows often 64-B multiples (sector completion applies), sometimes not
            dx = int(rng.choice([64 // b * int(rng.integers(1, 4)), int(rng.integers(5, 90))]))
            ddims = (dx, int(rng.integers(1, 9)), int(rng.integers(1, 6)))
            sdims = (int(rng.integers(1, 90)), int(rng.integers(1, 9)), int(rng.integers(1, 6)))
            src = rand_codes(rng, sf, sdims[::-1])
            dinit = rand_codes(rng, df, ddims[::-1])
            n = [int(rng.integers(1, ddims[i] + 1)) for i in range(3)]
            off = tuple(int(rng.integers(0, ddims[i] - n[i] + 1)) for i in range(3))
            first = tuple(int(rng.integers(-3, max(-2, sdims[i] - n[i] + 4))) for i in range(3))
            last = tuple(first[i] + n[i] for i in range(3))
            smap = [(0.0, 1.0), (-1.0, 3.0)][int(rng.integers(0, 2))]
            dmap = [(0.0, 1.0), (0.25, 7.5)][int(rng.integers(0, 2))]
            spad = int(rng.choice([0, 0, BPV[sf], 3 * BPV[sf]]))
            dpad = int(rng.choice([0, 0, 0, b]))
            what = f"fuzz{seed}.{case} {kname}={kval} {sf}->{df} s{sdims} d{ddims} {first}->{last}+{off} pads {spad},{dpad}"
            copy_case(lib, o, sf, df, smap, dmap, src, dinit, first, last, off, spad, dpad, what=what)
            # fill and arithmetic on boxes inside the destination / sources
            ff = off
            fl = tuple(off[i] + n[i] for i in range(3))
            dd = Dev(dinit, df, dmap, dpad)
            assert L.vktHipFillRange(dd.view, vec(ff), vec(fl), C.c_float(0.37)) == 0
            ref = o.fill_range(df, dmap, ddims, dinit.copy(), ff, fl, 0.37)
            assert_codes_equal(dd.read(), ref, df, "fill " + what)
            a = rand_codes(rng, df, ddims[::-1])
            a2 = rand_codes(rng, df, ddims[::-1])
            op = OPS[int(rng.integers(0, len(OPS)))]
            box0 = tuple(int(rng.integers(0, ddims[i])) for i in range(3))
            box1 = tuple(int(rng.integers(box0[i] + 1, ddims[i] + 1)) for i in range(3))
            da, db, dd = Dev(a, df, dmap, spad * b // BPV[sf]), Dev(a2, df, dmap), Dev(dinit, df, dmap, dpad)
            assert L.vktHipArithmeticRange(OPS.index(op), dd.view, da.view, db.view, vec(box0), vec(box1),
                                           vec((0, 0, 0))) == 0
            ref = o.arith(op, [df] * 3, [dmap] * 3, a, a2, dinit.copy(), box0, box1, (0, 0, 0))
            assert_codes_equal(dd.read(), ref, df, f"{op} {box0}->{box1} " + what)
            assert lib.vktHipSetTuningKnob(kname, -1) == 0
    finally:
        for kname, _ in knobs:
            lib.vktHipSetTuningKnob(kname, -1)


@pytest.mark.parametrize("k", [1, 2, 3])
def test_uint8_long_edge_free_rows_on_the_general_path(lib, o, k):
    """UInt8 copies over multi-row boxes of long rows without row edges (whole-x planes of a y
    sub-range: rows merge to >= 4096 voxels per plane) take the general path's wide items by
    default (knob pointwise.u8_pairs = 1), the pair grid with 2, the general path for every
    UInt8 multi-row box with 3: same bytes as the oracle, including shorter rows and row edges."""
    from volkit_amd._lib import lib as L
    rng = np.random.default_rng(91 + k)
    dims = (6, 40, 256)
    a = rand_codes(rng, 4, dims)
    dinit = rand_codes(rng, 4, dims)
    L.vktHipSetTuningKnob(b"pointwise.u8_pairs", k)
    try:
        for first, last in (((0, 3, 1), (256, 37, 5)), ((0, 0, 0), (256, 40, 6)), ((0, 5, 0), (256, 6, 6)),
                            ((16, 2, 1), (240, 39, 5)), ((3, 2, 1), (250, 39, 5))):
            copy_case(lib, o, 4, 4, (0.0, 1.0), (0.0, 1.0), a, dinit, first, last, (0, 0, 0), 0, 0,
                      f"u8 copy k={k} {first}->{last}")
            copy_case(lib, o, 4, 4, (0.0, 1.0), (0.0, 1.0), a, dinit, first, last, (0, 0, 0), 0, 64,
                      f"u8 copy k={k} {first}->{last} dst+64")
    finally:
        L.vktHipSetTuningKnob(b"pointwise.u8_pairs", -1)


@pytest.mark.parametrize("dword", [1, 0])
@pytest.mark.parametrize("wide", [0, 1, 2])
def test_float32_dword_shift(lib, o, dword, wide):
    """4-byte voxels at 4-B aligned addresses shift their windows by whole dwords (knob
    pointwise.dword_shift: the byte-align stage skipped), on the 8-voxel and the 16-B item layouts
    (knob pointwise.f32_wide): copies at every source x phase against several destination phases,
    an arithmetic dstOffset, 4-B aligned but not 16-B aligned view pointers (and, byte-offset
    pointers, which must keep the byte-align stage)."""
    rng = np.random.default_rng(5 + dword + 2 * wide)
    src = rand_codes(rng, 7, (4, 6, 45))
    b2 = rand_codes(rng, 7, (4, 6, 45))
    dinit = rand_codes(rng, 7, (5, 7, 53))
    assert lib.vktHipSetTuningKnob(b"pointwise.dword_shift", dword) == 0
    assert lib.vktHipSetTuningKnob(b"pointwise.f32_wide", wide) == 0
    try:
        for spad, dpad in ((0, 0), (4, 0), (0, 12), (8, 4)):
            for sx in range(5):
                for dx in (0, 1, 3, 6):
                    copy_case(lib, o, 7, 7, (0.0, 1.0), (0.0, 1.0), src, dinit, (sx, 1, 0), (sx + 37, 6, 4), (dx, 0, 1),
                              spad, dpad, what=f"dword={dword} wide={wide} pads {spad},{dpad} sx={sx} dx={dx}")
        for spad in (1, 2):   # byte-offset views (not 4-B aligned): the byte-align stage runs
            copy_case(lib, o, 7, 7, (0.0, 1.0), (0.0, 1.0), src, dinit, (3, 0, 0), (40, 6, 4), (0, 0, 0), spad, 0,
                      what=f"dword={dword} byte pad {spad}")
        for dx in range(8):
            da, db, dd = Dev(src, 7), Dev(b2, 7, pad=4), Dev(dinit, 7)
            assert lib.vktHipArithmeticRange(0, dd.view, da.view, db.view, vec((3, 1, 1)), vec((40, 5, 3)),
                                             vec((dx, 1, 1))) == 0
            ref = o.arith("Sum", [7] * 3, [(0.0, 1.0)] * 3, src, b2, dinit.copy(), (3, 1, 1), (40, 5, 3), (dx, 1, 1))
            assert_codes_equal(dd.read(), ref, 7, f"Sum dword={dword} wide={wide} dx={dx}")
    finally:
        lib.vktHipSetTuningKnob(b"pointwise.dword_shift", -1)
        lib.vktHipSetTuningKnob(b"pointwise.f32_wide", -1)


@pytest.mark.parametrize("dx", [0, 1, 3, 13, 16])
def test_float32_three_stream_sector_completion(lib, o, dx):
    """64-B sector completion for the 3-stream Float32 ops on the general path (the default;
    row-end items merged with the destination's own voxels, pads rewriting them): Sum / SafeDiff
    with phase-shifting dstOffsets on 192-voxel rows (768-B pitches, gaps >= 64 B between box
    rows), the destination outside the box intact, vs the oracle; knob pointwise.merge_sectors
    = 0 (per-voxel row ends) alongside."""
    rng = np.random.default_rng(300 + dx)
    a = rand_codes(rng, 7, (5, 6, 192))
    b = rand_codes(rng, 7, (5, 6, 192))
    dinit = rand_codes(rng, 7, (5, 6, 192))
    try:
        for mk in (1, 0):
            assert lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", mk) == 0
            for x0, w in ((0, 160), (5, 100), (17, 31), (40, 7), (3, 150)):
                first, last = (x0, 1, 0), (x0 + w, 5, 4)
                off = (dx - x0 + 2, 0, 1)   # arithmetic dstOffset: dst x = x + off
                if x0 + w + off[0] > 192:
                    continue
                for op in ("Sum", "SafeDiff"):
                    da, db, dd = Dev(a, 7), Dev(b, 7), Dev(dinit, 7)
                    assert lib.vktHipArithmeticRange(OPS.index(op), dd.view, da.view, db.view, vec(first), vec(last),
                                                     vec(off)) == 0, last_error()
                    ref = o.arith(op, [7] * 3, [(0.0, 1.0)] * 3, a, b, dinit.copy(), first, last, off)
                    assert_codes_equal(dd.read(), ref, 7, f"{op} merge={mk} dx={dx} x0={x0} w={w}")
    finally:
        lib.vktHipSetTuningKnob(b"pointwise.merge_sectors", -1)
