"""ComputeAggregates / ComputeHistogram against the oracle restatement of
reference src/vkt/Aggregates_serial.hpp:20-83 and src/vkt/Histogram_serial.hpp:20-50.

Parity contract:
  * histogram counts, min, max, argmin, argmax: bit-exact;
  * sum, mean, var, stddev, prod: the reference accumulates floats serially, the GPU
    accumulates the same per-voxel float terms in double and rounds once.  Tested bounds:
      |gpu - exact| <= 1 ulp(exact) + 2^-24 * sum|terms| * 1e-6     (GPU is accurate)
      |gpu - oracle| <= n * 2^-24 * sum|terms| + 1 ulp                (serial error bound)
    where exact is a float64 sum of the same float32 terms.
  * var under the one-pass moments paths (knob aggregates.moments, DESIGN §4.8: UInt16, Float32):
    the sum of squares is the EXACT sum (v - m)^2 (integer moments; float moments to ~2^-50), not
    a sum of float terms; each float term fl(fl(v - m)^2) lies within 3 * 2^-24 of (v - m)^2, so
      |var - var_terms| <= 3 * 2^-24 * var_terms + 2 ulp(var_terms)
    (var_terms: the float-terms value above); far inside the serial bound.
The oracle itself is pinned here against numpy's sequential float32 accumulation
(np.add.accumulate is strictly left-to-right) and a float32 restatement of the bin formula.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import binding as ob

vkt = pytest.importorskip("volkit_amd.volkit")
from volkit_amd import _lib  # noqa: E402
from volkit_amd._lib import lib  # noqa: E402

F32 = np.float32
EPS = 2.0 ** -24


def values_of(codes, fmt, lo, hi):
    """Unmapped float32 values of a code array through the oracle codec (vectorised for the
    formats used here)."""
    if fmt == 7:
        return codes.view(np.float32)
    flat = codes.reshape(-1)
    uniq, inv = np.unique(flat, return_inverse=True)
    vals = np.array([ob.unmap_voxel(int(c).to_bytes(ob.BPV[fmt], "little"), fmt, lo, hi) for c in uniq],
                    dtype=np.float32)
    return vals[inv].reshape(codes.shape)


# ---- oracle pinning (CPU) -----------------------------------------------------------------
def test_oracle_aggregates_follow_sequential_float32():
    rng = np.random.default_rng(1)
    codes = rng.integers(0, 65536, (6, 7, 9), dtype=np.uint16)
    v = ob.Volume(codes, 5, -1.0, 3.0)
    first, last = (1, 2, 0), (8, 7, 5)
    a = ob.aggregates_range(v, first, last)
    vals = values_of(codes, 5, -1.0, 3.0)[first[2]:last[2], first[1]:last[1], first[0]:last[0]].reshape(-1)
    seq = np.add.accumulate(vals, dtype=np.float32)[-1]
    assert a.sum == seq
    n = codes.size
    mean = F32(np.float64(seq) / n)
    assert a.mean == mean
    d = (vals - mean).astype(np.float32)
    var_acc = np.add.accumulate((d * d).astype(np.float32), dtype=np.float32)[-1]
    assert a.var == F32(np.float64(var_acc) / n)
    assert a.prod == np.multiply.accumulate(vals, dtype=np.float32)[-1]
    i = int(np.argmin(vals))   # first occurrence in z, y, x order
    box = (last[0] - first[0], last[1] - first[1])
    assert list(a.argmin) == [first[0] + i % box[0], first[1] + (i // box[0]) % box[1], first[2] + i // (box[0] * box[1])]


def test_oracle_histogram_formula():
    rng = np.random.default_rng(2)
    vals = rng.uniform(-0.2, 1.2, (5, 6, 7)).astype(np.float32)
    vals.reshape(-1)[:4] = [np.nan, np.inf, -0.0, 1.0]
    v = ob.Volume(vals.view(np.uint32), 7, 0.0, 1.0)
    bins, skipped = ob.histogram_range(v, (0, 0, 0), (7, 6, 5), 10)
    f = (vals.reshape(-1) - F32(0.0)) * (F32(10) / (F32(1.0) - F32(0.0)))
    ok = (f > -1) & (f < 10)
    assert skipped == int((~ok).sum())
    np.testing.assert_array_equal(bins, np.bincount(np.trunc(f[ok]).astype(np.int64), minlength=10))


def test_cpu_policy_is_refused():
    v = vkt.StructuredVolume(4, 4, 4, vkt.DataFormat_UInt8)
    assert vkt.ComputeAggregates(v, vkt.Aggregates()) == vkt.InvalidValue
    assert vkt.ComputeHistogram(v, vkt.Histogram(8)) == vkt.InvalidValue


def test_partial_combine_is_associative_and_tie_breaks_on_index():
    P = _lib.HipAggregatePartial_t

    def part(mn, mi, mx, xi, s, n):
        p = P()
        lib.vktHipAggregatePartialInit(C.byref(p))
        p.minValue, p.minIndex, p.maxValue, p.maxIndex, p.sum, p.count = mn, mi, mx, xi, s, n
        p.prod = 2.0
        return p

    a, b, c = part(1.0, 50, 5.0, 7, 1.5, 3), part(1.0, 20, 5.0, 9, 2.5, 4), part(0.5, 90, 4.0, 1, -1.0, 5)
    acc = P()
    lib.vktHipAggregatePartialInit(C.byref(acc))
    for p in (a, b):
        lib.vktHipAggregatePartialCombine(C.byref(acc), C.byref(p))
    assert (acc.minValue, acc.minIndex, acc.maxValue, acc.maxIndex) == (1.0, 20, 5.0, 7)
    lib.vktHipAggregatePartialCombine(C.byref(acc), C.byref(c))
    assert (acc.minValue, acc.minIndex, acc.sum, acc.count, acc.prod) == (0.5, 90, 3.0, 12, 8.0)
    out = _lib.Aggregates_t()
    lib.vktHipAggregatesFinish(C.byref(acc), C.byref(acc), 100, 10, 3, C.byref(out))
    assert (out.argmin.x, out.argmin.y, out.argmin.z) == (0, 0, 3)    # 90 = 3*30 + 0*10 + 0
    assert (out.argmax.x, out.argmax.y, out.argmax.z) == (7, 0, 0)


# ---- GPU parity -----------------------------------------------------------------------------
def set_device(dev):
    ep = vkt.GetThreadExecutionPolicy()
    ep.device = dev
    vkt.SetThreadExecutionPolicy(ep)


def gpu_volume(codes, fmt, lo, hi):
    z, y, x = codes.shape
    set_device(vkt.ExecutionPolicy.Device_CPU)
    v = vkt.StructuredVolume(x, y, z, fmt, 1.0, 1.0, 1.0, lo, hi)
    v.from_numpy(codes)
    return v


def gpu_aggregates(codes, fmt, lo, hi, first, last):
    v = gpu_volume(codes, fmt, lo, hi)
    a = vkt.Aggregates()
    set_device(vkt.ExecutionPolicy.Device_GPU)
    try:
        err = vkt.ComputeAggregatesRange(v, a, *first, *last)
    finally:
        set_device(vkt.ExecutionPolicy.Device_CPU)
    assert err == vkt.NoError, vkt.last_error()
    return a


def gpu_histogram(codes, fmt, lo, hi, first, last, nbins):
    v = gpu_volume(codes, fmt, lo, hi)
    h = vkt.Histogram(nbins)
    set_device(vkt.ExecutionPolicy.Device_GPU)
    try:
        err = vkt.ComputeHistogramRange(v, h, *first, *last)
    finally:
        set_device(vkt.ExecutionPolicy.Device_CPU)
    assert err == vkt.NoError, vkt.last_error()
    return h.getBinCounts()    # migrates back under the CPU policy


def rand_codes(rng, fmt, shape, specials=False):
    if fmt == 7:
        vals = rng.uniform(-1.5, 2.5, shape).astype(np.float32)
        if specials:
            flat = vals.reshape(-1)
            k = min(12, flat.size)
            idx = rng.choice(flat.size, k, replace=False)
            flat[idx] = np.resize(np.array([np.nan, np.inf, -np.inf, -0.0, 3e38, -3e38], np.float32), k)
        return vals.view(np.uint32)
    info = np.iinfo(ob.CODE_DTYPE[fmt])
    return rng.integers(0, int(info.max) + 1, shape, dtype=np.uint64).astype(ob.CODE_DTYPE[fmt])


CASES = [
    ((40, 30, 20), (0, 0, 0), (40, 30, 20)),
    ((40, 30, 20), (3, 5, 2), (37, 29, 19)),
    ((129, 3, 70), (1, 0, 10), (129, 3, 11)),
    ((1, 1, 1), (0, 0, 0), (1, 1, 1)),
]

# ranges of the streaming histogram kernel (8-voxel-aligned rows): one contiguous span (whole
# volume with a partial last step, whole planes, part of one plane) and a strided box
FAST_CASES = [
    ((256, 33, 17), (0, 0, 0), (256, 33, 17)),
    ((64, 24, 10), (0, 0, 2), (64, 24, 9)),
    ((64, 24, 10), (0, 5, 4), (64, 17, 5)),
    ((64, 24, 10), (8, 3, 2), (56, 20, 9)),
    # padded rows (range rows starting / ending off the 8-voxel grid): masked end items
    ((64, 24, 10), (3, 3, 2), (61, 20, 9)),
    ((64, 24, 10), (5, 0, 0), (6, 24, 10)),
    ((64, 24, 10), (9, 1, 1), (15, 2, 2)),
    ((128, 8, 4), (1, 0, 0), (128, 8, 4)),
]


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [4, 5, 2, 6, 7])
@pytest.mark.parametrize("mapping", [(0.0, 1.0), (-1.0, 3.0)])
@pytest.mark.parametrize("nbins", [1, 7, 256, 1000, 10240, 10241, 20000, 65536, 100000, 400000])
def test_histogram_parity(fmt, mapping, nbins):
    rng = np.random.default_rng(fmt * 7 + nbins)
    for dims, first, last in CASES + FAST_CASES:
        codes = rand_codes(rng, fmt, dims[::-1], specials=True)
        got = gpu_histogram(codes, fmt, *mapping, first, last, nbins)
        ref, _ = ob.histogram_range(ob.Volume(codes, fmt, *mapping), first, last, nbins)
        np.testing.assert_array_equal(got, ref, err_msg=f"dims={dims} {first}->{last}")


@pytest.mark.gpu
def test_histogram_uint16_unit_mapping_every_code():
    """UInt16 + unit mapping + 2^k bins takes the integer path (bin = code >> (16 - k)): every
    code, each power of two up to 2^17, and the look-alike mappings that must not take it."""
    codes = np.arange(65536, dtype=np.uint16).reshape(16, 16, 256)
    near1 = float(np.nextafter(np.float32(1.0), np.float32(2.0)))
    for mapping in ((0.0, 1.0), (-0.0, 1.0), (0.0, near1)):
        for nbins in (1, 2, 16, 256, 1024, 4096, 65536, 131072, 3, 65535):
            got = gpu_histogram(codes, 5, *mapping, (0, 0, 0), (256, 16, 16), nbins)
            ref, _ = ob.histogram_range(ob.Volume(codes, 5, *mapping), (0, 0, 0), (256, 16, 16), nbins)
            np.testing.assert_array_equal(got, ref, err_msg=f"map={mapping} nbins={nbins}")
    # UInt8: the shift path is taken when the host evaluation of all 256 bins is c >> s
    codes = np.tile(np.arange(256, dtype=np.uint8), 64).reshape(8, 8, 256)
    for mapping in ((0.0, 1.0), (-0.0, 1.0), (-1.0, 3.0), (0.0, 0.5), (0.0, 2.0)):
        for nbins in (1, 2, 64, 128, 256, 512, 255, 1000):
            got = gpu_histogram(codes, 4, *mapping, (0, 0, 0), (256, 8, 8), nbins)
            ref, _ = ob.histogram_range(ob.Volume(codes, 4, *mapping), (0, 0, 0), (256, 8, 8), nbins)
            np.testing.assert_array_equal(got, ref, err_msg=f"u8 map={mapping} nbins={nbins}")


# (mapping, numBins) whose oracle bins are (code * numBins) >> 16 for every UInt16 code (the
# library's mul-shift bins) and ones whose float rounding breaks that (they keep the float formula)
MULSHIFT_CASES = [((0.0, 1.0), 10240), ((0.0, 1.0), 1000), ((0.0, 1.0), 40960), ((0.0, 1.0), 65535),
                  ((0.0, 2.0), 1000), ((0.0, 0.5), 768), ((-1.0, 3.0), 10240), ((0.25, 7.5), 3000)]
FLOATBIN_CASES = [((0.0, 1.0), 20000), ((0.0, 1.0), 3000), ((0.0, 2.0), 12000), ((0.25, 7.5), 30000)]


def test_histogram_mulshift_premise_against_oracle():
    """The premise of the UInt16 mul-shift bins, checked with the oracle's restatement of
    Histogram_serial.hpp: for the listed cases every code's bin is (c * numBins) >> 16, and for the
    others it is not (so the host check in the library must reject them)."""
    codes = np.arange(65536, dtype=np.uint16).reshape(16, 16, 256)
    c = np.arange(65536, dtype=np.uint64)
    for cases, expect in ((MULSHIFT_CASES, True), (FLOATBIN_CASES, False)):
        for mapping, nbins in cases:
            ref, _ = ob.histogram_range(ob.Volume(codes, 5, *mapping), (0, 0, 0), (256, 16, 16), nbins)
            ms = np.bincount((c * nbins) >> 16, minlength=nbins).astype(ref.dtype)
            assert np.array_equal(ref, ms) == expect, f"map={mapping} nbins={nbins}"


@pytest.mark.gpu
def test_histogram_uint16_mulshift_bins():
    """Mul-shift bins (knob histogram.mulshift) vs the float formula and the oracle: every code,
    both kinds of case, replicated (<= 10 240 bins) and tiled counters, and a strided padded box."""
    rng = np.random.default_rng(77)
    every = np.arange(65536, dtype=np.uint16).reshape(16, 16, 256)
    rand = rng.integers(0, 65536, (24, 40, 520), dtype=np.uint16)
    for codes, box in ((every, ((0, 0, 0), (256, 16, 16))), (rand, ((3, 1, 2), (517, 39, 23)))):
        for mapping, nbins in MULSHIFT_CASES + FLOATBIN_CASES:
            ref, _ = ob.histogram_range(ob.Volume(codes, 5, *mapping), *box, nbins)
            for k in (1, 0):
                lib.vktHipSetTuningKnob(b"histogram.mulshift", k)
                try:
                    got = gpu_histogram(codes, 5, *mapping, *box, nbins)
                finally:
                    lib.vktHipSetTuningKnob(b"histogram.mulshift", -1)
                np.testing.assert_array_equal(got, ref, err_msg=f"map={mapping} nbins={nbins} knob={k}")


@pytest.mark.gpu
def test_histogram_constant_volume_and_reference_example():
    """Wave-uniform bins (one atomic per wave) and src/examples/Histogram.cpp's 256 bins."""
    codes = np.full((33, 65, 130), 200, np.uint8)
    got = gpu_histogram(codes, 4, 0.0, 1.0, (0, 0, 0), (130, 65, 33), 256)
    ref, _ = ob.histogram_range(ob.Volume(codes, 4), (0, 0, 0), (130, 65, 33), 256)
    np.testing.assert_array_equal(got, ref)
    assert got.sum() == codes.size
    # the streaming kernel: every lane of every wave on the same bin (replicated counters)
    # (20000 / 65536 bins: the tiled and packed-16 paths, one add of the lane count per
    # wave-uniform bin; the box leaves a partial last step -- waves with inactive lanes)
    for fmt, code in ((4, 200), (5, 40000), (7, 0x3F000000)):
        codes = np.full((9, 40, 512), code, ob.CODE_DTYPE[fmt])
        codes[4, 7:9, 100:300] = code // 2   # one run of another bin, partly wave-uniform
        for nb in (256, 20000, 65536):
            for box in (((0, 0, 0), (512, 40, 9)), ((0, 0, 0), (512, 40, 8)), ((8, 1, 0), (504, 39, 9))):
                got = gpu_histogram(codes, fmt, 0.0, 1.0, *box, nb)
                ref, _ = ob.histogram_range(ob.Volume(codes, fmt), *box, nb)
                np.testing.assert_array_equal(got, ref, err_msg=f"fmt={fmt} nb={nb} box={box}")


@pytest.mark.gpu
@pytest.mark.parametrize("fmt,mapping,nbins,fill", [
    (5, (0.0, 1.0), 65536, (40000, 40001)),    # integer bins, a low and a high 16-bit half
    (5, (0.0, 1.0), 65536, (40001,)),
    (5, (-1.0, 3.0), 50000, (123, 124)),       # float bins
    (7, (0.0, 1.0), 60000, (0x3F000000, 0x3F000001)),
])
def test_histogram_packed16_counter_wraps(fmt, mapping, nbins, fill):
    """More bins than one LDS tile of 32-bit counters: one pass over packed 16-bit counters.
    64 Mi voxels on at most two bins: alternating bins (no wave-uniform voxel) cross the 2^14
    flush threshold of both halves of one counter word many times per workgroup; a single bin
    is counted in the waves' run registers; a sprinkle of random codes lands everywhere else."""
    rng = np.random.default_rng(nbins)
    codes = np.resize(np.array(fill, ob.CODE_DTYPE[fmt]), 1024 * 1024 * 64).reshape(64, 1024, 1024)
    flat = codes.reshape(-1)
    idx = rng.choice(flat.size, 100000, replace=False)
    flat[idx] = rand_codes(rng, fmt, (100000,))
    full = ((0, 0, 0), (1024, 1024, 64))
    lib.vktHipSetTuningKnob(b"histogram.u16_codes", 0)   # (UInt16 float bins: the P16 float path)
    try:
        got = gpu_histogram(codes, fmt, *mapping, *full, nbins)
    finally:
        lib.vktHipSetTuningKnob(b"histogram.u16_codes", -1)
    ref, _ = ob.histogram_range(ob.Volume(codes, fmt, *mapping), *full, nbins)
    np.testing.assert_array_equal(got, ref)
    # a padded sub-box (masked end items) through the same path
    box = ((3, 1, 2), (1021, 1000, 60))
    got = gpu_histogram(codes, fmt, *mapping, *box, nbins)
    ref, _ = ob.histogram_range(ob.Volume(codes, fmt, *mapping), *box, nbins)
    np.testing.assert_array_equal(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [5, 7])
def test_histogram_packed16_matches_tiled_passes(fmt):
    """Knob histogram.packed16 = 0: one pass per LDS tile of 32-bit counters, same counts; knob
    histogram.p16_step = 0: P16 threshold tests after every item instead of every wave-step."""
    rng = np.random.default_rng(fmt)
    codes = rand_codes(rng, fmt, (40, 100, 256), specials=True)
    runs = []
    for knob, k in ((b"histogram.packed16", 1), (b"histogram.packed16", 0), (b"histogram.p16_step", 0)):
        lib.vktHipSetTuningKnob(knob, k)
        try:
            runs.append(gpu_histogram(codes, fmt, 0.0, 1.0, (0, 0, 0), (256, 100, 40), 65536))
        finally:
            lib.vktHipSetTuningKnob(knob, -1)
    np.testing.assert_array_equal(runs[0], runs[1])
    np.testing.assert_array_equal(runs[0], runs[2])
    ref, _ = ob.histogram_range(ob.Volume(codes, fmt), (0, 0, 0), (256, 100, 40), 65536)
    np.testing.assert_array_equal(runs[0], ref)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt,mapping", [(5, (0.0, 1.0)), (5, (-1.0, 3.0)), (7, (0.0, 1.0))])
@pytest.mark.parametrize("nbins", [100000, 150001, 300000])
def test_histogram_packed16_tiles(fmt, mapping, nbins):
    """Knob histogram.packed16 = 2 (round 6): more bins than one packed-16 launch holds, in
    packed-16 tiles (one pass each, the tile boundary at an even bin) -- vs the oracle: whole
    volume, padded sub-box, a constant region (flushes inside one tile); UInt16 with the code
    counts off."""
    rng = np.random.default_rng(nbins + 3 * fmt)
    codes = rand_codes(rng, fmt, (40, 100, 256), specials=True)
    codes[5:9] = codes[5, 0, 0]
    vol = ob.Volume(codes, fmt, *mapping)
    lib.vktHipSetTuningKnob(b"histogram.packed16", 2)
    lib.vktHipSetTuningKnob(b"histogram.u16_codes", 0)
    try:
        for first, last in (((0, 0, 0), (256, 100, 40)), ((3, 1, 2), (250, 99, 37))):
            got = gpu_histogram(codes, fmt, *mapping, first, last, nbins)
            ref, _ = ob.histogram_range(vol, first, last, nbins)
            np.testing.assert_array_equal(got, ref, err_msg=f"{first}->{last}")
    finally:
        lib.vktHipSetTuningKnob(b"histogram.packed16", -1)
        lib.vktHipSetTuningKnob(b"histogram.u16_codes", -1)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt,mapping", [(5, (0.0, 1.0)), (5, (-1.0, 3.0)), (7, (0.0, 1.0))])
@pytest.mark.parametrize("nbins", [65536, 50001, 100000, 150000])
def test_histogram_pair_tiles(fmt, mapping, nbins):
    """Knob histogram.pair_tiles = 2: 2-4 tiles of 32-bit counters counted side by side in one
    launch (workgroup groups on one XCD; the default 1 takes it where P16 does not apply), vs the
    oracle: whole volume (integer / mul-shift /
    float bins), a padded sub-box, and a constant region (the per-wave run register)."""
    rng = np.random.default_rng(nbins + fmt)
    codes = rand_codes(rng, fmt, (40, 100, 256), specials=True)
    codes[5:9] = codes[5, 0, 0]      # constant planes: wave-uniform items
    vol = ob.Volume(codes, fmt, *mapping)
    lib.vktHipSetTuningKnob(b"histogram.pair_tiles", 2)   # also where P16 would take the bins
    lib.vktHipSetTuningKnob(b"histogram.u16_codes", 0)    # (UInt16 float bins: not the code counts)
    lib.vktHipSetTuningKnob(b"histogram.packed16", 1)     # (> 81 408 bins: not packed-16 tiles)
    try:
        for first, last in (((0, 0, 0), (256, 100, 40)), ((3, 1, 2), (250, 99, 37))):
            got = gpu_histogram(codes, fmt, *mapping, first, last, nbins)
            ref, _ = ob.histogram_range(vol, first, last, nbins)
            np.testing.assert_array_equal(got, ref, err_msg=f"{first}->{last}")
    finally:
        lib.vktHipSetTuningKnob(b"histogram.pair_tiles", -1)
        lib.vktHipSetTuningKnob(b"histogram.u16_codes", -1)
        lib.vktHipSetTuningKnob(b"histogram.packed16", -1)


@pytest.mark.gpu
@pytest.mark.parametrize("mapping,nbins", [((-1.0, 3.0), 20000), ((-1.0, 3.0), 50000), ((0.0, 1.0), 100000),
                                           ((0.25, 7.5), 150000), ((3.0, -1.0), 70000), ((0.0, 1e-3), 90000),
                                           ((0.0, 1.0), 3000000), ((-1.0, 3.0), 65536), ((0.0, 1.0), 256)])
@pytest.mark.parametrize("fmt", [5, 2])
def test_histogram_uint16_code_counts(fmt, mapping, nbins):
    """Knob histogram.u16_codes (round 6): UInt16 bins that are not integer functions of the code
    count the 65 536 codes in one pass (the packed-16 kernel with the identity bin) and fold the
    counts into the bins with the reference's bin of the decoded value -- vs the oracle and vs the
    per-voxel kernels (knob 0): float bins inside one tile (knob 2) and across 2-4 tiles, a
    decreasing mapping and one that sends most codes out of range, 3 M bins (more tiles than the
    streaming kernels take: the global-atomic kernel at knob 0), whole volume, padded sub-box, and
    a constant region (one code, counts past the 16-bit counters' flush).  Int16 (fmt 2) volumes
    take the counts of their raw codes for every bin count (knob 0: the per-row kernel)."""
    rng = np.random.default_rng(nbins + fmt)
    codes = rand_codes(rng, fmt, (40, 100, 256))
    codes[5:30] = 40000                       # 640 000 voxels of one code
    vol = ob.Volume(codes, fmt, *mapping)
    try:
        for first, last in (((0, 0, 0), (256, 100, 40)), ((3, 1, 2), (250, 99, 37))):
            ref, _ = ob.histogram_range(vol, first, last, nbins)
            for k in (1, 2, 0):
                lib.vktHipSetTuningKnob(b"histogram.u16_codes", k)
                got = gpu_histogram(codes, fmt, *mapping, first, last, nbins)
                np.testing.assert_array_equal(got, ref, err_msg=f"knob={k} {first}->{last}")
    finally:
        lib.vktHipSetTuningKnob(b"histogram.u16_codes", -1)


@pytest.mark.gpu
@pytest.mark.parametrize("partials", [1, 2, 0])
def test_histogram_partials(partials):
    """Knob histogram.partials (round 6): tiled histogram launches store per-workgroup counter words
    that one kernel sums (1: packed-16 launches, 2: every tiled launch) instead of 64-bit atomics
    per counter (0) -- vs the oracle on every tiled
    path: packed-16 integer bins (with the in-run 2^14 flushes of a constant region), packed-16
    float bins, single-tile and multi-tile (one launch per tile) 32-bit counters, the 16-bit code
    counts (UInt16 float bins, Int16), whole volumes, a padded sub-box and a one-plane volume
    (fewer workgroups than the grid cap)."""
    rng = np.random.default_rng(31 + partials)
    assert lib.vktHipSetTuningKnob(b"histogram.partials", partials) == 0
    try:
        for fmt, mapping, nbins, knobs in ((5, (0.0, 1.0), 65536, ()), (5, (-1.0, 3.0), 20000, ()),
                                           (7, (0.0, 1.0), 65536, ()), (7, (0.0, 1.0), 100000, ()),
                                           (7, (0.0, 1.0), 150000, ((b"histogram.pair_tiles", 0),)),
                                           (5, (0.0, 1.0), 100000, ()), (2, (-1.0, 3.0), 256, ()),
                                           (5, (-1.0, 3.0), 50000, ((b"histogram.u16_codes", 0),))):
            for dims in ((256, 100, 40), (512, 64, 1)):
                codes = rand_codes(rng, fmt, dims[::-1], specials=True)
                codes[:, 10:30] = codes[0, 0, 0]      # a constant slab (run registers, flushes)
                vol = ob.Volume(codes, fmt, *mapping)
                boxes = [((0, 0, 0), dims)]
                if dims[2] > 1:
                    boxes.append(((3, 1, 2), (dims[0] - 5, dims[1] - 1, dims[2] - 3)))
                for k, v in knobs:
                    lib.vktHipSetTuningKnob(k, v)
                try:
                    for first, last in boxes:
                        got = gpu_histogram(codes, fmt, *mapping, first, last, nbins)
                        ref, _ = ob.histogram_range(vol, first, last, nbins)
                        np.testing.assert_array_equal(got, ref, err_msg=f"fmt={fmt} nb={nbins} {first}->{last}")
                finally:
                    for k, _ in knobs:
                        lib.vktHipSetTuningKnob(k, -1)
    finally:
        lib.vktHipSetTuningKnob(b"histogram.partials", -1)


def takes_moments(fmt, mapping):
    """UInt16 (integer moments under the unit mapping, float moments otherwise), Float32, Int16 and
    UInt32 (float moments; the last two since round 6) take the one-pass moments paths
    (aggregates.moments)."""
    return fmt in (5, 7, 2, 6)


def check_var(got_var, var_terms, moments, what=""):
    """var against the float-terms value: 1 ulp, or the moments bound (module docstring)."""
    ulp = float(np.spacing(np.float32(abs(var_terms))))
    bound = 3 * EPS * abs(var_terms) + 2 * ulp if moments else ulp
    assert abs(got_var - var_terms) <= bound, f"var {got_var} vs {var_terms} {what}"


def check_float(name, gpu, oracle, exact, terms_abs_sum, n):
    ulp = float(np.spacing(np.float32(abs(exact)))) if np.isfinite(exact) else 0.0
    assert abs(gpu - exact) <= ulp + 1e-6 * EPS * terms_abs_sum, f"{name}: gpu {gpu} vs exact {exact}"
    assert abs(gpu - oracle) <= n * EPS * terms_abs_sum + ulp, f"{name}: gpu {gpu} vs oracle {oracle}"


@pytest.mark.gpu
@pytest.mark.parametrize("fmt,mapping", [(4, (0.0, 1.0)), (5, (-1.0, 3.0)), (5, (0.0, 1.0)), (4, (-0.0, 1.0)), (2, (0.0, 1.0)), (7, (0.0, 1.0)),
                                         (6, (0.25, 7.5))])
def test_aggregates_parity(fmt, mapping):
    rng = np.random.default_rng(fmt)
    for dims, first, last in CASES + FAST_CASES:
        codes = rand_codes(rng, fmt, dims[::-1])
        got = gpu_aggregates(codes, fmt, *mapping, first, last)
        ref = ob.aggregates_range(ob.Volume(codes, fmt, *mapping), first, last)
        what = f"fmt={fmt} dims={dims} {first}->{last}"
        assert (got.min, got.max) == (ref.min, ref.max), what
        assert tuple(got.argmin) == tuple(ref.argmin) and tuple(got.argmax) == tuple(ref.argmax), what
        vals = values_of(codes, fmt, *mapping)[first[2]:last[2], first[1]:last[1], first[0]:last[0]].reshape(-1)
        n, nall = vals.size, codes.size
        exact_sum = float(np.sum(vals, dtype=np.float64))
        abs_sum = float(np.sum(np.abs(vals), dtype=np.float64))
        check_float("sum", got.sum, ref.sum, exact_sum, abs_sum, n)
        assert got.mean == np.float32(np.float64(np.float32(got.sum)) / nall), what
        d = (vals - np.float32(got.mean)).astype(np.float32)
        d2 = (d * d).astype(np.float32)
        exact_var = float(np.float32(np.float64(np.float32(np.sum(d2, dtype=np.float64))) / nall))
        check_var(got.var, exact_var, takes_moments(fmt, mapping), what)
        assert abs(got.var - ref.var) <= n * EPS * 4 * (abs(ref.var) + 1e-30) + float(np.spacing(np.float32(ref.var)))
        assert got.stddev == np.float32(np.sqrt(np.float32(got.var))), what


@pytest.mark.gpu
def test_aggregates_float32_span_ties():
    """Float32 spans take contiguous 16-B lanes (a lane's voxels are the halves at 4l and
    256 + 4l of each 64-item block): ties of the minimum and maximum placed in one lane's two
    halves, across lanes, blocks and steps must still report the first occurrence."""
    rng = np.random.default_rng(3)
    vals = rng.uniform(-1.0, 1.0, (40, 64, 96)).astype(np.float32)
    flat = vals.reshape(-1)
    for i in (260 * 8 + 300, 259 * 8 + 3, 5000, 5000 + 256, 70001, 200003):   # minima
        flat[i] = -5.0
    for i in (4 * 512 + 256 + 7, 4 * 512 + 11, 99999, 123456):                  # maxima
        flat[i] = 6.0
    codes = vals.view(np.uint32)
    box = ((0, 0, 0), (96, 64, 40))
    got = gpu_aggregates(codes, 7, 0.0, 1.0, *box)
    ref = ob.aggregates_range(ob.Volume(codes, 7), *box)
    assert (got.min, tuple(got.argmin), got.max, tuple(got.argmax)) == (ref.min, tuple(ref.argmin), ref.max,
                                                                        tuple(ref.argmax))
    assert ref.min == -5.0 and ref.max == 6.0


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [4, 5])
def test_aggregates_integer_pass_unit_mapping(fmt):
    """UInt8 / UInt16 under the unit mapping (the decodeUnit streaming kernels): tied extremes in
    different lanes, waves and padded end items, a product that never reaches 0, and sums checked
    against the exact value (also the guard for the integer pass-1 variants of DESIGN §4.8)."""
    top = 255 if fmt == 4 else 65535
    dt = np.uint8 if fmt == 4 else np.uint16
    rng = np.random.default_rng(41 + fmt)
    cases = [((24, 40, 1040), (0, 0, 0), (1040, 40, 24)),       # one span
             ((24, 40, 1040), (3, 1, 2), (1037, 39, 23))]        # padded rows
    for dims, first, last in cases:
        codes = rng.integers(1, top, dims, dtype=dt)
        for z, y, x in ((5, 7, 9), (2, 3, 1000), (20, 30, 40)):   # tied minima, first is the answer
            codes[z, y, x] = 0
        for z, y, x in ((6, 1, 511), (6, 1, 513), (22, 38, 8)):   # tied maxima
            codes[z, y, x] = top
        for mapping in ((0.0, 1.0), (-0.0, 1.0)):                  # (-0, 1) keeps the float pass
            got = gpu_aggregates(codes, fmt, *mapping, first, last)
            ref = ob.aggregates_range(ob.Volume(codes, fmt, *mapping), first, last)
            what = f"fmt={fmt} box={first}->{last} map={mapping}"
            assert (got.min, got.max) == (ref.min, ref.max), what
            assert tuple(got.argmin) == tuple(ref.argmin) and tuple(got.argmax) == tuple(ref.argmax), what
            vals = values_of(codes, fmt, *mapping)[first[2]:last[2], first[1]:last[1], first[0]:last[0]].reshape(-1)
            exact = float(np.sum(vals, dtype=np.float64))
            check_float("sum", got.sum, ref.sum, exact, exact, vals.size)
    # product: all-top volume, (1 - 2^-16)^n stays far from 0; UInt8 top decodes to < 1 as well
    codes = np.full((4, 8, 64), top, dt)
    got = gpu_aggregates(codes, fmt, 0.0, 1.0, (0, 0, 0), (64, 8, 4))
    ref = ob.aggregates_range(ob.Volume(codes, fmt), (0, 0, 0), (64, 8, 4))
    v = float(values_of(codes[:1, :1, :1], fmt, 0.0, 1.0).reshape(-1)[0])
    exact_prod = v ** codes.size
    assert got.prod != 0.0 and abs(got.prod - exact_prod) <= codes.size * EPS * exact_prod, (got.prod, exact_prod)
    assert abs(got.prod - ref.prod) <= codes.size * EPS * exact_prod


def check_aggregates(got, codes, fmt, mapping, first, last, what):
    ref = ob.aggregates_range(ob.Volume(codes, fmt, *mapping), first, last)
    assert (got.min, got.max) == (ref.min, ref.max), what
    assert tuple(got.argmin) == tuple(ref.argmin) and tuple(got.argmax) == tuple(ref.argmax), what
    vals = values_of(codes, fmt, *mapping)[first[2]:last[2], first[1]:last[1], first[0]:last[0]].reshape(-1)
    n, nall = vals.size, codes.size
    check_float("sum", got.sum, ref.sum, float(np.sum(vals, dtype=np.float64)),
                float(np.sum(np.abs(vals), dtype=np.float64)), n)
    assert got.mean == np.float32(np.float64(np.float32(got.sum)) / nall), what
    d = (vals - np.float32(got.mean)).astype(np.float32)
    d2 = (d * d).astype(np.float32)
    exact_var = float(np.float32(np.float64(np.float32(np.sum(d2, dtype=np.float64))) / nall))
    moments = takes_moments(fmt, mapping) and lib_knob_moments_on()
    check_var(got.var, exact_var, moments, what)
    assert got.stddev == np.float32(np.sqrt(np.float32(got.var))), what
    return ref


_MOMENTS_OFF = []


def lib_knob_moments_on():
    return not _MOMENTS_OFF


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [4, 5])
@pytest.mark.parametrize("mapping", [(0.0, 1.0), (3.0, -1.0), (-2.0, 5.0), (1000.0, 1000.001), (0.25, 0.25)])
def test_aggregates_code_counts(fmt, mapping):
    """UInt8 / UInt16 ComputeAggregates from one pass of code counts (knob aggregates.codes):
    increasing and decreasing mappings (the value minimum is then the LARGEST code), a mapping
    that rounds neighbouring codes to one value and a constant one (extremes held by several
    codes: the library reruns the two float passes), tied extremes across lanes, waves and
    padded end items; equal to the oracle and to the two-pass path (knob 0)."""
    rng = np.random.default_rng(17 + fmt)
    top, dt = (255, np.uint8) if fmt == 4 else (65535, np.uint16)
    cases = [((24, 40, 1040), (0, 0, 0), (1040, 40, 24)),      # one span
             ((24, 40, 1040), (3, 1, 2), (1037, 39, 23)),       # padded rows
             ((10, 64, 256), (8, 3, 2), (200, 60, 9))]          # strided box
    for dims, first, last in cases:
        codes = rng.integers(2, top - 1, dims, dtype=dt)
        for z, y, x in ((5, 7, 9), (2, 3, 1000 % dims[2]), (8, 30, 40)):
            codes[z, y, x] = 1
        for z, y, x in ((6, 1, 511 % dims[2]), (6, 1, 13), (9, 38, 8)):
            codes[z, y, x] = top - 1
        runs = []
        for k in (3, 0):
            lib.vktHipSetTuningKnob(b"aggregates.codes", k)
            try:
                got = gpu_aggregates(codes, fmt, *mapping, first, last)
            finally:
                lib.vktHipSetTuningKnob(b"aggregates.codes", -1)
            check_aggregates(got, codes, fmt, mapping, first, last, f"fmt={fmt} map={mapping} {first}->{last} knob={k}")
            runs.append(got)
        a, b = runs
        assert (a.min, a.max, tuple(a.argmin), tuple(a.argmax), a.mean) == (b.min, b.max, tuple(b.argmin),
                                                                          tuple(b.argmax), b.mean)
    # extremes that first occur after the first 512 Ki voxels of the range (the whole-grid
    # second stage of the first-occurrence search), once in a span and once in a padded box
    codes = rng.integers(2, top - 1, (16, 64, 1024), dtype=dt)
    codes[12, 5, 700] = codes[14, 0, 3] = 1
    codes[15, 63, 1000] = codes[13, 9, 9] = top - 1
    for first, last in (((0, 0, 0), (1024, 64, 16)), ((3, 1, 0), (1021, 64, 16))):
        got = gpu_aggregates(codes, fmt, *mapping, first, last)
        check_aggregates(got, codes, fmt, mapping, first, last, f"late extremes map={mapping} {first}->{last}")
    # product through value^count: 256 voxels of ~1.01 (the top code under (0, 1.01)), ~12.8
    codes = np.full((2, 2, 64), top, dt)
    got = gpu_aggregates(codes, fmt, 0.0, 1.01, (0, 0, 0), (64, 2, 2))
    v = float(values_of(codes[:1, :1, :1], fmt, 0.0, 1.01).reshape(-1)[0])
    exact = v ** codes.size
    assert abs(got.prod - exact) <= codes.size * EPS * exact, (got.prod, exact)


@pytest.mark.gpu
def test_aggregates_ties_specials_and_whole_volume_mean():
    # duplicate minima / maxima: first occurrence in z, y, x order; NaN never min / max;
    # +-inf: -inf < FLT_MAX and +inf > -FLT_MAX, so both qualify (the reference starts from
    # +-FLT_MAX); NaN never compares
    vals = np.full((6, 5, 4), 0.5, np.float32)
    vals[1, 2, 3] = vals[4, 0, 0] = -2.0
    vals[2, 1, 1] = vals[0, 4, 3] = 7.0
    vals[3, 3, 3] = np.nan
    codes = vals.view(np.uint32)
    got = gpu_aggregates(codes, 7, 0.0, 1.0, (0, 0, 0), (4, 5, 6))
    ref = ob.aggregates_range(ob.Volume(codes, 7), (0, 0, 0), (4, 5, 6))
    assert (got.min, tuple(got.argmin), got.max, tuple(got.argmax)) == (-2.0, (3, 2, 1), 7.0, (3, 4, 0))
    assert (ref.min, tuple(ref.argmin), ref.max, tuple(ref.argmax)) == (-2.0, (3, 2, 1), 7.0, (3, 4, 0))
    assert np.isnan(got.sum) and np.isnan(ref.sum)
    vals2 = np.array([np.inf, -np.inf, np.nan, 1.0], np.float32).reshape(1, 1, 4)
    got = gpu_aggregates(vals2.view(np.uint32), 7, 0.0, 1.0, (0, 0, 0), (4, 1, 1))
    ref = ob.aggregates_range(ob.Volume(vals2.view(np.uint32), 7), (0, 0, 0), (4, 1, 1))
    assert (got.min, tuple(got.argmin), got.max, tuple(got.argmax)) == (ref.min, tuple(ref.argmin), ref.max,
                                                                        tuple(ref.argmax)) == (-np.inf, (1, 0, 0), np.inf, (0, 0, 0))
    # all NaN: min stays FLT_MAX, argmin {0,0,0}
    nan = np.full((1, 2, 3), np.nan, np.float32).view(np.uint32)
    got = gpu_aggregates(nan, 7, 0.0, 1.0, (0, 0, 0), (3, 2, 1))
    assert got.min == np.finfo(np.float32).max and tuple(got.argmin) == (0, 0, 0)
    assert got.max == -np.finfo(np.float32).max and tuple(got.argmax) == (0, 0, 0)
    # sub-range: mean divides by the WHOLE volume's voxel count (Aggregates_serial.hpp:61-63)
    codes = np.full((10, 10, 10), 128, np.uint8)
    got = gpu_aggregates(codes, 4, 0.0, 1.0, (0, 0, 0), (10, 10, 1))
    ref = ob.aggregates_range(ob.Volume(codes, 4), (0, 0, 0), (10, 10, 1))
    assert got.mean == np.float32(np.float64(np.float32(got.sum)) / 1000)
    assert abs(got.mean - ref.mean) <= 100 * EPS * abs(ref.mean)      # serial float sum of 100 terms


@pytest.mark.gpu
@pytest.mark.parametrize("nx", [33, 64])   # row kernel / streaming kernel
def test_aggregate_slab_partials_combine_to_the_whole(nx):
    """Z-slab partials (multi-GPU building block): two slabs with their global z offset,
    combined, mean of the whole, pass 2, finish == single-volume result."""
    rng = np.random.default_rng(3)
    codes = rng.integers(0, 65536, (20, 17, nx), dtype=np.uint16)
    codes[3, 5, 7] = codes[15, 2, 1] = 0          # tied minima in different slabs
    codes[12, 9, 2] = codes[16, 0, 0] = 65535     # tied maxima in the second slab
    whole = gpu_aggregates(codes, 5, -1.0, 3.0, (0, 0, 0), (nx, 17, 20))
    ref = ob.aggregates_range(ob.Volume(codes, 5, -1.0, 3.0), (0, 0, 0), (nx, 17, 20))
    assert tuple(whole.argmin) == tuple(ref.argmin) == (7, 5, 3)
    assert tuple(whole.argmax) == tuple(ref.argmax) == (2, 9, 12)
    P = _lib.HipAggregatePartial_t
    slabs = [(0, 7), (7, 20)]
    vols = [gpu_volume(np.ascontiguousarray(codes[z0:z1]), 5, -1.0, 3.0) for z0, z1 in slabs]
    set_device(vkt.ExecutionPolicy.Device_GPU)
    try:
        acc1 = P()
        lib.vktHipAggregatePartialInit(C.byref(acc1))
        for (z0, z1), v in zip(slabs, vols):
            p = P()
            assert lib.vktHipAggregatesPass(v.hip_view(), _lib.Vec3i_t(0, 0, 0), _lib.Vec3i_t(nx, 17, z1 - z0), z0, 1,
                                            0.0, C.byref(p)) == 0
            lib.vktHipAggregatePartialCombine(C.byref(acc1), C.byref(p))
        mean = lib.vktHipAggregatesMean(C.byref(acc1), codes.size)
        acc2 = P()
        lib.vktHipAggregatePartialInit(C.byref(acc2))
        for (z0, z1), v in zip(slabs, vols):
            p = P()
            assert lib.vktHipAggregatesPass(v.hip_view(), _lib.Vec3i_t(0, 0, 0), _lib.Vec3i_t(nx, 17, z1 - z0), z0, 2,
                                            mean, C.byref(p)) == 0
            lib.vktHipAggregatePartialCombine(C.byref(acc2), C.byref(p))
    finally:
        set_device(vkt.ExecutionPolicy.Device_CPU)
    out = _lib.Aggregates_t()
    lib.vktHipAggregatesFinish(C.byref(acc1), C.byref(acc2), codes.size, nx, 17, C.byref(out))
    assert (out.min, out.max) == (whole.min, whole.max)
    assert (out.argmin.x, out.argmin.y, out.argmin.z) == tuple(whole.argmin)
    assert (out.argmax.x, out.argmax.y, out.argmax.z) == tuple(whole.argmax)
    assert out.mean == whole.mean
    check_var(whole.var, out.var, True, "whole (moments) vs slab partials (two passes)")


@pytest.mark.gpu
@pytest.mark.parametrize("rows16", [1, 2, 0])
def test_u8_code_counts_over_rows_exact(rows16):
    """UInt8 code counts over range rows (vktHipAggregateCodeCounts): the 16-voxel
    row walk counts every byte of each row's 16-aligned cover and subtracts the bytes outside
    the range again, inside the main loop (knob reduce.u8_rows16 = 1; rows of >= 9 items) or in
    a row walk after it (2); the 8-voxel walk masks them (0).  Exact against
    np.bincount of the box: row starts and ends at every phase mod 16, boxes touching x = 0 and
    x = dimX, one-row / one-plane boxes, rows of fewer than 16 voxels inside one item, a volume
    whose dimX is a multiple of 8 but not 16 (8-voxel walk either way), and ranges whose item
    count leaves a partial wave-step."""
    import torch
    rng = np.random.default_rng(71)
    vols = {(12, 21, 256): None, (9, 7, 1040): None, (5, 6, 200): None}
    boxes = {(12, 21, 256): [((100, 3, 1), (228, 20, 12)), ((0, 0, 0), (256, 21, 12)), ((1, 0, 0), (255, 21, 12)),
                             ((15, 2, 3), (17, 3, 4)), ((16, 5, 2), (32, 6, 11)), ((33, 4, 4), (47, 16, 9)),
                             ((241, 0, 0), (256, 21, 12)), ((0, 7, 5), (1, 8, 6))],
             (9, 7, 1040): [((3, 1, 2), (1037, 6, 8)), ((17, 0, 0), (1039, 7, 9)), ((0, 3, 4), (1040, 4, 5))],
             (5, 6, 200): [((3, 1, 1), (197, 5, 4)), ((8, 0, 0), (200, 6, 5))]}
    for dims, bl in boxes.items():
        codes = rng.integers(0, 256, dims, dtype=np.uint8)
        v = gpu_volume(codes, 4, 0.0, 1.0)
        set_device(vkt.ExecutionPolicy.Device_GPU)
        lib.vktHipSetTuningKnob(b"reduce.u8_rows16", rows16)
        try:
            for first, last in bl:
                counts = torch.zeros(256, dtype=torch.int64, device="cuda")
                err = lib.vktHipAggregateCodeCounts(v.hip_view(), _lib.Vec3i_t(*first), _lib.Vec3i_t(*last),
                                                    C.c_void_p(counts.data_ptr()))
                assert err == 0, _lib.last_error()
                box = codes[first[2]:last[2], first[1]:last[1], first[0]:last[0]]
                want = np.bincount(box.reshape(-1), minlength=256)
                got = counts.cpu().numpy()
                assert np.array_equal(got, want), (dims, first, last, np.nonzero(got != want)[0][:8])
        finally:
            lib.vktHipSetTuningKnob(b"reduce.u8_rows16", -1)
            set_device(vkt.ExecutionPolicy.Device_CPU)


@pytest.mark.gpu
@pytest.mark.parametrize("rows16", [1, 2, 0])
def test_u8_histogram_over_rows_from_code_counts(rows16):
    """UInt8 histograms over range rows from the 16-voxel code counts folded into the bins with
    the streaming kernel's bin formula (knob reduce.u8_rows16 1 / 2; 0 = the 8-voxel item walk):
    padded and unpadded rows of >= 9 items (end bytes subtracted inside the main loop), bin
    counts below, at and above 256, and mappings that drop codes outside [0, numBins)."""
    rng = np.random.default_rng(5 + rows16)
    codes = rng.integers(0, 256, (8, 20, 320), dtype=np.uint8)
    lib.vktHipSetTuningKnob(b"reduce.u8_rows16", rows16)
    try:
        for first, last in (((3, 1, 1), (317, 19, 7)), ((16, 0, 0), (304, 20, 8)), ((100, 2, 3), (250, 3, 8))):
            for mapping, nbins in (((0.0, 1.0), 256), ((0.0, 1.0), 7), ((-1.0, 3.0), 1000), ((0.25, 0.75), 64)):
                got = gpu_histogram(codes, 4, *mapping, first, last, nbins)
                ref, _ = ob.histogram_range(ob.Volume(codes, 4, *mapping), first, last, nbins)
                np.testing.assert_array_equal(got, ref, err_msg=f"{first}->{last} map={mapping} nbins={nbins}")
    finally:
        lib.vktHipSetTuningKnob(b"reduce.u8_rows16", -1)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5])
def test_aggregates_uint16_moment_variants(variant):
    """Every integer-moments kernel variant (knob aggregates.moments_pipe: buffers x items per lane,
    5 = the two-buffer kernel bound to 7 waves per SIMD) against the oracle over spans, padded
    rows and extremes first occurring late in a lane's walk."""
    rng = np.random.default_rng(77 + variant)
    late = rng.integers(100, 60000, (16, 64, 1024), dtype=np.uint16)
    late[12, 5, 700] = late[14, 0, 3] = 3
    late[15, 63, 1000] = late[13, 9, 9] = 65000
    assert lib.vktHipSetTuningKnob(b"aggregates.moments_pipe", variant) == 0
    try:
        for first, last in (((0, 0, 0), (1024, 64, 16)), ((3, 1, 0), (1021, 64, 16)), ((9, 5, 3), (1001, 60, 14))):
            got = gpu_aggregates(late, 5, 0.0, 1.0, first, last)
            check_aggregates(got, late, 5, (0.0, 1.0), first, last, f"variant={variant} {first}->{last}")
    finally:
        lib.vktHipSetTuningKnob(b"aggregates.moments_pipe", -1)


@pytest.mark.gpu
def test_aggregates_uint16_moments():
    """UInt16 ComputeAggregates under the unit mapping from one pass of exact integer moments
    (knob aggregates.moments) against the oracle and against the code-count path
    (knob 0): every code once (min 0 / max 65535 at known places), random codes over spans,
    padded rows (row ends at every phase mod 8, masked end items), strided boxes, ranges with a
    partial wave-step, tied extremes across lanes / waves / steps, extremes first occurring late,
    constant volumes (var exactly 0 over the whole volume, as the float terms give), a constant volume whose first voxel
    differs (the cancellation case of a float moment form), a product that stays above 0.
    min / max / arg / sum / mean are identical to the code-count path; var within the stated bound."""
    rng = np.random.default_rng(2024)
    every = rng.permutation(np.arange(65536, dtype=np.uint16)).reshape(16, 16, 256)
    rand = rng.integers(0, 65536, (24, 40, 1040), dtype=np.uint16)
    for z, y, x in ((5, 7, 9), (2, 3, 1000), (20, 30, 40), (23, 39, 1039)):
        rand[z, y, x] = 7          # tied small codes (the minimum of rand below 7 is overwritten)
    rand[rand < 7] = 8
    for z, y, x in ((6, 1, 511), (6, 1, 513), (22, 38, 8)):
        rand[z, y, x] = 65535
    const = np.full((10, 20, 64), 40000, np.uint16)
    outlier = const.copy()
    outlier[0, 0, 0] = 1
    late = rng.integers(100, 60000, (16, 64, 1024), dtype=np.uint16)
    late[12, 5, 700] = late[14, 0, 3] = 3
    late[15, 63, 1000] = late[13, 9, 9] = 65000
    cases = [(every, [((0, 0, 0), (256, 16, 16)), ((3, 1, 2), (253, 15, 14)), ((8, 0, 0), (16, 16, 16))]),
             (rand, [((0, 0, 0), (1040, 40, 24)), ((3, 1, 2), (1037, 39, 23)), ((1, 0, 0), (2, 40, 24)),
                     ((9, 5, 3), (1031, 6, 4)), ((0, 0, 5), (1040, 40, 6)), ((512, 3, 3), (520, 9, 20))]),
             (const, [((0, 0, 0), (64, 20, 10)), ((5, 3, 1), (61, 19, 9))]),
             (outlier, [((0, 0, 0), (64, 20, 10))]),
             (late, [((0, 0, 0), (1024, 64, 16)), ((3, 1, 0), (1021, 64, 16))])]
    for codes, boxes in cases:
        for first, last in boxes:
            what = f"dims={codes.shape} {first}->{last}"
            got = gpu_aggregates(codes, 5, 0.0, 1.0, first, last)
            check_aggregates(got, codes, 5, (0.0, 1.0), first, last, what)
            lib.vktHipSetTuningKnob(b"aggregates.moments", 0)
            _MOMENTS_OFF.append(1)
            try:
                two = gpu_aggregates(codes, 5, 0.0, 1.0, first, last)
                check_aggregates(two, codes, 5, (0.0, 1.0), first, last, what + " knob=0")
            finally:
                _MOMENTS_OFF.clear()
                lib.vktHipSetTuningKnob(b"aggregates.moments", -1)
            assert (got.min, got.max, tuple(got.argmin), tuple(got.argmax), got.sum, got.mean) == \
                (two.min, two.max, tuple(two.argmin), tuple(two.argmax), two.sum, two.mean), what
            if codes is const and last == codes.shape[::-1] and first == (0, 0, 0):
                assert got.var == 0.0 and two.var == 0.0, what   # (a sub-box's mean divides by the whole count)
    # product through the pair products: all-top volume, (1 - 2^-16)^n stays far from 0
    codes = np.full((4, 8, 64), 65535, np.uint16)
    got = gpu_aggregates(codes, 5, 0.0, 1.0, (0, 0, 0), (64, 8, 4))
    exact = (65535 / 65536) ** codes.size
    assert got.prod != 0.0 and abs(got.prod - exact) <= codes.size * EPS * exact, (got.prod, exact)


@pytest.mark.gpu
def test_aggregates_uint16_moments_sum_of_squares_beyond_2_64():
    """The code sum of squares of > 2^32 voxels of code 65535 exceeds 2^64: the 128-bit combine of
    the workgroup partials (aggregatesMomentsU16FinalKernel).  Constant volume of 2048 x 2048 x
    1025 voxels (8.6 GB): sum = n * 65535 * 2^-16 exactly rounded, var = the float mean's offset
    from the value squared, as the float terms of the reference give it."""
    import torch
    dims = (2048, 2048, 1025)
    n = dims[0] * dims[1] * dims[2]
    t = torch.empty((2 * n,), dtype=torch.uint8, device="cuda")
    view = _lib.HipVolumeView_t(t.data_ptr(), dims[0], dims[1], dims[2], 5, 0.0, 1.0)
    out = _lib.Aggregates_t()
    try:
        assert lib.vktHipFillRange(view, _lib.Vec3i_t(0, 0, 0), _lib.Vec3i_t(*dims), C.c_float(65535 / 65536)) == 0
        assert lib.vktHipAggregatesRange(view, _lib.Vec3i_t(0, 0, 0), _lib.Vec3i_t(*dims), C.byref(out)) == 0, \
            _lib.last_error()
    finally:
        del t
        torch.cuda.empty_cache()
    v = np.float32(65535 / 65536)
    s = np.float32(n * (65535 / 65536))
    assert out.sum == s
    m = np.float32(np.float64(s) / n)
    assert out.mean == m
    d = np.float32(v - m)
    var_terms = float(np.float32(np.float64(np.float32(np.float64(d * d) * n)) / n))
    check_var(out.var, var_terms, True, "2^32+ voxels")
    assert (out.min, out.max) == (v, v)
    assert (out.argmin.x, out.argmin.y, out.argmin.z) == (0, 0, 0) == (out.argmax.x, out.argmax.y, out.argmax.z)


@pytest.mark.gpu
def test_aggregates_float_moments_and_fallbacks():
    """UInt16 under other mappings and Float32 from one pass of floating-point moments (knob
    aggregates.moments bit 1): against the oracle and the two-pass path (knob 0) over
    spans, padded rows and strided boxes, a narrow mapping (1000, 1000.001) whose values sit far
    from 0 relative to their spread, and a first lane value far from the rest (the pivot case).
    Volumes whose float terms may leave the normal float range must give the two-pass result
    exactly: NaN / Inf voxels, |v - m| beyond 2^62 (3e30), values with a nonzero |v| < 2^-40
    (1e-20, denormals), and a UInt16 mapping whose codes decode to such tiny values."""
    rng = np.random.default_rng(99)
    boxes = [((0, 0, 0), (520, 24, 12)), ((3, 1, 2), (517, 23, 11)), ((8, 3, 2), (200, 20, 9))]

    def both(codes, fmt, mapping, first, last):
        got = gpu_aggregates(codes, fmt, *mapping, first, last)
        lib.vktHipSetTuningKnob(b"aggregates.moments", 0)
        try:
            two = gpu_aggregates(codes, fmt, *mapping, first, last)
        finally:
            lib.vktHipSetTuningKnob(b"aggregates.moments", -1)
        return got, two

    for fmt, mapping in ((5, (-1.0, 3.0)), (5, (1000.0, 1000.001)), (5, (3.0, -1.0)), (7, (0.0, 1.0)),
                         (2, (-1.0, 3.0)), (2, (1000.0, 1000.001)), (6, (0.25, 7.5)), (6, (3.0, -1.0))):
        codes = rand_codes(rng, fmt, (12, 24, 520))
        if fmt == 7:
            vals = codes.view(np.float32)
            vals[0, 0, 0] = 2.0e6      # the first lane's pivot far from its other values
        for first, last in boxes:
            what = f"fmt={fmt} map={mapping} {first}->{last}"
            got, two = both(codes, fmt, mapping, first, last)
            check_aggregates(got, codes, fmt, mapping, first, last, what)
            assert (got.min, got.max, tuple(got.argmin), tuple(got.argmax)) == \
                (two.min, two.max, tuple(two.argmin), tuple(two.argmax)), what
    # fallbacks: bit-identical to the two passes -- Int16 / UInt32 mappings whose values are tiny
    # (Int16: found per code on the host; UInt32: flagged per voxel)
    for fmt, mapping in ((2, (-1e-20, 1e-20)), (6, (-1e-20, 1e-20))):
        codes = rand_codes(rng, fmt, (8, 16, 256))
        got, two = both(codes, fmt, mapping, (0, 0, 0), (256, 16, 8))
        for f in ("min", "max", "sum", "mean", "var", "stddev", "prod"):
            assert np.array_equal(np.float32(getattr(got, f)), np.float32(getattr(two, f)), equal_nan=True), \
                f"fmt={fmt} {f}"
        assert tuple(got.argmin) == tuple(two.argmin) and tuple(got.argmax) == tuple(two.argmax)
    base = rng.uniform(-1.0, 1.0, (8, 16, 256)).astype(np.float32)
    specials = {"nan": np.nan, "inf": np.inf, "huge": 3.0e30, "tiny": 1.0e-20, "denormal": 1.0e-40}
    for name, val in specials.items():
        vals = base.copy()
        vals[3, 5, 100] = val
        codes = vals.view(np.uint32)
        for first, last in ((((0, 0, 0), (256, 16, 8))), (((3, 1, 1), (250, 15, 7)))):
            got, two = both(codes, 7, (0.0, 1.0), first, last)
            for f in ("min", "max", "sum", "mean", "var", "stddev", "prod"):
                a, b = getattr(got, f), getattr(two, f)
                assert (a == b) or (np.isnan(a) and np.isnan(b)), (name, f, a, b)
            assert tuple(got.argmin) == tuple(two.argmin) and tuple(got.argmax) == tuple(two.argmax)
    # a UInt16 mapping with codes decoding to tiny nonzero values: (-2^-41 * 65536 ... ) around 0
    codes = rng.integers(0, 65536, (8, 16, 256), dtype=np.uint16)
    tiny_map = (-1.0e-13, 1.0e-13)
    got, two = both(codes, 5, tiny_map, (0, 0, 0), (256, 16, 8))
    for f in ("min", "max", "sum", "mean", "var", "prod"):
        assert getattr(got, f) == getattr(two, f), f


@pytest.mark.gpu
def test_moments_first_occurrence_across_wave_steps():
    """The moment kernels keep each lane's extremes per wave-step and look up the first voxel of
    the extreme code in its step after the walk.  Volumes large enough that every wave walks many
    steps, with the extreme values repeated at scattered positions (ties within and across steps,
    lanes and workgroups), +0 / -0 both minimal for Float32: arg positions are the first
    occurrences in linear order and min keeps the first zero's sign -- as the reference's strict
    in-order updates (Aggregates_serial.hpp:40-49).  Spans and a padded sub-box."""
    rng = np.random.default_rng(4242)
    shape = (128, 256, 1024)   # (z, y, x): 32 Mi voxels, ~4 Mi items, many steps per wave
    n = shape[0] * shape[1] * shape[2]

    def first_xyz(flat, idx_box):
        z, y, x = np.unravel_index(flat, idx_box)
        return int(x), int(y), int(z)

    # UInt16, unit mapping (integer moments): codes in [1, 65534], then 0 and 65535 at 300
    # random places each
    codes = rng.integers(1, 65535, shape, dtype=np.uint16)
    flat = codes.reshape(-1)
    flat[rng.choice(n, 300, replace=False)] = 0
    flat[rng.choice(n, 300, replace=False)] = 65535
    for first, last in (((0, 0, 0), (1024, 256, 128)), ((100, 3, 5), (900, 250, 120))):
        (x0, y0, z0), (x1, y1, z1) = first, last
        sub = codes[z0:z1, y0:y1, x0:x1]
        a = gpu_aggregates(codes, 5, 0.0, 1.0, first, last)
        lo, hi = np.argmin(sub), np.argmax(sub)
        ex, ey, ez = first_xyz(lo, sub.shape)
        assert tuple(a.argmin) == (ex + x0, ey + y0, ez + z0), (first, "argmin")
        ex, ey, ez = first_xyz(hi, sub.shape)
        assert tuple(a.argmax) == (ex + x0, ey + y0, ez + z0), (first, "argmax")
        assert a.min == 0.0 and a.max == np.float32(65535 / 65536)
    # Float32 (float moments): values in [1, 2), zeros of random sign and a repeated maximum 5.0
    vals = rng.uniform(1.0, 2.0, shape).astype(np.float32)
    fv = vals.reshape(-1)
    zeros = rng.choice(n, 200, replace=False)
    fv[zeros] = np.where(rng.random(200) < 0.5, np.float32(0.0), np.float32(-0.0))
    fv[rng.choice(n, 200, replace=False)] = 5.0
    for first, last in (((0, 0, 0), (1024, 256, 128)), ((100, 3, 5), (900, 250, 120))):
        (x0, y0, z0), (x1, y1, z1) = first, last
        sub = vals[z0:z1, y0:y1, x0:x1]
        a = gpu_aggregates(vals.view(np.uint32), 7, 0.0, 1.0, first, last)
        lo, hi = np.argmin(sub), np.argmax(sub)
        ex, ey, ez = first_xyz(lo, sub.shape)
        assert tuple(a.argmin) == (ex + x0, ey + y0, ez + z0), (first, "argmin f32")
        assert np.signbit(np.float32(a.min)) == np.signbit(sub.reshape(-1)[lo]), (first, "sign of the first zero")
        ex, ey, ez = first_xyz(hi, sub.shape)
        assert tuple(a.argmax) == (ex + x0, ey + y0, ez + z0), (first, "argmax f32")
        assert a.max == 5.0
