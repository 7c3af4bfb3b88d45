"""Random-geometry fuzz of Resample (HIP path through the C ABI) vs the oracle: random source
and destination dims (integer ratios, non-integer up/down-sampling, mixed per axis, 1-voxel
axes), every format pair of the hot path, both filter modes, unit and non-unit mappings, and
Float32 sources with sparse specials (NaN, +-inf, -0) so the Linear chain's fix-up path runs.
Bit-exact (NaN matches NaN), DESIGN.md §3."""
import numpy as np
import pytest

from backends import GpuBackend, OracleBackend
from test_gpu_parity import assert_codes_equal, rand_codes

pytestmark = pytest.mark.gpu

FMTS = [4, 5, 7, 2, 6]


@pytest.fixture(scope="module")
def g():
    return GpuBackend()


@pytest.fixture(scope="module")
def o():
    return OracleBackend()


def dims_pair(rng):
    src, dst = [], []
    for _ in range(3):
        kind = rng.integers(0, 5)
        s = int(rng.integers(1, 40 if rng.random() < 0.8 else 140))
        if kind == 0:
            d = s * int(rng.choice([1, 2, 4]))            # integer up-sampling ratio
        elif kind == 1:
            d = max(1, s // int(rng.choice([2, 3])))      # down-sampling
        elif kind == 2:
            d = 1                                         # collapse an axis
        else:
            d = int(rng.integers(1, 70))                  # any ratio
        src.append(s)
        dst.append(d)
    return tuple(src), tuple(dst)


@pytest.mark.parametrize("seed", range(6))
def test_resample_random_geometry(g, o, seed):
    rng = np.random.default_rng(5000 + seed)
    for case in range(25):
        sd, dd = dims_pair(rng)
        sf = int(rng.choice(FMTS))
        df = sf if rng.random() < 0.6 else int(rng.choice(FMTS))
        smap = [(0.0, 1.0), (-1.0, 3.0), (0.25, 7.5)][int(rng.integers(0, 3))]
        dmap = [(0.0, 1.0), (-1.0, 3.0)][int(rng.integers(0, 2))]
        src = rand_codes(rng, sf, sd[::-1], floats="mixed")
        for fm in (0, 1):
            out = g.resample(df, dmap, dd, sf, smap, src, fm)
            ref = o.resample(df, dmap, dd, sf, smap, src, fm)
            assert_codes_equal(out, ref, df, f"fuzz{seed}.{case} {sd}->{dd} {sf}->{df} {smap}->{dmap} fm={fm}")


@pytest.mark.parametrize("prefetch", [2, 1, 0])
def test_resample_gather_prefetch_multi_task_waves(g, o, prefetch):
    """Knob resample.prefetch: UInt8 destinations cap the LDS gather's grid, so with more source
    rows than waves (260 x 260 rows here, 65 536 waves) a wave runs several tasks and loads the
    next task's row while it gathers the current one (knob 2; the default 1 prefetches for 2-byte
    destinations only) -- UInt8 and UInt8 -> UInt16 vs the oracle, every knob value."""
    from volkit_amd._lib import lib
    rng = np.random.default_rng(77)
    src = rand_codes(rng, 4, (260, 260, 32))
    assert lib.vktHipSetTuningKnob(b"resample.prefetch", prefetch) == 0
    try:
        for fm in (0, 1):
            for df in (4, 5):
                out = g.resample(df, (0.0, 1.0), (48, 300, 300), 4, (0.0, 1.0), src, fm)
                ref = o.resample(df, (0.0, 1.0), (48, 300, 300), 4, (0.0, 1.0), src, fm)
                assert_codes_equal(out, ref, df, f"prefetch={prefetch} df={df} fm={fm}")
    finally:
        lib.vktHipSetTuningKnob(b"resample.prefetch", -1)


@pytest.mark.parametrize("anyrows", [1, 0])
@pytest.mark.parametrize("sd,dd,sf,df", [((37, 20, 10), (64, 30, 14), 4, 4), ((21, 13, 9), (40, 20, 11), 5, 5),
                                         ((13, 9, 7), (20, 11, 9), 7, 7), ((100, 8, 6), (128, 9, 7), 4, 4),
                                         ((250, 12, 5), (176, 7, 9), 4, 5), ((19, 33, 4), (32, 17, 6), 7, 4)])
def test_resample_gather_rows_not_16_byte_multiples(g, o, sd, dd, sf, df, anyrows):
    """Knob resample.any_rows: source rows that are not 16-B multiples are staged in LDS too (the
    chunk past the row end taken at rowBytes - 16, overlapping its neighbour), Float32 Linear
    with specials included -- vs the oracle, knob on and off."""
    from volkit_amd._lib import lib
    rng = np.random.default_rng(sum(sd) * 3 + sum(dd) + sf * 11 + df)
    src = rand_codes(rng, sf, sd[::-1], floats="mixed")
    assert lib.vktHipSetTuningKnob(b"resample.any_rows", anyrows) == 0
    try:
        for fm in (0, 1):
            for dmap in ((0.0, 1.0), (-1.0, 3.0)):
                out = g.resample(df, dmap, dd, sf, (0.0, 1.0), src, fm)
                ref = o.resample(df, dmap, dd, sf, (0.0, 1.0), src, fm)
                assert_codes_equal(out, ref, df, f"anyrows={anyrows} {sd}->{dd} {sf}->{df} {dmap} fm={fm}")
    finally:
        lib.vktHipSetTuningKnob(b"resample.any_rows", -1)


PC_SHAPES = [
    ((48, 40, 24), (64, 52, 30), 4, 4),
    ((64, 40, 24), (48, 30, 20), 4, 4),
    ((1000, 6, 5), (1024, 7, 6), 4, 4),        # 1000-B rows: the chunk at rowBytes - 16
    ((70, 9, 11), (50, 13, 8), 5, 5),
    ((300, 7, 6), (512, 5, 9), 5, 5),
    ((130, 6, 7), (97, 8, 5), 7, 7),
    ((260, 5, 9), (300, 6, 4), 4, 5),          # UInt8 -> UInt16 (conversion)
    ((1024, 3, 4), (768, 5, 3), 5, 5),         # 2-KiB rows, several chunks per lane
    ((1024, 3, 4), (1500, 5, 3), 7, 7),        # 4-KiB rows
]


@pytest.mark.parametrize("pad", [1, 2])
@pytest.mark.parametrize("prefetch", [0, 2])
def test_resample_padded_lds_rows(g, o, pad, prefetch):
    """Knob resample.lds_pad (round 6): staged rows with 16 B of padding after every 256 B
    (UInt8 sources: 1; every format: 2), with and without the next-row prefetch -- the
    PC_SHAPES cases (rows of 48 B to 4 KiB, 16-B multiples padded, others not) vs the oracle."""
    from volkit_amd._lib import lib
    rng = np.random.default_rng(500 + pad + prefetch)
    assert lib.vktHipSetTuningKnob(b"resample.lds_pad", pad) == 0
    assert lib.vktHipSetTuningKnob(b"resample.prefetch", prefetch) == 0
    try:
        for sd, dd, sf, df in PC_SHAPES + [((1024, 20, 9), (768, 25, 7), 4, 4), ((512, 9, 9), (700, 9, 9), 4, 4)]:
            src = rand_codes(rng, sf, sd[::-1])
            for fm in (0, 1):
                out = g.resample(df, (0.0, 1.0), dd, sf, (0.0, 1.0), src, fm)
                ref = o.resample(df, (0.0, 1.0), dd, sf, (0.0, 1.0), src, fm)
                assert_codes_equal(out, ref, df, f"pad={pad} {sd}->{dd} {sf}->{df} fm={fm}")
    finally:
        lib.vktHipSetTuningKnob(b"resample.lds_pad", -1)
        lib.vktHipSetTuningKnob(b"resample.prefetch", -1)


@pytest.mark.parametrize("cap", [2, 64, 1, 0])
def test_resample_dst_row_gather(g, o, cap):
    """Knob resample.dst_rows (round 6): the LDS gather over destination-row tasks -- a fixed number
    of loads and stores per task, the next row's loads in flight across this task's stores
    (resampleGatherDstRowKernel) -- vs the oracle: UInt8 (padded and unpadded rows, a conversion)
    and UInt16, one and two store groups and source chunks, destination rows that are not whole
    store groups (lanes repeat the last lane's store), a small grid (cap 2: waves loop over many
    tasks) and a large one, the default (1: UInt8 rows that are not 16-B multiples) and off (0).
    Rows beyond the kernel's limits take the source-row gather."""
    from volkit_amd._lib import lib
    rng = np.random.default_rng(700 + cap)
    assert lib.vktHipSetTuningKnob(b"resample.dst_rows", cap) == 0
    shapes = PC_SHAPES + [((1024, 9, 7), (768, 11, 5), 4, 4), ((768, 7, 6), (1024, 9, 8), 4, 4),
                          ((1000, 5, 6), (1024, 7, 5), 4, 4), ((768, 6, 5), (1024, 8, 7), 5, 5),
                          ((1001, 4, 5), (1000, 6, 4), 5, 5), ((40, 30, 20), (24, 40, 30), 4, 4)]
    try:
        for sd, dd, sf, df in shapes:
            src = rand_codes(rng, sf, sd[::-1])
            for dmap in ((0.0, 1.0), (-1.0, 3.0)):
                out = g.resample(df, dmap, dd, sf, (0.0, 1.0), src, 0)
                ref = o.resample(df, dmap, dd, sf, (0.0, 1.0), src, 0)
                assert_codes_equal(out, ref, df, f"dst_rows={cap} {sd}->{dd} {sf}->{df} dmap={dmap}")
    finally:
        lib.vktHipSetTuningKnob(b"resample.dst_rows", -1)
