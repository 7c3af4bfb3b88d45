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


@pytest.mark.parametrize("xreg", [1, 0])
@pytest.mark.parametrize("sd,dd,sf,df", [((48, 20, 10), (64, 27, 13), 5, 5), ((64, 30, 20), (48, 17, 9), 4, 4),
                                         ((32, 16, 8), (48, 20, 12), 7, 7), ((96, 11, 7), (128, 5, 9), 5, 4),
                                         ((160, 9, 6), (96, 14, 6), 4, 5)])
def test_resample_gather_xtab_regs(g, o, sd, dd, sf, df, xreg):
    """Knob resample.xtab_regs: the LDS-staged gather with the x table loaded per lane from the
    device table (1) or staged in LDS (0) -- non-integer ratios with 16-B rows, vs the oracle."""
    from volkit_amd._lib import lib
    rng = np.random.default_rng(sum(sd) + 7 * sum(dd) + sf + df)
    src = rand_codes(rng, sf, sd[::-1], floats="mixed")
    assert lib.vktHipSetTuningKnob(b"resample.xtab_regs", xreg) == 0
    try:
        for fm in (0, 1):
            for dmap in ((0.0, 1.0), (-1.0, 3.0)):
                out = g.resample(df, dmap, dd, sf, (0.0, 1.0), src, fm)
                ref = o.resample(df, dmap, dd, sf, (0.0, 1.0), src, fm)
                assert_codes_equal(out, ref, df, f"xreg={xreg} {sd}->{dd} {sf}->{df} {dmap} fm={fm}")
    finally:
        lib.vktHipSetTuningKnob(b"resample.xtab_regs", -1)
