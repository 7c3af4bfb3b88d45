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
