"""Known-answer vectors recorded from the compiled reference (tests/golden/reference_kat.json,
see tests/golden/make_reference_kat.py for provenance), run against the oracle (CPU) and
against the HIP library (gpu marker)."""
import json
import math
import os

import numpy as np
import pytest

from backends import codes_of

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kat.json")))["kats"]
BY_ID = {k["id"]: k for k in KAT}


def _f(v):
    return {"inf": math.inf, "nan": math.nan, "-0": -0.0}.get(v, v) if isinstance(v, str) else v


@pytest.mark.parametrize("kid", [k["id"] for k in KAT if k["op"] == "map"])
def test_map_kat(backend, kid):
    k = BY_ID[kid]
    assert backend.map(k["value"], k["fmt"], *k["mapping"]) == k["expect_code"]


def test_safesum_saturated_wraps(backend):
    k = BY_ID["safesum_u16_saturated_wraps_to_zero"]
    a = np.array(k["a"], dtype=np.uint16).reshape(1, 1, 1)
    b = np.array(k["b"], dtype=np.uint16).reshape(1, 1, 1)
    d = np.array(k["dst_init"], dtype=np.uint16).reshape(1, 1, 1)
    out = backend.arith(k["name"], [k["fmt"]] * 3, [k["mapping"]] * 3, a, b, d, k["first"], k["last"], k["off"])
    assert out.ravel().tolist() == k["expect"]


def test_sumrange_writes_absolute_index(backend):
    k = BY_ID["sumrange_absolute_destination_index"]
    a = np.arange(27, dtype=np.uint8).reshape(3, 3, 3)
    b = np.zeros((3, 3, 3), np.uint8)
    d = np.full((3, 3, 3), 255, np.uint8)
    out = backend.arith(k["name"], [k["fmt"]] * 3, [k["mapping"]] * 3, a, b, d, k["first"], k["last"], k["off"])
    changed = np.argwhere(out != 255)
    assert [list(map(int, c[::-1])) for c in changed] == k["expect_changed_voxels"]
    assert out[2, 2, 2] == a[2, 2, 2]


@pytest.mark.parametrize("kid", ["codec_roundtrip_all_u8_codes", "codec_roundtrip_all_u16_codes"])
def test_sum_with_zero_roundtrips_every_code(backend, kid):
    k = BY_ID[kid]
    n = 256 if k["fmt"] == 4 else 65536
    dt = np.uint8 if k["fmt"] == 4 else np.uint16
    a = np.arange(n, dtype=dt).reshape(1, 1, n)
    z = np.zeros_like(a)
    out = backend.arith("Sum", [k["fmt"]] * 3, [k["mapping"]] * 3, a, z, z.copy(), (0, 0, 0), (n, 1, 1), (0, 0, 0))
    np.testing.assert_array_equal(out, a)


@pytest.mark.parametrize("kid", ["resample_10_to_7", "resample_4_to_8_duplicates"])
def test_resample_index_table(backend, kid):
    k = BY_ID[kid]
    sx, sy, sz = k["src_dims"]
    src = np.array(k["src"], dtype=np.uint8).reshape(sz, sy, sx)
    out = backend.resample(k["fmt"], k["mapping"], k["dst_dims"], k["fmt"], k["mapping"], src, k["filter"])
    assert out.ravel().tolist() == k["expect"]


def test_resample_float_inf_row(backend):
    k = BY_ID["resample_float_inf_linear_vs_nearest"]
    sx, sy, sz = k["src_dims"]
    src = codes_of([_f(v) for v in k["src"]], 7).reshape(sz, sy, sx)
    for fm, key in ((1, "expect_linear_row0"), (0, "expect_nearest_row0")):
        out = backend.resample(7, k["mapping"], k["dst_dims"], 7, k["mapping"], src, fm)
        row0 = out[0, 0, :].view(np.float32)
        exp = np.array([_f(v) for v in k[key]], dtype=np.float32)
        np.testing.assert_array_equal(np.isnan(row0), np.isnan(exp))
        np.testing.assert_array_equal(row0[~np.isnan(exp)], exp[~np.isnan(exp)])


def test_resample_linear_equals_nearest_integer(backend):
    k = BY_ID["resample_linear_equals_nearest_for_integer_formats"]
    rng = np.random.default_rng(7)
    for fmt in k["fmts"]:
        dt = np.uint8 if fmt == 4 else np.uint16
        for (s, d) in k["pairs"]:
            src = rng.integers(0, np.iinfo(dt).max + 1, size=(s[2], s[1], s[0]), dtype=dt)
            lin = backend.resample(fmt, k["mapping"], d, fmt, k["mapping"], src, 1)
            nea = backend.resample(fmt, k["mapping"], d, fmt, k["mapping"], src, 0)
            np.testing.assert_array_equal(lin, nea)


def test_resample_negative_zero(backend):
    k = BY_ID["resample_linear_negative_zero_becomes_positive"]
    sx, sy, sz = k["src_dims"]
    src = codes_of([_f(v) for v in k["src"]], 7).reshape(sz, sy, sx)
    out = backend.resample(7, k["mapping"], k["dst_dims"], 7, k["mapping"], src, 1)
    signs = (out.ravel()[:2] >> 31).tolist()
    assert signs == k["expect_linear_signbits_first2"]
