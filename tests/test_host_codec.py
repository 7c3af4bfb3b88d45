"""The codec header the kernels use (include/volkit_codec.hpp), compiled for the host
inside libvolkit (vktMapVoxel / vktUnmapVoxel), against the oracle's restatement of
reference src/vkt/VoxelMapping.hpp -- every code of the 8/16-bit formats and a spread of
float inputs including the reference's traps.  CPU only."""
import ctypes as C
import struct

import numpy as np
import pytest

from oracle import binding as ob

MAPPINGS = [(0.0, 1.0), (-1.0, 3.0), (0.25, 7.5), (1.0, 0.0), (-0.0, 0.0), (0.0, 1e-38), (-3e38, 3e38)]
FORMATS = [1, 2, 3, 4, 5, 6, 7]


def special_floats():
    vals = [0.0, -0.0, 0.1, 0.5, 1.0, 1.5, -0.25, 0.99999994, 1.0000001, 255.999, 65535.999, 1e-45, -1e-45, 1e-38,
            3.4e38, -3.4e38, float("inf"), float("-inf"), float("nan"), 2147483520.0, 2147483648.0, -2147483648.0,
            -2147483904.0, 4294967040.0, 4294967296.0, 9.2e18, 9.3e18, -9.3e18, 32767.0, 32768.0, -32768.0]
    rng = np.random.default_rng(3)
    vals += list(rng.uniform(-2, 3, 300).astype(np.float32))
    vals += list((rng.integers(0, 2**32, 300, dtype=np.uint64).astype(np.uint32)).view(np.float32))
    return [float(np.float32(v)) for v in vals]


@pytest.fixture(scope="module")
def vkt():
    import volkit_amd.volkit as v
    return v


def lib_unmap(vkt, code_bytes, fmt, lo, hi):
    return vkt.UnmapVoxel(code_bytes, fmt, lo, hi)


def same_float(a, b):
    return struct.pack("<f", a) == struct.pack("<f", b) or (np.isnan(a) and np.isnan(b))


@pytest.mark.parametrize("fmt", [4, 5, 2])
@pytest.mark.parametrize("mapping", MAPPINGS[:4])
def test_unmap_every_code(vkt, fmt, mapping):
    n = 256 if fmt == 4 else 65536
    width = 1 if fmt == 4 else 2
    for c in range(0, n, 1 if n == 256 else 7):
        b = c.to_bytes(width, "little")
        got = vkt.UnmapVoxel(b, fmt, *mapping)
        ref = ob.unmap_voxel(b, fmt, *mapping)
        assert same_float(got, ref), (fmt, mapping, c, got, ref)


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("mapping", MAPPINGS)
def test_map_floats(vkt, fmt, mapping):
    for v in special_floats():
        got = vkt.MapVoxel(v, fmt, *mapping)
        ref = ob.map_voxel(v, fmt, *mapping)
        if fmt in (1, 3):   # Int8/Int32: the reference writes nothing
            continue
        assert got == ref, (fmt, mapping, v, got.hex(), ref.hex())


def test_map_unmap_roundtrip_u16_all_codes(vkt):
    for c in range(65536):
        b = c.to_bytes(2, "little")
        assert vkt.MapVoxel(vkt.UnmapVoxel(b, 5), 5) == b


def test_uint32_unmap_samples(vkt):
    rng = np.random.default_rng(1)
    for c in list(rng.integers(0, 2**32, 2000, dtype=np.uint64)) + [0, 1, 2**31, 2**32 - 1, 2**24 + 1]:
        b = int(c).to_bytes(4, "little")
        for m in MAPPINGS[:3]:
            assert same_float(vkt.UnmapVoxel(b, 6, *m), ob.unmap_voxel(b, 6, *m))


def test_float32_unmap_is_raw_bits(vkt):
    for bits in (0x7FC00001, 0xFF800000, 0x00000001, 0x80000000, 0x3F800000):
        b = bits.to_bytes(4, "little")
        got = vkt.UnmapVoxel(b, 7, -1.0, 3.0)
        assert struct.pack("<f", got) == b or np.isnan(got)


def test_uint8_unmap_division_equals_reciprocal_product():
    """Codec.hpp decodes UInt8 with code * 0x3B800021 instead of the reference's IEEE division
    code / 255.999f (VoxelMapping.hpp:122-127): equal for every one of the 256 codes."""
    codes = np.arange(256, dtype=np.float32)
    inv = np.float32(1.0) / np.float32(255.999)
    assert struct.unpack("<I", struct.pack("<f", inv))[0] == 0x3B800021
    np.testing.assert_array_equal((codes / np.float32(255.999)).view(np.uint32), (codes * inv).view(np.uint32))
