"""Writes tests/golden/reference_kat.json: known-answer vectors observed on the COMPILED
REFERENCE serial path during the survey, transcribed as data.

Why transcription instead of regeneration: the reference's hot-path TUs include the CMake-
generated <vkt/config.h> (reference src/vkt/macros.hpp:4) and, for Fill/Resample, the
un-vendored visionaray headers (src/vkt/HierarchicalVolumeView.hpp:10-14).  Building them
here would need stand-ins for generated code and a missing library, which this project does
not write, so the reference is unbuildable in this container.  The survey ran the reference
and recorded these outputs; they are the only reference-produced vectors available.

Each entry names the SURVEY.md line that records it.  Inputs that the survey does not spell
out (e.g. which finite values sat in a source row) are chosen so that the recorded output is
independent of them, and the entry says so.

Run: python tests/golden/make_reference_kat.py
"""
import json
import os

UINT8, UINT16, UINT32, FLOAT32 = 4, 5, 6, 7
NEAREST, LINEAR = 0, 1
INF = "inf"
NAN = "nan"

KATS = [
    {
        "id": "fill_u16_one_wraps_to_zero",
        "source": "SURVEY.md:447-448 (A.1: 65535.999f == 65536.0f, Fill(UInt16,1.0) -> 0 [probe])",
        "op": "map", "fmt": UINT16, "mapping": [0.0, 1.0], "value": 1.0, "expect_code": 0,
    },
    {
        "id": "fill_u32_one_wraps_to_zero",
        "source": "SURVEY.md:450 (A.1: 4294967295.999f == 2^32, 1.0 -> 0 [probe])",
        "op": "map", "fmt": UINT32, "mapping": [0.0, 1.0], "value": 1.0, "expect_code": 0,
    },
    {
        "id": "safesum_u16_saturated_wraps_to_zero",
        "source": "SURVEY.md:31-32, 447-448 (saturated SafeSum wraps to code 0 [probe])",
        "op": "arith", "name": "SafeSum", "fmt": UINT16, "mapping": [0.0, 1.0],
        "dims": [1, 1, 1], "a": [65535], "b": [65535], "first": [0, 0, 0], "last": [1, 1, 1],
        "off": [0, 0, 0], "dst_init": [12345], "expect": [0],
    },
    {
        "id": "sumrange_absolute_destination_index",
        "source": "SURVEY.md:464 (A.2: SumRange(first=2,...,off=0) writes d(2,2,2), not d(0,0,0) [probe])",
        "op": "arith", "name": "Sum", "fmt": UINT8, "mapping": [0.0, 1.0],
        "dims": [3, 3, 3], "a": "iota", "b": "zeros", "first": [2, 2, 2], "last": [3, 3, 3],
        "off": [0, 0, 0], "dst_init": "fill:255",
        "expect_changed_voxels": [[2, 2, 2]],
        "note": "a = iota codes, b = zeros, dst prefilled 255: only d(2,2,2) changes, to a(2,2,2)",
    },
    {
        "id": "codec_roundtrip_all_u8_codes",
        "source": "SURVEY.md:458-459 (A.1: x+0 round-trips for all 256 UInt8 codes [probe])",
        "op": "sum_zero_roundtrip", "fmt": UINT8, "mapping": [0.0, 1.0], "codes": "all",
    },
    {
        "id": "codec_roundtrip_all_u16_codes",
        "source": "SURVEY.md:458-459 (A.1: x+0 round-trips for all 65,536 UInt16 codes [probe])",
        "op": "sum_zero_roundtrip", "fmt": UINT16, "mapping": [0.0, 1.0], "codes": "all",
    },
    {
        "id": "resample_10_to_7",
        "source": "SURVEY.md:484 (A.3: 10->7 gives 0 10 20 40 50 70 80 [probe])",
        "op": "resample", "fmt": UINT8, "mapping": [0.0, 1.0], "filter": NEAREST,
        "src_dims": [10, 1, 1], "dst_dims": [7, 1, 1],
        "src": [0, 10, 20, 30, 40, 50, 60, 70, 80, 90], "expect": [0, 10, 20, 40, 50, 70, 80],
    },
    {
        "id": "resample_4_to_8_duplicates",
        "source": "SURVEY.md:484 (A.3: 4->8 duplicates [probe])",
        "op": "resample", "fmt": UINT8, "mapping": [0.0, 1.0], "filter": NEAREST,
        "src_dims": [4, 1, 1], "dst_dims": [8, 1, 1],
        "src": [3, 7, 11, 13], "expect": [3, 3, 7, 7, 11, 11, 13, 13],
    },
    {
        "id": "resample_float_inf_linear_vs_nearest",
        "source": "SURVEY.md:485-487 (A.3: 4x2x1 source, +Inf at (0,1,0), to 8x4x2: row y=0 = "
                  "NaN NaN 2 2 3 3 NaN NaN (Linear) vs 1 1 2 2 3 3 4 4 (Nearest) [probe])",
        "op": "resample_float_row0", "fmt": FLOAT32, "mapping": [0.0, 1.0],
        "src_dims": [4, 2, 1], "dst_dims": [8, 4, 2],
        "src": [1.0, 2.0, 3.0, 4.0, INF, 6.0, 7.0, 8.0],
        "note": "row y=1 x=1..3 are not recorded by the survey; any finite values give the same row 0",
        "expect_linear_row0": [NAN, NAN, 2.0, 2.0, 3.0, 3.0, NAN, NAN],
        "expect_nearest_row0": [1.0, 1.0, 2.0, 2.0, 3.0, 3.0, 4.0, 4.0],
    },
    {
        "id": "resample_linear_equals_nearest_for_integer_formats",
        "source": "SURVEY.md:482-484 (A.3: byte-identical Linear and Nearest for UInt8/UInt16 on "
                  "10x9x8->7x6x5, 37x23x11->64x40x19, 16^3->32^3, 33x17x9->16x8x4, 5x7x3->13x19x11 [probe])",
        "op": "resample_linear_eq_nearest", "fmts": [UINT8, UINT16], "mapping": [0.0, 1.0],
        "pairs": [[[10, 9, 8], [7, 6, 5]], [[37, 23, 11], [64, 40, 19]], [[16, 16, 16], [32, 32, 32]],
                  [[33, 17, 9], [16, 8, 4]], [[5, 7, 3], [13, 19, 11]]],
    },
    {
        "id": "resample_linear_negative_zero_becomes_positive",
        "source": "SURVEY.md:488 (A.3: -0 becomes +0 (signbit cleared) [probe])",
        "op": "resample_float_signbit", "fmt": FLOAT32, "mapping": [0.0, 1.0],
        "src_dims": [2, 1, 1], "dst_dims": [4, 1, 1], "src": ["-0", 1.0],
        "note": "dst x=0,1 read sx=0 whose neighbours are finite and non-negative: -0 + 0*1 = +0; "
                "dst x=2,3 read the voxel past the buffer end (undefined in the reference) and are not checked",
        "expect_linear_signbits_first2": [0, 0],
    },
]


def main():
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kat.json")
    with open(path, "w") as f:
        json.dump({"generated_by": "tests/golden/make_reference_kat.py", "kats": KATS}, f, indent=1)
    print(f"wrote {path} ({len(KATS)} vectors)")


if __name__ == "__main__":
    main()
