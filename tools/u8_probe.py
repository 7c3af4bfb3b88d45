"""UInt8 / Float32 multi-row copies under the pointwise knobs (one process, same buffers)."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch  # noqa: E402,F401
from volkit_amd._lib import lib, Vec3i_t  # noqa: E402
sys.path.insert(0, os.path.dirname(__file__))
from bench_configs import alloc, free, timed  # noqa: E402

o = Vec3i_t(0, 0, 0)
e = 1024
for fmt, bpv in ((4, 1), (7, 4)):
    A, D = alloc((e,) * 3, fmt, seed=1), alloc((e,) * 3, fmt)
    for lab, f0, f1 in (("x 0..800", Vec3i_t(0, 100, 100), Vec3i_t(800, 900, 900)),
                        ("x 0..768", Vec3i_t(0, 100, 100), Vec3i_t(768, 900, 900)),
                        ("x 0..1024 (planes)", Vec3i_t(0, 100, 100), Vec3i_t(1024, 900, 900))):
        for knobs in ({}, {"pointwise.merge_sectors": 0}, {"pointwise.padded_rows": 0},
                      {"pointwise.merge_sectors": 0, "pointwise.padded_rows": 0}, {"pointwise.general": 0}):
            for k, v in knobs.items():
                lib.vktHipSetTuningKnob(k.encode(), v)
            ms = timed(lambda: lib.vktHipCopyRange(D, A, f0, f1, o), 20)
            for k in knobs:
                lib.vktHipSetTuningKnob(k.encode(), -1)
            nv = (f1.x - f0.x) * (f1.y - f0.y) * (f1.z - f0.z)
            print(json.dumps({"fmt": fmt, "box": lab, "knobs": knobs, "ms": round(ms, 4),
                              "GB/s": round(2 * bpv * nv / ms / 1e6, 1)}), flush=True)
    free(A, D)
