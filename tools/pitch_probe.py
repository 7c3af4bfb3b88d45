"""Strided-row streaming rate vs row pitch: SafeSumRange over 800 x 800 x 800 boxes whose
rows are 1600 B, in volumes of different x pitch (power of two or not).  One process, same
kernel; prints one JSON line per case."""
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
for dx in (1024, 1000, 1040, 1088, 1152, 2048):
    A, B, D = alloc((dx, 900, 820), 5, seed=1), alloc((dx, 900, 820), 5, seed=2), alloc((dx, 900, 820), 5)
    f0, f1 = Vec3i_t(0, 100, 20), Vec3i_t(800, 900, 820)
    ms = timed(lambda: lib.vktHipArithmeticRange(5, D, A, B, f0, f1, o), 20)
    nv = 800 ** 3
    print(json.dumps({"pitch_bytes": 2 * dx, "row_bytes": 1600, "ms": round(ms, 4),
                      "GB/s": round(6 * nv / ms / 1e6, 1)}), flush=True)
    free(A, B, D)
