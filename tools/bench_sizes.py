"""Size sweep of the metric pipeline on one GPU (development/report tool, not the driver's bench).

BASELINE.json's north star asks for Gvoxels/s "on synthetic 256^3-2048^3 grids" as absolute
numbers and as a fraction of the HBM roofline.  For each dst edge E in {256, 512, 1024, 2048}:
    Resample(R, S, Linear)   S = (E/2)^3 UInt16 -> R = E^3 UInt16
    SumRange(D, R, B)        E^3 UInt16
on device-resident synthetic codes, timed with HIP events on the backend's compute stream
(warm-up, then the mean of `reps` steps).  One JSON line per size:
    pipeline Gvox/s = E^3 / step time; algorithmic bytes = 2(E/2)^3 + 2E^3 + 6E^3.
    python tools/bench_sizes.py [--sizes 256,512,1024,2048]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from volkit_amd._lib import lib, HipVolumeView_t, Vec3i_t  # noqa: E402
from volkit_amd import _lib  # noqa: E402

HBM_PEAK_GBS = 8000.0


def alloc(e, seed=None):
    p = C.c_void_p()
    if lib.vktHipAllocate(C.byref(p), 2 * e ** 3) != 0:
        raise RuntimeError(_lib.last_error())
    v = HipVolumeView_t(p.value, e, e, e, 5, 0.0, 1.0)
    if seed is not None:
        lib.vktHipSynthesize(v, C.c_uint64(seed))
    return v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="256,512,1024,2048")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    lib.vktHipSetComputeStream(C.c_void_p(stream.cuda_stream))
    o = Vec3i_t(0, 0, 0)
    for e in (int(x) for x in args.sizes.split(",")):
        s = e // 2
        S, B, R, D = alloc(s, 0x5EED), alloc(e, 0x5EEE), alloc(e), alloc(e)
        last = Vec3i_t(e, e, e)

        def step():
            if lib.vktHipResample(R, S, 1) or lib.vktHipArithmeticRange(0, D, R, B, o, last, o):
                raise RuntimeError(_lib.last_error())

        reps = max(10, min(2000, int(2e10 // (8 * e ** 3))))   # ~ >= 20 ms of work per size
        for _ in range(max(5, reps // 4)):
            step()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            step()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        nbytes = 2 * s ** 3 + 2 * e ** 3 + 6 * e ** 3
        gbs = nbytes / (ms / 1e3) / 1e9
        print(json.dumps({"case": f"Resample {s}^3->{e}^3 + SumRange {e}^3 UInt16", "dst_voxels": e ** 3,
                          "ms_per_step": round(ms, 4), "Gvox/s": round(e ** 3 / (ms / 1e3) / 1e9, 1),
                          "GB/s": round(gbs, 1), "frac_of_8TBs": round(gbs / HBM_PEAK_GBS, 4), "reps": reps}),
              flush=True)
        for v in (S, B, R, D):
            lib.vktHipFree(C.c_void_p(v.data))


if __name__ == "__main__":
    main()
