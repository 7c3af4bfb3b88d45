"""Per-call fixed cost of ComputeAggregates / ComputeHistogram (tiny 64^3 box of a 1024^3 volume):
host wall time per call, for reading beside a rocprofv3 kernel trace of the same run
(kernels per call, their durations and the gaps between them).

    python3 tools/agg_fixed.py [calls]
"""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from volkit_amd import _lib  # noqa: E402
from volkit_amd._lib import HipVolumeView_t, Vec3i_t, lib  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    n = 1024
    torch.cuda.init()
    agg = _lib.Aggregates_t()
    bins = C.c_void_p()
    assert lib.vktHipAllocate(C.byref(bins), 65536 * 8) == 0
    for fmt, bpv in ((4, 1), (5, 2)):
        p = C.c_void_p()
        assert lib.vktHipAllocate(C.byref(p), n ** 3 * bpv) == 0
        v = HipVolumeView_t(p.value, n, n, n, fmt, 0.0, 1.0)
        lib.vktHipSynthesize(v, C.c_uint64(7))
        for what, a0, a1 in (("64^3 box", Vec3i_t(3, 0, 0), Vec3i_t(67, 64, 64)),
                             ("1024^3", Vec3i_t(0, 0, 0), Vec3i_t(n, n, n))):
            for op in ("aggregates", "histogram256"):
                fn = (lambda: lib.vktHipAggregatesRange(v, a0, a1, C.byref(agg))) if op == "aggregates" else \
                     (lambda: lib.vktHipHistogramRange(v, a0, a1, bins, 256, 0))
                for _ in range(5):
                    assert fn() == 0, _lib.last_error()
                torch.cuda.synchronize()
                ts = []
                for _ in range(calls):
                    t0 = time.perf_counter()
                    assert fn() == 0, _lib.last_error()
                    torch.cuda.synchronize()
                    ts.append((time.perf_counter() - t0) * 1e3)
                ts.sort()
                print(json.dumps({"case": f"{op} fmt={fmt} {what}", "calls": calls,
                                  "median_ms": round(ts[len(ts) // 2], 4), "p10_ms": round(ts[len(ts) // 10], 4)}),
                      flush=True)
        lib.vktHipFree(p)
    lib.vktHipFree(bins)


if __name__ == "__main__":
    main()
