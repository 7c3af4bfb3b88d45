"""Dev probe: SumRange 2048^3 UInt16 over three volumes re-allocated through
the library K times in ONE process (the arena carves the three 16-GiB volumes from one chunk
each time), printing one JSON line per allocation with the event time of its timed launches.
Run it under `rocprofv3 --pmc <counters>` (one process per pass): every allocation's launches
get the pass's counters, and scripts/pmc_dispatch.py joins them with the line of the same
allocation -- the fast (~7.9 ms) and slow (~8.4 ms) placement states side by side.

  PROBE_ITERS=6 PROBE_EDGE=2048 python tools/placement_pmc.py
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from volkit_amd._lib import lib, last_error, HipVolumeView_t, Vec3i_t  # noqa: E402

torch.cuda.set_device(0)
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
lib.vktHipSetComputeStream(C.c_void_p(stream.cuda_stream))
n = int(os.environ.get("PROBE_EDGE", "2048"))
nb = 2 * n ** 3
o, last = Vec3i_t(0, 0, 0), Vec3i_t(n, n, n)
WARM, TIMED = 1, 3          # SumRange launches per allocation: pmc_dispatch.py <log> 4
for it in range(int(os.environ.get("PROBE_ITERS", "6"))):
    ptrs = []
    for _ in range(3):
        p = C.c_void_p()
        assert lib.vktHipAllocate(C.byref(p), nb) == 0, last_error()
        ptrs.append(p.value)
    A, B, D = (HipVolumeView_t(p, n, n, n, 5, 0.0, 1.0) for p in ptrs)
    lib.vktHipSynthesize(A, C.c_uint64(1))
    lib.vktHipSynthesize(B, C.c_uint64(2))
    for _ in range(WARM):
        assert lib.vktHipArithmeticRange(0, D, A, B, o, last, o) == 0, last_error()
    ts = []
    for _ in range(TIMED):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        assert lib.vktHipArithmeticRange(0, D, A, B, o, last, o) == 0, last_error()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    print(json.dumps({"case": f"alloc {it} base {min(ptrs):#x}", "ms": round(ts[len(ts) // 2], 4),
                      "offsets_mib": [(p - min(ptrs)) >> 20 for p in ptrs]}), flush=True)
    torch.cuda.synchronize()
    for p in ptrs:
        assert lib.vktHipFree(C.c_void_p(p)) == 0, last_error()
