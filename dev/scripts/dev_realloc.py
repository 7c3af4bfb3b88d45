"""Dev probe: SumRange 1024^3 UInt16 time across re-allocations within one process."""
import ctypes as C, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from volkit_amd._lib import lib, HipVolumeView_t, Vec3i_t

torch.cuda.set_device(0)
stream = torch.cuda.Stream(); torch.cuda.set_stream(stream)
lib.vktHipSetComputeStream(C.c_void_p(stream.cuda_stream))
n = 1024; nb = 2 * n ** 3
o, last = Vec3i_t(0, 0, 0), Vec3i_t(n, n, n)
keep = []
for it in range(6):
    ptrs = []
    for k in range(3):
        p = C.c_void_p(); assert lib.vktHipAllocate(C.byref(p), nb) == 0; ptrs.append(p.value)
    A, B, D = (HipVolumeView_t(p, n, n, n, 5, 0.0, 1.0) for p in ptrs)
    lib.vktHipSynthesize(A, C.c_uint64(1)); lib.vktHipSynthesize(B, C.c_uint64(2))
    for _ in range(20): lib.vktHipArithmeticRange(0, D, A, B, o, last, o)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); a.record()
    for _ in range(30): lib.vktHipArithmeticRange(0, D, A, B, o, last, o)
    b.record(); b.synchronize()
    print(it, [hex(p) for p in ptrs], round(a.elapsed_time(b) / 30, 4), flush=True)
    if it % 2 == 0:
        keep.append(ptrs)            # hold some allocations so the next ones land elsewhere
    else:
        for p in ptrs: lib.vktHipFree(C.c_void_p(p))
