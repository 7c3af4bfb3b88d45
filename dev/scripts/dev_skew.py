"""Dev probe: SumRange 1024^3 UInt16 time vs relative offset (skew) of the three streams."""
import ctypes as C, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from volkit_amd import _lib
from volkit_amd._lib import lib, HipVolumeView_t, Vec3i_t

torch.cuda.set_device(0)
stream = torch.cuda.Stream(); torch.cuda.set_stream(stream)
lib.vktHipSetComputeStream(C.c_void_p(stream.cuda_stream))
n = 1024; nb = 2 * n ** 3; pad = 64 << 20
bufs = []
for k in range(3):
    p = C.c_void_p(); assert lib.vktHipAllocate(C.byref(p), nb + pad) == 0; bufs.append(p.value)
o, last = Vec3i_t(0, 0, 0), Vec3i_t(n, n, n)

def view(base, off):
    return HipVolumeView_t(base + off, n, n, n, 5, 0.0, 1.0)

for k in range(2):
    lib.vktHipSynthesize(view(bufs[k], 0), C.c_uint64(k + 1))
    lib.vktHipSynthesize(view(bufs[k], pad), C.c_uint64(k + 1))

def t(offs, reps=20):
    A, B, D = (view(bufs[i], offs[i]) for i in range(3))
    for _ in range(10): lib.vktHipArithmeticRange(0, D, A, B, o, last, o)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); a.record()
    for _ in range(reps): lib.vktHipArithmeticRange(0, D, A, B, o, last, o)
    b.record(); b.synchronize()
    return a.elapsed_time(b) / reps

print("ptrs", [hex(b) for b in bufs])
for rnd in range(2):
    for offs in ((0, 0, 0), (0, 4096, 8192), (0, 65536, 131072), (0, 1 << 20, 2 << 20), (0, 3 << 20, 7 << 20),
                 (0, 8 << 20, 16 << 20), (0, 1 << 25, 1 << 24), (0, 12288, 40960)):
        print(rnd, offs, round(t(offs), 4), flush=True)
