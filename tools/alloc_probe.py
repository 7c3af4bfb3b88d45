"""Dev probe: SumRange 1024^3 UInt16 event time per allocation mode, across re-allocations
(the launch alternates between two placement states).  Modes: the library's
hipMalloc per volume, hipExtMallocWithFlags(hipDeviceMallocContiguous) per volume, one
hipMalloc block carved into the three volumes."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from volkit_amd._lib import lib, HipVolumeView_t, Vec3i_t  # noqa: E402

hip = C.CDLL("libamdhip64.so")
hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
hip.hipFree.argtypes = [C.c_void_p]

torch.cuda.set_device(0)
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
lib.vktHipSetComputeStream(C.c_void_p(stream.cuda_stream))
n = int(os.environ.get("PROBE_EDGE", "1024"))   # 2048: the config-4 volumes (16 GiB each)
nb = 2 * n ** 3
o, last = Vec3i_t(0, 0, 0), Vec3i_t(n, n, n)


def alloc(mode):
    if mode in ("library", "library0"):   # vktHipAllocate (arena on / off: knob memory.arena)
        lib.vktHipSetTuningKnob(b"memory.arena", 1 if mode == "library" else 0)
        ptrs = []
        for _ in range(3):
            p = C.c_void_p()
            assert lib.vktHipAllocate(C.byref(p), nb) == 0
            ptrs.append(p.value)
        return ptrs, [("lib", q) for q in ptrs]
    if mode == "block":
        p = C.c_void_p()
        assert hip.hipMalloc(C.byref(p), 3 * nb + 4096) == 0
        return [p.value, p.value + nb, p.value + 2 * nb], [p.value]
    ptrs = []
    for _ in range(3):
        p = C.c_void_p()
        if mode == "contig":
            err = hip.hipExtMallocWithFlags(C.byref(p), nb, 0x4)
        else:
            err = hip.hipMalloc(C.byref(p), nb)
        assert err == 0, (mode, err)
        ptrs.append(p.value)
    return ptrs, ptrs


res = {}
for it in range(int(os.environ.get("PROBE_ITERS", "5"))):
    for mode in os.environ.get("PROBE_MODES", "default,contig,block").split(","):
        ptrs, frees = alloc(mode)
        A, B, D = (HipVolumeView_t(p, n, n, n, 5, 0.0, 1.0) for p in ptrs)
        lib.vktHipSynthesize(A, C.c_uint64(1))
        lib.vktHipSynthesize(B, C.c_uint64(2))
        for _ in range(10):
            lib.vktHipArithmeticRange(0, D, A, B, o, last, o)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for _ in range(30):
            lib.vktHipArithmeticRange(0, D, A, B, o, last, o)
        b.record()
        b.synchronize()
        ms = a.elapsed_time(b) / 30
        res.setdefault(mode, []).append(round(ms, 4))
        print(it, mode, round(ms, 4), flush=True)
        torch.cuda.synchronize()
        for p in frees:
            if isinstance(p, tuple):
                lib.vktHipFree(C.c_void_p(p[1]))
            else:
                hip.hipFree(C.c_void_p(p))
print({k: sorted(v) for k, v in res.items()})
for k, v in res.items():
    print(k, "spread", round((max(v) - min(v)) / min(v) * 100, 2), "%", flush=True)
