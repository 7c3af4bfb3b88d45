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


class _Loc(C.Structure):
    _fields_ = [("type", C.c_int), ("id", C.c_int)]


class _Flags(C.Structure):
    _fields_ = [("compressionType", C.c_ubyte), ("gpuDirectRDMACapable", C.c_ubyte), ("usage", C.c_ushort)]


class _Prop(C.Structure):
    _fields_ = [("type", C.c_int), ("requestedHandleType", C.c_int), ("location", _Loc),
                ("win32HandleMetaData", C.c_void_p), ("allocFlags", _Flags)]


class _Access(C.Structure):
    _fields_ = [("location", _Loc), ("flags", C.c_int)]


def vmm_alloc(sizes):
    """Virtual-memory-management allocation: one VA reservation for all volumes, one physical
    allocation (hipMemCreate) per entry of `sizes`, mapped back to back (hipMemMap)."""
    prop = _Prop(1, 0, _Loc(1, 0), None, _Flags(0, 0, 0))
    gran = C.c_size_t(0)
    assert hip.hipMemGetAllocationGranularity(C.byref(gran), C.byref(prop), 0) == 0
    g = gran.value
    total = sum((sz + g - 1) // g * g for sz in sizes)
    va = C.c_void_p()
    assert hip.hipMemAddressReserve(C.byref(va), C.c_size_t(total), C.c_size_t(max(g, 1 << 30)), None, C.c_ulonglong(0)) == 0
    off, handles, ptrs = 0, [], []
    for sz in sizes:
        sz = (sz + g - 1) // g * g
        h = C.c_void_p()
        assert hip.hipMemCreate(C.byref(h), C.c_size_t(sz), C.byref(prop), C.c_ulonglong(0)) == 0
        assert hip.hipMemMap(C.c_void_p(va.value + off), C.c_size_t(sz), C.c_size_t(0), h, C.c_ulonglong(0)) == 0
        handles.append((h, va.value + off, sz))
        ptrs.append(va.value + off)
        off += sz
    acc = _Access(_Loc(1, 0), 3)
    assert hip.hipMemSetAccess(va, C.c_size_t(total), C.byref(acc), C.c_size_t(1)) == 0
    return ptrs, [("vmm", va.value, total, handles)]


def vmm_free(rec):
    _, va, total, handles = rec
    for h, p, sz in handles:
        hip.hipMemUnmap(C.c_void_p(p), C.c_size_t(sz))
        hip.hipMemRelease(h)
    hip.hipMemAddressFree(C.c_void_p(va), C.c_size_t(total))


def alloc(mode):
    if mode == "vmm":      # one physical allocation for the three volumes
        ptrs, rec = vmm_alloc([3 * nb])
        return [ptrs[0], ptrs[0] + nb, ptrs[0] + 2 * nb], rec
    if mode == "vmm3":     # one physical allocation per volume, one VA range
        return vmm_alloc([nb, nb, nb])
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
            if isinstance(p, tuple) and p[0] == "vmm":
                vmm_free(p)
            elif isinstance(p, tuple):
                lib.vktHipFree(C.c_void_p(p[1]))
            else:
                hip.hipFree(C.c_void_p(p))
print({k: sorted(v) for k, v in res.items()})
for k, v in res.items():
    print(k, "spread", round((max(v) - min(v)) / min(v) * 100, 2), "%", flush=True)
