"""Dev probe (DESIGN.md §6, round-4 VMM fault): the HIP runtime alone -- no libvolkit loaded --
on memory mapped with the VMM API (hipMemAddressReserve / hipMemCreate / hipMemMap).  Each step
prints before it runs, so a crash names its step.

  python tools/vmm_probe.py reuse   # hipMalloc + hipFree a block, then map at that VA
  python tools/vmm_probe.py fresh   # map at a VA the runtime picks (no prior allocation)
  python tools/vmm_probe.py fresh torch   # the same under PyTorch's bundled HIP runtime
  python tools/vmm_probe.py lib torch     # libvolkit arena chunk released, mapping at its VA,
                                          # library kernels + vktHipMemcpy on the mapping
"""
import ctypes as C
import faulthandler
import sys

import numpy as np

faulthandler.enable()
mode = sys.argv[1] if len(sys.argv) > 1 else "fresh"
if "torch" in sys.argv[2:]:
    # PyTorch's wheel bundles its own HIP runtime (torch/lib/libamdhip64.so, torch.version.hip);
    # once torch is imported, "libamdhip64.so" resolves to that copy for every library in the
    # process (libvolkit's libamdhip64.so.7 included) instead of /opt/rocm's
    import torch  # noqa: F401
    mode += f" (torch {torch.version.hip} runtime)"
hip = C.CDLL("libamdhip64.so")
print(mode, "runtime:", sorted({ln.split()[-1] for ln in open("/proc/self/maps") if "amdhip64" in ln}), flush=True)
SIZE = 256 << 20


class Loc(C.Structure):
    _fields_ = [("type", C.c_int), ("id", C.c_int)]


class Flags(C.Structure):
    _fields_ = [("compressionType", C.c_ubyte), ("gpuDirectRDMACapable", C.c_ubyte), ("usage", C.c_ushort)]


class Prop(C.Structure):
    _fields_ = [("type", C.c_int), ("requestedHandleType", C.c_int), ("location", Loc),
                ("win32HandleMetaData", C.c_void_p), ("allocFlags", Flags)]


class Access(C.Structure):
    _fields_ = [("location", Loc), ("flags", C.c_int)]


def step(name, rc):
    print(f"{mode}: {name} -> {rc}", flush=True)
    if rc != 0:
        sys.exit(f"{name} failed: {rc}")


def say(name):
    print(f"{mode}: {name} ...", flush=True)


step("hipSetDevice", hip.hipSetDevice(0))
hint = None
lib = None
N = (256, 256, 512)                                  # UInt16: 64 MiB per volume (lib mode)
NB = 2 * N[0] * N[1] * N[2]
if sys.argv[1:2] == ["lib"]:
    # the round-5 test's sequence through libvolkit: three arena volumes carved from one
    # 256-MiB chunk, Synthesize + SumRange, freed (the chunk goes back to HIP); the mapping below
    # asks for the chunk's VA and the library runs the same kernels and its D2H copy on it
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from volkit_amd._lib import lib, last_error, HipVolumeView_t, Vec3i_t   # noqa: E402
    step("arena_chunk_mib", lib.vktHipSetTuningKnob(b"memory.arena_chunk_mib", 256))

    def lib_sumrange(ptrs, tag):
        A, B, D = (HipVolumeView_t(p, N[0], N[1], N[2], 5, 0.0, 1.0) for p in ptrs)
        o, last = Vec3i_t(0, 0, 0), Vec3i_t(*N)
        step(f"{tag} Synthesize", lib.vktHipSynthesize(A, C.c_uint64(11)) or lib.vktHipSynthesize(B, C.c_uint64(12)))
        step(f"{tag} SumRange", lib.vktHipArithmeticRange(0, D, A, B, o, last, o))
        step(f"{tag} device sync", hip.hipDeviceSynchronize())
        out = np.empty(NB, np.uint8)
        say(f"{tag} vktHipMemcpy D2H 64 MiB from the third volume")
        step(f"{tag} vktHipMemcpy", lib.vktHipMemcpy(out.ctypes.data, C.c_void_p(ptrs[2]), NB, 2))
        return out

    ptrs = []
    for _ in range(3):
        q = C.c_void_p()
        step("vktHipAllocate", lib.vktHipAllocate(C.byref(q), NB))
        ptrs.append(q.value)
    want = lib_sumrange(ptrs, "arena")
    for q in ptrs:
        step("vktHipFree", lib.vktHipFree(C.c_void_p(q)))
    hint = min(ptrs)
elif mode == "reuse":
    p = C.c_void_p()
    step("hipMalloc", hip.hipMalloc(C.byref(p), C.c_size_t(SIZE)))
    step("hipMemset", hip.hipMemset(p, 1, C.c_size_t(SIZE)))
    step("hipDeviceSynchronize", hip.hipDeviceSynchronize())
    step("hipFree", hip.hipFree(p))
    hint = p.value
prop = Prop(1, 0, Loc(1, 0), None, Flags(0, 0, 0))
gran = C.c_size_t(0)
step("hipMemGetAllocationGranularity", hip.hipMemGetAllocationGranularity(C.byref(gran), C.byref(prop), 0))
va = C.c_void_p()
step("hipMemAddressReserve", hip.hipMemAddressReserve(C.byref(va), C.c_size_t(SIZE), C.c_size_t(gran.value),
                                                      C.c_void_p(hint), C.c_ulonglong(0)))
print(f"{mode}: VA {va.value:#x} (hint {hint and hex(hint)}, reused: {va.value == hint})", flush=True)
h = C.c_void_p()
step("hipMemCreate", hip.hipMemCreate(C.byref(h), C.c_size_t(SIZE), C.byref(prop), C.c_ulonglong(0)))
step("hipMemMap", hip.hipMemMap(va, C.c_size_t(SIZE), C.c_size_t(0), h, C.c_ulonglong(0)))
acc = Access(Loc(1, 0), 3)
step("hipMemSetAccess", hip.hipMemSetAccess(va, C.c_size_t(SIZE), C.byref(acc), C.c_size_t(1)))
step("hipMemset(vmm)", hip.hipMemset(va, 7, C.c_size_t(SIZE)))
step("hipDeviceSynchronize", hip.hipDeviceSynchronize())
if lib is not None:
    got = lib_sumrange([va.value, va.value + NB, va.value + 2 * NB], "mapping")
    print(f"{mode}: SumRange on the mapping equals the arena run: {np.array_equal(got, want)}", flush=True)
s = C.c_void_p()
step("hipStreamCreate", hip.hipStreamCreate(C.byref(s)))
# D2H copies into pageable memory: 1 MiB / 64 MiB, from the mapping's first byte and from an
# offset inside it (the round-5 test crashed in a 64-MiB copy from offset 128 MiB)
for mib, off_mib in ((1, 0), (64, 0), (1, 128), (64, 128)):
    host = np.zeros(mib << 20, np.uint8)
    src = C.c_void_p(va.value + (off_mib << 20))
    say(f"hipMemcpy D2H {mib} MiB from offset {off_mib} MiB (pageable)")
    step(f"hipMemcpy D2H {mib}@{off_mib}", hip.hipMemcpy(C.c_void_p(host.ctypes.data), src, C.c_size_t(host.nbytes), 2))
    say(f"hipMemcpyAsync D2H {mib} MiB from offset {off_mib} MiB on a created stream")
    step(f"hipMemcpyAsync D2H {mib}@{off_mib}", hip.hipMemcpyAsync(C.c_void_p(host.ctypes.data), src,
                                                                  C.c_size_t(host.nbytes), 2, s))
    step("hipStreamSynchronize", hip.hipStreamSynchronize(s))
    print(f"{mode}: bytes {np.unique(host)}", flush=True)
say("hipMemsetAsync 64 MiB at offset 128 MiB")
step("hipMemsetAsync interior", hip.hipMemsetAsync(C.c_void_p(va.value + (128 << 20)), 9, C.c_size_t(64 << 20), s))
step("hipStreamSynchronize", hip.hipStreamSynchronize(s))
step("hipMemUnmap", hip.hipMemUnmap(va, C.c_size_t(SIZE)))
step("hipMemRelease", hip.hipMemRelease(h))
step("hipMemAddressFree", hip.hipMemAddressFree(va, C.c_size_t(SIZE)))
step("hipDeviceSynchronize", hip.hipDeviceSynchronize())
print(f"{mode}: done", flush=True)
