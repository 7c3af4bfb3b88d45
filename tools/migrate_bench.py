"""Host <-> HBM migration throughput of ManagedBuffer::migrate (deferred policy switch),
pageable (reference behaviour) vs pinned host allocations.  Development/reporting tool."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import volkit_amd.volkit as vkt  # noqa: E402
from volkit_amd._lib import lib  # noqa: E402


def policy(dev):
    ep = vkt.GetThreadExecutionPolicy()
    ep.device = dev
    vkt.SetThreadExecutionPolicy(ep)


def run(pinned, edge=1024):
    lib.vktHipSetPinnedHostAllocation(1 if pinned else 0)
    policy(vkt.ExecutionPolicy.Device_CPU)
    v = vkt.StructuredVolume(edge, edge, edge, vkt.DataFormat_UInt16)
    v.from_numpy(np.ones((edge, edge, edge), np.uint16))
    nbytes = v.getSizeInBytes()
    out = {}
    for rep in range(2):
        policy(vkt.ExecutionPolicy.Device_GPU)
        t0 = time.perf_counter()
        v.migrate()
        lib.vktHipSynchronize()
        h2d = time.perf_counter() - t0
        policy(vkt.ExecutionPolicy.Device_CPU)
        t0 = time.perf_counter()
        v.migrate()
        d2h = time.perf_counter() - t0
        out = {"pinned": pinned, "bytes": nbytes, "H2D_GBs": round(nbytes / h2d / 1e9, 2),
               "D2H_GBs": round(nbytes / d2h / 1e9, 2)}
    print(json.dumps(out), flush=True)


def breakdown(nbytes=2 << 30, reps=3):
    """Where a migrate's time goes: the copies alone between preallocated buffers (pageable
    numpy memory written beforehand, an untouched pageable buffer whose pages the copy faults in,
    pinned memory) and the allocations a migrate makes on the new side and frees on the old one."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    hip.hipHostFree.argtypes = [C.c_void_p]
    out = {"bytes": nbytes}

    def best(fn):
        ts = []
        for _ in range(reps):
            lib.vktHipSynchronize()
            t0 = time.perf_counter()
            fn()
            lib.vktHipSynchronize()
            ts.append(time.perf_counter() - t0)
        return min(ts)

    d = C.c_void_p()
    t0 = time.perf_counter()
    assert lib.vktHipAllocate(C.byref(d), nbytes) == 0
    out["device_alloc_ms_first"] = round((time.perf_counter() - t0) * 1e3, 2)
    host = np.ones(nbytes, np.uint8)          # pageable, pages written
    ph = C.c_void_p()
    t0 = time.perf_counter()
    assert hip.hipHostMalloc(C.byref(ph), nbytes, 0) == 0
    out["pinned_alloc_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    C.memset(ph, 1, nbytes)
    for name, ptr in (("pageable", host.ctypes.data), ("pinned", ph.value)):
        h2d = best(lambda: lib.vktHipMemcpy(d, C.c_void_p(ptr), nbytes, 1))
        d2h = best(lambda: lib.vktHipMemcpy(C.c_void_p(ptr), d, nbytes, 2))
        out[f"copy_{name}"] = {"H2D_GBs": round(nbytes / h2d / 1e9, 2), "D2H_GBs": round(nbytes / d2h / 1e9, 2)}

    def fresh_d2h():
        f = np.empty(nbytes, np.uint8)        # untouched pages: the copy faults them in
        lib.vktHipMemcpy(C.c_void_p(f.ctypes.data), d, nbytes, 2)
        return f
    t = best(fresh_d2h)
    out["copy_pageable_D2H_into_fresh_GBs"] = round(nbytes / t / 1e9, 2)
    t0 = time.perf_counter()
    hip.hipHostFree(ph)
    out["pinned_free_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    lib.vktHipFree(d)
    t0 = time.perf_counter()
    assert lib.vktHipAllocate(C.byref(d), nbytes) == 0
    lib.vktHipSynchronize()
    out["device_alloc_ms_again"] = round((time.perf_counter() - t0) * 1e3, 2)
    lib.vktHipFree(d)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    torch.cuda.set_device(0)
    run(False)
    run(True)
    breakdown()
