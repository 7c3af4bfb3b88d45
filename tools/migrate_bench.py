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


if __name__ == "__main__":
    torch.cuda.set_device(0)
    run(False)
    run(True)
