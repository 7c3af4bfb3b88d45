"""Dev probe: host-side (enqueue) time of BrickDecompose vs. the synchronised time."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import volkit_amd.volkit as vkt

ep = vkt.GetThreadExecutionPolicy(); ep.device = vkt.ExecutionPolicy.Device_GPU; vkt.SetThreadExecutionPolicy(ep)
n = 1024
for bs in (32, 64):
    V = vkt.StructuredVolume(n, n, n, vkt.DataFormat_UInt16)
    vkt.Synthesize(V, 77)
    arr = vkt.Array3D_StructuredVolume()
    b3, h3 = vkt.Vec3i(bs, bs, bs), vkt.Vec3i(1, 1, 1)
    vkt.BrickDecomposeResize(arr, V, b3, h3, h3)
    vkt.BrickDecompose(arr, V, b3, h3, h3); torch.cuda.synchronize()
    t0 = time.perf_counter(); vkt.BrickDecompose(arr, V, b3, h3, h3); t1 = time.perf_counter()
    torch.cuda.synchronize(); t2 = time.perf_counter()
    t3 = time.perf_counter()
    for _ in range(10):
        vkt.BrickDecompose(arr, V, b3, h3, h3)
    t4 = time.perf_counter(); torch.cuda.synchronize(); t5 = time.perf_counter()
    print(f"{bs}^3: enqueue {1e3*(t1-t0):.3f} ms, sync total {1e3*(t2-t0):.3f} ms; 10 back-to-back: enqueue {1e2*(t4-t3):.3f} ms/call, total {1e2*(t5-t3):.3f} ms/call", flush=True)
    del arr, V
