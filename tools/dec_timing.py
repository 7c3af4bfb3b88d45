import sys, time, os
sys.path.insert(0, '/root/repo')
import torch
import volkit_amd.volkit as vkt
ep = vkt.GetThreadExecutionPolicy(); ep.device = vkt.ExecutionPolicy.Device_GPU; vkt.SetThreadExecutionPolicy(ep)
n = 1024
V = vkt.StructuredVolume(n, n, n, vkt.DataFormat_UInt16)
vkt.Synthesize(V, 77)
arr = vkt.Array3D_StructuredVolume()
b3, h3 = vkt.Vec3i(16, 16, 16), vkt.Vec3i(1, 1, 1)
vkt.BrickDecomposeResize(arr, V, b3, h3, h3)
for i in range(6):
    torch.cuda.synchronize()
    t = time.perf_counter()
    vkt.BrickDecompose(arr, V, b3, h3, h3)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"call {1e3*(t1-t):.3f} ms, +sync {1e3*(t2-t):.3f} ms", file=sys.stderr, flush=True)
