"""Dev probe: public-API calls under rocprofv3 --marker-trace show one roctx range per call."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import volkit_amd.volkit as vkt

ep = vkt.GetThreadExecutionPolicy(); ep.device = vkt.ExecutionPolicy.Device_GPU; vkt.SetThreadExecutionPolicy(ep)
S = vkt.StructuredVolume(256, 256, 256, vkt.DataFormat_UInt16)
R = vkt.StructuredVolume(512, 512, 512, vkt.DataFormat_UInt16)
B = vkt.StructuredVolume(512, 512, 512, vkt.DataFormat_UInt16)
D = vkt.StructuredVolume(512, 512, 512, vkt.DataFormat_UInt16)
assert vkt.Fill(S, 0.25) == 0 and vkt.Fill(B, 0.5) == 0
assert vkt.Resample(R, S, vkt.FilterMode_Linear) == 0
assert vkt.SumRange(D, R, B, 0, 0, 0, 512, 512, 512) == 0
ep.device = vkt.ExecutionPolicy.Device_CPU; vkt.SetThreadExecutionPolicy(ep)
print("value", D.getValue(3, 4, 5))
