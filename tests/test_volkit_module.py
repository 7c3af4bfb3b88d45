"""``import volkit as vkt`` (the reference's module name, src/vkt/volkit.i:11) and the
VKT_DEFAULT_DEVICE=GPU switch that lets unmodified reference scripts -- which never set an
execution policy -- run on this GPU backend.  The GPU case follows the call sequences of the
reference's Python examples (src/examples/Arithmetic.py:5-18, Aggregates.py:28-75), written
here for the test, in a subprocess (the switch is read when libvolkit.so loads)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# names the reference's Python examples use (src/examples/*.py)
EXAMPLE_NAMES = ["Vec3i", "StructuredVolume", "DataFormat_UInt8", "DataFormat_Unspecified", "RenderState",
                 "RenderAlgo_MultiScattering", "Render", "ExecutionPolicy", "GetThreadExecutionPolicy",
                 "SetThreadExecutionPolicy", "RawFile", "InputStream", "Aggregates", "ComputeAggregates",
                 "ComputeAggregatesRange", "Array3D_StructuredVolume", "BrickDecompose", "BrickDecomposeResize",
                 "LookupTable", "ColorFormat_RGBA32F", "Fill", "CopyRange", "SafeSum", "Resample"]


def _run(code, env_extra):
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, cwd="/tmp",
                          env=env)


def test_import_volkit_exposes_the_swig_names():
    r = _run("import volkit as vkt; print(' '.join(n for n in %r if not hasattr(vkt, n)))" % EXAMPLE_NAMES, {})
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "", f"missing: {r.stdout}"


@pytest.mark.parametrize("value,expect", [("GPU", "GPU"), ("", "CPU"), ("CPU", "CPU")])
def test_default_device_switch(value, expect):
    code = ("import volkit as vkt; ep = vkt.GetThreadExecutionPolicy(); "
            "print('GPU' if ep.device == vkt.ExecutionPolicy.Device_GPU else 'CPU')")
    r = _run(code, {"VKT_DEFAULT_DEVICE": value})
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == expect


@pytest.mark.gpu
def test_reference_example_sequences_run_unmodified_on_gpu(tmp_path):
    raw = tmp_path / "vol_32x32x32_uint8.raw"
    code = f"""
import numpy as np
import volkit as vkt

# Arithmetic.py's sequence: a 32^3 UInt8 volume, a render state, MultiScattering, Render
dims = vkt.Vec3i()
dims.x = 32
dims.y = 32
dims.z = 32
dataFormat = vkt.DataFormat_UInt8
volume1 = vkt.StructuredVolume(dims.x, dims.y, dims.z, dataFormat)
renderState = vkt.RenderState()
renderState.renderAlgo = vkt.RenderAlgo_MultiScattering
assert vkt.Render(volume1, renderState) == vkt.NoError, vkt.last_error()

# Aggregates.py's sequence: RawFile -> InputStream.read -> ComputeAggregates(+Range)
np.arange(32 ** 3, dtype=np.uint32).astype(np.uint8).tofile({str(raw)!r})
file = vkt.RawFile({str(raw)!r}, "r")
d = file.getDims()
volume = vkt.StructuredVolume(d.x, d.y, d.z, file.getDataFormat())
ips = vkt.InputStream(file)
ips.read(volume)
aggr = vkt.Aggregates()
assert vkt.ComputeAggregates(volume, aggr) == vkt.NoError, vkt.last_error()
print(aggr.min, aggr.max, aggr.argmax.x, aggr.argmax.y, aggr.argmax.z)
assert vkt.ComputeAggregatesRange(volume, aggr, 2, 2, 2, 10, 10, 10) == vkt.NoError
print("ok")
"""
    r = _run(code, {"VKT_DEFAULT_DEVICE": "GPU", "VKT_RENDER_FRAMES": "2"})
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.strip().splitlines()
    assert lines[-1] == "ok"
    mn, mx, ax, ay, az = lines[-2].split()
    assert float(mn) == 0.0 and abs(float(mx) - 255 / 255.999) < 1e-6 and (int(ax), int(ay), int(az)) == (31, 7, 0)
