"""BASELINE.json configs 1 and 4 on the HIP path.

* Config 1 -- the exact workload of reference src/examples/CoreAlgorithms.c:57-93 (64^3 UInt8
  Fill 0.1f, then CopyRange (10..34)^3 into a 24^3 volume), plus the example's next steps
  (TransformRangeSV1 diagonal marker over (2..22)^3, CreateCopy), through the public C API with
  the GPU policy, against the oracle's serial restatement.  This library is the GPU backend, so
  the reference's CPU-policy run becomes a GPU-policy run of the same calls.
* Config 4 -- one rank's share of the 8-GPU Z-slab layout (2048^3 UInt16 from 1024^3, then
  SumRange 2048^3): rank r resamples its 2048x2048x256 dst slab from its 1024x1024x128 source
  slab with vktHipResampleSlab and runs SumRange on the slab, as bench.py --layout-gpus 8 does
  for rank 0.  Full-size properties (the exact index table of this ratio is d // 2 and Linear
  == Nearest for integer data, so the slab is the 2x2x2 replication of its source planes; Sum
  with a zero volume is the identity) and oracle parity on sampled planes.
"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import binding as ob
from test_gpu_large import DevVol, v3

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def hip():
    import torch
    assert torch.cuda.is_available()
    from volkit_amd import _lib
    return _lib


@pytest.fixture(scope="module")
def vkt():
    import volkit_amd.volkit as v
    return v


def _gpu_policy(vkt):
    ep = vkt.GetThreadExecutionPolicy()
    ep.device = vkt.ExecutionPolicy.Device_GPU
    vkt.SetThreadExecutionPolicy(ep)


def _cpu_policy(vkt):
    ep = vkt.GetThreadExecutionPolicy()
    ep.device = vkt.ExecutionPolicy.Device_CPU
    vkt.SetThreadExecutionPolicy(ep)


def test_config1_core_algorithms_exact(vkt):
    _gpu_policy(vkt)
    try:
        v1 = vkt.StructuredVolume(64, 64, 64, vkt.DataFormat_UInt8, 1.0, 1.0, 1.0, 0.0, 1.0)
        assert vkt.Fill(v1, 0.1) == 0
        v2 = vkt.StructuredVolume(24, 24, 24, vkt.DataFormat_UInt8, 1.0, 1.0, 1.0, 0.0, 1.0)
        assert vkt.CopyRange(v2, v1, 10, 10, 10, 34, 34, 34, 0, 0, 0) == 0

        def diag(x, y, z, voxel):
            if x == y and y == z:
                voxel.bytes[0] = 0xFF

        assert vkt.TransformRange(v2, 2, 2, 2, 22, 22, 22, diag) == 0
        v3_ = vkt.StructuredVolume.CreateCopy(v2)
        _cpu_policy(vkt)
        got1, got2, got3 = v1.to_numpy(), v2.to_numpy(), v3_.to_numpy()
    finally:
        _cpu_policy(vkt)

    r1 = ob.Volume.zeros((64, 64, 64), 4)
    ob.fill_range(r1, (0, 0, 0), (64, 64, 64), 0.1)
    r2 = ob.Volume.zeros((24, 24, 24), 4)
    ob.copy_range(r2, r1, (10, 10, 10), (34, 34, 34), (0, 0, 0))

    def odiag(x, y, z, b, f, lo, hi):
        if x == y and y == z:
            b[0] = 0xFF

    ob.transform_range1(r2, (2, 2, 2), (22, 22, 22), odiag)
    np.testing.assert_array_equal(got1, r1.codes)
    np.testing.assert_array_equal(got2, r2.codes)
    np.testing.assert_array_equal(got3, r2.codes)
    # 0.1f encodes to code 25 (0.1 * 255.999 = 25.6 -> 25); the copy of (10..34)^3 clamps at 63
    assert got1.min() == got1.max() == 25
    assert got2[0, 0, 0] == 25 and got2[5, 5, 5] == 0xFF


@pytest.mark.parametrize("rank", [0, 7])
def test_config4_rank_slab_full_size(hip, rank):
    from volkit_amd import slab
    world, e, s = 8, 2048, 1024
    plan = slab.plan_resample(e, s, world, rank, 1, chain=False)
    ls0, ls1 = plan.local_src
    dz0, dz1 = plan.dst
    assert (dz1 - dz0, ls1 - ls0) == (256, 128) and not plan.recvs and not plan.sends
    S = DevVol(hip, (s, s, ls1 - ls0), 5)
    R, B, D = (DevVol(hip, (e, e, dz1 - dz0), 5) for _ in range(3))
    try:
        S.synth(0x5EED + 1000 * rank)
        B.synth(0x5EED + 1 + 1000 * rank)
        assert hip.lib.vktHipResampleSlab(R.view, S.view, 1, e, dz0, s, ls0) == 0, hip.last_error()
        src, r = S.download(), R.download()
        for dz in (0, 1):
            for dy in (0, 1):
                for dx in (0, 1):
                    np.testing.assert_array_equal(r[dz::2, dy::2, dx::2], src, err_msg=f"rank {rank} {dz}{dy}{dx}")
        # oracle parity of the slab resample on sampled dst planes: the oracle gets source planes
        # [sg, sg + 2) (the Linear chain's clamped z + 1 neighbour; a plane another rank owns is
        # given as zeros -- with fractions 0 and integer data it contributes 0 * finite = 0)
        for zl in (0, 1, 254, 255):
            zg = dz0 + zl
            sg = zg // 2
            planes = src[sg - ls0:sg - ls0 + 2]
            if planes.shape[0] < 2 and sg + 1 < s:
                planes = np.concatenate([planes, np.zeros_like(planes)])
            ref = ob.Volume.zeros((e, e, 1), 5)
            ob.resample_slab(ref, ob.Volume(planes, 5), 1, e, zg, s, sg)
            np.testing.assert_array_equal(r[zl:zl + 1], ref.codes, err_msg=f"rank {rank} plane {zg}")
        del src
        last = v3(e, e, dz1 - dz0, hip)
        o = v3(0, 0, 0, hip)
        assert hip.lib.vktHipFillRange(D.view, o, last, C.c_float(0.0)) == 0
        assert hip.lib.vktHipArithmeticRange(0, D.view, R.view, D.view, o, last, o) == 0   # R + 0
        np.testing.assert_array_equal(D.download(), r)
        assert hip.lib.vktHipArithmeticRange(0, D.view, R.view, B.view, o, last, o) == 0
        d, b = D.download(), B.download()
        for zl in (0, 128, 255):
            ref = ob.Volume.zeros((e, e, 1), 5)
            ob.arith_range("Sum", ref, ob.Volume(r[zl:zl + 1], 5), ob.Volume(b[zl:zl + 1], 5), (0, 0, 0), (e, e, 1))
            np.testing.assert_array_equal(d[zl:zl + 1], ref.codes, err_msg=f"rank {rank} SumRange plane {zl}")
    finally:
        for v in (S, R, B, D):
            v.free()


def test_bench_layout8_rank0_runs():
    """bench.py --layout-gpus 8: rank 0's config-4 slab (2048x2048x256 dst) in the bench harness."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--layout-gpus", "8", "--steps", "5",
                          "--warmup", "2", "--no-cpu-baseline", "--no-copy-peak"], capture_output=True, text=True,
                         timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["config"]["slab_dst_per_rank"] == [2048, 2048, 256]
    assert line["config"]["global_dst"] == [2048, 2048, 2048]
    assert line["value"] > 100.0
