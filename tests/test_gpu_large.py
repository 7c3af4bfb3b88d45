"""GPU tests at BASELINE.json sizes and for the Z-slab path, through the backend C ABI
(include/volkit_hip.h) on device-resident volumes.

* full-size parity where the oracle finishes in seconds (512^3 UInt16 arithmetic, config 2);
* size-independent properties at the metric sizes: 2x Resample of integer (and finite,
  non-negative float) data is exact replication; config 3 at full size (1024^3 -> 2048^3
  Float32 Linear, 32 GiB) with a non-finite source voxel, checked plane by plane on the device; Sum with a zero volume is the identity for
  every UInt16 code; Fill writes one code everywhere; Copy reproduces its source;
* Z-slab resample: P slabs of a global volume, each resampled from its local planes (owned +
  exchanged halo, per volkit_amd.slab's plan), equal the whole-volume oracle resample.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import binding as ob

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    import torch
    assert torch.cuda.is_available()
    from volkit_amd import _lib
    return _lib


class DevVol:
    """A device allocation + backend view."""

    def __init__(self, L, dims, fmt, lo=0.0, hi=1.0):
        self.L = L
        self.dims, self.fmt = tuple(dims), fmt
        x, y, z = dims
        self.nbytes = x * y * z * ob.BPV[fmt]
        p = C.c_void_p()
        assert L.lib.vktHipAllocate(C.byref(p), self.nbytes) == 0, L.last_error()
        self.ptr = p.value
        self.view = L.HipVolumeView_t(self.ptr, x, y, z, fmt, lo, hi)

    def upload(self, codes):
        a = np.ascontiguousarray(codes)
        assert a.nbytes == self.nbytes
        assert self.L.lib.vktHipMemcpy(self.ptr, a.ctypes.data, a.nbytes, 1) == 0

    def download(self):
        x, y, z = self.dims
        out = np.empty((z, y, x), dtype=ob.CODE_DTYPE[self.fmt])
        assert self.L.lib.vktHipMemcpy(out.ctypes.data, self.ptr, self.nbytes, 2) == 0
        return out

    def synth(self, seed):
        assert self.L.lib.vktHipSynthesize(self.view, C.c_uint64(seed)) == 0

    def free(self):
        if self.ptr:
            self.L.lib.vktHipFree(C.c_void_p(self.ptr))
            self.ptr = None


def v3(x, y, z, L):
    return L.Vec3i_t(x, y, z)


def test_config2_arith_512_full_parity(hip):
    """512^3 UInt16 SafeSum / SafeDiff / SumRange (BASELINE config 2), bit-exact vs oracle."""
    n = 512
    A, B, D = (DevVol(hip, (n, n, n), 5) for _ in range(3))
    A.synth(0x5EED)
    B.synth(0x5EED + 1)
    a, b = A.download(), B.download()
    np.testing.assert_array_equal(a.view(np.uint8).reshape(-1)[:64], ob.synth(64, 0x5EED))   # same generator
    for op, code in (("SafeSum", 5), ("SafeDiff", 6), ("Sum", 0)):
        assert hip.lib.vktHipArithmeticRange(code, D.view, A.view, B.view, v3(0, 0, 0, hip), v3(n, n, n, hip),
                                             v3(0, 0, 0, hip)) == 0
        got = D.download()
        ref = ob.Volume.zeros((n, n, n), 5)
        ob.arith_range(op, ref, ob.Volume(a, 5), ob.Volume(b, 5), (0, 0, 0), (n, n, n))
        np.testing.assert_array_equal(got, ref.codes, err_msg=op)
    for v in (A, B, D):
        v.free()


def test_metric_pipeline_1024_properties(hip):
    """Resample 512^3 -> 1024^3 UInt16 Linear + SumRange 1024^3: the exact index table for
    this ratio is x//2, and Linear == Nearest for integer data, so R must be the 2x2x2
    replication of S; SumRange(R, 0) must return R (every code round-trips);
    SumRange(R, B) is checked plane-sampled against the oracle."""
    s, e = 512, 1024
    S = DevVol(hip, (s, s, s), 5)
    R, B, D = (DevVol(hip, (e, e, e), 5) for _ in range(3))
    S.synth(7)
    B.synth(8)
    assert hip.lib.vktHipResample(R.view, S.view, 1) == 0
    src = S.download()
    r = R.download()
    for dz in (0, 1):
        for dy in (0, 1):
            for dx in (0, 1):
                np.testing.assert_array_equal(r[dz::2, dy::2, dx::2], src)
    del src
    Z = DevVol(hip, (e, e, e), 5)
    assert hip.lib.vktHipFillRange(Z.view, v3(0, 0, 0, hip), v3(e, e, e, hip), C.c_float(0.0)) == 0
    assert hip.lib.vktHipArithmeticRange(0, D.view, R.view, Z.view, v3(0, 0, 0, hip), v3(e, e, e, hip),
                                         v3(0, 0, 0, hip)) == 0
    np.testing.assert_array_equal(D.download(), r)
    assert hip.lib.vktHipArithmeticRange(0, D.view, R.view, B.view, v3(0, 0, 0, hip), v3(e, e, e, hip),
                                         v3(0, 0, 0, hip)) == 0
    d, b = D.download(), B.download()
    for z in (0, 1, 511, 1023):
        ref = ob.Volume.zeros((e, e, 1), 5)
        ob.arith_range("Sum", ref, ob.Volume(r[z:z + 1], 5), ob.Volume(b[z:z + 1], 5), (0, 0, 0), (e, e, 1))
        np.testing.assert_array_equal(d[z:z + 1], ref.codes, err_msg=f"plane {z}")
    for v in (S, R, B, D, Z):
        v.free()


def test_float_resample_replication_512_to_1024(hip):
    """Config-3 kernel at half size: finite non-negative Float32 data -> Linear == Nearest ==
    replication (bitwise)."""
    s, e = 512, 1024
    rng = np.random.default_rng(3)
    S = DevVol(hip, (s, s, s), 7)
    R = DevVol(hip, (e, e, e), 7)
    src = rng.random((s, s, s), dtype=np.float32)
    S.upload(src.view(np.uint32))
    assert hip.lib.vktHipResample(R.view, S.view, 1) == 0
    r = R.download()
    for dz in (0, 1):
        for dy in (0, 1):
            for dx in (0, 1):
                np.testing.assert_array_equal(r[dz::2, dy::2, dx::2], src.view(np.uint32))
    S.free()
    R.free()


def test_config3_full_size_linear_with_specials(hip):
    """BASELINE config 3 at full size: Resample 1024^3 -> 2048^3 Float32 Linear (32 GiB dst),
    source uniform in [0, 1) plus +inf at one interior voxel p, checked on the device plane by
    plane.  With fractions 0 the sampleLinear chain of source voxel s is v(s) + 0 * (its 7
    neighbours, hi.x = next voxel in memory): inf where s == p (inf + 0 * finite), NaN where p is
    one of s's 7 neighbours (0 * inf), else v(s) -- and dst(d) = chain(d // 2)."""
    import torch
    s, e = 1024, 2048
    p = (517, 301, 700)   # (x, y, z), interior
    S = DevVol(hip, (s, s, s), 7)
    R = DevVol(hip, (e, e, e), 7)
    gen = torch.Generator(device="cuda").manual_seed(3)
    src = torch.rand((s, s, s), device="cuda", dtype=torch.float32, generator=gen)
    src[p[2], p[1], p[0]] = float("inf")
    assert hip.lib.vktHipMemcpy(S.ptr, src.data_ptr(), S.nbytes, 3) == 0
    assert hip.lib.vktHipResample(R.view, S.view, 1) == 0
    assert hip.lib.vktHipSynchronize() == 0
    expect = src.clone()
    for dz in (0, 1):
        for dy in (0, 1):
            for dx in (0, 1):
                if dx or dy or dz:
                    expect[p[2] - dz, p[1] - dy, p[0] - dx] = float("nan")
    # copy the dst out plane pair by plane pair (device to device) and compare on the device
    plane = e * e
    for z in range(s):
        t = torch.empty((2, e, e), device="cuda", dtype=torch.float32)
        assert hip.lib.vktHipMemcpy(t.data_ptr(), R.ptr + 2 * z * plane * 4, 2 * plane * 4, 3) == 0
        ref = expect[z].repeat_interleave(2, 0).repeat_interleave(2, 1)
        for k in (0, 1):
            got = t[k]
            nan_g, nan_r = torch.isnan(got), torch.isnan(ref)
            assert torch.equal(nan_g, nan_r), f"NaN mask differs in dst plane {2 * z + k}"
            assert torch.equal(got[~nan_g], ref[~nan_r]), f"dst plane {2 * z + k}"
    assert int(torch.isnan(expect).sum()) == 7
    S.free()
    R.free()


def test_fill_and_copy_1024(hip):
    e = 1024
    V, W = DevVol(hip, (e, e, e), 5), DevVol(hip, (e, e, e), 5)
    assert hip.lib.vktHipFillRange(V.view, v3(0, 0, 0, hip), v3(e, e, e, hip), C.c_float(0.1)) == 0
    code = int.from_bytes(ob.map_voxel(0.1, 5), "little")
    v = V.download()
    assert (v == code).all()
    V.synth(99)
    assert hip.lib.vktHipCopyRange(W.view, V.view, v3(0, 0, 0, hip), v3(e, e, e, hip), v3(0, 0, 0, hip)) == 0
    np.testing.assert_array_equal(W.download(), V.download())
    V.free()
    W.free()


def test_float32_4gib_operands_shifted_parity(hip):
    """1024^3 Float32 operands are exactly 4 GiB: the general path's 32-bit addressing admits
    them (byte offsets from the 16-B aligned base <= 2^32).  Phase-shifted CopyRange and an
    arithmetic dstOffset on the 800^3 sub-box at x0 = 100 (the f32shift bench cases, whose last
    rows end at the volume's last bytes when shifted to the far corner), bit-exact vs the oracle."""
    import torch
    e = 1024
    A, B, D = (DevVol(hip, (e, e, e), 7) for _ in range(3))
    gen = torch.Generator(device="cuda").manual_seed(11)
    for v in (A, B, D):
        t = torch.rand((e, e, e), device="cuda", dtype=torch.float32, generator=gen)
        assert hip.lib.vktHipMemcpy(v.ptr, t.data_ptr(), v.nbytes, 3) == 0
        del t
    assert hip.lib.vktHipSynchronize() == 0
    a, b, d0 = A.download(), B.download(), D.download()
    f0, f1 = (100, 100, 100), (900, 900, 900)
    cases = (("copy dst 0", None, (0, 0, 0)), ("copy dst x0=3", None, (3, 100, 100)),
             ("copy to the volume end", None, (224, 224, 224)), ("Sum dstOffset x=-97", 0, (-97, 0, 0)),
             ("Sum dstOffset to the end", 0, (124, 124, 124)))
    for what, op, off in cases:
        assert hip.lib.vktHipMemcpy(D.ptr, d0.ctypes.data, D.nbytes, 1) == 0
        if op is None:
            rc = hip.lib.vktHipCopyRange(D.view, A.view, v3(*f0, hip), v3(*f1, hip), v3(*off, hip))
            ref = ob.Volume(d0.copy(), 7)
            ob.copy_range(ref, ob.Volume(a, 7), f0, f1, off)
        else:
            rc = hip.lib.vktHipArithmeticRange(op, D.view, A.view, B.view, v3(*f0, hip), v3(*f1, hip), v3(*off, hip))
            ref = ob.Volume(d0.copy(), 7)
            ob.arith_range("Sum", ref, ob.Volume(a, 7), ob.Volume(b, 7), f0, f1, off)
        assert rc == 0, hip.last_error()
        got = D.download()
        assert np.array_equal(got, ref.codes), what
        del got, ref
    for v in (A, B, D):
        v.free()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("fmt,fm", [(5, 1), (7, 1), (4, 0)])
@pytest.mark.parametrize("sdims,ddims", [((64, 48, 40), (128, 96, 80)), ((37, 23, 29), (64, 40, 53)),
                                         ((32, 32, 64), (16, 16, 21))])
def test_zslab_resample_matches_whole_volume(hip, world, fmt, fm, sdims, ddims):
    from volkit_amd import slab
    rng = np.random.default_rng(world * 100 + fmt)
    sx, sy, sz = sdims
    dx, dy, dz = ddims
    if fmt == 7:
        g = rng.uniform(-1, 2, (sz, sy, sx)).astype(np.float32)
        g.reshape(-1)[::131] = np.nan
        glob = g.view(np.uint32)
    else:
        glob = rng.integers(0, 2 ** (8 * ob.BPV[fmt]), (sz, sy, sx), dtype=np.uint64).astype(ob.CODE_DTYPE[fmt])
    ref = ob.Volume.zeros(ddims, fmt)
    ob.resample(ref, ob.Volume(glob, fmt), fm)
    chain = fm == 1 and fmt == 7
    for rank in range(world):
        plan = slab.plan_resample(dz, sz, world, rank, fm, chain)
        d0, d1 = plan.dst
        if d1 <= d0:
            continue
        l0, l1 = plan.local_src
        Sl = DevVol(hip, (sx, sy, l1 - l0), fmt)
        Sl.upload(glob[l0:l1])          # owned planes + the halo the exchange would deliver
        Dl = DevVol(hip, (dx, dy, d1 - d0), fmt)
        assert slab.resample_slab(Dl.view, Sl.view, fm, plan) == 0, hip.last_error()
        got = Dl.download()
        exp = ref.codes[d0:d1]
        if fmt == 7:
            fg, fe = got.view(np.float32), exp.view(np.float32)
            np.testing.assert_array_equal(np.isnan(fg), np.isnan(fe))
            np.testing.assert_array_equal(got[~np.isnan(fe)], exp[~np.isnan(fe)])
        else:
            np.testing.assert_array_equal(got, exp)
        Sl.free()
        Dl.free()


@pytest.mark.parametrize("world", [2, 3])
def test_zslab_linear_specials_in_halo_planes(hip, world):
    """Float32 Linear (optimistic convert + fix-up path): non-finite values and -0 only in the
    planes just above each slab boundary (the z+1 halo a slab reads but does not own) and in
    the first row after a plane end (hi.x of the previous plane's last voxel)."""
    from volkit_amd import slab
    sx, sy, sz = 32, 16, 12
    dx, dy, dz = 64, 32, 24
    g = np.random.default_rng(world).uniform(0, 1, (sz, sy, sx)).astype(np.float32)
    for rank in range(1, world):
        z0, _ = slab.slab_bounds(sz, world, rank)
        g[z0, 3, 5] = np.inf
        g[z0, 0, 0] = np.nan
        g[z0 - 1, sy - 1, sx - 1] = -0.0
    glob = g.view(np.uint32)
    ref = ob.Volume.zeros((dx, dy, dz), 7)
    ob.resample(ref, ob.Volume(glob, 7), 1)
    for rank in range(world):
        plan = slab.plan_resample(dz, sz, world, rank, 1, True)
        d0, d1 = plan.dst
        l0, l1 = plan.local_src
        Sl = DevVol(hip, (sx, sy, l1 - l0), 7)
        Sl.upload(glob[l0:l1])
        Dl = DevVol(hip, (dx, dy, d1 - d0), 7)
        assert slab.resample_slab(Dl.view, Sl.view, 1, plan) == 0, hip.last_error()
        got, exp = Dl.download(), ref.codes[d0:d1]
        fg, fe = got.view(np.float32), exp.view(np.float32)
        np.testing.assert_array_equal(np.isnan(fg), np.isnan(fe))
        np.testing.assert_array_equal(got[~np.isnan(fe)], exp[~np.isnan(fe)])
        Sl.free()
        Dl.free()
