"""Z-slab partitions held by ONE process on one GPU, through the native C ABI with the
in-process transport (comm = NULL: every move is a device-to-device hipMemcpyAsync on the
compute stream, include/volkit_hip.h):

* vktHipSlabExchangeHaloLocal + vktHipResampleSlab per slab -- a Float32 Linear chain over 4
  and 8 slabs whose halo planes hold non-finite values and -0 (the planes the exchange must
  deliver), byte-equal to the whole-volume oracle resample.  Each slab buffer starts with its
  owned planes only; the halo planes start as garbage, so a missed or misplaced move shows.
  This runs the transfer list's pointer math (runtime/Comm.cpp planeSpan), the same code the
  RCCL exchange uses.
* vktHipSlab{Fill,Copy,Arithmetic}Range over 1-8 slabs: global first/last/dstOffset with
  dstOffset.z moving planes across slab boundaries, clamped halo copies past both z borders,
  format conversion, three different partitions in one arithmetic call; each slab's owned dst
  planes equal one whole-volume oracle call, the dst halo planes are untouched.
* slab.py's torch.distributed executor with one rank (vktHipSlabRangePieces on the GPU).
Reference semantics: Resample_serial.hpp:26-71, Fill_serial.hpp:20-26, Copy_serial.hpp:38-47,
Arithmetic_serial.hpp:25-41.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import binding as ob
from test_slab_range_gloo import CASES, _codes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    import torch
    from volkit_amd._lib import lib
    torch.cuda.set_device(0)
    return lib


def err(L):
    from volkit_amd import _lib
    return _lib.last_error()


class DevSlab:
    """Rank `rank`'s slab of a global (G, y, x) code array on the device: owned planes, plus
    `halo` planes on each side filled with a garbage byte."""

    def __init__(self, glob, fmt, world, rank, halo=0, extra=None):
        import torch
        from volkit_amd import _lib, slab
        G, y, x = glob.shape
        o0, o1 = slab.slab_bounds(G, world, rank)
        lo, hi = (o0, o1) if o1 > o0 else (o0, o0)
        if extra is not None:          # explicit held range (Resample: owned + read planes)
            lo, hi = extra
        elif o1 > o0:
            lo, hi = max(0, o0 - halo), min(G, o1 + halo)
        self.z0, self.owned = lo, (o0, o1)
        host = np.full((hi - lo, y, x), 0x5A, dtype=glob.dtype)
        if o1 > o0:
            host[o0 - lo:o1 - lo] = glob[o0:o1]
        self.before = host.copy()
        raw = host.view(np.uint8).reshape(-1)
        self.t = torch.zeros(max(raw.size, 1) + 64, dtype=torch.uint8, device="cuda")
        self.t[:raw.size].copy_(torch.from_numpy(raw.copy()))
        self.shape, self.dtype = host.shape, glob.dtype
        self.view = _lib.HipVolumeView_t(self.t.data_ptr(), x, y, hi - lo, fmt, 0.0, 1.0)
        self.slab = _lib.HipSlab_t(self.view, lo, G)

    def read(self):
        import torch
        torch.cuda.synchronize()
        n = int(np.prod(self.shape)) * np.dtype(self.dtype).itemsize
        return self.t[:n].cpu().numpy().view(self.dtype).reshape(self.shape)


def same_codes(got, want, fmt):
    if fmt == 7:
        fg, fw = got.view(np.float32), want.view(np.float32)
        return np.array_equal(np.isnan(fg), np.isnan(fw)) and np.array_equal(got[~np.isnan(fw)], want[~np.isnan(fw)])
    return np.array_equal(got, want)


@pytest.mark.parametrize("transport", ["local", "peer", "overlapped"])
@pytest.mark.parametrize("nslabs", [4, 8])
@pytest.mark.parametrize("sdims,ddims", [((40, 24, 32), (80, 48, 64)), ((37, 19, 29), (64, 40, 53)),
                                         ((32, 16, 64), (16, 16, 21))])
def test_local_halo_exchange_linear_chain(L, nslabs, sdims, ddims, transport):
    """vktHipSlabExchangeHaloLocal (device copies) and vktHipSlabExchangeHaloPeer (peer copies into
    each slab's device; every slab on device 0 of the one-GPU pool) deliver every rank's halo."""
    from volkit_amd import _lib, slab
    sx, sy, sz = sdims
    dx, dy, dz = ddims
    g = np.random.default_rng(nslabs * 7 + sz).uniform(0, 1, (sz, sy, sx)).astype(np.float32)
    # non-finite values and -0 in every plane a slab receives (the first plane of every slab but
    # slab 0 -- the z+1 neighbour of the slab below) and the hi.x voxel before it
    for r in range(1, nslabs):
        z0, z1 = slab.slab_bounds(sz, nslabs, r)
        if z1 > z0:
            g[z0, 1, 2] = np.inf
            g[z0, 0, 0] = np.nan
            g[z0, sy - 1, sx - 1] = -np.inf
            g[z0, 2, 3] = -0.0
    glob = g.view(np.uint32)
    ref = ob.Volume.zeros(ddims, 7)
    ob.resample(ref, ob.Volume(glob, 7), 1)
    plans = [slab.plan_resample(dz, sz, nslabs, r, 1, True) for r in range(nslabs)]
    srcs = [DevSlab(glob, 7, nslabs, r, extra=p.local_src) for r, p in enumerate(plans)]
    moved = sum(p.halo_planes for p in plans)
    assert moved > 0, "the chain must exchange planes"
    views = (_lib.HipVolumeView_t * nslabs)(*[s.view for s in srcs])
    z0s = (C.c_int32 * nslabs)(*[s.z0 for s in srcs])
    if transport == "overlapped":
        # vktHipResampleSlabsOverlappedLocal: each slab's receives on the copy stream while its
        # interior planes resample, then the rest -- equal to the whole-volume resample
        dsts = [DevSlab(np.zeros((max(p.dst[1] - p.dst[0], 0), dy, dx), np.uint32), 7, 1, 0) for p in plans]
        dviews = (_lib.HipVolumeView_t * nslabs)(*[d.view for d in dsts])
        assert L.vktHipResampleSlabsOverlappedLocal(nslabs, dviews, views, z0s, dz, sz, 1, 1) == 0, err(L)
        for r, (p, s, d) in enumerate(zip(plans, srcs, dsts)):
            l0, l1 = p.local_src
            assert np.array_equal(s.read(), glob[l0:l1]), f"slab {r}: halo planes not delivered"
            d0, d1 = p.dst
            if d1 > d0:
                assert same_codes(d.read(), ref.codes[d0:d1], 7), f"slab {r}: overlapped resample differs"
        return
    if transport == "local":
        assert L.vktHipSlabExchangeHaloLocal(nslabs, views, z0s, dz, sz, 1, 1) == 0, err(L)
    else:
        devs = (C.c_int32 * nslabs)(*([0] * nslabs))
        assert L.vktHipSlabExchangeHaloPeer(nslabs, views, z0s, devs, dz, sz, 1, 1) == 0, err(L)
    for r, (p, s) in enumerate(zip(plans, srcs)):
        l0, l1 = p.local_src
        assert np.array_equal(s.read(), glob[l0:l1]), f"slab {r}: halo planes not delivered"
        d0, d1 = p.dst
        if d1 <= d0:
            continue
        D = DevSlab(np.zeros((d1 - d0, dy, dx), np.uint32), 7, 1, 0)
        assert slab.resample_slab(D.view, s.view, 1, p) == 0, err(L)
        assert same_codes(D.read(), ref.codes[d0:d1], 7), f"slab {r}: resample differs from the whole volume"


def test_peer_halo_exchange_across_two_devices_waits_for_the_compute_stream(L):
    """vktHipSlabExchangeHaloPeer with slabs on devices 0 and 1: the slab on device 1 receives
    its halo plane by a peer copy on a stream of device 1, which must first wait for the work
    queued on the library's compute stream -- here a FillRange of the source slab (device 0)
    enqueued right before the exchange, with no host synchronisation in between.  Source depth
    15 -> dst 30 over two ranks: slab 1 (dst planes [15, 30)) reads source plane 7, owned by
    slab 0; slab 0 reads planes 8 and 9 from slab 1.  Needs two GPUs (skipped on the one-GPU pool)."""
    import torch
    from volkit_amd import _lib
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    x, y = 64, 32
    plane = x * y * 4
    t0 = torch.zeros(10 * plane, dtype=torch.uint8, device="cuda:0")   # global planes [0, 10)
    t1 = torch.zeros(8 * plane, dtype=torch.uint8, device="cuda:1")   # global planes [7, 15)
    t1.view(torch.float32).fill_(0.25)
    torch.cuda.synchronize(1)
    torch.cuda.synchronize(0)
    v0 = _lib.HipVolumeView_t(t0.data_ptr(), x, y, 10, 7, 0.0, 1.0)
    v1 = _lib.HipVolumeView_t(t1.data_ptr(), x, y, 8, 7, 0.0, 1.0)
    assert L.vktHipFillRange(v0, _lib.Vec3i_t(0, 0, 0), _lib.Vec3i_t(x, y, 8), C.c_float(0.75)) == 0, err(L)
    views = (_lib.HipVolumeView_t * 2)(v0, v1)
    z0s = (C.c_int32 * 2)(0, 7)
    devs = (C.c_int32 * 2)(0, 1)
    assert L.vktHipSlabExchangeHaloPeer(2, views, z0s, devs, 30, 15, 1, 1) == 0, err(L)
    torch.cuda.synchronize(0)
    torch.cuda.synchronize(1)
    g0 = t0.cpu().numpy().view(np.float32).reshape(10, y, x)
    g1 = t1.cpu().numpy().view(np.float32).reshape(8, y, x)
    assert (g0[:8] == 0.75).all() and (g0[8:] == 0.25).all()
    assert (g1[0] == 0.75).all() and (g1[1:] == 0.25).all()


def test_local_halo_exchange_rejects_short_buffers(L):
    import torch
    from volkit_amd import _lib
    t = torch.zeros(2 * 8 * 8 * 4 * 4, dtype=torch.uint8, device="cuda")
    v0 = _lib.HipVolumeView_t(t.data_ptr(), 8, 8, 4, 7, 0.0, 1.0)
    v1 = _lib.HipVolumeView_t(t.data_ptr() + 8 * 8 * 4 * 4, 8, 8, 4, 7, 0.0, 1.0)
    views = (_lib.HipVolumeView_t * 2)(v0, v1)
    z0s = (C.c_int32 * 2)(0, 4)
    # slab 0 holds planes [0, 4) but must also hold plane 4 (the chain's z+1 neighbour)
    assert L.vktHipSlabExchangeHaloLocal(2, views, z0s, 16, 8, 1, 1) != 0
    devs = (C.c_int32 * 2)(0, 0)
    assert L.vktHipSlabExchangeHaloPeer(2, views, z0s, devs, 16, 8, 1, 1) != 0
    bad = (C.c_int32 * 2)(0, 99)
    assert L.vktHipSlabExchangeHaloPeer(2, views, z0s, bad, 16, 8, 1, 1) != 0   # no such device


@pytest.mark.parametrize("nslabs", [1, 2, 3, 4, 8])
def test_local_slab_range_calls(L, nslabs):
    from volkit_amd import _lib
    bad = []
    X, Y = 72, 20      # rows of several 16-B chunks, phases per first.x
    for ci, (kind, dfmt, sfmt, dG, s1G, s2G, first, last, off, op) in enumerate(CASES):
        for halo in (0, 1):
            rng = np.random.default_rng(2000 + ci)
            # the z extents of the CPU cases; x / y boxes for the wider planes (row phases 3, 8, 13)
            if kind == "fill":
                f, l_, o = (5, 2, first[2]), (67, 18, last[2]), (0, 0, 0)
            elif kind == "copy":    # clamped x / y where the CPU case clamps; dst box x [4, 68), y [2, 18)
                f = (first[0] * 5 + 3, first[1] * 3, first[2])
                l_, o = (f[0] + 64, f[1] + 16, last[2]), (4, 2, off[2])
            else:
                f, l_, o = (first[0] * 5 + 3, first[1] * 3, first[2]), (69, 20, last[2]), (0, 0, off[2])
            dglob = _codes(rng, dfmt, (dG, Y, X))
            s1 = _codes(rng, sfmt, (s1G, Y, X)) if s1G else None
            s2 = _codes(rng, sfmt, (s2G, Y, X)) if s2G else None
            ref = ob.Volume(dglob.copy(), dfmt)
            D = [DevSlab(dglob, dfmt, nslabs, r, halo) for r in range(nslabs)]
            darr = (_lib.HipSlab_t * nslabs)(*[d.slab for d in D])
            F, La, O = _lib.Vec3i_t(*f), _lib.Vec3i_t(*l_), _lib.Vec3i_t(*o)
            if kind == "fill":
                ob.fill_range(ref, f, l_, 0.375)
                e = L.vktHipSlabFillRange(None, nslabs, darr, F, La, C.c_float(0.375))
            elif kind == "copy":
                ob.copy_range(ref, ob.Volume(s1, sfmt), f, l_, o)
                S = [DevSlab(s1, sfmt, nslabs, r, halo) for r in range(nslabs)]
                sarr = (_lib.HipSlab_t * nslabs)(*[s.slab for s in S])
                e = L.vktHipSlabCopyRange(None, nslabs, darr, sarr, F, La, O)
            else:
                ob.arith_range(op, ref, ob.Volume(s1, sfmt), ob.Volume(s2, sfmt), f, l_, o)
                A = [DevSlab(s1, sfmt, nslabs, r, halo) for r in range(nslabs)]
                B = [DevSlab(s2, sfmt, nslabs, r, halo) for r in range(nslabs)]
                aarr = (_lib.HipSlab_t * nslabs)(*[s.slab for s in A])
                barr = (_lib.HipSlab_t * nslabs)(*[s.slab for s in B])
                e = L.vktHipSlabArithmeticRange(None, _lib.ARITH_OPS.index(op), nslabs, darr, aarr, barr, F, La, O)
            if e != 0:
                bad.append(f"case {ci} {kind} halo={halo}: error {err(L)}")
                continue
            for r, d in enumerate(D):
                o0, o1 = d.owned
                got = d.read()
                if not same_codes(got[o0 - d.z0:o1 - d.z0], ref.codes[o0:o1], dfmt):
                    bad.append(f"case {ci} {kind} halo={halo} slab {r}: owned planes differ")
                keep = np.ones(got.shape[0], bool)
                keep[o0 - d.z0:o1 - d.z0] = False
                if not np.array_equal(got[keep], d.before[keep]):
                    bad.append(f"case {ci} {kind} halo={halo} slab {r}: halo planes written")
    assert not bad, "; ".join(bad)


def test_slab_range_in_place_arithmetic(L):
    """Sum(A, A, B) over slabs (dest aliases source 1, dstOffset 0): every piece is own, the
    local op runs in place like the whole-volume call."""
    from volkit_amd import _lib
    rng = np.random.default_rng(5)
    a = _codes(rng, 5, (19, 16, 64))
    b = _codes(rng, 5, (19, 16, 64))
    ref = ob.Volume(a.copy(), 5)
    ob.arith_range("Sum", ref, ob.Volume(a.copy(), 5), ob.Volume(b, 5), (0, 0, 0), (64, 16, 19), (0, 0, 0))
    A = [DevSlab(a, 5, 3, r) for r in range(3)]
    B = [DevSlab(b, 5, 3, r) for r in range(3)]
    aarr = (_lib.HipSlab_t * 3)(*[s.slab for s in A])
    barr = (_lib.HipSlab_t * 3)(*[s.slab for s in B])
    assert L.vktHipSlabArithmeticRange(None, 0, 3, aarr, aarr, barr, _lib.Vec3i_t(0, 0, 0), _lib.Vec3i_t(64, 16, 19),
                                       _lib.Vec3i_t(0, 0, 0)) == 0, err(L)
    for s in A:
        o0, o1 = s.owned
        assert np.array_equal(s.read(), ref.codes[o0:o1])


def test_slab_py_executor_one_rank(L):
    """slab.copy_range / arithmetic_range without torch.distributed (world 1): the pieces run
    through vktHipSlabRangePieces on device tensors."""
    import torch
    from volkit_amd import _lib, slab
    rng = np.random.default_rng(6)
    s = _codes(rng, 4, (11, 12, 48))
    d = _codes(rng, 4, (14, 12, 48))
    ref = ob.Volume(d.copy(), 4)
    ob.copy_range(ref, ob.Volume(s, 4), (3, -1, -2), (45, 11, 10), (0, 0, 2))
    S, D = DevSlab(s, 4, 1, 0), DevSlab(d, 4, 1, 0)
    slab.copy_range(slab.Slab(D.view, 0, 14), slab.Slab(S.view, 0, 11), (3, -1, -2), (45, 11, 10), (0, 0, 2))
    torch.cuda.synchronize()
    assert np.array_equal(D.read(), ref.codes)


@pytest.mark.parametrize("nslabs", [1, 3, 4])
def test_slab_transform_host_callback(L, nslabs):
    """vktHipSlabTransformRange1 (and slab.transform_range for one rank): each slab runs the
    host callback over its owned planes of the global range with global z; the slabs put
    together equal the whole-volume oracle TransformRange_serial (Transform_serial.hpp:15-48),
    halo planes untouched."""
    from volkit_amd import _lib, slab
    from volkit_amd.volkit import VoxelView
    rng = np.random.default_rng(nslabs)
    G, y, x = 11, 6, 13
    glob = rng.integers(0, 256, (G, y, x), dtype=np.uint8)
    first, last = (2, 1, 1), (12, 6, 10)

    def op(xx, yy, zz, v):
        v.bytes[0] = (v.bytes[0] ^ (xx + 3 * yy + 17 * zz)) & 0xFF

    def oracle_op(xx, yy, zz, b, fmt, lo, hi):
        b[0] = (b[0] ^ (xx + 3 * yy + 17 * zz)) & 0xFF

    ref = ob.Volume(glob.copy(), 4, 0.0, 1.0)
    ob.transform_range1(ref, first, last, oracle_op)
    slabs = [DevSlab(glob, 4, nslabs, r, halo=1) for r in range(nslabs)]
    seen = []

    def record(xx, yy, zz, v):
        seen.append(zz)
        op(xx, yy, zz, v)
    cb = _lib.UnaryOp(lambda xx, yy, zz, v: record(xx, yy, zz, VoxelView(v)))
    for r, s in enumerate(slabs):
        assert L.vktHipSlabTransformRange1(nslabs, r, s.slab, _lib.Vec3i_t(*first), _lib.Vec3i_t(*last), cb) == 0, err(L)
    assert seen == sorted(seen)            # ranks 0..n-1 in turn: the serial z order
    for s in slabs:
        got, o0, o1 = s.read(), *s.owned
        np.testing.assert_array_equal(got[o0 - s.z0:o1 - s.z0], ref.codes[o0:o1])
        keep = np.ones(got.shape[0], bool)
        keep[o0 - s.z0:o1 - s.z0] = False
        np.testing.assert_array_equal(got[keep], s.before[keep])
    if nslabs == 1:
        s = DevSlab(glob, 4, 1, 0)
        slab.transform_range(slab.Slab(s.view, s.z0, G), first, last, op)
        np.testing.assert_array_equal(s.read(), ref.codes)
    bad = slabs[0]
    assert L.vktHipSlabTransformRange1(nslabs, 0, bad.slab, _lib.Vec3i_t(0, 0, 0), _lib.Vec3i_t(x, y, G + 1), cb) != 0
