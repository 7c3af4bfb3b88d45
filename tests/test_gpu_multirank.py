"""Multi-rank GPU path rehearsed on one MI355X: 2 processes (both on cuda:0, gloo for the
exchange -- the driver's 8-GPU node uses RCCL), each holding only its own Z-slab in HBM and
running the real HIP kernels:
  * slab.aggregates (pass 1 / all_gather / mean / pass 2 / all_gather) == whole-volume oracle;
    on UInt8 / UInt16 slabs the one-pass code-count form (all_reduce of the code counts, first-
    occurrence search per slab, all_reduce MIN of the indices), also == the oracle;
  * slab.histogram (local counts on the device, all_reduce) == whole-volume oracle, exactly;
  * Float32 "Linear" Resample with the z+1 halo received from the neighbour rank == the
    rank's slab of the whole-volume oracle resample;
  * slab.copy_range / slab.arithmetic_range with a dstOffset.z that moves planes across the
    slab boundary (device slabs, the moved planes staged through gloo) == the rank's planes of
    one whole-volume oracle call.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORLD = 2
RANGE_COPY = ((1, 2, 3), (30, 18, 20), (0, 1, 4))       # first, last, dstOffset: planes move up 1
RANGE_ARITH = ((0, 0, 2), (32, 20, 20), (0, 0, -2))     # ... and down 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _global_volume():
    rng = np.random.default_rng(2024)
    vals = rng.uniform(-0.25, 1.25, (24, 20, 32)).astype(np.float32)   # (z, y, x)
    vals[5, 3, 7] = vals[20, 0, 1] = np.float32(-0.5)
    return vals


def _code_volume(fmt):
    top = 255 if fmt == 4 else 65535
    rng = np.random.default_rng(31 + fmt)
    codes = rng.integers(2, top - 1, (20, 24, 64)).astype(np.uint8 if fmt == 4 else np.uint16)
    codes[15, 3, 9] = codes[18, 0, 0] = 1              # the minimum only in the second slab
    codes[4, 20, 60] = codes[14, 2, 2] = top - 1
    return codes


def _worker(rank, port, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        import volkit_amd.volkit as vkt
        from volkit_amd import slab

        vals = _global_volume()
        gz, gy, gx = vals.shape
        z0, z1 = slab.slab_bounds(gz, WORLD, rank)
        ep = vkt.GetThreadExecutionPolicy()
        ep.device = vkt.ExecutionPolicy.Device_GPU
        vkt.SetThreadExecutionPolicy(ep)
        v = vkt.StructuredVolume(gx, gy, z1 - z0, vkt.DataFormat_Float32)
        v.from_numpy(np.ascontiguousarray(vals[z0:z1]).view(np.uint32))    # H2D of the own slab only
        view = v.hip_view()
        out = {}
        for first, last in (((0, 0, 0), (gx, gy, gz)), ((3, 2, 5), (30, 19, 17))):
            a = slab.aggregates(view, (gx, gy, gz), z0, first, last, device="cuda")
            bins = torch.zeros(64, dtype=torch.int64, device="cuda")
            slab.histogram(view, z0, first, last, bins, 64)
            out[(first, last)] = ((a.min, a.max, (a.argmin.x, a.argmin.y, a.argmin.z),
                                   (a.argmax.x, a.argmax.y, a.argmax.z), a.sum, a.mean, a.var),
                                  bins.cpu().numpy().copy())
        # UInt8 / UInt16 slabs: the one-pass code-count form (counts on the device, all_reduce,
        # first-occurrence search per slab, all_reduce MIN of the indices)
        # (UInt16 / Float32 take the one-pass moments form: one all_gather of moment partials)
        for fmt, mapping in ((5, (-1.0, 3.0)), (5, (0.0, 1.0)), (4, (0.0, 1.0)), (4, (3.0, -1.0))):
            codes = _code_volume(fmt)
            cz, cy, cx = codes.shape
            c0, c1 = slab.slab_bounds(cz, WORLD, rank)
            cv = vkt.StructuredVolume(cx, cy, c1 - c0, fmt, 1.0, 1.0, 1.0, *mapping)
            cv.from_numpy(np.ascontiguousarray(codes[c0:c1]))
            for first, last in (((0, 0, 0), (cx, cy, cz)), ((3, 1, 2), (cx - 5, cy, cz - 1))):
                a = slab.aggregates(cv.hip_view(), (cx, cy, cz), c0, first, last, device="cuda")
                out[("codes", fmt, mapping, first, last)] = (a.min, a.max, (a.argmin.x, a.argmin.y, a.argmin.z),
                                                             (a.argmax.x, a.argmax.y, a.argmax.z), a.sum, a.mean, a.var)
        # Float32 Linear resample 2x with the halo exchanged over the process group
        dz = 2 * gz
        plan = slab.plan_resample(dz, gz, WORLD, rank, vkt.FilterMode_Linear, chain=True)
        l0, l1 = plan.local_src
        src = vkt.StructuredVolume(gx, gy, l1 - l0, vkt.DataFormat_Float32)
        local = np.zeros((l1 - l0, gy, gx), np.float32)
        local[z0 - l0:z1 - l0] = vals[z0:z1]
        src.from_numpy(local.view(np.uint32))
        sview = src.hip_view()
        plane = gx * gy * 4

        def planes(g0, g1):
            host = torch.from_numpy(local.view(np.uint8).reshape(-1)[(g0 - l0) * plane:(g1 - l0) * plane].copy())
            return host

        # gloo moves host tensors: send our planes, receive into host buffers, upload
        ops = []
        for peer, g0, g1 in plan.sends:
            ops.append(dist.P2POp(dist.isend, planes(g0, g1), peer))
        recv = []
        for peer, g0, g1 in plan.recvs:
            t = torch.empty((g1 - g0) * plane, dtype=torch.uint8)
            recv.append((g0, t))
            ops.append(dist.P2POp(dist.irecv, t, peer))
        if ops:
            for r in dist.batch_isend_irecv(ops):
                r.wait()
        for g0, t in recv:
            local.view(np.uint8).reshape(-1)[(g0 - l0) * plane:(g0 - l0) * plane + t.numel()] = t.numpy()
        src.from_numpy(local.view(np.uint32))
        sview = src.hip_view()
        d0, d1 = plan.dst
        dst = vkt.StructuredVolume(2 * gx, 2 * gy, d1 - d0, vkt.DataFormat_Float32)
        err = slab.resample_slab(dst.hip_view(), sview, vkt.FilterMode_Linear, plan)
        assert err == 0, vkt.last_error()
        # the overlapped form on device planes: exchange issued, interior dst planes resampled
        # from the owned source planes, then the boundary planes once the halo has landed
        own = np.zeros((l1 - l0, gy, gx), np.float32)
        own[z0 - l0:z1 - l0] = vals[z0:z1]
        src2 = vkt.StructuredVolume(gx, gy, l1 - l0, vkt.DataFormat_Float32)
        src2.from_numpy(own.view(np.uint32))
        sv2 = src2.hip_view()
        dst2 = vkt.StructuredVolume(2 * gx, 2 * gy, d1 - d0, vkt.DataFormat_Float32)

        def dev_planes(g0, g1):
            return slab.device_tensor(sv2.data + (g0 - l0) * plane, (g1 - g0) * plane)

        dk = slab.interior_split(plan, vkt.FilterMode_Linear, True)
        err = slab.resample_slab_overlapped(dst2.hip_view(), sv2, vkt.FilterMode_Linear, plan, True, dev_planes)
        assert err == 0, vkt.last_error()
        torch.cuda.synchronize()
        assert np.array_equal(dst2.to_numpy(), dst.to_numpy()), f"rank {rank}: overlapped != single call (dk={dk})"
        out["split"] = (d0, dk, d1)
        # Range calls over the slabs: planes cross the rank boundary (dstOffset.z)
        from volkit_amd import _lib

        def dev_slab(glob):
            t = torch.from_numpy(np.ascontiguousarray(glob[z0:z1]).view(np.uint8).reshape(-1).copy()).cuda()
            view = _lib.HipVolumeView_t(t.data_ptr(), gx, gy, z1 - z0, vkt.DataFormat_Float32, 0.0, 1.0)
            return slab.Slab(view, z0, gz, t)

        a_sl, b_sl = dev_slab(vals), dev_slab(vals[::-1] * 0.5)
        c_sl, s_sl = dev_slab(np.zeros_like(vals)), dev_slab(np.zeros_like(vals))
        slab.copy_range(c_sl, a_sl, *RANGE_COPY)
        slab.arithmetic_range("SafeSum", s_sl, a_sl, b_sl, *RANGE_ARITH)
        torch.cuda.synchronize()
        out["range"] = (z0, z1, c_sl.tensor.cpu().numpy().view(np.uint32).copy(),
                        s_sl.tensor.cpu().numpy().view(np.uint32).copy())
        ep.device = vkt.ExecutionPolicy.Device_CPU
        vkt.SetThreadExecutionPolicy(ep)
        q.put((rank, out, (d0, d1, dst.to_numpy()), plan.halo_planes))
        dist.destroy_process_group()
    except Exception as e:   # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc(), None, None))


def test_two_ranks_on_one_gpu():
    import torch.multiprocessing as mp
    from oracle import binding as ob

    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=400) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r, out, _, _ in res:
        assert not isinstance(out, str), out
    vals = _global_volume()
    gz, gy, gx = vals.shape
    whole = ob.Volume(vals.view(np.uint32), 7)
    whole_b = np.ascontiguousarray(vals[::-1] * 0.5)
    ref_c = ob.Volume(np.zeros_like(vals).view(np.uint32), 7)
    ob.copy_range(ref_c, ob.Volume(vals.view(np.uint32), 7), *RANGE_COPY)
    ref_s = ob.Volume(np.zeros_like(vals).view(np.uint32), 7)
    ob.arith_range("SafeSum", ref_s, ob.Volume(vals.view(np.uint32), 7), ob.Volume(whole_b.view(np.uint32), 7),
                   *RANGE_ARITH)
    for r, out, _, halo in res:
        assert not isinstance(out, str), out
        z0, z1, got_c, got_s = out.pop("range")
        assert np.array_equal(got_c, ref_c.codes[z0:z1].reshape(-1)), f"rank {r}: slab copy_range differs"
        assert np.array_equal(got_s, ref_s.codes[z0:z1].reshape(-1)), f"rank {r}: slab arithmetic_range differs"
        d0, dk, d1 = out.pop("split")
        assert d0 < dk < d1 or not halo, (r, d0, dk, d1)   # a rank with a halo has an interior
    for key in [k for k in res[0][1] if k[0] == "codes"]:
        _, fmt, mapping, first, last = key
        codes = _code_volume(fmt)
        ref = ob.aggregates_range(ob.Volume(codes, fmt, *mapping), first, last)
        for r, out, _, _ in res:
            mn, mx, amin, amax, s, mean, var = out.pop(key)
            assert (mn, mx, amin, amax) == (ref.min, ref.max, tuple(ref.argmin), tuple(ref.argmax)), (r, key)
            n = np.prod(np.subtract(last, first))
            assert abs(s - ref.sum) <= n * 2.0 ** -24 * abs(ref.sum) + 1e-6, (r, key)
            assert abs(var - ref.var) <= 4 * n * 2.0 ** -24 * abs(ref.var) + 1e-7, (r, key)
    for key in res[0][1]:
        first, last = key
        ref = ob.aggregates_range(whole, first, last)
        ref_bins, _ = ob.histogram_range(ob.Volume(vals.view(np.uint32), 7, 0.0, 1.0), first, last, 64)
        for r, out, _, _ in res:
            (mn, mx, amin, amax, s, mean, var), bins = out[key]
            assert (mn, mx, amin, amax) == (ref.min, ref.max, tuple(ref.argmin), tuple(ref.argmax)), (r, key)
            n = np.prod(np.subtract(last, first))
            assert abs(s - ref.sum) <= n * 2.0 ** -24 * 1.25 * n
            assert abs(var - ref.var) <= 4 * n * 2.0 ** -24 * abs(ref.var) + 1e-7
            np.testing.assert_array_equal(bins, ref_bins.astype(np.int64))
    ref_dst = ob.Volume.zeros((2 * gx, 2 * gy, 2 * gz), 7)
    ob.resample(ref_dst, whole, 1)
    halos = 0
    for r, _, (d0, d1, got), halo in res:
        halos += halo
        exp = ref_dst.codes[d0:d1]
        same = (got == exp) | (np.isnan(got.view(np.float32)) & np.isnan(exp.view(np.float32)))
        assert same.all(), f"rank {r}: {int((~same).sum())} voxels differ"
    assert halos > 0    # the Float32 chain needed the neighbour's plane
