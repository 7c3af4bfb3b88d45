"""Z-slab partitioning and halo exchange of volkit_amd.slab with real torch.distributed ranks
(gloo, 127.0.0.1) on the CPU.

Each rank holds only its owned source planes, computes the exchange plan from the exact z
index table (vktHipResampleSlabSourceRange, a host function of libvolkit), and receives the
planes it reads from their owners.  Checks: (1) after the exchange every rank's local buffer
equals the global planes it claims to hold; (2) the oracle's slab resample of the local
buffer (the checker; on the GPU box the HIP kernel does this step, see
tests/test_gpu_large.py) equals the rank's slab of the whole-volume oracle resample -- i.e. the
plan always covers what the dst slab reads, including the float "Linear" chain's z+1 plane.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

CASES = [
    # (world, src dims, dst dims, fmt, filter, chain)
    (2, (16, 12, 8), (32, 24, 16), 5, 1, False),   # 2x, UInt16: reads stay local, no halo
    (2, (16, 12, 8), (32, 24, 16), 7, 1, True),    # 2x, Float32 Linear: one-plane halo
    (3, (10, 9, 37), (7, 6, 64), 4, 0, False),     # non-integer z ratio, uneven slabs
    (3, (10, 9, 37), (7, 6, 64), 7, 1, True),
    (2, (8, 8, 40), (8, 8, 13), 7, 1, True),       # downsampling
    (4, (12, 10, 21), (12, 10, 50), 7, 1, True),   # 4 ranks, uneven slabs, Float32 chain halos
    (8, (8, 6, 16), (16, 12, 32), 7, 1, True),     # 8 ranks (the node's GPU count), 2x
]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, case, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle import binding as ob
        from volkit_amd import slab

        _, sdims, ddims, fmt, fm, chain = case
        sx, sy, sz = sdims
        dx, dy, dz = ddims
        bpv = ob.BPV[fmt]
        rng = np.random.default_rng(1234)          # same global volume on every rank
        if fmt == 7:
            glob_src = rng.uniform(-1, 2, (sz, sy, sx)).astype(np.float32)
            glob_src.reshape(-1)[::97] = np.inf
            glob_src = glob_src.view(np.uint32)
        else:
            glob_src = rng.integers(0, 2 ** (8 * bpv), (sz, sy, sx), dtype=np.uint64).astype(ob.CODE_DTYPE[fmt])

        plan = slab.plan_resample(dz, sz, world, rank, fm, chain)
        l0, l1 = plan.local_src
        local = np.zeros((l1 - l0, sy, sx), dtype=glob_src.dtype)
        o0, o1 = plan.owned_src
        local[o0 - l0:o1 - l0] = glob_src[o0:o1]    # a rank starts with its own planes only
        flat = torch.from_numpy(local.view(np.uint8).reshape(-1))
        pb = sx * sy * bpv

        def planes(g0, g1):
            return flat[(g0 - l0) * pb:(g1 - l0) * pb]

        slab.exchange_planes(plan, planes)
        ok_planes = bool(np.array_equal(local, glob_src[l0:l1]))

        # checker: oracle slab resample of the local buffer vs whole-volume oracle resample
        d0, d1 = plan.dst
        ref = ob.Volume.zeros((dx, dy, dz), fmt)
        ob.resample(ref, ob.Volume(glob_src, fmt), fm)
        ok_vals = True
        if d1 > d0:
            mine = ob.Volume.zeros((dx, dy, d1 - d0), fmt)
            ob.resample_slab(mine, ob.Volume(local, fmt), fm, dz, d0, sz, l0)
            a, b = mine.codes, ref.codes[d0:d1]
            if fmt == 7:
                fa, fb = a.view(np.float32), b.view(np.float32)
                ok_vals = bool(np.array_equal(np.isnan(fa), np.isnan(fb)) and
                               np.array_equal(a[~np.isnan(fb)], b[~np.isnan(fb)]))
            else:
                ok_vals = bool(np.array_equal(a, b))
        q.put((rank, ok_planes, ok_vals, plan.halo_planes))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface worker errors in the parent
        q.put((rank, False, False, repr(e)))


@pytest.mark.parametrize("case", CASES, ids=[f"w{c[0]}-{c[1]}->{c[2]}-fmt{c[3]}-fm{c[4]}" for c in CASES])
def test_slab_exchange_gloo(case):
    world = case[0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok_planes, ok_vals, info in sorted(results, key=lambda r: r[0]):
        assert ok_planes, f"rank {rank}: local source planes differ after exchange ({info})"
        assert ok_vals, f"rank {rank}: slab resample differs from the global resample ({info})"
    halos = [r[3] for r in results]
    if case[5]:
        assert any(h > 0 for h in halos), "float Linear case should exchange at least one halo plane"


def test_plan_partition_covers_volume():
    from volkit_amd import slab
    for world in (1, 2, 3, 4, 8):
        for n in (1, 7, 64, 1000):
            spans = [slab.slab_bounds(n, world, r) for r in range(world)]
            covered = [z for a, b in spans for z in range(a, b)]
            assert covered == list(range(n))


def test_metric_config_needs_no_halo():
    """bench.py's weak-scaling layout (N=8: 1024^3 -> 2048^3, BASELINE config 4), UInt16 ->
    no exchange; every rank owns the same number of dst voxels."""
    import bench
    from volkit_amd import slab
    assert bench.global_dims(1024, 1) == [1024, 1024, 1024]
    assert bench.global_dims(1024, 2) == [2048, 1024, 1024]
    assert bench.global_dims(1024, 4) == [2048, 2048, 1024]
    assert bench.global_dims(1024, 8) == [2048, 2048, 2048]
    for world in (2, 4, 8):
        dx, dy, dz = bench.global_dims(1024, world)
        for rank in range(world):
            p = slab.plan_resample(dz, dz // 2, world, rank, 1, chain=False)
            assert p.recvs == [] and p.sends == []
            z0, z1 = p.dst
            assert dx * dy * (z1 - z0) == 1024 ** 3
            pf = slab.plan_resample(dz, dz // 2, world, rank, 1, chain=True)
            assert pf.halo_planes == (0 if rank == world - 1 else 2)


@pytest.mark.parametrize("world,src,dst,fmt,fm,chain", CASES + [(8, (16, 16, 256), (32, 32, 512), 7, 1, True),
                                                            (8, (16, 16, 128), (32, 32, 2048), 7, 1, True)])
def test_interior_split_reads_only_owned_planes(world, src, dst, fmt, fm, chain):
    """The overlapped slab resample (slab.resample_slab_overlapped) computes dst planes
    [dst0, dk) while the halo is in flight: they must read owned source planes only, dk must be
    the largest such plane, and the boundary [dk, dst1) must read planes of the local buffer."""
    from volkit_amd import slab
    for rank in range(world):
        plan = slab.plan_resample(dst[2], src[2], world, rank, fm, chain)
        d0, d1 = plan.dst
        dk = slab.interior_split(plan, fm, chain)
        assert d0 <= dk <= d1
        if not plan.recvs:
            assert dk == d1
            continue
        o0, o1 = plan.owned_src
        l0, l1 = plan.local_src
        if dk > d0:
            b, e = slab.source_range(dst[2], d0, dk, src[2], fm, chain)
            assert o0 <= b and e <= o1, (rank, dk, b, e)
        if dk < d1:
            b, e = slab.source_range(dst[2], d0, dk + 1, src[2], fm, chain)
            assert b < o0 or e > o1, (rank, "dk is not maximal")
            b, e = slab.source_range(dst[2], dk, d1, src[2], fm, chain)
            assert l0 <= b and e <= l1
