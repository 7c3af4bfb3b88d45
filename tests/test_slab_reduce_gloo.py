"""Z-slab reductions of volkit_amd.slab with real torch.distributed ranks (gloo, 127.0.0.1) on
the CPU: each rank reduces only its owned planes, partials / bin counts are exchanged
(all_gather / all_reduce), and the result must equal the whole-volume oracle: min, max,
argmin, argmax and histogram counts exactly; sum / mean / var within the serial error bound.

The per-slab step here is a numpy restatement of the backend's pass semantics (double
accumulation of the reference's float terms) -- on the GPU box that step is the HIP kernel
(tests/test_reduce.py::test_aggregate_slab_partials_combine_to_the_whole and
tests/test_gpu_multirank.py run it).
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

FLT_MAX = float(np.finfo(np.float32).max)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class NumpySlab:
    """Stands in for a device view: .dimZ plus the host values of the owned planes."""

    def __init__(self, vals):
        self.vals = vals
        self.dimZ = vals.shape[0]


def numpy_pass(view, first, last, z0, pass_no, mean):
    from volkit_amd import _lib
    from volkit_amd._lib import lib
    p = _lib.HipAggregatePartial_t()
    lib.vktHipAggregatePartialInit(C.byref(p))
    box = view.vals[first[2]:last[2], first[1]:last[1], first[0]:last[0]]
    gz, gy, gx = view.vals.shape[0], view.vals.shape[1], view.vals.shape[2]
    zz, yy, xx = np.meshgrid(np.arange(first[2], last[2]) + z0, np.arange(first[1], last[1]),
                             np.arange(first[0], last[0]), indexing="ij")
    gidx = ((zz.astype(np.uint64) * gy + yy) * gx + xx).reshape(-1)
    v = box.reshape(-1)
    if pass_no == 1:
        ok = v < np.float32(FLT_MAX)
        if ok.any():
            m = v[ok].min()
            p.minValue, p.minIndex = float(m), int(gidx[ok][np.argmax(v[ok] == m)])
        ok = v > np.float32(-FLT_MAX)
        if ok.any():
            m = v[ok].max()
            p.maxValue, p.maxIndex = float(m), int(gidx[ok][np.argmax(v[ok] == m)])
        p.sum = float(np.sum(v, dtype=np.float64))
        p.prod = float(np.prod(v, dtype=np.float64))
        p.count = v.size
    else:
        d = (v - np.float32(mean)).astype(np.float32)
        p.sumSq = float(np.sum((d * d).astype(np.float32), dtype=np.float64))
    return p


def numpy_count(view, first, last, bins, num_bins):
    from oracle import binding as ob
    box = np.ascontiguousarray(view.vals[first[2]:last[2], first[1]:last[1], first[0]:last[0]])
    got, _ = ob.histogram_range(ob.Volume(box.view(np.uint32), 7, 0.0, 1.0), (0, 0, 0), box.shape[::-1], num_bins)
    bins.copy_(torch.from_numpy(got.astype(np.int64)))


def _worker(rank, world, port, case, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from volkit_amd import slab
        dims, first, last, nbins = case
        gx, gy, gz = dims
        rng = np.random.default_rng(99)
        vals = rng.uniform(-0.25, 1.25, (gz, gy, gx)).astype(np.float32)
        vals[3, 1, 2] = vals[gz - 1, 0, 0] = np.float32(-0.5)     # tied minima across slabs
        z0, z1 = slab.slab_bounds(gz, world, rank)
        view = NumpySlab(vals[z0:z1])
        agg = slab.aggregates(view, dims, z0, first, last, pass_fn=numpy_pass)
        bins = torch.zeros(nbins, dtype=torch.int64)
        slab.histogram(view, z0, first, last, bins, nbins, count_fn=numpy_count)
        q.put((rank, (agg.min, agg.max, (agg.argmin.x, agg.argmin.y, agg.argmin.z),
                      (agg.argmax.x, agg.argmax.y, agg.argmax.z), agg.sum, agg.mean, agg.var), bins.numpy().copy()))
        dist.destroy_process_group()
    except Exception as e:   # pragma: no cover - reported to the parent
        q.put((rank, repr(e), None))


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", [((12, 9, 10), (0, 0, 0), (12, 9, 10), 16),
                                  ((12, 9, 10), (2, 1, 3), (11, 9, 9), 7)])
def test_slab_reductions_match_whole_volume(world, case):
    from oracle import binding as ob
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r, agg, _ in res:
        assert not isinstance(agg, str), agg
    dims, first, last, nbins = case
    gx, gy, gz = dims
    vals = np.random.default_rng(99).uniform(-0.25, 1.25, (gz, gy, gx)).astype(np.float32)
    vals[3, 1, 2] = vals[gz - 1, 0, 0] = np.float32(-0.5)
    ref = ob.aggregates_range(ob.Volume(vals.view(np.uint32), 7), first, last)
    ref_bins, _ = ob.histogram_range(ob.Volume(vals.view(np.uint32), 7, 0.0, 1.0), first, last, nbins)
    aggs = {r: a for r, a, _ in res}
    assert len(set(aggs.values())) == 1                       # every rank has the same answer
    mn, mx, amin, amax, s, mean, var = aggs[0]
    assert (mn, mx, amin, amax) == (ref.min, ref.max, tuple(ref.argmin), tuple(ref.argmax))
    n = (last[0] - first[0]) * (last[1] - first[1]) * (last[2] - first[2])
    assert abs(s - ref.sum) <= n * 2.0 ** -24 * 1.25 * n + abs(ref.sum) * 1e-6
    assert abs(mean - ref.mean) <= n * 2.0 ** -24 * abs(ref.mean) + 1e-7
    assert abs(var - ref.var) <= 4 * n * 2.0 ** -24 * abs(ref.var) + 1e-7
    for r, _, b in res:
        np.testing.assert_array_equal(b, ref_bins.astype(np.int64))
