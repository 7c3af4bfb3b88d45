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


# ---- UInt8 / UInt16 slabs in one data pass (slab._aggregates_codes) ------------------------------
class NumpyCodeSlab(NumpySlab):
    """A UInt8 / UInt16 slab: .codes (z, y, x), .vals their oracle-decoded float32 values (for the
    two-pass fallback), and the view fields the code-count form reads."""

    def __init__(self, codes, fmt, lo, hi, values):
        super().__init__(values)
        self.codes = codes
        self.dataFormat, self.mappingLo, self.mappingHi = fmt, lo, hi


def code_values(fmt, lo, hi, ncodes):
    from oracle import binding as ob
    return np.array([ob.unmap_voxel(int(c).to_bytes(ob.BPV[fmt], "little"), fmt, lo, hi) for c in range(ncodes)],
                    dtype=np.float32)


class NumpyCodeFns:
    """numpy restatement of the three GPU steps (vktHipAggregateCodeCounts, vktHipAggregatesFrom-
    Codes -- aggregatesCodesFinalKernel's float terms --, vktHipAggregateFirstCodes)."""

    @staticmethod
    def supported(view, first, last):
        return True

    @staticmethod
    def count(view, first, last, counts):
        box = view.codes[first[2]:last[2], first[1]:last[1], first[0]:last[0]]
        counts.copy_(torch.from_numpy(np.bincount(box.reshape(-1).astype(np.int64), minlength=counts.numel())))

    @staticmethod
    def from_codes(counts, fmt, lo, hi, n):
        from volkit_amd import _lib
        from volkit_amd._lib import lib
        cnt = counts.numpy().astype(np.float64)
        v = code_values(fmt, lo, hi, cnt.size)
        present = cnt > 0
        p1, p2 = _lib.HipAggregatePartial_t(), _lib.HipAggregatePartial_t()
        lib.vktHipAggregatePartialInit(C.byref(p1))
        lib.vktHipAggregatePartialInit(C.byref(p2))
        vp, cp = v[present], cnt[present]
        p1.sum = float(np.sum(cp * vp.astype(np.float64)))
        p1.prod = float(np.prod(vp.astype(np.float64) ** cp))
        p1.count = int(cp.sum())
        p1.minValue, p1.maxValue = float(vp.min()), float(vp.max())
        mean = np.float32(np.float64(np.float32(p1.sum)) / n)
        d = (vp - mean).astype(np.float32)
        p2.sumSq = float(np.sum(cp * (d * d).astype(np.float32).astype(np.float64)))
        codes = np.nonzero(present)[0]
        lo_c, hi_c = codes[vp == vp.min()], codes[vp == vp.max()]
        ok = len(lo_c) == 1 and len(hi_c) == 1 and np.all(np.abs(vp) < np.float32(FLT_MAX))
        return p1, p2, ((int(lo_c[0]), int(hi_c[0])) if ok else (-1, -1))

    @staticmethod
    def first_codes(view, first, last, z0, cmin, cmax):
        box = view.codes[first[2]:last[2], first[1]:last[1], first[0]:last[0]]
        gy, gx = view.codes.shape[1], view.codes.shape[2]
        out = []
        for c in (cmin, cmax):
            hits = np.argwhere(box == c)   # z, y, x in row-major (serial) order
            if len(hits) == 0:
                out.append((1 << 64) - 1)
            else:
                z, y, x = hits[0]
                out.append(int(((z + first[2] + z0) * gy + (y + first[1])) * gx + (x + first[0])))
        return tuple(out)


def _codes_volume(fmt, dims):
    gx, gy, gz = dims
    top = 255 if fmt == 4 else 65535
    rng = np.random.default_rng(7 + fmt)
    codes = rng.integers(3, top - 2, (gz, gy, gx)).astype(np.uint8 if fmt == 4 else np.uint16)
    codes[2, 1, 3] = codes[gz - 2, 0, 1] = 1           # tied minima in different slabs
    codes[gz - 1, gy - 1, gx - 1] = codes[5, 4, 4] = top - 1
    return codes


def _codes_worker(rank, world, port, case, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from volkit_amd import slab
        fmt, (lo, hi), dims, first, last = case
        codes = _codes_volume(fmt, dims)
        vals = code_values(fmt, lo, hi, 256 if fmt == 4 else 65536)[codes.astype(np.int64)]
        z0, z1 = slab.slab_bounds(dims[2], world, rank)
        view = NumpyCodeSlab(codes[z0:z1], fmt, lo, hi, vals[z0:z1])
        agg = slab.aggregates(view, dims, z0, first, last, pass_fn=numpy_pass, code_fns=NumpyCodeFns)
        q.put((rank, (agg.min, agg.max, (agg.argmin.x, agg.argmin.y, agg.argmin.z),
                      (agg.argmax.x, agg.argmax.y, agg.argmax.z), agg.sum, agg.mean, agg.var)))
        dist.destroy_process_group()
    except Exception:   # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", [(4, (0.0, 1.0), (12, 9, 10), (0, 0, 0), (12, 9, 10)),
                                  (4, (3.0, -1.0), (12, 9, 10), (2, 1, 3), (11, 9, 9)),
                                  (5, (-1.0, 3.0), (12, 9, 10), (1, 0, 1), (12, 8, 10)),
                                  (4, (0.25, 0.25), (12, 9, 10), (0, 0, 0), (12, 9, 10))])   # -> two passes
def test_slab_code_count_aggregates(world, case):
    """slab.aggregates on UInt8 / UInt16 slabs: local code counts, one all_reduce(SUM), the
    aggregates from the global counts, first-occurrence search per slab + all_reduce(MIN) of the
    indices == the whole-volume oracle (a constant mapping falls back to the two passes)."""
    from oracle import binding as ob
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_codes_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r, agg in res:
        assert not isinstance(agg, str), agg
    fmt, (lo, hi), dims, first, last = case
    codes = _codes_volume(fmt, dims)
    ref = ob.aggregates_range(ob.Volume(codes, fmt, lo, hi), first, last)
    aggs = {r: a for r, a in res}
    assert len(set(aggs.values())) == 1
    mn, mx, amin, amax, s, mean, var = aggs[0]
    assert (mn, mx, amin, amax) == (ref.min, ref.max, tuple(ref.argmin), tuple(ref.argmax))
    n = (last[0] - first[0]) * (last[1] - first[1]) * (last[2] - first[2])
    assert abs(s - ref.sum) <= n * 2.0 ** -24 * abs(ref.sum) + 1e-6
    assert abs(mean - ref.mean) <= n * 2.0 ** -24 * abs(ref.mean) + 1e-7
    assert abs(var - ref.var) <= 4 * n * 2.0 ** -24 * abs(ref.var) + 1e-7


# ---- UInt16 / Float32 slabs in one pass of moments (slab._aggregates_moments) --------------------
class NumpyMomentFns:
    """numpy restatement of the per-rank step vktHipAggregateMoments (aggregatesMomentsU16Kernel /
    aggregatesMomentsFKernel + their combine): form 1 exact integer sums of the UInt16 codes under the
    unit mapping, form 2 the mean and the sum of squared deviations of the values (float64), min / max
    with first-occurrence global indices; the combine across ranks and the finish are the library's
    own host code (vktHipAggregatesFromMoments)."""

    @staticmethod
    def supported(view, first, last):
        return True

    @staticmethod
    def moments(view, first, last, z0):
        from volkit_amd import _lib
        p = _lib.HipMomentPartial_t()
        unit = view.dataFormat == 5 and view.mappingLo == 0.0 and view.mappingHi == 1.0 \
            and np.copysign(1.0, view.mappingLo) > 0
        p.form = 1 if unit else 2
        p.prod, p.minValue, p.maxValue = 1.0, FLT_MAX, -FLT_MAX
        p.minIndex = p.maxIndex = (1 << 64) - 1
        if first == last or any(a >= b for a, b in zip(first, last)):
            return p
        box = view.vals[first[2]:last[2], first[1]:last[1], first[0]:last[0]]
        v = box.reshape(-1)
        gy, gx = view.vals.shape[1], view.vals.shape[2]
        zz, yy, xx = np.meshgrid(np.arange(first[2], last[2]) + z0, np.arange(first[1], last[1]),
                                 np.arange(first[0], last[0]), indexing="ij")
        gidx = ((zz.astype(np.uint64) * gy + yy) * gx + xx).reshape(-1)
        p.count = v.size
        m = v.min()
        p.minValue, p.minIndex = float(m), int(gidx[np.argmax(v == m)])
        m = v.max()
        p.maxValue, p.maxIndex = float(m), int(gidx[np.argmax(v == m)])
        p.prod = float(np.prod(v.astype(np.float64)))
        if unit:
            c = view.codes[first[2]:last[2], first[1]:last[1], first[0]:last[0]].reshape(-1).astype(object)
            s2 = int(sum(int(x) * int(x) for x in c))
            p.codeSum = int(sum(int(x) for x in c))
            p.codeSumSqLo, p.codeSumSqHi = s2 & ((1 << 64) - 1), s2 >> 64
        else:
            d = v.astype(np.float64)
            p.mean = float(d.mean())
            p.m2 = float(np.sum((d - p.mean) ** 2))
            p.sum = float(np.sum(d))
            a = np.abs(v)
            p.flags = (1 if not np.all(np.isfinite(v)) else 0) | (2 if np.any((a < 2.0 ** -40) & (a != 0)) else 0)
        return p


def _moments_worker(rank, world, port, case, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from volkit_amd import slab
        fmt, (lo, hi), dims, first, last = case
        gx, gy, gz = dims
        if fmt == 7:
            codes = np.random.default_rng(5).uniform(-2.0, 3.0, (gz, gy, gx)).astype(np.float32)
            codes[2, 1, 3] = codes[gz - 2, 0, 1] = -2.5
            vals = codes
        else:
            codes = _codes_volume(fmt, dims)
            vals = code_values(fmt, lo, hi, 65536)[codes.astype(np.int64)]
        z0, z1 = slab.slab_bounds(gz, world, rank)
        view = NumpyCodeSlab(codes[z0:z1], fmt, lo, hi, vals[z0:z1])
        agg = slab.aggregates(view, dims, z0, first, last, pass_fn=numpy_pass, moment_fns=NumpyMomentFns)
        q.put((rank, (agg.min, agg.max, (agg.argmin.x, agg.argmin.y, agg.argmin.z),
                      (agg.argmax.x, agg.argmax.y, agg.argmax.z), agg.sum, agg.mean, agg.var)))
        dist.destroy_process_group()
    except Exception:   # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", [(5, (0.0, 1.0), (12, 9, 10), (0, 0, 0), (12, 9, 10)),     # integer form
                                  (5, (0.0, 1.0), (12, 9, 10), (2, 1, 3), (11, 9, 9)),
                                  (5, (-1.0, 3.0), (12, 9, 10), (1, 0, 1), (12, 8, 10)),    # float form
                                  (7, (0.0, 1.0), (12, 9, 10), (0, 0, 0), (12, 9, 10)),
                                  (7, (0.0, 1.0), (12, 9, 10), (3, 0, 8), (9, 9, 10))])     # a rank with none
def test_slab_moment_aggregates(world, case):
    """slab.aggregates on UInt16 / Float32 slabs: per-rank moment partials, ONE all_gather, the
    library's in-order combine and finish (vktHipAggregatesFromMoments, host code) == the
    whole-volume oracle; var within the moments bound of tests/test_reduce.py."""
    from oracle import binding as ob
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_moments_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r, agg in res:
        assert not isinstance(agg, str), agg
    fmt, (lo, hi), dims, first, last = case
    gx, gy, gz = dims
    if fmt == 7:
        codes = np.random.default_rng(5).uniform(-2.0, 3.0, (gz, gy, gx)).astype(np.float32)
        codes[2, 1, 3] = codes[gz - 2, 0, 1] = -2.5
        ref = ob.aggregates_range(ob.Volume(codes.view(np.uint32), 7), first, last)
        vals = codes
    else:
        codes = _codes_volume(fmt, dims)
        ref = ob.aggregates_range(ob.Volume(codes, fmt, lo, hi), first, last)
        vals = code_values(fmt, lo, hi, 65536)[codes.astype(np.int64)]
    aggs = {r: a for r, a in res}
    assert len(set(aggs.values())) == 1
    mn, mx, amin, amax, s, mean, var = aggs[0]
    assert (mn, mx, amin, amax) == (ref.min, ref.max, tuple(ref.argmin), tuple(ref.argmax))
    box = vals[first[2]:last[2], first[1]:last[1], first[0]:last[0]].reshape(-1)
    n, nall = box.size, codes.size
    assert abs(s - ref.sum) <= n * 2.0 ** -24 * float(np.sum(np.abs(box), dtype=np.float64)) + 1e-6
    assert mean == np.float32(np.float64(np.float32(s)) / nall)
    d = (box - np.float32(mean)).astype(np.float32)
    var_terms = float(np.float32(np.float64(np.float32(np.sum((d * d).astype(np.float32), dtype=np.float64))) / nall))
    ulp = float(np.spacing(np.float32(var_terms)))
    assert abs(var - var_terms) <= 3 * 2.0 ** -24 * var_terms + 2 * ulp, (var, var_terms)
