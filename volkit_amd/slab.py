"""Z-slab partitioning of StructuredVolumes across one process per GPU.

The reference is single-device (no NCCL/MPI anywhere).  Its nearest
analogue is BrickDecompose with halos (reference include/cpp/vkt/Decompose.hpp:16-50).  This
module adds the multi-GPU layout the north star asks for:

* every rank owns the contiguous global z-planes [z0, z1) of each volume (ceil partition);
* pointwise ops (Fill, Copy, the ten arithmetic ops) are independent per plane: each rank
  runs them on its own slab, no communication;
* Resample reads source planes through the exact z index table; the planes a rank's dst slab
  reads that another rank owns are exchanged point-to-point (torch.distributed isend/irecv:
  RCCL over xGMI with the "nccl" backend, gloo on CPU).  For integer formats (and any Nearest
  resample) with slab-aligned ratios the reads stay inside the own slab and nothing moves;
  the float "Linear" chain reads the z+1 neighbour plane, i.e. a one-plane halo.

Local compute always goes through the HIP backend (include/volkit_hip.h: vktHipResampleSlab,
vktHipArithmeticRange, ...).  The exchange functions only move bytes and work on any tensors
(CPU tensors with gloo, device tensors with RCCL), which is what the CPU tests exercise.
"""
from __future__ import annotations

import contextlib
import ctypes as C
from dataclasses import dataclass, field
from typing import Callable, List, Tuple

from . import _lib
from ._lib import lib


def slab_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Planes [z0, z1) owned by `rank` (ceil partition; trailing ranks may be empty)."""
    size = -(-n // world)
    z0 = min(rank * size, n)
    return z0, min(z0 + size, n)


def source_range(dst_gdz: int, dz0: int, dz1: int, src_gdz: int, filter_mode: int, chain: bool) -> Tuple[int, int]:
    """Global source planes [s0, s1) that dst planes [dz0, dz1) read (exact index table)."""
    b, e = C.c_int32(), C.c_int32()
    err = lib.vktHipResampleSlabSourceRange(dst_gdz, dz0, dz1, src_gdz, filter_mode, 1 if chain else 0,
                                            C.byref(b), C.byref(e))
    if err != 0:
        raise RuntimeError(_lib.last_error())
    return b.value, e.value


@dataclass
class ResamplePlan:
    world: int
    rank: int
    dst_gdz: int
    src_gdz: int
    dst: Tuple[int, int]                 # owned dst planes
    owned_src: Tuple[int, int]           # owned source planes
    local_src: Tuple[int, int]           # planes held in the local source buffer (owned + halo)
    recvs: List[Tuple[int, int, int]] = field(default_factory=list)   # (peer, g0, g1)
    sends: List[Tuple[int, int, int]] = field(default_factory=list)   # (peer, g0, g1)
    filter_mode: int = 0                 # the filter and chain the plan's source ranges assume
    chain: bool = False

    def check(self, filter_mode, chain) -> Tuple[int, bool]:
        """The plan's (filter_mode, chain), or ValueError when a caller passes others: the
        source sub-views would then miss the z+1 neighbour planes the chain reads."""
        fm = self.filter_mode if filter_mode is None else filter_mode
        ch = self.chain if chain is None else bool(chain)
        if fm != self.filter_mode or ch != self.chain:
            raise ValueError(f"plan made for filter_mode={self.filter_mode}, chain={self.chain}; "
                             f"called with filter_mode={fm}, chain={ch}")
        return fm, ch

    @property
    def halo_planes(self) -> int:
        return sum(g1 - g0 for _, g0, g1 in self.recvs)


def plan_resample(dst_gdz: int, src_gdz: int, world: int, rank: int, filter_mode: int, chain: bool) -> ResamplePlan:
    """Every rank computes the same global plan; sends are the peers' needs we own."""
    needs = []
    for r in range(world):
        d0, d1 = slab_bounds(dst_gdz, world, r)
        needs.append(source_range(dst_gdz, d0, d1, src_gdz, filter_mode, chain) if d1 > d0 else (0, 0))
    owned = [slab_bounds(src_gdz, world, r) for r in range(world)]

    def intersect(a, b):
        lo, hi = max(a[0], b[0]), min(a[1], b[1])
        return (lo, hi) if hi > lo else None

    o = owned[rank]
    n = needs[rank]
    lo = min(o[0], n[0]) if n[1] > n[0] else o[0]
    hi = max(o[1], n[1]) if n[1] > n[0] else o[1]
    plan = ResamplePlan(world, rank, dst_gdz, src_gdz, slab_bounds(dst_gdz, world, rank), o, (lo, hi),
                        filter_mode=filter_mode, chain=bool(chain))
    for peer in range(world):
        if peer == rank:
            continue
        got = intersect(n, owned[peer]) if n[1] > n[0] else None
        if got:
            plan.recvs.append((peer, got[0], got[1]))
        give = intersect(needs[peer], o) if needs[peer][1] > needs[peer][0] else None
        if give:
            plan.sends.append((peer, give[0], give[1]))
    return plan


@contextlib.contextmanager
def library_stream(enabled: bool = True):
    """Make the library's compute stream (vktHipGetComputeStream) torch's current stream for the
    block.  torch.distributed orders a nccl (RCCL) isend/irecv after the work queued on torch's
    current stream and a later wait() makes the current stream wait for it; the library's
    kernels run on its compute stream.  Inside this block the two are one stream, so a send
    sees the kernels that produced its planes and a kernel enqueued after finish_exchange sees
    the received planes, whatever stream the caller had current.  No-op when disabled (host
    tensors, gloo on CPU)."""
    if not enabled:
        yield
        return
    import torch
    s = C.c_void_p()
    if lib.vktHipGetComputeStream(C.byref(s)) != 0:
        raise RuntimeError(_lib.last_error())
    with torch.cuda.stream(torch.cuda.ExternalStream(s.value or 0)):
        yield


def start_exchange(plan: ResamplePlan, planes: Callable[[int, int], "torch.Tensor"], group=None):
    """Issue the halo exchange (one batched isend/irecv round) without waiting for it; returns
    the pending round for finish_exchange.  `planes(g0, g1)` returns a writable uint8 tensor
    view of global source planes [g0, g1) in the local buffer.

    With the nccl backend (RCCL over xGMI) device planes move device to device on RCCL's own
    stream, which starts after the work already queued on torch's current stream; kernels
    enqueued on that stream before finish_exchange run concurrently with the transfer.  Call it
    inside library_stream() (resample_slab_overlapped does) so that stream is the library's.  gloo
    moves host tensors only, so device planes are staged through host copies there (CPU tests,
    1-GPU rehearsals)."""
    import torch.distributed as dist

    staged = dist.get_backend(group) == "gloo"
    ops, landing = [], []
    for peer, g0, g1 in plan.sends:
        t = planes(g0, g1).contiguous()
        ops.append(dist.P2POp(dist.isend, t.cpu() if staged and t.is_cuda else t, peer, group))
    for peer, g0, g1 in plan.recvs:
        t = planes(g0, g1)
        if staged and t.is_cuda:
            host = t.new_empty(t.shape, device="cpu")
            landing.append((t, host))
            t = host
        ops.append(dist.P2POp(dist.irecv, t, peer, group))
    return (dist.batch_isend_irecv(ops) if ops else [], landing)


_EXCHANGE_TIMEOUT_S = None


def set_exchange_timeout(seconds) -> None:
    """Bound every wait of an exchange round (finish_exchange, the Range calls' moves) to
    `seconds` (None: the backend's default -- the process group's timeout for gloo; a
    stream-ordered wait for nccl).  A peer that never joins its side of a round then raises
    RuntimeError on the waiting rank instead of hanging it (SURVEY §5 failure detection; with
    nccl the wait also blocks the host until the receives land or the deadline passes)."""
    global _EXCHANGE_TIMEOUT_S
    _EXCHANGE_TIMEOUT_S = None if seconds is None else float(seconds)


def _wait(req) -> None:
    if _EXCHANGE_TIMEOUT_S is None:
        req.wait()
        return
    import datetime
    try:
        ok = req.wait(datetime.timedelta(seconds=_EXCHANGE_TIMEOUT_S))
    except RuntimeError as e:
        raise RuntimeError(f"slab exchange: a peer did not complete its side within {_EXCHANGE_TIMEOUT_S} s: "
                           f"{e}") from e
    if ok is False:
        raise RuntimeError(f"slab exchange: a peer did not complete its side within {_EXCHANGE_TIMEOUT_S} s")


def finish_exchange(pending) -> None:
    """Wait for a round from start_exchange: with RCCL the current stream waits for the
    receives (the host does not block unless set_exchange_timeout bounds the wait), so a kernel
    enqueued next reads the halo."""
    reqs, landing = pending
    for req in reqs:
        _wait(req)
    for dev, host in landing:
        dev.copy_(host)


def exchange_planes(plan: ResamplePlan, planes: Callable[[int, int], "torch.Tensor"], group=None) -> None:
    """Point-to-point halo exchange, issued and waited for (start_exchange + finish_exchange)."""
    finish_exchange(start_exchange(plan, planes, group))


def interior_split(plan: ResamplePlan, filter_mode: int = None, chain: bool = None) -> int:
    """dk such that dst planes [dst0, dk) read only source planes this rank owns (the interior:
    computable while the halo is in flight) and [dk, dst1) read the halo.  dst0 when even the
    first plane needs a received one; dst1 when nothing is received.  filter_mode / chain
    default to the plan's (others raise ValueError)."""
    filter_mode, chain = plan.check(filter_mode, chain)
    d0, d1 = plan.dst
    o0, o1 = plan.owned_src
    if d1 <= d0 or not plan.recvs:
        return d1

    def owned(dk):
        b, e = source_range(plan.dst_gdz, d0, dk, plan.src_gdz, filter_mode, chain)
        return b >= o0 and e <= o1

    lo, hi = d0, d1          # owned(lo) holds trivially for the empty range; find the largest
    while lo < hi:
        mid = (lo + hi + 1) // 2
        if owned(mid):
            lo = mid
        else:
            hi = mid - 1
    return lo


_BYTES_PER_VOXEL = {1: 1, 2: 2, 3: 4, 4: 1, 5: 2, 6: 4, 7: 4}   # DataFormat Int8 .. Float32


def sub_view(view, g0: int, g1: int, z0: int):
    """View of global planes [g0, g1) of a slab view whose first plane is global plane z0."""
    plane = view.dimX * view.dimY * _BYTES_PER_VOXEL[view.dataFormat]
    v = _lib.HipVolumeView_t.from_buffer_copy(view)
    v.data = (view.data or 0) + (g0 - z0) * plane
    v.dimZ = g1 - g0
    return v


def resample_slab_overlapped(dst_view, src_view, filter_mode: int, plan: ResamplePlan, chain: bool,
                             planes: Callable[[int, int], "torch.Tensor"], group=None,
                             on_library_stream: bool = True) -> int:
    """Halo exchange overlapped with the interior: issue the exchange, resample the dst planes
    that read only owned source planes (source sub-view of exactly those planes, so nothing
    touches the planes in flight), wait for the receives on the stream, then resample the
    boundary planes from the source planes they read.  Each call is a slab resample of its own
    (the same exact index tables), so the result equals resample_slab's.  The exchange runs with
    the library's compute stream as torch's current stream (library_stream; pass
    on_library_stream=False only for host-tensor planes)."""
    filter_mode, chain = plan.check(filter_mode, chain)
    d0, d1 = plan.dst
    ls0 = plan.local_src[0]
    if not plan.recvs and not plan.sends:
        return resample_slab(dst_view, src_view, filter_mode, plan)
    with library_stream(on_library_stream):
        pending = start_exchange(plan, planes, group)
        dk = interior_split(plan, filter_mode, chain)
        err = 0
        for a, b, wait in ((d0, dk, False), (dk, d1, True)):
            if wait:
                finish_exchange(pending)
            if b <= a or err:
                continue
            s0, s1 = source_range(plan.dst_gdz, a, b, plan.src_gdz, filter_mode, chain)
            err = lib.vktHipResampleSlab(sub_view(dst_view, a, b, d0), sub_view(src_view, s0, s1, ls0), filter_mode,
                                         plan.dst_gdz, a, plan.src_gdz, s0)
    return err


class DeviceBytes:
    """Zero-copy torch view of a device allocation (via __cuda_array_interface__)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 3, "strides": None}


def device_tensor(ptr: int, nbytes: int):
    import torch
    return torch.as_tensor(DeviceBytes(ptr, nbytes), device="cuda")


def resample_slab(dst_view, src_view, filter_mode: int, plan: ResamplePlan) -> int:
    """Run the HIP slab resample for this rank (views from StructuredVolume.hip_view())."""
    return lib.vktHipResampleSlab(dst_view, src_view, filter_mode, plan.dst_gdz, plan.dst[0], plan.src_gdz,
                                  plan.local_src[0])


# ---- Range calls over Z-slabs (ranges intersected with each slab, planes a
#      dstOffset.z or a clamped halo moves across slab boundaries sent to their owner) --------------
FILL, COPY, ARITHMETIC = 0, 1, 2


@dataclass
class Slab:
    """One rank's part of a Z-slab partitioned volume (include/volkit_hip.h vktHipSlab_t):
    `view` (HipVolumeView_t, X/Y dims global) holds global planes [z0, z0 + view.dimZ), which
    include the planes the rank owns in the ceil partition of global_dim_z planes.  `tensor`
    (optional) is a flat uint8 tensor over the view's bytes -- host memory for gloo on CPU;
    by default a zero-copy device tensor over view.data."""
    view: object
    z0: int
    global_dim_z: int
    tensor: object = None

    def c(self):
        return _lib.HipSlab_t(self.view, self.z0, self.global_dim_z)

    @property
    def plane_bytes(self) -> int:
        return self.view.dimX * self.view.dimY * _BYTES_PER_VOXEL[self.view.dataFormat]

    def flat(self):
        if self.tensor is None:
            self.tensor = device_tensor(self.view.data, self.plane_bytes * self.view.dimZ)
        return self.tensor

    def planes(self, g0: int, g1: int):
        """uint8 tensor view of global planes [g0, g1) of this slab."""
        if g0 < self.z0 or g1 > self.z0 + self.view.dimZ:
            raise ValueError(f"slab holds planes [{self.z0}, {self.z0 + self.view.dimZ}), not [{g0}, {g1})")
        pb = self.plane_bytes
        return self.flat()[(g0 - self.z0) * pb:(g1 - self.z0) * pb]


def range_plan(kind: int, world: int, rank: int, dst_gdz: int, src1_gdz: int, src2_gdz: int, first, last,
               dst_offset=(0, 0, 0)):
    """The C plan (vktHipSlabRangePlan): this rank's pieces, its moves in the global order, and
    the plane counts of its two gather buffers."""
    args = [kind, world, rank, dst_gdz, src1_gdz, src2_gdz, _lib.Vec3i_t(*first), _lib.Vec3i_t(*last),
            _lib.Vec3i_t(*dst_offset)]
    n, m, bp = C.c_int32(), C.c_int32(), (C.c_int32 * 2)()
    if lib.vktHipSlabRangePlan(*args, None, 0, C.byref(n), None, 0, C.byref(m), bp) != 0:
        raise RuntimeError(_lib.last_error())
    pieces, moves = (_lib.HipSlabPiece_t * max(n.value, 1))(), (_lib.HipSlabMove_t * max(m.value, 1))()
    if lib.vktHipSlabRangePlan(*args, pieces, n.value, C.byref(n), moves, m.value, C.byref(m), bp) != 0:
        raise RuntimeError(_lib.last_error())
    return list(pieces[:n.value]), list(moves[:m.value]), (bp[0], bp[1])


def _world_rank(group):
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def _gpu_pieces(kind, op, world, rank, dst, srcs, first, last, off, value, bufs):
    s1 = C.byref(srcs[0].c()) if len(srcs) > 0 else None
    s2 = C.byref(srcs[1].c()) if len(srcs) > 1 else None
    g = [b.data_ptr() if b is not None else None for b in bufs]
    return lib.vktHipSlabRangePieces(kind, op, world, rank, dst.c(), s1, s2, _lib.Vec3i_t(*first),
                                     _lib.Vec3i_t(*last), _lib.Vec3i_t(*off), C.c_float(value), g[0], g[1])


def _range(kind, op, dst: Slab, srcs, first, last, off, value, group, run_pieces):
    import torch
    import torch.distributed as dist

    world, rank = _world_rank(group)
    gz = [s.global_dim_z for s in srcs] + [0, 0]
    pieces, moves, bp = range_plan(kind, world, rank, dst.global_dim_z, gz[0], gz[1], first, last, off)
    tensors = [dst.flat()] + [s.flat() for s in srcs]
    on_gpu = any(t.is_cuda for t in tensors)
    bufs = [None, None]
    with library_stream(on_gpu):
        # gather buffers allocated on the library's stream: torch returns their blocks to that
        # stream, so no later user reuses them while the library's kernels still read them
        for k, s in enumerate(srcs):
            if bp[k]:
                bufs[k] = torch.empty(bp[k] * s.plane_bytes, dtype=torch.uint8, device=s.flat().device)
        if moves:
            staged = dist.get_backend(group) == "gloo"
            ops, landing = [], []
            for m in moves:
                s = srcs[m.source]
                if m.send:
                    t = s.planes(m.z0, m.z1).contiguous()
                    ops.append(dist.P2POp(dist.isend, t.cpu() if staged and t.is_cuda else t, m.peer, group))
                else:
                    pb = s.plane_bytes
                    t = bufs[m.source][m.bufPlane * pb:(m.bufPlane + m.z1 - m.z0) * pb]
                    if staged and t.is_cuda:
                        host = t.new_empty(t.shape, device="cpu")
                        landing.append((t, host))
                        t = host
                    ops.append(dist.P2POp(dist.irecv, t, m.peer, group))
            finish_exchange((dist.batch_isend_irecv(ops), landing))
        err = (run_pieces or _gpu_pieces)(kind, op, world, rank, dst, srcs, first, last, off, value, bufs)
    if err:
        raise RuntimeError(_lib.last_error() if err != 0 else "slab range failed")
    return 0


def fill_range(dst: Slab, first, last, value: float, group=None, run_pieces=None) -> int:
    """FillRange over a Z-slab partitioned volume (global first/last): each rank fills the
    owned planes of the range; nothing moves."""
    return _range(FILL, 0, dst, [], first, last, (0, 0, 0), value, group, run_pieces)


def copy_range(dst: Slab, src: Slab, first, last, dst_offset=(0, 0, 0), group=None, run_pieces=None) -> int:
    """CopyRange over Z-slabs (global first/last/dstOffset, source clamped to the global volume,
    Copy_serial.hpp:38-47): the source planes a rank's dst planes read that other ranks own move
    to it (one batched isend/irecv round), then the local pieces run."""
    return _range(COPY, 0, dst, [src], first, last, dst_offset, 0.0, group, run_pieces)


def arithmetic_range(op, dst: Slab, s1: Slab, s2: Slab, first, last, dst_offset=(0, 0, 0), group=None,
                     run_pieces=None) -> int:
    """{Sum, ..., SafeAbsDiff}Range over Z-slabs (absolute-x reads, dst[x + dstOffset] writes,
    Arithmetic_serial.hpp:25-41); `op` is an index or a name of _lib.ARITH_OPS."""
    code = _lib.ARITH_OPS.index(op) if isinstance(op, str) else int(op)
    return _range(ARITHMETIC, code, dst, [s1, s2], first, last, dst_offset, 0.0, group, run_pieces)


def transform_range(dst: Slab, first, last, fn, group=None) -> int:
    """TransformRange with a host callback over Z-slabs (Transform shards with no exchange):
    each rank runs fn(x, y, z, VoxelView) over the owned planes of the global range, z global
    (vktHipSlabTransformRange1; Transform_serial.hpp:15-48 per slab)."""
    from .volkit import VoxelView
    world, rank = _world_rank(group)
    cb = _lib.UnaryOp(lambda x, y, z, v: fn(x, y, z, VoxelView(v)))
    if lib.vktHipSlabTransformRange1(world, rank, dst.c(), _lib.Vec3i_t(*first), _lib.Vec3i_t(*last), cb) != 0:
        raise RuntimeError(_lib.last_error())
    return 0


# ---- reductions over Z-slabs (the first all-reduce users) -------------------
PARTIAL_BYTES = C.sizeof(_lib.HipAggregatePartial_t)


def slab_range(first, last, z0: int, z1: int):
    """Intersect the global range [first, last) with the owned planes [z0, z1): local
    (first, last) of this slab's buffer, or None when the slab holds none of it."""
    lo, hi = max(first[2], z0), min(last[2], z1)
    if hi <= lo or last[0] <= first[0] or last[1] <= first[1]:
        return None
    return (first[0], first[1], lo - z0), (last[0], last[1], hi - z0)


def _gpu_pass(view, first, last, z0, pass_no, mean):
    p = _lib.HipAggregatePartial_t()
    err = lib.vktHipAggregatesPass(view, _lib.Vec3i_t(*first), _lib.Vec3i_t(*last), z0, pass_no, C.c_float(mean),
                                   C.byref(p))
    if err != 0:
        raise RuntimeError(_lib.last_error())
    return p


def _allgather_partials(p, group=None, device=None):
    """Every rank's partial (a ctypes structure), in rank order (one all_gather of its bytes per
    rank; on a device tensor for nccl, a host tensor for gloo)."""
    import torch
    import torch.distributed as dist

    mine = torch.frombuffer(bytearray(bytes(p)), dtype=torch.uint8)
    if device is not None and dist.get_backend(group) != "gloo":
        mine = mine.to(device)
    world = dist.get_world_size(group)
    out = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(out, mine, group=group)
    return [type(p).from_buffer_copy(bytes(t.cpu().numpy())) for t in out]


def combine_partials(parts):
    acc = _lib.HipAggregatePartial_t()
    lib.vktHipAggregatePartialInit(C.byref(acc))
    for p in parts:
        lib.vktHipAggregatePartialCombine(C.byref(acc), C.byref(p))
    return acc


def _all_reduce(t, op, group=None):
    """all_reduce of a (device or host) tensor; gloo reduces a host copy of a device tensor."""
    import torch.distributed as dist
    if t.is_cuda and dist.get_backend(group) == "gloo":
        host = t.cpu()
        dist.all_reduce(host, op=op, group=group)
        t.copy_(host)
    else:
        dist.all_reduce(t, op=op, group=group)
    return t


NO_INDEX = (1 << 64) - 1
_I64_MAX = (1 << 63) - 1


class GpuCodeFns:
    """The code-count form's per-rank steps on the GPU (include/volkit_hip.h)."""

    @staticmethod
    def supported(view, first, last) -> bool:
        return bool(lib.vktHipAggregateCodesSupported(view, _lib.Vec3i_t(*first), _lib.Vec3i_t(*last)))

    @staticmethod
    def count(view, first, last, counts) -> None:
        if lib.vktHipAggregateCodeCounts(view, _lib.Vec3i_t(*first), _lib.Vec3i_t(*last),
                                         C.c_void_p(counts.data_ptr())) != 0:
            raise RuntimeError(_lib.last_error())

    @staticmethod
    def from_codes(counts, fmt, lo, hi, n):
        p1, p2, codes = _lib.HipAggregatePartial_t(), _lib.HipAggregatePartial_t(), (C.c_int32 * 2)()
        if lib.vktHipAggregatesFromCodes(C.c_void_p(counts.data_ptr()), fmt, C.c_float(lo), C.c_float(hi), n,
                                         C.byref(p1), C.byref(p2), codes) != 0:
            raise RuntimeError(_lib.last_error())
        return p1, p2, (codes[0], codes[1])

    @staticmethod
    def first_codes(view, first, last, z0, cmin, cmax):
        idx = (C.c_uint64 * 2)()
        if lib.vktHipAggregateFirstCodes(view, _lib.Vec3i_t(*first), _lib.Vec3i_t(*last), z0, cmin, cmax, idx) != 0:
            raise RuntimeError(_lib.last_error())
        return idx[0], idx[1]


class GpuMomentFns:
    """The moments form's per-rank steps on the GPU (include/volkit_hip.h vktHipAggregateMoments)."""

    @staticmethod
    def supported(view, first, last) -> bool:
        return bool(lib.vktHipAggregateMomentsSupported(view, _lib.Vec3i_t(*first), _lib.Vec3i_t(*last)))

    @staticmethod
    def moments(view, first, last, z0):
        p = _lib.HipMomentPartial_t()
        if lib.vktHipAggregateMoments(view, _lib.Vec3i_t(*first), _lib.Vec3i_t(*last), z0, C.byref(p)) != 0:
            raise RuntimeError(_lib.last_error())
        return p


def _aggregates_moments(view, global_dims, z0, first, last, rng, group, device, fns):
    """UInt16 / Float32 slabs in one data pass: every rank's 96-byte moments partial (exact
    integer sums under the UInt16 unit mapping, float moments otherwise), ONE all_gather, combined
    in rank order (deterministic, identical on every rank) and finished on the host.  None when
    the float form says its terms may leave the float range (the caller runs the two passes; every
    rank reaches the same answer from the same partials)."""
    gx, gy, gz = global_dims
    p = fns.moments(view, *(rng or (first, first)), z0)
    parts = _allgather_partials(p, group, device)
    arr = (_lib.HipMomentPartial_t * len(parts))(*parts)
    out, complete = _lib.Aggregates_t(), C.c_int32(0)
    if lib.vktHipAggregatesFromMoments(arr, len(parts), gx * gy * gz, gx, gy, C.byref(out), C.byref(complete)) != 0:
        raise RuntimeError(_lib.last_error())
    return out if complete.value else None


def _aggregates_codes(view, global_dims, z0, rng, group, device, fns):
    """UInt8 / UInt16 slabs in one data pass: local code counts, ONE all_reduce(SUM) of them, the
    aggregates from the global counts (identical on every rank), a first-occurrence search of
    the two extremes' codes in each slab and an all_reduce(MIN) of the indices.  None when the
    counts cannot tell which voxel comes first (the caller runs the two passes; every rank
    reaches the same answer, from the same counts)."""
    import torch
    import torch.distributed as dist

    gx, gy, gz = global_dims
    ncodes = 256 if view.dataFormat == 4 else 65536
    dev = device if device is not None else "cpu"
    # the library writes `counts` on its compute stream and the collectives run after torch's
    # current stream: inside library_stream the two are one stream, whatever the caller has
    # current; the tensors are allocated there too, so their memory is tied to it
    with library_stream(torch.device(dev).type == "cuda"):
        counts = torch.zeros(ncodes, dtype=torch.int64, device=dev)
        if rng:
            fns.count(view, rng[0], rng[1], counts)
        _all_reduce(counts, dist.ReduceOp.SUM, group)
        p1, p2, (cmin, cmax) = fns.from_codes(counts, view.dataFormat, view.mappingLo, view.mappingHi, gx * gy * gz)
        if cmin < 0 or cmax < 0:
            return None
        imin, imax = fns.first_codes(view, rng[0], rng[1], z0, cmin, cmax) if rng else (NO_INDEX, NO_INDEX)
        idx = torch.tensor([min(imin, _I64_MAX), min(imax, _I64_MAX)], dtype=torch.int64, device=dev)
        _all_reduce(idx, dist.ReduceOp.MIN, group)
        imin, imax = (int(i) if int(i) != _I64_MAX else NO_INDEX for i in idx.cpu())
    p1.minIndex, p1.maxIndex = imin, imax
    out = _lib.Aggregates_t()
    lib.vktHipAggregatesFinish(C.byref(p1), C.byref(p2), gx * gy * gz, gx, gy, C.byref(out))
    return out


def aggregates(view, global_dims, z0: int, first, last, group=None, device=None, pass_fn=None, code_fns=None,
               moment_fns=None):
    """ComputeAggregatesRange over a Z-slab partitioned volume: each rank reduces its planes
    (pass 1), partials are all-gathered and combined in rank order (deterministic), the
    reference's float mean of the WHOLE volume follows, then pass 2 and a second exchange.
    UInt16 / Float32 volumes whose every slab takes the moments walk use ONE data pass and one
    all_gather of 96-byte moment partials (_aggregates_moments; `moment_fns` replaces the GPU
    steps), UInt8 (and UInt16 when that is off) one pass of code counts (_aggregates_codes;
    `code_fns` replaces the GPU steps, e.g. in CPU tests); a custom `pass_fn` alone keeps the two
    passes.  `view` is this rank's slab (global planes [z0, z0 + view.dimZ)); returns Aggregates_t."""
    import torch
    import torch.distributed as dist

    gx, gy, gz = global_dims
    rng = slab_range(first, last, z0, z0 + view.dimZ)
    fmt = getattr(view, "dataFormat", None)
    if fmt in (5, 7) and (moment_fns is not None or (code_fns is None and pass_fn is None)):
        fns = moment_fns or GpuMomentFns
        ok = torch.tensor([1 if fns.supported(view, *(rng or (first, first))) else 0], dtype=torch.int64,
                          device=device if device is not None else "cpu")
        _all_reduce(ok, dist.ReduceOp.MIN, group)
        if int(ok.item()):
            out = _aggregates_moments(view, global_dims, z0, first, last, rng, group, device, fns)
            if out is not None:
                return out
    if fmt in (4, 5) and (code_fns is not None or pass_fn is None):
        fns = code_fns or GpuCodeFns
        ok = torch.tensor([1 if fns.supported(view, *(rng or (first, first))) else 0], dtype=torch.int64,
                          device=device if device is not None else "cpu")
        _all_reduce(ok, dist.ReduceOp.MIN, group)
        if int(ok.item()):
            out = _aggregates_codes(view, global_dims, z0, rng, group, device, fns)
            if out is not None:
                return out
    pass_fn = pass_fn or _gpu_pass
    empty = _lib.HipAggregatePartial_t()
    lib.vktHipAggregatePartialInit(C.byref(empty))
    p1 = pass_fn(view, *rng, z0, 1, 0.0) if rng else empty
    acc1 = combine_partials(_allgather_partials(p1, group, device))
    n = gx * gy * gz
    mean = lib.vktHipAggregatesMean(C.byref(acc1), n)
    p2 = pass_fn(view, *rng, z0, 2, mean) if rng else empty
    acc2 = combine_partials(_allgather_partials(p2, group, device))
    out = _lib.Aggregates_t()
    lib.vktHipAggregatesFinish(C.byref(acc1), C.byref(acc2), n, gx, gy, C.byref(out))
    return out


def _gpu_count(view, first, last, bins, num_bins):
    err = lib.vktHipHistogramRange(view, _lib.Vec3i_t(*first), _lib.Vec3i_t(*last), C.c_void_p(bins.data_ptr()),
                                   num_bins, 0)
    if err != 0:
        raise RuntimeError(_lib.last_error())


def histogram(view, z0: int, first, last, bins, num_bins: int, group=None, count_fn=None):
    """ComputeHistogramRange over a Z-slab partitioned volume: each rank counts its planes
    into `bins` (an int64 tensor of num_bins counters; a device tensor for the GPU backend),
    then one all_reduce(SUM) -- RCCL over xGMI with the nccl backend (gloo reduces a host
    copy).  Counts are integers: the result is exact."""
    import torch.distributed as dist

    rng = slab_range(first, last, z0, z0 + view.dimZ)
    with library_stream(bins.is_cuda):   # the counting kernel and the all_reduce on one stream
        if rng:
            (count_fn or _gpu_count)(view, rng[0], rng[1], bins, num_bins)
        else:
            bins.zero_()
        if bins.is_cuda and dist.get_backend(group) == "gloo":
            host = bins.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
            bins.copy_(host)
        else:
            dist.all_reduce(bins, op=dist.ReduceOp.SUM, group=group)
    return bins
