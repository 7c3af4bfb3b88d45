"""Native Z-slab plan and RCCL halo exchange (include/volkit_hip.h: vktHipSlabResamplePlan,
vktHipComm*, vktHipSlabExchangeHalo; volkit_amd/csrc/runtime/Comm.cpp).

CPU: the C plan equals volkit_amd/slab.py:plan_resample (which the gloo tests exercise) for
every rank of many layouts, transfers pair up across ranks, and argument errors are
returned.  GPU: a one-rank communicator (create, exchange -- nothing to move -- destroy).
The multi-rank exchange needs one GPU per rank (RCCL refuses two ranks on one device):
`test_two_rank_exchange` runs only where two GPUs are visible, i.e. not on the 1-GPU pool
this round's GPU tests ran on.
"""
import ctypes as C
import os

import pytest

from volkit_amd import _lib, slab
from volkit_amd._lib import HipCommId_t, HipSlabTransfer_t, HipVolumeView_t, lib

NEAREST, LINEAR = 0, 1


def c_plan(dst_gdz, src_gdz, world, rank, fm, chain):
    z0, z1, n = C.c_int32(), C.c_int32(), C.c_int32()
    assert lib.vktHipSlabResamplePlan(dst_gdz, src_gdz, world, rank, fm, int(chain), C.byref(z0), C.byref(z1),
                                      None, 0, C.byref(n)) == 0, _lib.last_error()
    xs = (HipSlabTransfer_t * max(1, n.value))()
    assert lib.vktHipSlabResamplePlan(dst_gdz, src_gdz, world, rank, fm, int(chain), C.byref(z0), C.byref(z1),
                                      xs, n.value, C.byref(n)) == 0, _lib.last_error()
    recvs = [(x.peer, x.z0, x.z1) for x in xs[:n.value] if not x.send]
    sends = [(x.peer, x.z0, x.z1) for x in xs[:n.value] if x.send]
    return (z0.value, z1.value), sorted(recvs), sorted(sends)


LAYOUTS = [(2048, 1024), (1024, 512), (1024, 1024), (1000, 768), (768, 1000), (64, 7), (7, 64), (3, 17), (17, 3),
           (256, 128), (129, 64)]


@pytest.mark.parametrize("dst_gdz,src_gdz", LAYOUTS)
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("fm,chain", [(NEAREST, False), (LINEAR, False), (LINEAR, True)])
def test_native_plan_matches_slab_py(dst_gdz, src_gdz, world, fm, chain):
    for rank in range(world):
        py = slab.plan_resample(dst_gdz, src_gdz, world, rank, fm, chain)
        local, recvs, sends = c_plan(dst_gdz, src_gdz, world, rank, fm, chain)
        assert local == tuple(py.local_src), (rank, local, py.local_src)
        assert recvs == sorted(py.recvs), rank
        assert sends == sorted(py.sends), rank


def test_every_plane_received_is_sent_once():
    """Across all ranks the transfers pair up: each (receiver, sender, planes) appears as a send."""
    for dst_gdz, src_gdz in LAYOUTS:
        for world in (2, 3, 8):
            recvs, sends = set(), set()
            for rank in range(world):
                _, r, s = c_plan(dst_gdz, src_gdz, world, rank, LINEAR, True)
                recvs |= {(rank, p, a, b) for p, a, b in r}
                sends |= {(p, rank, a, b) for p, a, b in s}
            assert recvs == sends


def test_plan_errors_are_returned():
    z0, z1, n = C.c_int32(), C.c_int32(), C.c_int32()
    assert lib.vktHipSlabResamplePlan(64, 32, 4, 4, LINEAR, 1, C.byref(z0), C.byref(z1), None, 0, C.byref(n)) != 0
    assert "invalid rank" in _lib.last_error()
    assert lib.vktHipSlabResamplePlan(64, 32, 4, 1, LINEAR, 1, None, C.byref(z1), None, 0, C.byref(n)) != 0
    # too small a transfer array
    assert lib.vktHipSlabResamplePlan(64, 32, 4, 1, LINEAR, 1, C.byref(z0), C.byref(z1), None, 0, C.byref(n)) == 0
    assert n.value > 0
    xs = (HipSlabTransfer_t * 1)()
    assert lib.vktHipSlabResamplePlan(64, 32, 4, 1, LINEAR, 1, C.byref(z0), C.byref(z1), xs, n.value - 1,
                                      C.byref(n)) != 0
    assert "too small" in _lib.last_error()
    assert lib.vktHipSlabExchangeHalo(None, HipVolumeView_t(), 0, 64, 32, LINEAR, 1) != 0
    assert "null communicator" in _lib.last_error()
    assert lib.vktHipCommSetTimeout(None, 1000) != 0


@pytest.mark.gpu
def test_one_rank_communicator():
    import torch
    torch.cuda.init()
    uid = HipCommId_t()
    assert lib.vktHipCommGetUniqueId(C.byref(uid)) == 0, _lib.last_error()
    comm = C.c_void_p()
    assert lib.vktHipCommInitRank(C.byref(comm), 1, uid, 0) == 0, _lib.last_error()
    try:
        assert lib.vktHipCommSetTimeout(comm, -1) != 0
        assert lib.vktHipCommSetTimeout(comm, 5000) == 0, _lib.last_error()
        buf = torch.zeros(16 * 16 * 8 * 2, dtype=torch.uint8, device="cuda")
        view = HipVolumeView_t(buf.data_ptr(), 16, 16, 8, 5, 0.0, 1.0)
        # one rank owns every plane: nothing to move
        assert lib.vktHipSlabExchangeHalo(comm, view, 0, 16, 8, LINEAR, 1) == 0, _lib.last_error()
        torch.cuda.synchronize()
    finally:
        assert lib.vktHipCommDestroy(comm) == 0, _lib.last_error()


def _two_rank_worker(rank, uid_bytes, result_q):
    import torch
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(rank)
    assert lib.vktHipSetDevice(rank) == 0
    uid = HipCommId_t()
    C.memmove(C.addressof(uid), uid_bytes, 128)
    comm = C.c_void_p()
    assert lib.vktHipCommInitRank(C.byref(comm), 2, uid, rank) == 0, _lib.last_error()
    dst_gdz, src_gdz, dx, dy = 64, 32, 32, 8
    (lo, hi), recvs, sends = c_plan(dst_gdz, src_gdz, 2, rank, LINEAR, True)
    own = slab.slab_bounds(src_gdz, 2, rank)
    plane = dx * dy * 4
    buf = torch.zeros((hi - lo) * plane, dtype=torch.uint8, device="cuda")
    # every owned plane z holds the byte pattern z + 1; halo planes start at 0
    for z in range(*own):
        buf[(z - lo) * plane:(z - lo + 1) * plane] = z + 1
    view = HipVolumeView_t(buf.data_ptr(), dx, dy, hi - lo, 7, 0.0, 1.0)
    err = lib.vktHipSlabExchangeHalo(comm, view, lo, dst_gdz, src_gdz, LINEAR, 1)
    torch.cuda.synchronize()
    got = buf.view(hi - lo, plane)[:, 0].cpu().numpy().tolist()
    lib.vktHipCommDestroy(comm)
    result_q.put((rank, err, lo, got))


@pytest.mark.gpu
def test_two_rank_exchange():
    """Two processes, one GPU each: every halo plane arrives with its owner's pattern."""
    import torch
    import torch.multiprocessing as mp
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs (RCCL refuses two ranks on one device)")
    uid = HipCommId_t()
    assert lib.vktHipCommGetUniqueId(C.byref(uid)) == 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_two_rank_worker, args=(r, C.string_at(C.addressof(uid), 128), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, err, lo, got in res:
        assert err == 0
        assert got == [lo + i + 1 for i in range(len(got))], (rank, got)


@pytest.mark.gpu
def test_round_deadline_aborts_without_blocking_the_host():
    """Failure detection on one GPU: a one-rank communicator exchanges with itself
    (vktHipCommExchange, peer = own rank).  A plain round completes and vktHipCommSynchronize
    returns 0.  Then knob comm.test_stall_ms keeps the round's stream busy for 4 s after its
    transfers, under a 300 ms deadline: the call returns at once (enqueued, the host is not
    blocked), the watcher times the round from its start and aborts the communicator, so
    vktHipCommSynchronize returns vktInvalidValue well before the stall ends, naming the
    deadline, and the next round is refused."""
    import time
    import torch
    torch.cuda.init()
    uid = HipCommId_t()
    assert lib.vktHipCommGetUniqueId(C.byref(uid)) == 0, _lib.last_error()
    comm = C.c_void_p()
    assert lib.vktHipCommInitRank(C.byref(comm), 1, uid, 0) == 0, _lib.last_error()
    n = 1 << 20
    a = torch.arange(n, dtype=torch.int32, device="cuda").view(torch.uint8)
    b = torch.zeros_like(a)
    torch.cuda.synchronize()
    try:
        assert lib.vktHipCommSetTimeout(comm, 5000) == 0
        assert lib.vktHipCommExchange(comm, 0, C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()), a.numel()) == 0, \
            _lib.last_error()
        assert lib.vktHipCommSynchronize(comm) == 0, _lib.last_error()
        torch.cuda.synchronize()
        assert torch.equal(a, b)
        assert lib.vktHipCommExchange(comm, 1, C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()), 16) != 0  # no rank 1

        assert lib.vktHipSetTuningKnob(b"comm.test_stall_ms", 4000) == 0
        assert lib.vktHipCommSetTimeout(comm, 300) == 0
        t0 = time.monotonic()
        assert lib.vktHipCommExchange(comm, 0, C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()), a.numel()) == 0, \
            _lib.last_error()
        enqueue_s = time.monotonic() - t0
        lib.vktHipSetTuningKnob(b"comm.test_stall_ms", 0)
        err = lib.vktHipCommSynchronize(comm)
        judged_s = time.monotonic() - t0
        msg = _lib.last_error()
        assert err != 0 and "within 300 ms" in msg, msg
        assert enqueue_s < 0.2, enqueue_s
        assert judged_s < 3.0, judged_s          # the deadline fired; the 4-s stall had not ended
        # later rounds are refused at once
        assert lib.vktHipCommExchange(comm, 0, C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()), 16) != 0
        assert "aborted" in _lib.last_error()
    finally:
        lib.vktHipSetTuningKnob(b"comm.test_stall_ms", 0)
        torch.cuda.synchronize()                 # (the stall kernel leaves after its 4 s)
        assert lib.vktHipCommDestroy(comm) == 0, _lib.last_error()


@pytest.mark.gpu
def test_round_deadline_fails_the_issuing_call_when_synchronous():
    """with async execution off (vktHipSetAsyncExecution(0)) every call
    synchronises, so the call whose round outlived its deadline returns vktInvalidValue itself,
    naming the deadline (comm::finishRound -> vktHipCommSynchronize after the stream drained) --
    not vktNoError with garbage in the halo and the failure surfacing on a later call."""
    import torch
    torch.cuda.init()
    was = C.c_int32()
    assert lib.vktHipGetAsyncExecution(C.byref(was)) == 0
    uid = HipCommId_t()
    assert lib.vktHipCommGetUniqueId(C.byref(uid)) == 0, _lib.last_error()
    comm = C.c_void_p()
    assert lib.vktHipCommInitRank(C.byref(comm), 1, uid, 0) == 0, _lib.last_error()
    a = torch.arange(1 << 18, dtype=torch.int32, device="cuda").view(torch.uint8)
    b = torch.zeros_like(a)
    torch.cuda.synchronize()
    try:
        assert lib.vktHipSetAsyncExecution(0) == 0
        assert lib.vktHipCommSetTimeout(comm, 5000) == 0
        # a clean round: the synchronous call judges it and returns 0, the bytes have landed
        assert lib.vktHipCommExchange(comm, 0, C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()), a.numel()) == 0, \
            _lib.last_error()
        assert torch.equal(a, b)
        assert lib.vktHipSetTuningKnob(b"comm.test_stall_ms", 1500) == 0
        assert lib.vktHipCommSetTimeout(comm, 300) == 0
        err = lib.vktHipCommExchange(comm, 0, C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()), a.numel())
        msg = _lib.last_error()
        assert err != 0 and "within 300 ms" in msg, (err, msg)
    finally:
        lib.vktHipSetTuningKnob(b"comm.test_stall_ms", 0)
        lib.vktHipSetAsyncExecution(was.value)
        torch.cuda.synchronize()
        assert lib.vktHipCommDestroy(comm) == 0, _lib.last_error()


@pytest.mark.gpu
def test_overlapped_resample_on_one_rank_matches_resample_slab():
    """vktHipResampleSlabOverlapped on a one-rank communicator (the C entry had no
    test): the whole volume is the rank's slab, nothing moves, the interior split covers every
    dst plane -- bytes equal one vktHipResampleSlab of the same volume (Float32 Linear, the
    z+1 chain, with non-finite voxels), in async and synchronous mode."""
    import numpy as np
    import torch
    torch.cuda.init()
    rng = np.random.default_rng(77)
    vals = rng.uniform(-1, 2, (24, 20, 36)).astype(np.float32)
    vals[7, 3, 5], vals[23, 19, 35], vals[0, 0, 0] = np.inf, np.nan, -0.0
    src = torch.from_numpy(vals).cuda()
    dd = (50, 31, 40)                                     # dst (x, y, z)
    want = torch.zeros((dd[2], dd[1], dd[0]), dtype=torch.float32, device="cuda")
    got = torch.full_like(want, 7.0)
    sv = HipVolumeView_t(src.data_ptr(), 36, 20, 24, 7, 0.0, 1.0)
    wv = HipVolumeView_t(want.data_ptr(), dd[0], dd[1], dd[2], 7, 0.0, 1.0)
    gv = HipVolumeView_t(got.data_ptr(), dd[0], dd[1], dd[2], 7, 0.0, 1.0)
    assert lib.vktHipResampleSlab(wv, sv, LINEAR, dd[2], 0, 24, 0) == 0, _lib.last_error()
    was = C.c_int32()
    assert lib.vktHipGetAsyncExecution(C.byref(was)) == 0
    uid = HipCommId_t()
    assert lib.vktHipCommGetUniqueId(C.byref(uid)) == 0, _lib.last_error()
    comm = C.c_void_p()
    assert lib.vktHipCommInitRank(C.byref(comm), 1, uid, 0) == 0, _lib.last_error()
    try:
        for mode in (1, 0):
            assert lib.vktHipSetAsyncExecution(mode) == 0
            got.fill_(7.0)
            torch.cuda.synchronize()
            assert lib.vktHipResampleSlabOverlapped(comm, gv, sv, 0, dd[2], 24, LINEAR, 1) == 0, _lib.last_error()
            torch.cuda.synchronize()
            assert torch.equal(got.view(torch.int32), want.view(torch.int32)), mode
        # a dst view that is not the rank's slab is refused
        bad = HipVolumeView_t(got.data_ptr(), dd[0], dd[1], dd[2] - 1, 7, 0.0, 1.0)
        assert lib.vktHipResampleSlabOverlapped(comm, bad, sv, 0, dd[2], 24, LINEAR, 1) != 0
        assert "dst slab" in _lib.last_error()
    finally:
        lib.vktHipSetAsyncExecution(was.value)
        assert lib.vktHipCommDestroy(comm) == 0, _lib.last_error()


def _two_rank_overlapped_worker(rank, uid_bytes, result_q):
    """One rank of test_two_rank_overlapped_resample (one GPU per rank)."""
    import numpy as np
    import torch
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(rank)
    assert lib.vktHipSetDevice(rank) == 0
    uid = HipCommId_t()
    C.memmove(C.addressof(uid), uid_bytes, 128)
    comm = C.c_void_p()
    assert lib.vktHipCommInitRank(C.byref(comm), 2, uid, rank) == 0, _lib.last_error()
    dst_gdz, src_gdz, dx, dy, sx, sy = 64, 32, 40, 12, 24, 10
    rng = np.random.default_rng(5)
    vals = rng.uniform(-1, 2, (src_gdz, sy, sx)).astype(np.float32)
    (lo, hi), recvs, _ = c_plan(dst_gdz, src_gdz, 2, rank, LINEAR, True)
    o0, o1 = slab.slab_bounds(src_gdz, 2, rank)
    d0, d1 = slab.slab_bounds(dst_gdz, 2, rank)
    out = []
    for path in ("overlapped", "exchange"):
        src = torch.zeros((hi - lo, sy, sx), dtype=torch.float32, device="cuda")
        src[o0 - lo:o1 - lo] = torch.from_numpy(vals[o0:o1]).cuda()     # halo planes start at 0
        dst = torch.zeros((d1 - d0, dy, dx), dtype=torch.float32, device="cuda")
        sv = HipVolumeView_t(src.data_ptr(), sx, sy, hi - lo, 7, 0.0, 1.0)
        dv = HipVolumeView_t(dst.data_ptr(), dx, dy, d1 - d0, 7, 0.0, 1.0)
        if path == "overlapped":
            err = lib.vktHipResampleSlabOverlapped(comm, dv, sv, lo, dst_gdz, src_gdz, LINEAR, 1)
        else:
            err = lib.vktHipSlabExchangeHalo(comm, sv, lo, dst_gdz, src_gdz, LINEAR, 1)
            if err == 0:
                err = lib.vktHipResampleSlab(dv, sv, LINEAR, dst_gdz, d0, src_gdz, lo)
        torch.cuda.synchronize()
        out.append((err, dst.cpu().numpy().view(np.uint32).copy()))
    lib.vktHipCommDestroy(comm)
    result_q.put((rank, len(recvs), out[0][0], out[1][0], bool(np.array_equal(out[0][1], out[1][1]))))


@pytest.mark.gpu
def test_two_rank_overlapped_resample():
    """vktHipResampleSlabOverlapped between two processes (one GPU each) equals
    vktHipSlabExchangeHalo + vktHipResampleSlab on the same slabs; rank 0 receives the z+1 halo
    plane, rank 1 receives nothing (its interior split covers its whole slab)."""
    import torch
    import torch.multiprocessing as mp
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs (RCCL refuses two ranks on one device)")
    uid = HipCommId_t()
    assert lib.vktHipCommGetUniqueId(C.byref(uid)) == 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_two_rank_overlapped_worker, args=(r, C.string_at(C.addressof(uid), 128), q))
             for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert [r[1] > 0 for r in res] == [True, False]
    for rank, _, e_ov, e_ex, same in res:
        assert e_ov == 0 and e_ex == 0 and same, rank
