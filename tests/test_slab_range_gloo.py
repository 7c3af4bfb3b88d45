"""FillRange / CopyRange / arithmetic Range over Z-slab partitioned volumes (volkit_amd.slab,
include/volkit_hip.h vktHipSlab*), with real torch.distributed ranks (gloo, 127.0.0.1) on the CPU.

Every rank holds its owned planes of each volume (plus garbage halo planes in some cases), runs
the C plan (vktHipSlabRangePlan: pieces + moves), moves the source planes its dst planes read
that other ranks own (dstOffset.z across slab boundaries, clamped halo planes) with one batched
isend/irecv round, and runs its pieces.  Pieces run here on the ORACLE (the checker; on the GPU
the library's vktHipSlabRangePieces does this step, tests/test_gpu_slab_range.py), so the test
checks the plan and the exchange: each rank's owned dst planes must equal the same planes of
one whole-volume oracle call with the same global first/last/dstOffset (reference semantics
Fill_serial.hpp:20-26, Copy_serial.hpp:38-47, Arithmetic_serial.hpp:25-41), and halo planes of
the dst slab must be left alone.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

# (kind, dst fmt, src fmt, dst G, src1 G, src2 G, first, last, dstOffset, op)
#   x/y: dst (12, 5), sources (12, 5) -- global dims; G = depth of each volume
CASES = [
    ("fill", 5, 5, 13, 0, 0, (1, 0, 2), (11, 5, 12), (0, 0, 0), None),
    ("fill", 7, 7, 9, 0, 0, (0, 1, 0), (12, 4, 9), (0, 0, 0), None),
    ("copy", 5, 5, 16, 13, 0, (0, 0, 0), (12, 5, 13), (0, 0, 3), None),           # planes move up 3
    ("copy", 5, 5, 16, 13, 0, (1, 1, 4), (11, 4, 13), (0, 0, 0), None),           # ... down 4
    ("copy", 5, 5, 16, 13, 0, (-2, -1, -3), (10, 4, 12), (0, 0, 1), None),        # clamped halo below
    ("copy", 4, 4, 20, 9, 0, (0, 0, 5), (12, 5, 17), (0, 0, 2), None),            # clamped halo above
    ("copy", 4, 4, 20, 9, 0, (-1, 0, -4), (11, 5, 15), (0, 0, 0), None),          # both clamps
    ("copy", 7, 5, 11, 13, 0, (0, 0, 2), (12, 5, 12), (0, 0, 1), None),           # UInt16 -> Float32
    ("arith", 5, 5, 13, 13, 13, (0, 0, 1), (12, 5, 9), (0, 0, 3), "Sum"),
    ("arith", 5, 5, 13, 13, 13, (2, 1, 4), (10, 5, 13), (0, 0, -4), "SafeDiff"),
    ("arith", 5, 5, 15, 13, 17, (0, 0, 0), (12, 5, 13), (0, 0, 2), "SafeSum"),    # 3 different partitions
    ("arith", 7, 7, 12, 12, 12, (0, 0, 0), (12, 5, 12), (0, 0, 0), "Prod"),
    ("arith", 4, 4, 10, 14, 14, (1, 0, 5), (12, 5, 14), (0, 0, -5), "AbsDiff"),
]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _codes(rng, fmt, shape):
    from oracle import binding as ob
    if fmt == 7:
        return rng.uniform(-1, 2, shape).astype(np.float32).view(np.uint32)
    return rng.integers(0, 2 ** (8 * ob.BPV[fmt]), shape, dtype=np.uint64).astype(ob.CODE_DTYPE[fmt])


class Local:
    """A rank's slab of one volume in host memory: owned planes (+ `halo` garbage planes on
    each side inside [0, G))."""

    def __init__(self, glob, fmt, world, rank, halo, lo_hi=(0.0, 1.0)):
        from volkit_amd import _lib, slab
        G = glob.shape[0]
        o0, o1 = slab.slab_bounds(G, world, rank)
        self.z0 = max(0, o0 - halo) if o1 > o0 else o0
        z1 = min(G, o1 + halo) if o1 > o0 else o1
        self.owned = (o0, o1)
        self.arr = np.full((z1 - self.z0,) + glob.shape[1:], 0xA5, dtype=glob.dtype)   # garbage
        self.arr[o0 - self.z0:o1 - self.z0] = glob[o0:o1]
        self.tensor = torch.from_numpy(self.arr.view(np.uint8).reshape(-1))
        y, x = glob.shape[1:]
        view = _lib.HipVolumeView_t(self.tensor.data_ptr(), x, y, z1 - self.z0, fmt, *lo_hi)
        self.slab = slab.Slab(view, self.z0, G, self.tensor)


def oracle_pieces(kind, op, world, rank, dst, srcs, first, last, off, value, bufs):
    """Test-side restatement of the C piece runner (Slab.cpp runPiece) on the oracle: each piece
    reads its source planes from the own slab or the gather buffer, as sub-volumes of exactly
    those planes."""
    from oracle import binding as ob
    from volkit_amd import slab
    gz = [s.global_dim_z for s in srcs] + [0, 0]
    pieces, _, _ = slab.range_plan(kind, world, rank, dst.global_dim_z, gz[0], gz[1], first, last, off)

    def vol(s, flat, plane0, n):
        v = s.view
        dt = ob.CODE_DTYPE[v.dataFormat]
        pb = s.plane_bytes
        raw = flat[plane0 * pb:(plane0 + n) * pb].numpy()
        return ob.Volume(raw.view(dt).reshape(n, v.dimY, v.dimX), v.dataFormat, v.mappingLo, v.mappingHi)

    dv = vol(dst, dst.tensor, 0, dst.view.dimZ)
    for p in pieces:
        if kind == slab.FILL:
            ob.fill_range(dv, (first[0], first[1], p.zBegin - dst.z0), (last[0], last[1], p.zEnd - dst.z0), value)
            continue
        sv = []
        for k, s in enumerate(srcs):
            if p.bufPlane[k] < 0:
                sv.append(vol(s, s.tensor, p.srcZ[k] - s.z0, p.srcPlanes[k]))
            else:
                sv.append(vol(s, bufs[k], p.bufPlane[k], p.srcPlanes[k]))
        dz = p.dstZ - dst.z0
        if kind == slab.COPY:
            ob.copy_range(dv, sv[0], (first[0], first[1], p.zBegin - p.srcZ[0]),
                          (last[0], last[1], p.zEnd - p.srcZ[0]), (off[0], off[1], dz))
        else:
            ob.arith_range(op, dv, sv[0], sv[1], (first[0], first[1], 0), (last[0], last[1], p.zEnd - p.zBegin),
                           (off[0], off[1], dz))
    assert dst.view.dimZ == 0 or np.shares_memory(dv.codes, dst.tensor.numpy())
    return 0


def _worker(rank, world, port, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle import binding as ob
        from volkit_amd import slab
        bad = []
        for ci, (kind, dfmt, sfmt, dG, s1G, s2G, first, last, off, op) in enumerate(CASES):
            for halo in (0, 1):
                rng = np.random.default_rng(1000 + ci)        # the same global volumes on every rank
                dglob = _codes(rng, dfmt, (dG, 5, 12))
                s1 = _codes(rng, sfmt, (s1G, 5, 12)) if s1G else None
                s2 = _codes(rng, sfmt, (s2G, 5, 12)) if s2G else None
                # whole-volume oracle
                ref = ob.Volume(dglob.copy(), dfmt)
                if kind == "fill":
                    ob.fill_range(ref, first, last, 0.375)
                elif kind == "copy":
                    ob.copy_range(ref, ob.Volume(s1, sfmt), first, last, off)
                else:
                    ob.arith_range(op, ref, ob.Volume(s1, sfmt), ob.Volume(s2, sfmt), first, last, off)
                # slabs
                D = Local(dglob, dfmt, world, rank, halo)
                halo_before = D.arr.copy()
                if kind == "fill":
                    slab.fill_range(D.slab, first, last, 0.375, run_pieces=oracle_pieces)
                elif kind == "copy":
                    S = Local(s1, sfmt, world, rank, halo)
                    slab.copy_range(D.slab, S.slab, first, last, off, run_pieces=oracle_pieces)
                else:
                    A, B = Local(s1, sfmt, world, rank, halo), Local(s2, sfmt, world, rank, halo)
                    slab.arithmetic_range(op, D.slab, A.slab, B.slab, first, last, off, run_pieces=oracle_pieces)
                o0, o1 = D.owned
                got = D.arr[o0 - D.z0:o1 - D.z0]
                want = ref.codes[o0:o1]
                if dfmt == 7:
                    fa, fb = got.view(np.float32), want.view(np.float32)
                    same = np.array_equal(np.isnan(fa), np.isnan(fb)) and np.array_equal(got[~np.isnan(fb)],
                                                                                         want[~np.isnan(fb)])
                else:
                    same = np.array_equal(got, want)
                keep = np.ones(D.arr.shape[0], bool)
                keep[o0 - D.z0:o1 - D.z0] = False
                if not same:
                    bad.append(f"case {ci} {kind} halo={halo}: owned planes [{o0},{o1}) differ")
                if not np.array_equal(D.arr[keep], halo_before[keep]):
                    bad.append(f"case {ci} {kind} halo={halo}: dst halo planes written")
        q.put((rank, bad))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface worker errors in the parent
        import traceback
        q.put((rank, [traceback.format_exc()]))


@pytest.mark.parametrize("world", [1, 2, 3, 4, 6])
def test_slab_range_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, bad in sorted(results, key=lambda r: r[0]):
        assert not bad, f"world {world} rank {rank}: " + "; ".join(bad)


def test_range_plan_moves_pair_up():
    """Every receive in any rank's plan is a send in its peer's plan, in the same order per
    pair of ranks (the RCCL group matches them in issue order), with the same plane range."""
    from volkit_amd import slab
    for kind, dfmt, sfmt, dG, s1G, s2G, first, last, off, op in CASES:
        k = {"fill": slab.FILL, "copy": slab.COPY, "arith": slab.ARITHMETIC}[kind]
        for world in (2, 3, 4, 5, 8):
            plans = [slab.range_plan(k, world, r, dG, s1G, s2G, first, last, off) for r in range(world)]
            for r in range(world):
                for peer in range(world):
                    recvs = [(m.source, m.z0, m.z1) for m in plans[r][1] if not m.send and m.peer == peer]
                    sends = [(m.source, m.z0, m.z1) for m in plans[peer][1] if m.send and m.peer == r]
                    assert recvs == sends, (kind, world, r, peer)
                # gather buffers hold exactly the received planes
                for src in (0, 1):
                    n = sum(m.z1 - m.z0 for m in plans[r][1] if not m.send and m.source == src)
                    assert n == plans[r][2][src]


def test_range_plan_rejects_out_of_bounds():
    from volkit_amd import slab
    with pytest.raises(RuntimeError):
        slab.range_plan(slab.ARITHMETIC, 2, 0, 10, 10, 10, (0, 0, 0), (4, 4, 10), (0, 0, 1))
    with pytest.raises(RuntimeError):
        slab.range_plan(slab.COPY, 2, 0, 10, 10, 0, (0, 0, -3), (4, 4, 8), (0, 0, 0))   # 11 planes into 10
    with pytest.raises(RuntimeError):
        slab.range_plan(slab.FILL, 2, 0, 10, 0, 0, (0, 0, 2), (4, 4, 11), (0, 0, 0))
    # empty and reversed ranges plan nothing
    assert slab.range_plan(slab.COPY, 2, 1, 10, 10, 0, (0, 0, 5), (4, 4, 5), (0, 0, 0))[:2] == ([], [])
    assert slab.range_plan(slab.COPY, 2, 1, 10, 10, 0, (4, 0, 0), (0, 4, 9), (0, 0, 0))[:2] == ([], [])
