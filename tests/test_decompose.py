"""BrickDecompose / BrickDecomposeResize against the oracle restatement
of reference src/vkt/Decompose.cpp:96-150 and src/vkt/Decompose_serial.hpp:15-46.

CPU tests: the brick layout that BrickDecomposeResize allocates (host logic), the C Array3D
handle API, and that the GPU backend refuses the CPU policy.  GPU tests: bit-exact brick
contents (clamped halos at the volume border) for every voxel format, the reference example
(src/examples/Decompose.c: 120x66x49 UInt8, 16^3 bricks, halo 1), the conversion path for a
brick whose mapping differs from the source's, and argument validation.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import binding as ob

vkt = pytest.importorskip("volkit_amd.volkit")
from volkit_amd._lib import Vec3i_t, lib  # noqa: E402

LAYOUTS = [
    ((10, 9, 8), (4, 4, 4), (0, 0, 0), (0, 0, 0)),
    ((10, 9, 8), (4, 4, 4), (1, 1, 1), (1, 1, 1)),
    ((120, 66, 49), (16, 16, 16), (1, 1, 1), (1, 1, 1)),      # src/examples/Decompose.c
    ((33, 17, 5), (8, 32, 2), (2, 0, 1), (0, 3, 0)),
    ((64, 64, 64), (64, 64, 64), (0, 0, 0), (0, 0, 0)),
    ((7, 5, 3), (1, 2, 3), (0, 1, 0), (1, 0, 2)),
    # 16-byte items spanning two brick rows (linear mode), clamped halos on every face
    ((70, 40, 33), (20, 20, 20), (1, 2, 1), (3, 1, 2)),
    ((100, 37, 19), (37, 13, 7), (2, 2, 2), (2, 2, 2)),
    ((131, 9, 4), (64, 4, 4), (5, 0, 0), (7, 0, 0)),
    # bricks of many 16-KiB workgroup chunks, chunk boundaries inside rows
    ((150, 97, 61), (64, 48, 40), (1, 1, 1), (2, 1, 3)),
    # halos wider than a brick: interior bricks clamped at the x ends (no uniform-grid descriptors)
    ((70, 20, 10), (8, 8, 8), (10, 1, 0), (12, 0, 1)),
]


def set_device(dev):
    ep = vkt.GetThreadExecutionPolicy()
    ep.device = dev
    vkt.SetThreadExecutionPolicy(ep)


@pytest.fixture
def cpu():
    set_device(vkt.ExecutionPolicy.Device_CPU)
    yield
    set_device(vkt.ExecutionPolicy.Device_CPU)


@pytest.mark.parametrize("dims,brick,neg,pos", LAYOUTS)
def test_resize_layout_matches_reference(cpu, dims, brick, neg, pos):
    src = vkt.StructuredVolume(*dims, vkt.DataFormat_UInt16, 0.5, 1.0, 2.0, -1.0, 3.0)
    arr = vkt.Array3D_StructuredVolume()
    assert vkt.BrickDecomposeResize(arr, src, vkt.Vec3i(*brick), vkt.Vec3i(*neg), vkt.Vec3i(*pos)) == vkt.NoError
    nb, layout = ob.brick_layout(dims, brick, neg, pos)
    assert tuple(arr.dims()) == nb and len(arr) == len(layout)
    for idx, bdims in layout.items():
        b = arr[idx]
        assert tuple(b.getDims()) == bdims, idx
        assert b.getDataFormat() == vkt.DataFormat_UInt16
        assert b.getDist() == (0.5, 1.0, 2.0)
        m = b.getVoxelMapping()
        assert (m.x, m.y) == (-1.0, 3.0)


def test_c_array3d_api(cpu):
    h = C.c_void_p()
    lib.vktArray3D_vktStructuredVolume_Create(C.byref(h), Vec3i_t(2, 3, 4))
    try:
        assert lib.vktArray3D_vktStructuredVolume_NumElements(h) == 24
        d = lib.vktArray3D_vktStructuredVolume_Dims(h)
        assert (d.x, d.y, d.z) == (2, 3, 4)
        assert not lib.vktArray3D_vktStructuredVolume_Empty(h)
        begin = C.cast(lib.vktArray3D_vktStructuredVolume_Begin(h), C.c_void_p).value
        end = C.cast(lib.vktArray3D_vktStructuredVolume_End(h), C.c_void_p).value
        assert end - begin == 24 * C.sizeof(C.c_void_p)
        slot = C.cast(lib.vktArray3D_vktStructuredVolume_Access(h, Vec3i_t(1, 2, 3)), C.c_void_p).value
        assert slot - begin == (3 * 6 + 2 * 2 + 1) * C.sizeof(C.c_void_p)
        lib.vktArray3D_vktStructuredVolume_Resize(h, Vec3i_t(0, 0, 0))
        assert lib.vktArray3D_vktStructuredVolume_Empty(h)
    finally:
        lib.vktArray3D_vktStructuredVolume_Destroy(h)


def test_cpu_policy_is_refused(cpu):
    src = vkt.StructuredVolume(8, 8, 8, vkt.DataFormat_UInt8)
    arr = vkt.Array3D_StructuredVolume()
    assert vkt.BrickDecomposeResize(arr, src, vkt.Vec3i(4, 4, 4)) == vkt.NoError
    assert vkt.BrickDecompose(arr, src, vkt.Vec3i(4, 4, 4)) == vkt.InvalidValue
    assert "CPU execution policy" in vkt.last_error()


def rand_codes(rng, fmt, shape):
    if fmt == 7:
        return rng.uniform(-2, 2, size=shape).astype(np.float32).view(np.uint32)
    info = np.iinfo(ob.CODE_DTYPE[fmt])
    return rng.integers(0, int(info.max) + 1, size=shape, dtype=np.uint64).astype(ob.CODE_DTYPE[fmt])


def gpu_decompose(codes, fmt, mapping, brick, neg, pos, tweak=None):
    """Source filled on the host, bricks allocated and decomposed under the GPU policy, read
    back under the CPU policy (deferred migration)."""
    z, y, x = codes.shape
    set_device(vkt.ExecutionPolicy.Device_CPU)
    src = vkt.StructuredVolume(x, y, z, fmt, 1.0, 1.0, 1.0, *mapping)
    src.from_numpy(codes)
    arr = vkt.Array3D_StructuredVolume()
    set_device(vkt.ExecutionPolicy.Device_GPU)
    try:
        assert vkt.BrickDecomposeResize(arr, src, vkt.Vec3i(*brick), vkt.Vec3i(*neg), vkt.Vec3i(*pos)) == vkt.NoError
        if tweak:
            tweak(arr)
        err = vkt.BrickDecompose(arr, src, vkt.Vec3i(*brick), vkt.Vec3i(*neg), vkt.Vec3i(*pos))
    finally:
        set_device(vkt.ExecutionPolicy.Device_CPU)
    if err != vkt.NoError:
        return err, None
    d = arr.dims()
    out = {(i, j, k): arr[(i, j, k)].to_numpy() for k in range(d.z) for j in range(d.y) for i in range(d.x)}
    return err, out


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [4, 5, 7, 6])
@pytest.mark.parametrize("dims,brick,neg,pos", LAYOUTS)
def test_brick_decompose_parity(fmt, dims, brick, neg, pos):
    rng = np.random.default_rng(fmt * 100 + sum(dims))
    codes = rand_codes(rng, fmt, dims[::-1])
    err, got = gpu_decompose(codes, fmt, (0.0, 1.0), brick, neg, pos)
    assert err == vkt.NoError, vkt.last_error()
    ref = ob.brick_decompose(ob.Volume(codes, fmt), brick, neg, pos)
    assert set(got) == set(ref)
    for idx, v in ref.items():
        np.testing.assert_array_equal(got[idx], v.codes, err_msg=f"brick {idx}")


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [4, 5, 7])
@pytest.mark.parametrize("dims,brick,neg,pos", LAYOUTS)
def test_brick_decompose_descriptor_table(fmt, dims, brick, neg, pos):
    """Knob decompose.grid = 0: uniform brick grids load one descriptor per brick instead of
    deriving it from the brick index (the default, tested by test_brick_decompose_parity)."""
    rng = np.random.default_rng(fmt * 100 + sum(dims) + 7)
    codes = rand_codes(rng, fmt, dims[::-1])
    assert lib.vktHipSetTuningKnob(b"decompose.grid", 0) == 0
    try:
        err, got = gpu_decompose(codes, fmt, (0.0, 1.0), brick, neg, pos)
    finally:
        assert lib.vktHipSetTuningKnob(b"decompose.grid", -1) == 0
    assert err == vkt.NoError, vkt.last_error()
    ref = ob.brick_decompose(ob.Volume(codes, fmt), brick, neg, pos)
    for idx, v in ref.items():
        np.testing.assert_array_equal(got[idx], v.codes, err_msg=f"brick {idx}")


@pytest.mark.gpu
@pytest.mark.parametrize("grid", [1, 0])
@pytest.mark.parametrize("fmt", [4, 5, 7])
@pytest.mark.parametrize("dims,brick,neg,pos", LAYOUTS)
def test_brick_decompose_128_thread_workgroups(fmt, dims, brick, neg, pos, grid):
    """Knob decompose.block = 128: each 16-KiB chunk copied by 128 threads (twice the items and
    staged words per thread), with grid-derived descriptors and with the descriptor table."""
    rng = np.random.default_rng(fmt * 100 + sum(dims) + 11)
    codes = rand_codes(rng, fmt, dims[::-1])
    assert lib.vktHipSetTuningKnob(b"decompose.block", 128) == 0
    assert lib.vktHipSetTuningKnob(b"decompose.grid", grid) == 0
    try:
        err, got = gpu_decompose(codes, fmt, (0.0, 1.0), brick, neg, pos)
    finally:
        assert lib.vktHipSetTuningKnob(b"decompose.block", -1) == 0
        assert lib.vktHipSetTuningKnob(b"decompose.grid", -1) == 0
    assert err == vkt.NoError, vkt.last_error()
    ref = ob.brick_decompose(ob.Volume(codes, fmt), brick, neg, pos)
    for idx, v in ref.items():
        np.testing.assert_array_equal(got[idx], v.codes, err_msg=f"brick {idx}")


@pytest.mark.gpu
@pytest.mark.parametrize("aligned", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("fmt", [4, 5, 7])
@pytest.mark.parametrize("dims,brick,neg,pos", LAYOUTS[1:4] + LAYOUTS[6:] + [
    ((96, 40, 33), (16, 16, 16), (1, 1, 1), (1, 1, 1)),     # 16-B row pitch: the edge mode (4) applies
    ((64, 24, 20), (5, 7, 6), (2, 1, 0), (1, 0, 2)),        # rows shorter than a word: all edge voxels
    ((128, 12, 10), (40, 6, 5), (3, 1, 1), (0, 1, 1))])
def test_brick_decompose_aligned_lds_pieces(fmt, dims, brick, neg, pos, aligned):
    """The staged copy's LDS writes of the words cut by a row end or the chunk, per knob
    decompose.aligned_lds: 0 per-voxel loop, 1 naturally aligned pieces (2: every word so), 3 all
    voxels written with the ones outside sent to the tile's unused tail (chunks that leave 16 B
    free; full chunks keep the loop), 4 the voxels at each row end in a loop of their own (one
    chunk per brick, 16-B row pitch; otherwise 0), 5 (default) 4 for UInt8 and 0 for the wider
    formats: the same bricks as the oracle."""
    rng = np.random.default_rng(fmt * 100 + sum(dims) + aligned)
    codes = rand_codes(rng, fmt, dims[::-1])
    assert lib.vktHipSetTuningKnob(b"decompose.aligned_lds", aligned) == 0
    try:
        err, got = gpu_decompose(codes, fmt, (0.0, 1.0), brick, neg, pos)
    finally:
        assert lib.vktHipSetTuningKnob(b"decompose.aligned_lds", -1) == 0
    assert err == vkt.NoError, vkt.last_error()
    ref = ob.brick_decompose(ob.Volume(codes, fmt), brick, neg, pos)
    for idx, v in ref.items():
        np.testing.assert_array_equal(got[idx], v.codes, err_msg=f"brick {idx}")


@pytest.mark.gpu
def test_reference_example_decompose():
    """src/examples/Decompose.c:16-88: Fill(.1) on 120x66x49 UInt8, 16^3 bricks with halo 1 --
    every brick voxel (halos clamped at the border) holds the code of 0.1."""
    codes = np.full((49, 66, 120), ob.map_voxel(0.1, 4)[0], dtype=np.uint8)
    err, got = gpu_decompose(codes, 4, (0.0, 1.0), (16, 16, 16), (1, 1, 1), (1, 1, 1))
    assert err == vkt.NoError
    assert len(got) == 8 * 5 * 4
    for idx, a in got.items():
        assert (a == 25).all(), idx
    assert got[(0, 0, 0)].shape == (18, 18, 18) and got[(7, 4, 3)].shape == (1 + 1 + 1, 2 + 2, 8 + 2)


@pytest.mark.gpu
def test_brick_with_other_mapping_converts():
    """A brick whose mapping differs from the source's takes CopyRange's unmap->map path
    (Copy_serial.hpp:21-22), the others stay bytewise in the batched launch."""
    rng = np.random.default_rng(5)
    codes = rand_codes(rng, 5, (12, 10, 9))

    def tweak(arr):
        arr[(1, 0, 1)].setVoxelMapping(-1.0, 3.0)

    err, got = gpu_decompose(codes, 5, (0.0, 1.0), (5, 5, 5), (1, 0, 1), (0, 1, 1), tweak)
    assert err == vkt.NoError, vkt.last_error()
    src = ob.Volume(codes, 5)
    nb, layout = ob.brick_layout(src.dims, (5, 5, 5), (1, 0, 1), (0, 1, 1))
    ranges = ob.brick_ranges(src.dims, nb, (5, 5, 5), (1, 0, 1), (0, 1, 1))
    for idx, bdims in layout.items():
        lo, hi = (-1.0, 3.0) if idx == (1, 0, 1) else (0.0, 1.0)
        ref = ob.Volume.zeros(bdims, 5, lo, hi)
        ob.copy_range(ref, src, *ranges[idx])
        np.testing.assert_array_equal(got[idx], ref.codes, err_msg=f"brick {idx}")


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [4, 5, 7])
def test_brick_larger_than_its_range(fmt):
    """A brick allocated larger than its copy box keeps its own row/plane pitch (row mode of
    the batched kernel): voxels outside the box are left untouched."""
    rng = np.random.default_rng(fmt)
    codes = rand_codes(rng, fmt, (11, 13, 41))

    def tweak(arr):
        arr[(0, 1, 1)].setDims(40, 9, 8)
        arr[(1, 0, 0)].setDims(23, 9, 6)

    err, got = gpu_decompose(codes, fmt, (0.0, 1.0), (20, 6, 5), (1, 1, 0), (2, 0, 1), tweak)
    assert err == vkt.NoError, vkt.last_error()
    src = ob.Volume(codes, fmt)
    nb, layout = ob.brick_layout(src.dims, (20, 6, 5), (1, 1, 0), (2, 0, 1))
    ranges = ob.brick_ranges(src.dims, nb, (20, 6, 5), (1, 1, 0), (2, 0, 1))
    for idx, bdims in layout.items():
        bdims = {(0, 1, 1): (40, 9, 8), (1, 0, 0): (23, 9, 6)}.get(idx, bdims)
        ref = ob.Volume.zeros(bdims, fmt)
        ob.copy_range(ref, src, *ranges[idx])
        g = got[idx]
        if idx in ((0, 1, 1), (1, 0, 0)):
            # the resized brick's bytes outside the box were never written: compare the box
            fz, fy, fx = [r1 - r0 for r0, r1 in zip(ranges[idx][0][::-1], ranges[idx][1][::-1])]
            np.testing.assert_array_equal(g[:fz, :fy, :fx], ref.codes[:fz, :fy, :fx], err_msg=f"brick {idx}")
        else:
            np.testing.assert_array_equal(g, ref.codes, err_msg=f"brick {idx}")


@pytest.mark.gpu
def test_brick_too_small_is_rejected_before_any_launch():
    codes = np.arange(8 * 8 * 8, dtype=np.uint16).reshape(8, 8, 8)

    def tweak(arr):
        arr[(1, 1, 1)].setDims(2, 2, 2)

    err, _ = gpu_decompose(codes, 5, (0.0, 1.0), (4, 4, 4), (0, 0, 0), (0, 0, 0), tweak)
    assert err == vkt.InvalidValue
    assert "smaller than its range" in vkt.last_error()


@pytest.mark.gpu
def test_repeated_decompositions_stay_exact():
    """Back-to-back decompositions with changing formats / layouts (bricks and descriptor
    tables re-allocated at recycled addresses): a stream-ordered-pool version of the table
    upload was intermittently read stale here."""
    rng = np.random.default_rng(0)
    for it in range(40):
        fmt = (4, 5, 7, 6)[it % 4]
        dims, brick = ((10, 9, 8), (4, 4, 4)) if it % 3 else ((33, 17, 5), (8, 32, 2))
        codes = rand_codes(rng, fmt, dims[::-1])
        err, got = gpu_decompose(codes, fmt, (0.0, 1.0), brick, (1, 0, 1), (0, 1, 0))
        assert err == vkt.NoError
        ref = ob.brick_decompose(ob.Volume(codes, fmt), brick, (1, 0, 1), (0, 1, 0))
        for idx, v in ref.items():
            np.testing.assert_array_equal(got[idx], v.codes, err_msg=f"iteration {it} brick {idx}")


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [4, 5, 7])
def test_brick_decompose_small_bricks_large_volume(fmt):
    """32^3 bricks with a 1-voxel halo over a 160x96x64 volume: many bricks per row, items
    spanning two brick rows in every brick, loads at the first and last source bytes."""
    rng = np.random.default_rng(fmt + 40)
    codes = rand_codes(rng, fmt, (64, 96, 160))
    err, got = gpu_decompose(codes, fmt, (0.0, 1.0), (32, 32, 32), (1, 1, 1), (1, 1, 1))
    assert err == vkt.NoError, vkt.last_error()
    ref = ob.brick_decompose(ob.Volume(codes, fmt), (32, 32, 32), (1, 1, 1), (1, 1, 1))
    for idx, v in ref.items():
        np.testing.assert_array_equal(got[idx], v.codes, err_msg=f"brick {idx}")


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [5, 7])
def test_brick_decompose_narrow_rows(fmt):
    """8-voxel brick rows (a 16-KiB chunk spans up to 1025 rows of the staged copy)."""
    rng = np.random.default_rng(fmt + 50)
    codes = rand_codes(rng, fmt, (64, 64, 64))
    err, got = gpu_decompose(codes, fmt, (0.0, 1.0), (8, 64, 64), (0, 0, 0), (0, 0, 0))
    assert err == vkt.NoError, vkt.last_error()
    ref = ob.brick_decompose(ob.Volume(codes, fmt), (8, 64, 64), (0, 0, 0), (0, 0, 0))
    for idx, v in ref.items():
        np.testing.assert_array_equal(got[idx], v.codes, err_msg=f"brick {idx}")


@pytest.mark.gpu
def test_grid_entry_point_parity_and_validation():
    """vktHipBrickDecomposeGrid (the front-ends' path for BrickDecomposeResize-shaped arrays)
    through the C ABI: a 37x23x19 UInt16 source, 8^3 bricks with halos (2,1,0)/(1,2,3), bricks
    allocated at their box sizes, bit-exact vs the oracle; a halo wider than a brick takes the
    range path inside the call (same bytes); a null brick pointer, a brick inside the source and
    a brick count that is not ceil(dims / brickSize) are refused before any copy."""
    from volkit_amd import _lib as L
    rng = np.random.default_rng(77)
    dims = (37, 23, 19)
    codes = rand_codes(rng, 5, dims[::-1])
    nbytes = codes.nbytes
    p = C.c_void_p()
    assert lib.vktHipAllocate(C.byref(p), nbytes) == 0
    src_ptr = p.value
    assert lib.vktHipMemcpy(C.c_void_p(src_ptr), codes.ctypes.data, nbytes, 1) == 0
    src = L.HipVolumeView_t(src_ptr, *dims, 5, 0.0, 1.0)
    for brick, neg, pos in (((8, 8, 8), (2, 1, 0), (1, 2, 3)), ((4, 4, 4), (6, 1, 1), (5, 0, 2))):
        ref = ob.brick_decompose(ob.Volume(codes, 5), brick, neg, pos)
        nb = tuple(-(-d // b) for d, b in zip(dims, brick))
        ptrs, shapes = [], []
        for k in range(nb[2]):
            for j in range(nb[1]):
                for i in range(nb[0]):
                    shape = ref[(i, j, k)].codes.shape
                    q = C.c_void_p()
                    assert lib.vktHipAllocate(C.byref(q), int(np.prod(shape)) * 2) == 0
                    ptrs.append(q.value)
                    shapes.append(((i, j, k), shape))
        arr = (C.c_void_p * len(ptrs))(*ptrs)
        grid = L.HipBrickGrid_t(L.Vec3i_t(*nb), L.Vec3i_t(*brick), L.Vec3i_t(*neg), L.Vec3i_t(*pos))
        assert lib.vktHipBrickDecomposeGrid(src, grid, arr) == 0, L.last_error()
        assert lib.vktHipSynchronize() == 0
        for q, (idx, shape) in zip(ptrs, shapes):
            got = np.empty(shape, np.uint16)
            assert lib.vktHipMemcpy(got.ctypes.data, C.c_void_p(q), got.nbytes, 2) == 0
            np.testing.assert_array_equal(got, ref[idx].codes, err_msg=f"{brick} {neg} {pos} brick {idx}")
        bad = list(ptrs)
        bad[3] = None
        assert lib.vktHipBrickDecomposeGrid(src, grid, (C.c_void_p * len(bad))(*bad)) != 0
        bad[3] = src_ptr + 64
        assert lib.vktHipBrickDecomposeGrid(src, grid, (C.c_void_p * len(bad))(*bad)) != 0
        wrong = L.HipBrickGrid_t(L.Vec3i_t(nb[0] + 1, nb[1], nb[2]), L.Vec3i_t(*brick), L.Vec3i_t(*neg),
                                 L.Vec3i_t(*pos))
        assert lib.vktHipBrickDecomposeGrid(src, wrong, arr) != 0
        for q in ptrs:
            lib.vktHipFree(C.c_void_p(q))
    lib.vktHipFree(C.c_void_p(src_ptr))


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [4, 5, 7])
@pytest.mark.parametrize("dims,brick,neg,pos", LAYOUTS)
def test_brick_decompose_staged_grid_kernel(fmt, dims, brick, neg, pos):
    """Knob decompose.gather = 0: uniform grids keep the staged kernel (source words scattered
    into the brick layout in LDS) instead of the gather kernel (the default, tested above)."""
    rng = np.random.default_rng(fmt * 100 + sum(dims) + 11)
    codes = rand_codes(rng, fmt, dims[::-1])
    assert lib.vktHipSetTuningKnob(b"decompose.gather", 0) == 0
    try:
        err, got = gpu_decompose(codes, fmt, (0.0, 1.0), brick, neg, pos)
    finally:
        assert lib.vktHipSetTuningKnob(b"decompose.gather", -1) == 0
    assert err == vkt.NoError, vkt.last_error()
    ref = ob.brick_decompose(ob.Volume(codes, fmt), brick, neg, pos)
    for idx, v in ref.items():
        np.testing.assert_array_equal(got[idx], v.codes, err_msg=f"brick {idx}")


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [4, 5, 7])
@pytest.mark.parametrize("dims,brick,neg,pos", LAYOUTS + [((70, 33, 21), (16, 16, 16), (1, 1, 1), (1, 1, 1)),
                                                        ((45, 9, 5), (9, 4, 2), (2, 0, 1), (1, 3, 0))])
def test_brick_decompose_pair_kernel(fmt, dims, brick, neg, pos):
    """Knob decompose.pair = 1: two x-neighbour bricks of <= 16 KiB per workgroup, the union of
    their rows staged once into two LDS tiles (odd last bricks alone; bricks of several chunks and
    other lists keep the other kernels) -- every layout, bit-exact vs the oracle."""
    rng = np.random.default_rng(fmt * 100 + sum(dims) + 23)
    codes = rand_codes(rng, fmt, dims[::-1])
    assert lib.vktHipSetTuningKnob(b"decompose.pair", 1) == 0
    try:
        err, got = gpu_decompose(codes, fmt, (0.0, 1.0), brick, neg, pos)
    finally:
        assert lib.vktHipSetTuningKnob(b"decompose.pair", -1) == 0
    assert err == vkt.NoError, vkt.last_error()
    ref = ob.brick_decompose(ob.Volume(codes, fmt), brick, neg, pos)
    for idx, v in ref.items():
        np.testing.assert_array_equal(got[idx], v.codes, err_msg=f"brick {idx}")


DIRECT_LAYOUTS = [
    ((64, 64, 64), (64, 64, 64), (0, 0, 0), (0, 0, 0)),
    ((128, 40, 33), (16, 8, 5), (0, 0, 0), (0, 0, 0)),     # border bricks along y and z
    ((96, 20, 12), (32, 7, 5), (0, 0, 0), (0, 0, 0)),
    ((160, 9, 130), (32, 9, 64), (0, 0, 0), (0, 0, 0)),    # one brick along y, bricks of several chunks
    ((100, 20, 12), (20, 7, 5), (0, 0, 0), (0, 0, 0)),     # rows not whole 16-B words: staged kernel
    ((64, 24, 16), (16, 8, 8), (0, 0, 0), (0, 1, 0)),      # a halo: staged kernel
    ((176, 48, 40), (16, 16, 16), (0, 0, 0), (0, 0, 0)),   # 16^3: 2 (UInt16) / 4 (UInt8) bricks per workgroup,
    ((144, 20, 24), (16, 8, 8), (0, 0, 0), (0, 0, 0)),     # odd brick counts (a partial last workgroup)
]


@pytest.mark.gpu
@pytest.mark.parametrize("direct", [1, 2, 0])
@pytest.mark.parametrize("fmt", [4, 5, 7])
@pytest.mark.parametrize("dims,brick,neg,pos", DIRECT_LAYOUTS)
def test_brick_decompose_direct_kernel(fmt, dims, brick, neg, pos, direct):
    """Knob decompose.direct: halo-free grids whose box rows are whole 16-B words at aligned
    source offsets copy each word with one load and one store (brickDirect, no LDS tile; 1:
    small bricks 2 or 4 per workgroup, 2: one per workgroup); the other layouts and direct = 0
    keep the staged kernel -- bit-exact vs the oracle either way."""
    rng = np.random.default_rng(fmt * 100 + sum(dims) + 31)
    codes = rand_codes(rng, fmt, dims[::-1])
    assert lib.vktHipSetTuningKnob(b"decompose.direct", direct) == 0
    try:
        err, got = gpu_decompose(codes, fmt, (0.0, 1.0), brick, neg, pos)
    finally:
        assert lib.vktHipSetTuningKnob(b"decompose.direct", -1) == 0
    assert err == vkt.NoError, vkt.last_error()
    ref = ob.brick_decompose(ob.Volume(codes, fmt), brick, neg, pos)
    assert set(got) == set(ref)
    for idx, v in ref.items():
        np.testing.assert_array_equal(got[idx], v.codes, err_msg=f"brick {idx}")


ROW_IMAGE_LAYOUTS = [
    ((64, 40, 36), (16, 16, 16), (1, 1, 1), (1, 1, 1)),    # 16^3 + halo 1: clamped voxels at every border
    ((70, 33, 21), (16, 8, 8), (1, 0, 2), (0, 1, 1)),      # asymmetric halos, partial last bricks
    ((96, 20, 18), (32, 8, 8), (2, 1, 0), (3, 0, 1)),      # wider halos (<= 16 B of the left halo)
    ((64, 24, 16), (16, 8, 8), (0, 0, 0), (0, 1, 0)),      # halo in y only
    ((48, 16, 16), (8, 8, 8), (1, 1, 1), (1, 1, 1)),       # 8^3 + halo: rows of 10 voxels
]


@pytest.mark.gpu
@pytest.mark.parametrize("knob", [1, 0])
@pytest.mark.parametrize("fmt", [4, 5, 7])
@pytest.mark.parametrize("dims,brick,neg,pos", ROW_IMAGE_LAYOUTS)
def test_brick_decompose_row_image_kernel(fmt, dims, brick, neg, pos, knob):
    """Knob decompose.row_image (round 6): one brick per workgroup through per-row LDS images --
    aligned source words in, one 16-B piece per 16 B of a destination row out (the last piece
    overlapping), clamped border voxels beside the span -- bit-exact vs the oracle for every format
    (layouts whose rows are under 16 B, UInt8 8^3 + halo, fall back to the staged kernel); knob 0
    is the staged kernel on the same layouts (the default, 2, takes the row image for UInt8 only)."""
    rng = np.random.default_rng(fmt * 10 + sum(dims) + 77)
    codes = rand_codes(rng, fmt, dims[::-1])
    assert lib.vktHipSetTuningKnob(b"decompose.row_image", knob) == 0
    try:
        err, got = gpu_decompose(codes, fmt, (0.0, 1.0), brick, neg, pos)
    finally:
        assert lib.vktHipSetTuningKnob(b"decompose.row_image", -1) == 0
    assert err == vkt.NoError, vkt.last_error()
    ref = ob.brick_decompose(ob.Volume(codes, fmt), brick, neg, pos)
    assert set(got) == set(ref)
    for idx, v in ref.items():
        np.testing.assert_array_equal(got[idx], v.codes, err_msg=f"brick {idx}")
