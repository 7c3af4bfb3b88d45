"""RawFile / InputStream / OutputStream and the CLI's StructuredVolume stream (SURVEY.md §8(f)
F3), against restatements of reference src/vkt/RawFile.cpp:36-106 (file-name parsing),
src/vkt/InputStream.cpp:22-75 / OutputStream.cpp:20-60 (whole-volume and row-range transfers:
each line lands at x = 0 of its row, the reference's offset omits firstX) and
src/cli/main.cpp:32-88 (header layout).

CPU policy: bytes go straight to host memory (as in the reference).  GPU policy: the volume
lives in HBM and the transfer streams through pinned double buffers on the copy stream --
sizes above the 64 MiB staging chunk exercise the double buffering.
"""
import os
import struct

import numpy as np
import pytest

vkt = pytest.importorskip("volkit_amd.volkit")


def parse_name(name):
    """Restatement of RawFile's name parsing (RawFile.cpp:43-106)."""
    dims, fmt = (0, 0, 0), 4
    for tok in name.split("_"):
        import re
        m = re.match(r"^\s*([+-]?\d+)x([+-]?\d+)x([+-]?\d+)", tok)
        if m:
            dims = tuple(int(g) for g in m.groups())
        m = re.match(r"^int(\d+)", tok)
        if m:
            fmt = {8: 1, 16: 2, 32: 3}.get(int(m.group(1)), 0)
        m = re.match(r"^uint(\d+)", tok)
        if m:
            fmt = {8: 4, 16: 5, 32: 6}.get(int(m.group(1)), 0)
    return dims, fmt


@pytest.mark.parametrize("name", ["head_256x256x128_uint16.raw", "a_7x5x3_int8.raw", "b_uint32_64x64x64",
                                  "plain.raw", "c_10x20x30_uint12.raw", "d_int16_9x9x9_uint8.raw"])
def test_raw_file_name_parsing(tmp_path, name):
    p = tmp_path / name
    p.write_bytes(b"")
    f = vkt.RawFile(str(p), "rb")
    dims, fmt = parse_name(name)
    assert tuple(f.getDims()) == dims and f.getDataFormat() == fmt


def set_device(dev):
    ep = vkt.GetThreadExecutionPolicy()
    ep.device = dev
    vkt.SetThreadExecutionPolicy(ep)


def read_range_ref(codes_file, dims, first, last, init):
    """InputStream::readRange restated: lines in z->y order, stored at x = 0 of each row."""
    out = init.copy()
    n = last[0] - first[0]
    pos = 0
    for z in range(first[2], last[2]):
        for y in range(first[1], last[1]):
            out[z, y, :n] = codes_file[pos:pos + n]
            pos += n
    return out


def write_range_ref(codes, first, last):
    n = last[0] - first[0]
    return np.concatenate([codes[z, y, :n] for z in range(first[2], last[2]) for y in range(first[1], last[1])])


def run_stream_cases(tmp_path, device, dims, fmt=5):
    x, y, z = dims
    dt = {4: np.uint8, 5: np.uint16, 7: np.uint32}[fmt]
    rng = np.random.default_rng(sum(dims))
    codes = rng.integers(0, np.iinfo(dt).max, (z, y, x), dtype=np.uint64).astype(dt)
    path = tmp_path / f"v_{x}x{y}x{z}.raw"
    codes.tofile(path)
    set_device(vkt.ExecutionPolicy.Device_CPU)
    v = vkt.StructuredVolume(x, y, z, fmt)
    set_device(device)
    try:
        # whole volume
        f = vkt.RawFile(str(path), "rb")
        assert vkt.InputStream(f).read(v) == vkt.NoError
        f.close()
        # row range (reference quirk: lines at x = 0)
        first, last = (x // 3, y // 3, z // 3), (x - x // 4, y - y // 4, z - z // 4)
        nline = (last[0] - first[0])
        stream = rng.integers(0, np.iinfo(dt).max, (last[2] - first[2]) * (last[1] - first[1]) * nline,
                              dtype=np.uint64).astype(dt)
        rpath = tmp_path / "range.raw"
        stream.tofile(rpath)
        w = vkt.StructuredVolume(x, y, z, fmt)
        w.from_numpy(codes)
        f = vkt.RawFile(str(rpath), "rb")
        assert vkt.InputStream(f).readRange(w, *first, *last) == vkt.NoError
        f.close()
        # write back: whole volume and a range
        opath = tmp_path / "out.raw"
        f = vkt.RawFile(str(opath), "wb")
        assert vkt.OutputStream(f).write(w) == vkt.NoError
        f.close()
        opath2 = tmp_path / "out_range.raw"
        f = vkt.RawFile(str(opath2), "wb")
        assert vkt.OutputStream(f).writeRange(w, *first, *last) == vkt.NoError
        f.close()
    finally:
        set_device(vkt.ExecutionPolicy.Device_CPU)
    np.testing.assert_array_equal(v.to_numpy(), codes)
    exp = read_range_ref(stream, dims, first, last, codes)
    np.testing.assert_array_equal(w.to_numpy(), exp)
    np.testing.assert_array_equal(np.fromfile(opath, dtype=dt).reshape(z, y, x), exp)
    np.testing.assert_array_equal(np.fromfile(opath2, dtype=dt), write_range_ref(exp, first, last))


def test_streams_cpu_policy(tmp_path):
    run_stream_cases(tmp_path, vkt.ExecutionPolicy.Device_CPU, (33, 20, 9))


def test_sv_stream_header_layout_and_roundtrip(tmp_path):
    """Header written by the reference CLI (main.cpp:71-88): u32 magic 1, u32 type 0, 3 x i32
    dims, u32 format, 3 x f32 dist, 2 x f32 mapping, then the voxels."""
    codes = np.arange(5 * 4 * 3, dtype=np.uint16).reshape(3, 4, 5)
    raw = struct.pack("<II3iI3f2f", 1, 0, 5, 4, 3, 5, 1.0, 2.0, 0.5, -1.0, 3.0) + codes.tobytes()
    p = tmp_path / "in.sv"
    p.write_bytes(raw)
    v = vkt.StructuredVolume()
    f = vkt.RawFile(str(p), "rb")
    assert vkt.ReadSVStream(f, v) == vkt.NoError
    f.close()
    assert tuple(v.getDims()) == (5, 4, 3) and v.getDataFormat() == 5 and v.getDist() == (1.0, 2.0, 0.5)
    np.testing.assert_array_equal(v.to_numpy(), codes)
    q = tmp_path / "out.sv"
    f = vkt.RawFile(str(q), "wb")
    assert vkt.WriteSVStream(f, v) == vkt.NoError
    f.close()
    assert q.read_bytes() == raw
    # wrong magic / truncated body / missing file
    bad = tmp_path / "bad.sv"
    bad.write_bytes(struct.pack("<II", 2, 0) + raw[8:])
    f = vkt.RawFile(str(bad), "rb")
    assert vkt.ReadSVStream(f, vkt.StructuredVolume()) == vkt.ReadError
    f.close()
    short = tmp_path / "short.sv"
    short.write_bytes(raw[:-3])
    f = vkt.RawFile(str(short), "rb")
    assert vkt.ReadSVStream(f, vkt.StructuredVolume()) == vkt.ReadError
    f.close()
    f = vkt.RawFile(str(tmp_path / "missing.raw"), "rb")
    assert not f.good()
    assert vkt.InputStream(f).read(vkt.StructuredVolume(2, 2, 2, 4)) == vkt.InvalidDataSource


@pytest.mark.gpu
@pytest.mark.parametrize("dims,fmt", [((33, 20, 9), 5), ((1, 1, 1), 4), ((512, 256, 260), 5), ((96, 2, 1), 7)])
def test_streams_gpu_policy(tmp_path, dims, fmt):
    """(512, 256, 260) UInt16 = 65 MiB: more than one 64 MiB staging chunk."""
    run_stream_cases(tmp_path, vkt.ExecutionPolicy.Device_GPU, dims, fmt)


@pytest.mark.gpu
def test_sv_stream_gpu_policy(tmp_path):
    codes = np.random.default_rng(0).integers(0, 256, (17, 9, 31), dtype=np.uint8)
    set_device(vkt.ExecutionPolicy.Device_GPU)
    try:
        v = vkt.StructuredVolume(31, 9, 17, vkt.DataFormat_UInt8)
        v.from_numpy(codes)
        f = vkt.RawFile(str(tmp_path / "g.sv"), "wb")
        assert vkt.WriteSVStream(f, v) == vkt.NoError
        f.close()
        w = vkt.StructuredVolume()
        f = vkt.RawFile(str(tmp_path / "g.sv"), "rb")
        assert vkt.ReadSVStream(f, w) == vkt.NoError   # allocated in HBM, streamed in
        f.close()
        assert vkt.SumRange(w, w, w, 0, 0, 0, 31, 9, 17) == vkt.NoError   # usable by kernels
    finally:
        set_device(vkt.ExecutionPolicy.Device_CPU)
    from oracle import binding as ob
    ref = ob.Volume.zeros((31, 9, 17), 4)
    ob.arith_range("Sum", ref, ob.Volume(codes, 4), ob.Volume(codes, 4), (0, 0, 0), (31, 9, 17))
    np.testing.assert_array_equal(w.to_numpy(), ref.codes)


def test_large_host_read_in_parallel_keeps_the_stream_position(tmp_path):
    """InputStream::read into a host volume of >= 64 MiB reads the file with parallel preads at
    the stream's position (RawFile::readParallel): the volume's bytes, then a second, small read
    from the same RawFile continues right after them (the FILE position advanced as fread would);
    a file shorter than the volume gives ReadError."""
    dims = (512, 288, 256)                         # 72 MiB of UInt16
    n = dims[0] * dims[1] * dims[2]
    rng = np.random.default_rng(5)
    head = rng.integers(0, 65535, 7, dtype=np.uint16)          # read first, small (fread)
    big = rng.integers(0, 65535, n, dtype=np.uint16)
    tail = rng.integers(0, 65535, 2 * 3 * 4, dtype=np.uint16)
    path = tmp_path / "big.raw"
    np.concatenate([head, big, tail]).tofile(path)
    set_device(vkt.ExecutionPolicy.Device_CPU)
    a = vkt.StructuredVolume(7, 1, 1, 5)
    v = vkt.StructuredVolume(*dims, 5)
    w = vkt.StructuredVolume(2, 3, 4, 5)
    f = vkt.RawFile(str(path), "rb")
    s = vkt.InputStream(f)
    assert s.read(a) == vkt.NoError
    assert s.read(v) == vkt.NoError
    assert s.read(w) == vkt.NoError
    f.close()
    np.testing.assert_array_equal(a.to_numpy().reshape(-1), head)
    np.testing.assert_array_equal(v.to_numpy().reshape(-1), big)
    np.testing.assert_array_equal(w.to_numpy().reshape(-1), tail)
    short = tmp_path / "short.raw"
    big[: n - 1000].tofile(short)
    f = vkt.RawFile(str(short), "rb")
    assert vkt.InputStream(f).read(v) == vkt.ReadError
    f.close()
