"""Context handles (include/volkit_hip.h vktHipContext*): the reference's vktCudaContext API
(include/c/vkt/CudaContext.h:17-65, declared but never defined there) for HIP -- streams owned
by the context or given by the caller, compute / copy stream ids, the async flag, bound to the
backend with vktHipContextMakeCurrent."""
import ctypes as C

import numpy as np
import pytest

from volkit_amd import _lib
from volkit_amd._lib import lib

pytestmark = pytest.mark.gpu


def _ok(e):
    assert e == 0, _lib.last_error()


def test_context_streams_ids_and_binding():
    import torch
    torch.cuda.set_device(0)
    ctx = C.c_void_p()
    _ok(lib.vktHipContextCreate(C.byref(ctx)))
    try:
        n, cid, pid, a = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int32()
        _ok(lib.vktHipContextGetNumStreams(ctx, C.byref(n)))
        _ok(lib.vktHipContextGetComputeStreamId(ctx, C.byref(cid)))
        _ok(lib.vktHipContextGetCopyStreamId(ctx, C.byref(pid)))
        assert (n.value, cid.value, pid.value) == (2, 0, 1)
        _ok(lib.vktHipContextSetNumStreams(ctx, 4))
        _ok(lib.vktHipContextSetComputeStreamId(ctx, 3))
        _ok(lib.vktHipContextSetCopyStreamId(ctx, 2))
        assert lib.vktHipContextSetComputeStreamId(ctx, 4) != 0          # out of range
        user = torch.cuda.Stream()
        _ok(lib.vktHipContextSetStream(ctx, 2, C.c_void_p(user.cuda_stream)))
        s3, s2 = C.c_void_p(), C.c_void_p()
        _ok(lib.vktHipContextGetStream(ctx, 3, C.byref(s3)))
        _ok(lib.vktHipContextGetStream(ctx, 2, C.byref(s2)))
        assert s2.value == user.cuda_stream and s3.value
        _ok(lib.vktHipContextSetAsyncExecution(ctx, 0))
        _ok(lib.vktHipContextGetAsyncExecution(ctx, C.byref(a)))
        assert a.value == 0
        # bound: the backend runs on stream 3, migrates on the caller's stream, synchronously
        own = C.c_void_p()
        _ok(lib.vktHipGetComputeStream(C.byref(own)))
        _ok(lib.vktHipContextMakeCurrent(ctx))
        cs, ps = C.c_void_p(), C.c_void_p()
        _ok(lib.vktHipGetComputeStream(C.byref(cs)))
        _ok(lib.vktHipGetCopyStream(C.byref(ps)))
        assert cs.value == s3.value and ps.value == user.cuda_stream
        _ok(lib.vktHipGetAsyncExecution(C.byref(a)))
        assert a.value == 0
        # an algorithm on the context's stream (synchronous: the result is there on return)
        t = torch.zeros(4096, dtype=torch.uint16, device="cuda")
        torch.cuda.synchronize()
        v = _lib.HipVolumeView_t(t.data_ptr(), 16, 16, 16, 5, 0.0, 1.0)
        _ok(lib.vktHipFillRange(v, _lib.Vec3i_t(0, 0, 0), _lib.Vec3i_t(16, 16, 16), C.c_float(1.0 / 65535.0 * 7)))
        assert (t.cpu().numpy() == 7).all()
        # a setter on the current context takes effect at once
        _ok(lib.vktHipContextSetComputeStreamId(ctx, 1))
        s1 = C.c_void_p()
        _ok(lib.vktHipContextGetStream(ctx, 1, C.byref(s1)))
        _ok(lib.vktHipGetComputeStream(C.byref(cs)))
        assert cs.value == s1.value
        _ok(lib.vktHipContextMakeCurrent(None))
        _ok(lib.vktHipGetComputeStream(C.byref(cs)))
        assert cs.value == own.value
        _ok(lib.vktHipContextMakeCurrent(ctx))
    finally:
        _ok(lib.vktHipContextDestroy(ctx))     # current: restores the backend's own streams
        _ok(lib.vktHipSetAsyncExecution(1))
    cs = C.c_void_p()
    _ok(lib.vktHipGetComputeStream(C.byref(cs)))
    assert cs.value == own.value


def test_context_argument_checks():
    assert lib.vktHipContextCreate(None) != 0
    assert lib.vktHipContextSetNumStreams(None, 2) != 0
    assert lib.vktHipContextDestroy(None) == 0
    ctx = C.c_void_p()
    _ok(lib.vktHipContextCreate(C.byref(ctx)))
    try:
        assert lib.vktHipContextSetNumStreams(ctx, 0) != 0
        assert lib.vktHipContextSetStream(ctx, 5, C.c_void_p(1)) != 0
        _ok(lib.vktHipContextSetNumStreams(ctx, 1))        # ids clamp to the remaining stream
        cid, pid = C.c_int32(), C.c_int32()
        _ok(lib.vktHipContextGetComputeStreamId(ctx, C.byref(cid)))
        _ok(lib.vktHipContextGetCopyStreamId(ctx, C.byref(pid)))
        assert (cid.value, pid.value) == (0, 0)
    finally:
        _ok(lib.vktHipContextDestroy(ctx))


def test_shrinking_the_current_context_with_work_queued():
    """SetNumStreams on the CURRENT context while kernels are queued on the compute stream it
    removes (and SetStream replacing a bound owned stream): the backend is rebound to a surviving
    stream and the old one is synchronised before it is destroyed, so the queued work finishes and
    later calls run on a live stream."""
    import torch
    torch.cuda.set_device(0)
    ctx = C.c_void_p()
    _ok(lib.vktHipContextCreate(C.byref(ctx)))
    n = 256
    t = torch.zeros(n * n * n, dtype=torch.uint16, device="cuda")
    torch.cuda.synchronize()
    v = _lib.HipVolumeView_t(t.data_ptr(), n, n, n, 5, 0.0, 1.0)
    o, last = _lib.Vec3i_t(0, 0, 0), _lib.Vec3i_t(n, n, n)
    try:
        _ok(lib.vktHipContextSetNumStreams(ctx, 4))
        _ok(lib.vktHipContextSetComputeStreamId(ctx, 3))
        _ok(lib.vktHipContextMakeCurrent(ctx))
        for k in range(40):   # queued on stream 3, asynchronously
            _ok(lib.vktHipFillRange(v, o, last, C.c_float((k + 1) / 65536.0)))
        _ok(lib.vktHipContextSetNumStreams(ctx, 2))        # stream 3 goes: rebind, sync, destroy
        cs, s1 = C.c_void_p(), C.c_void_p()
        _ok(lib.vktHipGetComputeStream(C.byref(cs)))
        _ok(lib.vktHipContextGetStream(ctx, 1, C.byref(s1)))
        assert cs.value == s1.value
        _ok(lib.vktHipFillRange(v, o, last, C.c_float(41 / 65536.0)))   # on the new stream
        for k in range(10):
            _ok(lib.vktHipFillRange(v, o, last, C.c_float((k + 100) / 65536.0)))
        user = torch.cuda.Stream()
        _ok(lib.vktHipContextSetStream(ctx, 1, C.c_void_p(user.cuda_stream)))   # replaces the bound stream
        _ok(lib.vktHipGetComputeStream(C.byref(cs)))
        assert cs.value == user.cuda_stream
        _ok(lib.vktHipFillRange(v, o, last, C.c_float(7 / 65536.0)))
        _ok(lib.vktHipSynchronize())
        assert (t.cpu().numpy() == 7).all()
    finally:
        _ok(lib.vktHipContextDestroy(ctx))
