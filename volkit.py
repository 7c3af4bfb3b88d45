"""``import volkit as vkt`` -- the reference's Python module name (reference
src/vkt/volkit.i:11, ``%module volkit``; its examples start with ``import volkit as vkt``).

Re-exports the SWIG-named API of ``volkit_amd.volkit`` (ctypes over libvolkit.so's C ABI), so
a reference script runs against this library with the repository on ``PYTHONPATH``.  This
library is the GPU backend: algorithms need ``ExecutionPolicy.Device_GPU`` -- set it in the
script, or run unmodified scripts (which never set a policy) with ``VKT_DEFAULT_DEVICE=GPU``.
"""
from volkit_amd.volkit import *  # noqa: F401,F403
