"""volkit_amd -- MI355X-native (gfx950) backend of volkit's StructuredVolume core path.

* ``volkit_amd.volkit``  -- the volkit Python API (SWIG names) over libvolkit.so's C ABI.
* ``volkit_amd.slab``    -- Z-slab partitioning across one process per GPU (torch.distributed).
* ``volkit_amd._lib``    -- raw ctypes binding; importing it fails loudly if the library is
                            not built (there is no CPU fallback).
"""
from . import _lib  # noqa: F401  (raises VolkitLibraryMissing if libvolkit.so is absent)
from . import volkit  # noqa: F401

__all__ = ["volkit"]
