"""Shared pytest setup.

Markers: ``gpu`` = needs an MI355X (run with ``-m gpu`` on the GPU box); everything else
runs on the CPU-only build container (oracle checks, host logic, ABI/export checks,
gloo multi-process tests).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X GPU (HIP device)")


@pytest.fixture(scope="session")
def oracle():
    from backends import OracleBackend
    return OracleBackend()


@pytest.fixture(scope="session")
def gpu():
    import torch  # noqa: F401  (only to probe for a device cheaply)
    from backends import GpuBackend
    b = GpuBackend()
    return b


@pytest.fixture(params=["oracle", "gpu"])
def backend(request):
    """Runs a test on the oracle (CPU) and, when selected with -m gpu, on the GPU library."""
    if request.param == "gpu":
        from backends import GpuBackend
        return GpuBackend()
    from backends import OracleBackend
    return OracleBackend()


def pytest_collection_modifyitems(config, items):
    # parametrised `backend` tests: the gpu variant carries the gpu marker
    for item in items:
        cs = getattr(item, "callspec", None)
        if cs is not None and cs.params.get("backend") == "gpu":
            item.add_marker(pytest.mark.gpu)
