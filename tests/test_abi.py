"""The C-ABI library loads and exports every function that include/*.h declares (CPU only:
no compute calls)."""
import ctypes
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DECL = re.compile(r"VKTAPI\s+[\w\s\*]+?\b(vkt\w+)\s*\(")
MACRO_ARITH = ["Sum", "Diff", "Prod", "Quot", "AbsDiff", "SafeSum", "SafeDiff", "SafeProd", "SafeQuot", "SafeAbsDiff"]


def declared_symbols():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        for m in DECL.finditer(text):
            if "##" not in m.group(0):
                names.add(m.group(1))
        if "VKT_DECLARE_ARITHMETIC_C_" in text:
            for op in MACRO_ARITH:
                names.add(f"vkt{op}SV")
                names.add(f"vkt{op}RangeSV")
    return sorted(names)


def test_headers_declare_the_hot_path():
    names = declared_symbols()
    for must in ["vktFillSV", "vktFillRangeSV", "vktCopyRangeSV", "vktSumRangeSV", "vktSafeSumRangeSV",
                 "vktSafeDiffRangeSV", "vktResampleSV", "vktTransformRangeSV2", "vktStructuredVolumeMigrate",
                 "vktHipResample", "vktHipArithmeticRange", "vktHipResampleSlab", "vktHipMemsetRange"]:
        assert must in names
    assert len(names) > 85


@pytest.mark.parametrize("name", declared_symbols())
def test_library_exports(name):
    lib = ctypes.CDLL(os.path.join(ROOT, "volkit_amd", "lib", "libvolkit.so"))
    assert hasattr(lib, name), f"{name} declared in include/*.h but not exported"


def test_python_binding_covers_every_export():
    from volkit_amd import _lib
    missing = [n for n in declared_symbols() if n not in _lib.SIGNATURES]
    assert not missing, missing


def test_forwarding_headers_point_at_the_api():
    # `#include <vkt/Fill.h>` / `<vkt/StructuredVolume.hpp>` keep working (reference include layout)
    for sub in ("c/vkt/Fill.h", "c/vkt/Arithmetic.h", "cpp/vkt/StructuredVolume.hpp", "cpp/vkt/Resample.hpp"):
        assert os.path.exists(os.path.join(ROOT, "include", sub)), sub
