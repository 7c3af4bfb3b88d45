"""Source compatibility: a C99 user and a C++ user written against the reference's include
layout (`#include <vkt/...>`) compile with gcc / g++ against include/, link libvolkit.so and
run their CPU-policy parts (CPU only: no kernels).  Modelled on reference
src/examples/Decompose.c and src/examples/Decompose.cpp."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = [f"-I{ROOT}/include/c", f"-I{ROOT}/include/cpp", f"-I{ROOT}/include"]
LIBDIR = os.path.join(ROOT, "volkit_amd", "lib")

C_USER = r"""
#include <stdio.h>
#include <vkt/Decompose.h>
#include <vkt/ExecutionPolicy.h>
#include <vkt/Fill.h>
#include <vkt/StructuredVolume.h>
int main(void)
{
    vktStructuredVolume volume;
    vktArray3D_vktStructuredVolume decomp;
    vktVec3i_t d, idx = {7, 4, 3};
    vktStructuredVolumeCreate(&volume, 120, 66, 49, vktDataFormatUInt8, 1.f, 1.f, 1.f, 0.f, 1.f);
    vktArray3D_vktStructuredVolume_CreateEmpty(&decomp);
    if (vktBrickDecomposeResizeSV(decomp, volume, 16, 16, 16, 1, 1, 1, 1, 1, 1) != vktNoError) return 1;
    d = vktArray3D_vktStructuredVolume_Dims(decomp);
    vktVec3i_t bd = vktStructuredVolumeGetDims3iv(*vktArray3D_vktStructuredVolume_Access(decomp, idx));
    /* CPU policy: this library is the GPU backend, algorithms refuse instead of falling back */
    int refused = vktFillSV(volume, .1f) == vktInvalidValue;
    printf("%d %d %d %d %d %d %d\n", d.x, d.y, d.z, bd.x, bd.y, bd.z, refused);
    vktArray3D_vktStructuredVolume_Destroy(decomp);
    vktStructuredVolumeDestroy(volume);
    return 0;
}
"""

CPP_USER = r"""
#include <cstdio>
#include <vkt/Array3D.hpp>
#include <vkt/Decompose.hpp>
#include <vkt/ExecutionPolicy.hpp>
#include <vkt/Resample.hpp>
#include <vkt/StructuredVolume.hpp>
int main()
{
    vkt::StructuredVolume volume(120, 66, 49, vkt::DataFormat::UInt16, 1.f, 1.f, 1.f, -1.f, 3.f);
    vkt::Array3D<vkt::StructuredVolume> decomp;
    vkt::BrickDecomposeResize(decomp, volume, {16, 16, 16}, {1, 1, 1}, {1, 1, 1});
    vkt::Vec3i d = decomp.dims();
    vkt::Vec3i bd = decomp[vkt::Vec3i{7, 4, 3}].getDims();
    vkt::Vec2f m = decomp[vkt::Vec3i{0, 0, 0}].getVoxelMapping();
    volume.setValue(3, 2, 1, 0.5f);
    float v = volume.getValue(3, 2, 1);
    int refused = vkt::Resample(volume, volume, vkt::FilterMode::Linear) == vkt::InvalidValue;
    std::printf("%d %d %d %d %d %d %g %g %g %d\n", d.x, d.y, d.z, bd.x, bd.y, bd.z, m.x, m.y, v, refused);
    return 0;
}
"""


def build_and_run(tmp_path, name, src, compiler, extra):
    path = tmp_path / name
    path.write_text(src)
    exe = tmp_path / (name + ".bin")
    subprocess.run([compiler, *extra, *INC, str(path), "-o", str(exe), f"-L{LIBDIR}", "-lvolkit",
                    f"-Wl,-rpath,{LIBDIR}"], check=True, capture_output=True, text=True)
    env = dict(os.environ, VKT_LOG_LEVEL="0")
    res = subprocess.run([str(exe)], check=True, capture_output=True, text=True, env=env, timeout=120)
    return res.stdout.strip().splitlines()[-1].split()   # last line: the program output (logs go before)


@pytest.mark.skipif(not os.path.exists(os.path.join(LIBDIR, "libvolkit.so")), reason="libvolkit.so not built")
def test_c99_user(tmp_path):
    out = build_and_run(tmp_path, "user.c", C_USER, "gcc", ["-std=c99", "-Wall", "-Werror"])
    assert out == ["8", "5", "4", "10", "4", "3", "1"]


@pytest.mark.skipif(not os.path.exists(os.path.join(LIBDIR, "libvolkit.so")), reason="libvolkit.so not built")
def test_cpp_user(tmp_path):
    out = build_and_run(tmp_path, "user.cpp", CPP_USER, "g++", ["-std=c++14", "-Wall", "-Werror"])
    assert out == ["8", "5", "4", "10", "4", "3", "-1", "3", "0.5", "1"]
