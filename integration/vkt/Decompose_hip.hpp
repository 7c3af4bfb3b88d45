// Decompose_hip.hpp -- replaces the C++ overload of src/vkt/Decompose_cuda.hpp (empty there,
// src/vkt/Decompose_cuda.cu:8-17) in src/vkt/Decompose.cpp: the brick ranges of
// BrickDecompose_serial (src/vkt/Decompose_serial.hpp:24-44), all bricks in one launch.
#pragma once
#include <algorithm>
#include <vector>

#include <vkt/Array3D.hpp>
#include "HipView.hpp"

namespace vkt
{
    inline void BrickDecompose_cuda(Array3D<StructuredVolume>& decomp, StructuredVolume& volume, Vec3i brickSize,
                                    Vec3i haloSizeNeg, Vec3i haloSizePos)
    {
        Vec3i dims = decomp.dims();
        Vec3i src = volume.getDims();
        std::vector<vktHipBrickRange_t> ranges;
        ranges.reserve(decomp.numElements());
        for (int z = 0; z < dims.z; ++z)
            for (int y = 0; y < dims.y; ++y)
                for (int x = 0; x < dims.x; ++x)
                {
                    Vec3i first{x * brickSize.x, y * brickSize.y, z * brickSize.z};
                    Vec3i last{std::min(first.x + brickSize.x, src.x), std::min(first.y + brickSize.y, src.y),
                               std::min(first.z + brickSize.z, src.z)};
                    first = {first.x - haloSizeNeg.x, first.y - haloSizeNeg.y, first.z - haloSizeNeg.z};
                    last = {last.x + haloSizePos.x, last.y + haloSizePos.y, last.z + haloSizePos.z};
                    ranges.push_back({HipView(decomp[Vec3i{x, y, z}]), C3(first), C3(last)});
                }
        vktHipBrickDecompose(HipView(volume), ranges.data(), static_cast<int32_t>(ranges.size()));
    }
} // vkt
