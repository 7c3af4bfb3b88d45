// ResampleRow2.hip -- row kernel instantiations, MODE 2 (Float32 source, lerp chain).
#include "ResampleRow.hpp"

namespace vkt
{
namespace hipk
{
    void launchRowMode2(ResampleArgs const& a, int32_t k, uint32_t bpvd, unsigned grid, int32_t instrPerRow,
                        hipStream_t s)
    {
        if (bpvd == 4)
            launchRowK<4, 4, 2, codec::FmtFloat32, -1>(a, k, grid, instrPerRow, s);
        else if (bpvd == 2)
            launchRowK<4, 2, 2, codec::FmtFloat32, -1>(a, k, grid, instrPerRow, s);
        else
            launchRowK<4, 1, 2, codec::FmtFloat32, -1>(a, k, grid, instrPerRow, s);
    }
} // hipk
} // vkt
