// ResampleRow1.hip -- row kernel instantiations, MODE 1 (convert each source code).
#include "ResampleRow.hpp"

namespace vkt
{
namespace hipk
{
    void launchRowMode1(ResampleArgs const& a, int32_t k, uint32_t bpv, int32_t fs, int32_t fd, unsigned grid,
                        int32_t instrPerRow, hipStream_t s)
    {
        if (fs == codec::FmtUInt16 && fd == codec::FmtUInt16)
            launchRowK<2, 2, 1, codec::FmtUInt16, codec::FmtUInt16>(a, k, grid, instrPerRow, s);
        else if (fs == codec::FmtFloat32 && fd == codec::FmtFloat32)   // config 3 Nearest
            launchRowK<4, 4, 1, codec::FmtFloat32, codec::FmtFloat32>(a, k, grid, instrPerRow, s);
        else if (fs == codec::FmtUInt8 && fd == codec::FmtUInt8)
            launchRowK<1, 1, 1, codec::FmtUInt8, codec::FmtUInt8>(a, k, grid, instrPerRow, s);
        else if (bpv == 1) launchRowK<1, 1, 1, -1, -1>(a, k, grid, instrPerRow, s);
        else if (bpv == 2) launchRowK<2, 2, 1, -1, -1>(a, k, grid, instrPerRow, s);
        else launchRowK<4, 4, 1, -1, -1>(a, k, grid, instrPerRow, s);
    }
} // hipk
} // vkt
