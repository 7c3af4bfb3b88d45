// ResampleRow0.hip -- row kernel instantiations, MODE 0 (identity codes).
#include "ResampleRow.hpp"

namespace vkt
{
namespace hipk
{
    void launchRowMode0(ResampleArgs const& a, int32_t k, uint32_t bpv, unsigned grid, int32_t instrPerRow,
                        hipStream_t s)
    {
        if (bpv == 1) launchRowK<1, 1, 0, -1, -1>(a, k, grid, instrPerRow, s);
        else if (bpv == 2) launchRowK<2, 2, 0, -1, -1>(a, k, grid, instrPerRow, s);
        else launchRowK<4, 4, 0, -1, -1>(a, k, grid, instrPerRow, s);
    }
} // hipk
} // vkt
