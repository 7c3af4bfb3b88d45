// PointwiseArith2.hip -- instantiations of the arithmetic kernels for ops 4 and 5.
#include "PointwiseOps.hpp"

namespace vkt
{
namespace hipk
{
    vktError arithmeticPair2(int op, PwPlan const& p, vktHipVolumeView_t const& d, vktHipVolumeView_t const& a,
                             vktHipVolumeView_t const& b, hipStream_t s)
    {
        return op == 4 ? arithmetic<4>(p, d, a, b, s) : arithmetic<5>(p, d, a, b, s);
    }
} // hipk
} // vkt
