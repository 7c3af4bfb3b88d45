// PointwiseArith0.hip -- instantiations of the arithmetic kernels for ops 0 and 1.
#include "PointwiseOps.hpp"

namespace vkt
{
namespace hipk
{
    vktError arithmeticPair0(int op, PwPlan const& p, vktHipVolumeView_t const& d, vktHipVolumeView_t const& a,
                             vktHipVolumeView_t const& b, hipStream_t s)
    {
        return op == 0 ? arithmetic<0>(p, d, a, b, s) : arithmetic<1>(p, d, a, b, s);
    }
} // hipk
} // vkt
