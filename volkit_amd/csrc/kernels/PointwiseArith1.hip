// PointwiseArith1.hip -- instantiations of the arithmetic kernels for ops 2 and 3.
#include "PointwiseOps.hpp"

namespace vkt
{
namespace hipk
{
    vktError arithmeticPair1(int op, PwPlan const& p, vktHipVolumeView_t const& d, vktHipVolumeView_t const& a,
                             vktHipVolumeView_t const& b, hipStream_t s)
    {
        return op == 2 ? arithmetic<2>(p, d, a, b, s) : arithmetic<3>(p, d, a, b, s);
    }
} // hipk
} // vkt
