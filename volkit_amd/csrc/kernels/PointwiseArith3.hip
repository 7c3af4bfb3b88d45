// PointwiseArith3.hip -- instantiations of the arithmetic kernels for ops 6 and 7.
#include "PointwiseOps.hpp"

namespace vkt
{
namespace hipk
{
    vktError arithmeticPair3(int op, PwPlan const& p, vktHipVolumeView_t const& d, vktHipVolumeView_t const& a,
                             vktHipVolumeView_t const& b, hipStream_t s)
    {
        return op == 6 ? arithmetic<6>(p, d, a, b, s) : arithmetic<7>(p, d, a, b, s);
    }
} // hipk
} // vkt
