// PointwiseArith4.hip -- instantiations of the arithmetic kernels for ops 8 and 9.
#include "PointwiseOps.hpp"

namespace vkt
{
namespace hipk
{
    vktError arithmeticPair4(int op, PwPlan const& p, vktHipVolumeView_t const& d, vktHipVolumeView_t const& a,
                             vktHipVolumeView_t const& b, hipStream_t s)
    {
        return op == 8 ? arithmetic<8>(p, d, a, b, s) : arithmetic<9>(p, d, a, b, s);
    }
} // hipk
} // vkt
