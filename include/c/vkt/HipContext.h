/* HIP context handles: vktHipContext* (reference include/c/vkt/CudaContext.h:17-65, for HIP streams). */
#pragma once
#include "../../volkit_hip.h"
