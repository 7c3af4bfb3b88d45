/* HIP context/backend API (design intent of reference include/c/vkt/CudaContext.h). */
#pragma once
#include "../../volkit_hip.h"
