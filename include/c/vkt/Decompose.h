/* Forwarding header: reference include layout (include/c/vkt/Decompose.h) -> the combined C API. */
#pragma once
#include "../../volkit_c.h"
