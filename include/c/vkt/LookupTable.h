/* Forwarding header: reference include layout (include/c/vkt/LookupTable.h) -> the combined C API. */
#pragma once
#include "../../volkit_c.h"
