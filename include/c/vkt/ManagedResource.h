/* Forwarding header: reference include layout (include/c/vkt/ManagedResource.h) -> the combined C API. */
#pragma once
#include "../../volkit_c.h"
