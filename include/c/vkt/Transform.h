/* Forwarding header: reference include layout (include/c/vkt/Transform.h) -> the combined C API. */
#pragma once
#include "../../volkit_c.h"
