/* Forwarding header: reference include layout (include/c/vkt/Render.h) -> the combined C API. */
#pragma once
#include "../../volkit_c.h"
