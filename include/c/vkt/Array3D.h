/* Forwarding header: reference include layout (include/c/vkt/Array3D.h) -> the combined C API. */
#pragma once
#include "../../volkit_c.h"
