/* Forwarding header: reference include layout (include/c/vkt/OutputStream.h) -> the combined C API. */
#pragma once
#include "../../volkit_c.h"
