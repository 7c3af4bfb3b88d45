/* Forwarding header: reference include layout (include/c/vkt/InputStream.h) -> the combined C API. */
#pragma once
#include "../../volkit_c.h"
