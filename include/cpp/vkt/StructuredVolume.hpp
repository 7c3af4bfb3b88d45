// Forwarding header: reference include layout (include/cpp/vkt/StructuredVolume.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
