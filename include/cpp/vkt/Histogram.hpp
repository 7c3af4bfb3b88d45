// Forwarding header: reference include layout (include/cpp/vkt/Histogram.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
