// Forwarding header: reference include layout (include/cpp/vkt/Fill.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
