// Forwarding header: reference include layout (include/cpp/vkt/Copy.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
