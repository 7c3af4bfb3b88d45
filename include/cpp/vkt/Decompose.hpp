// Forwarding header: reference include layout (include/cpp/vkt/Decompose.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
