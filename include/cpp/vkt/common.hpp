// Forwarding header: reference include layout (include/cpp/vkt/common.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
