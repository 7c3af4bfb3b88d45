// Forwarding header: reference include layout (include/cpp/vkt/forward.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
