// Forwarding header: reference include layout (include/cpp/vkt/linalg.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
