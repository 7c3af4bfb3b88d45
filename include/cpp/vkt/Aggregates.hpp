// Forwarding header: reference include layout (include/cpp/vkt/Aggregates.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
