// Forwarding header: reference include layout (include/cpp/vkt/Memory.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
