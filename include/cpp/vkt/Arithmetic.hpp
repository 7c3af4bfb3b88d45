// Forwarding header: reference include layout (include/cpp/vkt/Arithmetic.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
