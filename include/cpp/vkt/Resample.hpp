// Forwarding header: reference include layout (include/cpp/vkt/Resample.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
