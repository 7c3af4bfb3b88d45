// Forwarding header: reference include layout (include/cpp/vkt/Array3D.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
