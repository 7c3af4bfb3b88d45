// Forwarding header: reference include layout (include/cpp/vkt/Voxel.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
