// Forwarding header: reference include layout (include/cpp/vkt/Render.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
