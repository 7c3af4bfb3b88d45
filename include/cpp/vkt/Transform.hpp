// Forwarding header: reference include layout (include/cpp/vkt/Transform.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
