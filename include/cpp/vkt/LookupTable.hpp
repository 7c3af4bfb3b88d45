// Forwarding header: reference include layout (include/cpp/vkt/LookupTable.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
