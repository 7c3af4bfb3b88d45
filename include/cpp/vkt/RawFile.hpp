// Forwarding header: reference include layout (include/cpp/vkt/RawFile.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
