// Forwarding header: reference include layout (include/cpp/vkt/OutputStream.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
