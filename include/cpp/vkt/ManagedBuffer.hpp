// Forwarding header: reference include layout (include/cpp/vkt/ManagedBuffer.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
