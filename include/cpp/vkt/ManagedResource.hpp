// Forwarding header: reference include layout (include/cpp/vkt/ManagedResource.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
