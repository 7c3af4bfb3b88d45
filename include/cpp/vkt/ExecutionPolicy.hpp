// Forwarding header: reference include layout (include/cpp/vkt/ExecutionPolicy.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
