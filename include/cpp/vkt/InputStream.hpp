// Forwarding header: reference include layout (include/cpp/vkt/InputStream.hpp) -> the combined C++ API.
#pragma once
#include "../../volkit.hpp"
