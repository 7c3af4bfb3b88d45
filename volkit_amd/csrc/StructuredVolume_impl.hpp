// StructuredVolume_impl.hpp -- the C handle wraps the C++ object
// (reference src/vkt/StructuredVolume_impl.hpp:10-33).
#pragma once

#include <utility>

#include "volkit.hpp"

struct vktStructuredVolume_impl
{
    template <typename... Args>
    explicit vktStructuredVolume_impl(Args&&... args) : volume(std::forward<Args>(args)...)
    {
    }

    vkt::StructuredVolume volume;
};
