// Memory_hip.hpp -- replaces src/vkt/Memory_cuda.hpp (:16-31) in src/vkt/Memory.cpp; the
// cudaMemcpy of Memcpy() (src/vkt/Memory.cpp:40-75) becomes vktHipMemcpy(dst, src, size,
// (vktCopyKind)ck) (same CopyKind values).
#pragma once
#include <cstddef>
#include <volkit_hip.h>

namespace vkt
{
    inline void Allocate_cuda(void** ptr, std::size_t size) { vktHipAllocate(ptr, size); }

    inline void Free_cuda(void* ptr) { vktHipFree(ptr); }

    inline void MemsetRange_cuda(void* dst, void const* src, std::size_t dstSize, std::size_t srcSize)
    {
        vktHipMemsetRange(dst, src, dstSize, srcSize);
    }
} // vkt
