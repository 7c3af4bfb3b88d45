// HostPool.hpp -- a small persistent pool of host threads for the library's host-side planning
// loops (BrickDecompose walks and describes up to 262 144 bricks per call, 30 ns each).
#pragma once

#include <cstddef>
#include <functional>

namespace vkt
{
namespace rt
{
    // Runs fn(begin, end) over [0, n) in contiguous chunks of at least minChunk items on up to
    // hostThreads() threads (the caller is one of them) and returns when every chunk is done.
    // Chunks may run in any order and concurrently: fn must only write state of its own items.
    // A call while another thread's parallelFor is running (or from inside fn) runs serially on
    // the calling thread.  Worker threads start with the calling thread's HIP device.
    void parallelFor(size_t n, size_t minChunk, std::function<void(size_t, size_t)> const& fn);

    // Threads parallelFor uses: VKT_HOST_THREADS if set (1 = serial), else min(16, cores).
    int hostThreads();
} // rt
} // vkt
