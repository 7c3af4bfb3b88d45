// kbench7.hip -- workgroup shape sweep for the 3-stream UInt16 Sum (2 reads + 1 write per
// voxel, 1024^3 voxels = 6 GiB) -- the SumRange kernel of the metric (development tool).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -I../volkit_amd/csrc kbench7.hip -o kbench7
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "kernels/KernelCommon.hpp"

using namespace vkt::hipk;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); std::exit(1);} } while (0)

static float timeIt(std::function<void()> fn, int reps = 9)
{
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    fn();
    CHECK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int i = 0; i < reps; ++i)
    {
        CHECK(hipEventRecord(a));
        fn();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

// u16 saturating-free add stand-in with the codec's cost profile removed: the point is the
// memory shape.  U items of 16 B per lane, WPB waves per workgroup, workgroups in order.
template <int U, int WPB, bool NTL>
__global__ __launch_bounds__(64 * WPB) void sum3(u32x4 const* __restrict__ a, u32x4 const* __restrict__ b,
                                                 u32x4* __restrict__ d)
{
    uint64_t const base = (uint64_t(blockIdx.x) * WPB + threadIdx.x / 64) * 64 * U + (threadIdx.x & 63);
    u32x4 va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
        if constexpr (NTL)
        {
            va[u] = __builtin_nontemporal_load(a + base + 64 * u);
            vb[u] = __builtin_nontemporal_load(b + base + 64 * u);
        }
        else
        {
            va[u] = a[base + 64 * u];
            vb[u] = b[base + 64 * u];
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
        u32x4 r;
        r.x = ((va[u].x & 0xFFFFu) + (vb[u].x & 0xFFFFu)) & 0xFFFFu | ((va[u].x >> 16) + (vb[u].x >> 16)) << 16;
        r.y = ((va[u].y & 0xFFFFu) + (vb[u].y & 0xFFFFu)) & 0xFFFFu | ((va[u].y >> 16) + (vb[u].y >> 16)) << 16;
        r.z = ((va[u].z & 0xFFFFu) + (vb[u].z & 0xFFFFu)) & 0xFFFFu | ((va[u].z >> 16) + (vb[u].z >> 16)) << 16;
        r.w = ((va[u].w & 0xFFFFu) + (vb[u].w & 0xFFFFu)) & 0xFFFFu | ((va[u].w >> 16) + (vb[u].w >> 16)) << 16;
        __builtin_nontemporal_store(r, d + base + 64 * u);
    }
}

int main()
{
    uint64_t const nv = 1024ull * 1024 * 1024, n16 = nv * 2 / 16;
    u32x4 *A, *B, *D;
    CHECK(hipMalloc(&A, nv * 2));
    CHECK(hipMalloc(&B, nv * 2));
    CHECK(hipMalloc(&D, nv * 2));
    CHECK(hipMemset(A, 0x11, nv * 2));
    CHECK(hipMemset(B, 0x22, nv * 2));
    double const bytes = 6.0 * nv;
#define R(U, W, NT)                                                                                                 \
    {                                                                                                               \
        float ms = timeIt([&] { hipLaunchKernelGGL((sum3<U, W, NT>), dim3(n16 / (64 * U * W)), dim3(64 * W), 0, 0, A, B, D); }); \
        std::printf("U%d WPB%d nt%d %8.4f ms %8.1f GB/s\n", U, W, NT, ms, bytes * 1e-9 / (ms * 1e-3));            \
    }
    for (int rep = 0; rep < 2; ++rep)
    {
        R(4, 4, true) R(4, 4, false) R(1, 4, true) R(1, 4, false) R(2, 2, true) R(2, 2, false)
        R(2, 4, true) R(1, 8, true) R(1, 2, true) R(2, 1, true) R(4, 1, true) R(4, 2, true) R(1, 16, true)
    }
    return 0;
}
