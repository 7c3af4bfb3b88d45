// kbench4.hip -- does the number of concurrent address streams per wave change HBM throughput?
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "kernels/KernelCommon.hpp"
#include "volkit_codec.hpp"

using namespace vkt::hipk;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); std::exit(1);} } while (0)

static float timeIt(std::function<void()> fn, int reps = 15)
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

// STREAMS independent regions of n/STREAMS vectors; each wave owns a chunk of every region and
// writes (or copies) U consecutive 1 KB pieces per region per iteration.
template <int MODE, int STREAMS, int U>
__global__ __launch_bounds__(256) void multi(u32x4 const* __restrict__ a, u32x4 const* __restrict__ b,
                                             u32x4* __restrict__ d, uint64_t n)
{
    uint64_t region = n / STREAMS;
    uint64_t waves = uint64_t(gridDim.x) * 4;
    uint64_t w = blockIdx.x * 4ull + threadIdx.x / 64;
    uint64_t per = (region + waves - 1) / waves;
    per = (per + 64 * U - 1) / (64 * U) * (64 * U);
    uint64_t beg = w * per, end = beg + per < region ? beg + per : region;
    int lane = threadIdx.x & 63;
    for (uint64_t i = beg + lane; i + 64 * (U - 1) < end; i += 64 * U)
    {
        u32x4 va[STREAMS][U], vb[STREAMS][U];
#pragma unroll
        for (int s = 0; s < STREAMS; ++s)
#pragma unroll
            for (int u = 0; u < U; ++u)
            {
                uint64_t k = s * region + i + 64 * u;
                if constexpr (MODE >= 1)
                    va[s][u] = __builtin_nontemporal_load(a + k);
                if constexpr (MODE >= 2)
                    vb[s][u] = __builtin_nontemporal_load(b + k);
            }
#pragma unroll
        for (int s = 0; s < STREAMS; ++s)
#pragma unroll
            for (int u = 0; u < U; ++u)
            {
                uint64_t k = s * region + i + 64 * u;
                u32x4 v = {1, 2, 3, 4};
                if constexpr (MODE == 1)
                    v = va[s][u];
                if constexpr (MODE == 2)
                    v = va[s][u] + vb[s][u];
                __builtin_nontemporal_store(v, d + k);
            }
    }
}

int main()
{
    const uint64_t NV = 1024ull * 1024 * 1024;
    uint16_t *A, *B, *D;
    CHECK(hipMalloc(&A, NV * 2));
    CHECK(hipMalloc(&B, NV * 2));
    CHECK(hipMalloc(&D, NV * 2));
    CHECK(hipMemset(A, 0x11, NV * 2));
    CHECK(hipMemset(B, 0x22, NV * 2));
    uint64_t n16 = NV * 2 / 16;
    auto report = [&](char const* name, int grid, float ms, double bytes) {
        std::printf("%-28s grid=%6d %8.4f ms %8.1f GB/s\n", name, grid, ms, bytes * 1e-9 / (ms * 1e-3));
    };
#define RUN(MODE, S, U, G)                                                                                      \
    report("mode" #MODE " streams" #S " U" #U, G,                                                              \
           timeIt([&] { hipLaunchKernelGGL((multi<MODE, S, U>), dim3(G), dim3(256), 0, 0, (u32x4*)A, (u32x4*)B, \
                                           (u32x4*)D, n16); }),                                                 \
           (MODE == 0 ? 2.0 : MODE == 1 ? 4.0 : 6.0) * NV)
    for (int g : {1024, 2048, 4096})
    {
        RUN(0, 1, 4, g); RUN(0, 2, 2, g); RUN(0, 4, 1, g); RUN(0, 4, 2, g); RUN(0, 8, 1, g);
        RUN(1, 1, 4, g); RUN(1, 2, 2, g); RUN(1, 4, 1, g); RUN(1, 4, 2, g); RUN(1, 8, 1, g);
        RUN(2, 1, 4, g); RUN(2, 2, 2, g); RUN(2, 4, 1, g); RUN(2, 2, 1, g);
    }
    return 0;
}
