// kbench9.hip -- pacing sweep of the 3-stream UInt16 pointwise kernel: functor cost
// (integer add / Sum with the run-time division test / Sum with the division fixed) x
// workgroup shape, after a 300 ms warm-up so clocks have settled (development tool).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../include -I../volkit_amd/csrc kbench9.hip -o kbench9
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "kernels/PointwiseOps.hpp"

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

struct IntAdd
{
    __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t b) const { return (a + b) & 0xFFFFu; }
};

template <int U, int WPB, int SLEEP, class F>
__global__ __launch_bounds__(64 * WPB) void gk(uint8_t const* __restrict__ a, uint8_t const* __restrict__ b,
                                               uint8_t* __restrict__ d, F f)
{
    uint64_t const item = (uint64_t(blockIdx.x) * WPB + threadIdx.x / 64) * 64 * U + (threadIdx.x & 63);
    uint32_t va[U][8], vb[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
        load8<2, true>(a, (item + 64 * u) * 8, va[u]);
        load8<2, true>(b, (item + 64 * u) * 8, vb[u]);
    }
    if constexpr (SLEEP > 0)
        __builtin_amdgcn_s_sleep(SLEEP);
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
        uint32_t o[8];
#pragma unroll
        for (int v = 0; v < 8; ++v)
            o[v] = f(va[u][v], vb[u][v]);
        store8<2, true>(d, (item + 64 * u) * 8, o);
    }
}

__global__ void fillRandom(uint64_t* p, uint64_t n, uint64_t seed)
{
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    {
        uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

int main()
{
    uint64_t const nv = 1024ull * 1024 * 1024;
    uint8_t *A, *B, *D;
    CHECK(hipMalloc(&A, nv * 2));
    CHECK(hipMalloc(&B, nv * 2));
    CHECK(hipMalloc(&D, nv * 2));
    hipLaunchKernelGGL(fillRandom, dim3(4096), dim3(256), 0, 0, (uint64_t*)A, nv / 4, 1ull);
    hipLaunchKernelGGL(fillRandom, dim3(4096), dim3(256), 0, 0, (uint64_t*)B, nv / 4, 99ull);
    double const bytes = 6.0 * nv;
    vkt::codec::MapParams dm = vkt::codec::makeMapParams(0.f, 1.f);
    ArithF<0, 5, 5, 5, 1> fp{5, 5, 5, 0.f, 1.f, 0.f, 1.f, dm};
    ArithF<0, 5, 5, 5, 0> fd{5, 5, 5, 0.f, 1.f, 0.f, 1.f, dm};
    IntAdd fi;
    // warm-up: ~300 ms of sustained streaming
    auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 0.3)
    {
        for (int i = 0; i < 20; ++i)
            hipLaunchKernelGGL((gk<1, 2, 0, IntAdd>), dim3(nv / 8 / 128), dim3(128), 0, 0, A, B, D, fi);
        CHECK(hipDeviceSynchronize());
    }
#define R(U, W, S, F, NAME)                                                                                           \
    {                                                                                                                 \
        float ms = timeIt([&] { hipLaunchKernelGGL((gk<U, W, S, decltype(F)>), dim3(nv / 8 / (64 * U * W)), dim3(64 * W), 0, 0, A, B, D, F); }); \
        std::printf("%-6s U%d WPB%d sleep%d %8.4f ms %8.1f GB/s\n", NAME, U, W, S, ms, bytes * 1e-9 / (ms * 1e-3));  \
    }
    for (int rep = 0; rep < 2; ++rep)
    {
        R(1, 2, 0, fi, "int") R(1, 2, 0, fd, "dyn") R(1, 2, 0, fp, "pow2")
        R(1, 1, 0, fi, "int") R(1, 1, 0, fd, "dyn") R(1, 1, 0, fp, "pow2")
        R(1, 4, 0, fi, "int") R(1, 4, 0, fd, "dyn") R(1, 4, 0, fp, "pow2")
        R(2, 1, 0, fi, "int") R(2, 1, 0, fd, "dyn") R(2, 1, 0, fp, "pow2")
        R(2, 2, 0, fd, "dyn") R(2, 2, 0, fp, "pow2") R(4, 4, 0, fd, "dyn") R(4, 4, 0, fp, "pow2")
        R(1, 2, 1, fi, "int") R(1, 2, 2, fi, "int") R(1, 2, 4, fi, "int") R(1, 2, 1, fp, "pow2") R(1, 2, 3, fp, "pow2")
    }
    return 0;
}
