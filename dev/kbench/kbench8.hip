// kbench8.hip -- the library's pointwise vector kernel (UInt16 Sum functor) against the bare
// 3-stream kernel of kbench7 on the same buffers, constant vs random contents (development tool).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../include -I../volkit_amd/csrc kbench8.hip -o kbench8
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "kernels/PointwiseOps.hpp"

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

template <int U, int WPB>
__global__ __launch_bounds__(64 * WPB) void sum3(u32x4 const* __restrict__ a, u32x4 const* __restrict__ b,
                                                 u32x4* __restrict__ d)
{
    uint64_t const base = (uint64_t(blockIdx.x) * WPB + threadIdx.x / 64) * 64 * U + (threadIdx.x & 63);
    u32x4 va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
        va[u] = __builtin_nontemporal_load(a + base + 64 * u);
        vb[u] = __builtin_nontemporal_load(b + base + 64 * u);
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

int main(int argc, char** argv)
{
    uint64_t const nv = 1024ull * 1024 * 1024, n16 = nv * 2 / 16;
    uint8_t *A, *B, *D;
    if (argc > 1)   // the allocation order of tools/bench_configs.py's metric group
    {
        void* S;
        CHECK(hipMalloc(&S, 512ull * 512 * 512 * 2));
    }
    CHECK(hipMalloc(&A, nv * 2));
    CHECK(hipMalloc(&B, nv * 2));
    CHECK(hipMalloc(&D, nv * 2));
    double const bytes = 6.0 * nv;
    Operand od{}, oa{}, ob{};
    od.data = D; oa.data = A; ob.data = B;
    Geom g{};
    g.nx = g.vnx = g.vnx8 = nv;
    g.ny = g.nz = g.vny = g.vnz = 1;
    vkt::codec::MapParams dm = vkt::codec::makeMapParams(0.f, 1.f);
    ArithF<0, 5, 5, 5, 1> f{5, 5, 5, 0.f, 1.f, 0.f, 1.f, dm};
    ArithF<0, 5, 5, 5, 0> f0{5, 5, 5, 0.f, 1.f, 0.f, 1.f, dm};
    PassF pass;
    unsigned const grid = unsigned(nv / 8 / kVecBlock);
    for (int data = 0; data < 2; ++data)
    {
        if (data == 0)
        {
            CHECK(hipMemset(A, 0x11, nv * 2));
            CHECK(hipMemset(B, 0x22, nv * 2));
        }
        else
        {
            hipLaunchKernelGGL(fillRandom, dim3(4096), dim3(256), 0, 0, (uint64_t*)A, nv / 4, 1ull);
            hipLaunchKernelGGL(fillRandom, dim3(4096), dim3(256), 0, 0, (uint64_t*)B, nv / 4, 99ull);
        }
        for (int rep = 0; rep < 2; ++rep)
        {
            float ms = timeIt([&] { hipLaunchKernelGGL((sum3<1, 2>), dim3(n16 / 128), dim3(128), 0, 0, (u32x4*)A, (u32x4*)B, (u32x4*)D); });
            std::printf("data%d bare U1 WPB2    %8.4f ms %8.1f GB/s\n", data, ms, bytes * 1e-9 / (ms * 1e-3));
            ms = timeIt([&] { hipLaunchKernelGGL((pointwiseVecKernel<2, 2, decltype(f)>), dim3(grid), dim3(kVecBlock), 0, 0, od, oa, ob, g, f); });
            std::printf("data%d lib ArithF pow2  %8.4f ms %8.1f GB/s\n", data, ms, bytes * 1e-9 / (ms * 1e-3));
            ms = timeIt([&] { hipLaunchKernelGGL((pointwiseVecKernel<2, 2, decltype(f0)>), dim3(grid), dim3(kVecBlock), 0, 0, od, oa, ob, g, f0); });
            std::printf("data%d lib ArithF dyn   %8.4f ms %8.1f GB/s\n", data, ms, bytes * 1e-9 / (ms * 1e-3));
            ms = timeIt([&] { hipLaunchKernelGGL((pointwiseVecKernel<2, 2, PassF>), dim3(grid), dim3(kVecBlock), 0, 0, od, oa, ob, g, pass); });
            std::printf("data%d lib PassF(2src)  %8.4f ms %8.1f GB/s\n", data, ms, bytes * 1e-9 / (ms * 1e-3));
            ms = timeIt([&] { hipLaunchKernelGGL((pointwiseVecKernel<1, 2, PassF>), dim3(grid), dim3(kVecBlock), 0, 0, od, oa, ob, g, pass); });
            std::printf("data%d lib copy         %8.4f ms %8.1f GB/s\n", data, ms, 4.0 * nv * 1e-9 / (ms * 1e-3));
        }
    }
    return 0;
}
