// kbench2.hip -- streaming-layout sweep for copy / UInt16 Sum (development tool, not shipped).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "kernels/KernelCommon.hpp"
#include "volkit_codec.hpp"

using namespace vkt::hipk;
using vkt::codec::MapParams;

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

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

struct SumU16
{
    float lo1, hi1, lo2, hi2;
    MapParams dm;
    __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t b) const
    {
        float v1 = vkt::codec::decode(a, 5, lo1, hi1);
        float v2 = vkt::codec::decode(b, 5, lo2, hi2);
        bool w;
        return vkt::codec::encode(v1 + v2, 5, dm, w);
    }
};

__device__ __forceinline__ u32x4 apply8(u32x4 a, u32x4 b, SumU16 const& f)
{
    uint32_t ca[8] = {a.x & 0xFFFF, a.x >> 16, a.y & 0xFFFF, a.y >> 16, a.z & 0xFFFF, a.z >> 16, a.w & 0xFFFF, a.w >> 16};
    uint32_t cb[8] = {b.x & 0xFFFF, b.x >> 16, b.y & 0xFFFF, b.y >> 16, b.z & 0xFFFF, b.z >> 16, b.w & 0xFFFF, b.w >> 16};
    uint32_t o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        o[i] = f(ca[i], cb[i]);
    u32x4 r;
    r.x = o[0] | o[1] << 16;
    r.y = o[2] | o[3] << 16;
    r.z = o[4] | o[5] << 16;
    r.w = o[6] | o[7] << 16;
    return r;
}

template <bool NTL>
__device__ __forceinline__ u32x4 ld(u32x4 const* p)
{
    if constexpr (NTL)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

template <bool NTS>
__device__ __forceinline__ void st(u32x4* p, u32x4 v)
{
    if constexpr (NTS)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

// MODE 0 = copy a->d ; MODE 1 = sum a+b -> d
// LAYOUT 0: block-contiguous span, U rows of blockDim in flight
// LAYOUT 1: wave-contiguous span (each wave owns span/waves), U x 64 lanes in flight
template <int MODE, int LAYOUT, int U, bool NTL, bool NTS>
__global__ void streamK(u32x4 const* __restrict__ a, u32x4 const* __restrict__ b, u32x4* __restrict__ d, uint64_t n,
                        SumU16 f)
{
    uint64_t beg, end, step, i0;
    if constexpr (LAYOUT == 0)
    {
        uint64_t per = (n + gridDim.x - 1) / gridDim.x;
        per = (per + blockDim.x * U - 1) / (blockDim.x * U) * (blockDim.x * U);
        beg = blockIdx.x * per;
        end = beg + per < n ? beg + per : n;
        step = blockDim.x;
        i0 = beg + threadIdx.x;
    }
    else
    {
        uint64_t waves = uint64_t(gridDim.x) * (blockDim.x / 64);
        uint64_t w = blockIdx.x * uint64_t(blockDim.x / 64) + threadIdx.x / 64;
        uint64_t per = (n + waves - 1) / waves;
        per = (per + 64 * U - 1) / (64 * U) * (64 * U);
        beg = w * per;
        end = beg + per < n ? beg + per : n;
        step = 64;
        i0 = beg + (threadIdx.x & 63);
    }
    for (uint64_t i = i0; i < end; i += step * U)
    {
        u32x4 va[U], vb[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * step < end)
            {
                va[u] = ld<NTL>(a + i + u * step);
                if constexpr (MODE == 1)
                    vb[u] = ld<NTL>(b + i + u * step);
            }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * step < end)
            {
                if constexpr (MODE == 1)
                    st<NTS>(d + i + u * step, apply8(va[u], vb[u], f));
                else
                    st<NTS>(d + i + u * step, va[u]);
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
    CHECK(hipMemset(D, 0, NV * 2));
    uint64_t n16 = NV * 2 / 16;
    SumU16 f{0.f, 1.f, 0.f, 1.f, vkt::codec::makeMapParams(0.f, 1.f)};
    auto report = [&](char const* name, int grid, int bs, float ms, double bytes) {
        std::printf("%-34s grid=%6d bs=%4d %8.4f ms %8.1f GB/s\n", name, grid, bs, ms, bytes * 1e-9 / (ms * 1e-3));
    };
#define RUN(MODE, LAYOUT, U, NTL, NTS, GRID, BS)                                                                    \
    report(#MODE " L" #LAYOUT " U" #U " ntl" #NTL " nts" #NTS, GRID, BS,                                              \
           timeIt([&] {                                                                                            \
               hipLaunchKernelGGL((streamK<MODE, LAYOUT, U, NTL, NTS>), dim3(GRID), dim3(BS), 0, 0, (u32x4*)A,   \
                                  (u32x4*)B, (u32x4*)D, n16, f);                                                   \
           }),                                                                                                      \
           (MODE ? 6.0 : 4.0) * NV)
    for (int g : {4096, 16384, 65536, 131072, 262144})
    {
        RUN(0, 0, 4, true, true, g, 256);
        RUN(0, 0, 2, true, true, g, 256);
        RUN(0, 0, 1, true, true, g, 256);
        RUN(1, 0, 4, true, true, g, 256);
        RUN(1, 0, 2, true, true, g, 256);
        RUN(1, 0, 1, true, true, g, 256);
        RUN(1, 0, 4, false, true, g, 256);
        RUN(1, 0, 2, true, true, g, 512);
    }
    return 0;
}
