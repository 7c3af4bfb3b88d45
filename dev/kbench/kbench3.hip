// kbench.hip -- standalone timing harness for kernel variants (development tool, not shipped).
// Times the achievable-HBM reference (16-B copy / write kernels) and variants of the
// pointwise UInt16 Sum and the 2x Resample replication on 1024^3 UInt16 volumes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../include -I../volkit_amd/csrc kbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "kernels/KernelCommon.hpp"
#include "volkit_codec.hpp"

using namespace vkt::hipk;
using vkt::codec::MapParams;

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

static float timeIt(std::function<void()> fn, int reps = 10)
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

// ---- references ------------------------------------------------------------------------
__global__ __launch_bounds__(256) void copy16(u32x4 const* __restrict__ s, u32x4* __restrict__ d, uint64_t n)
{
    uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += stride)
        d[i] = s[i];
}

template <int U>
__global__ __launch_bounds__(256) void copy16u(u32x4 const* __restrict__ s, u32x4* __restrict__ d, uint64_t n)
{
    uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride)
    {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = s[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_nontemporal_store(v[u], d + i + u * stride);
    }
    for (; i < n; i += stride)
        d[i] = s[i];
}

__global__ __launch_bounds__(256) void write16(u32x4* __restrict__ d, uint64_t n, u32x4 v)
{
    uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += stride)
        __builtin_nontemporal_store(v, d + i);
}

__global__ __launch_bounds__(256) void write16plain(u32x4* __restrict__ d, uint64_t n, u32x4 v)
{
    uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += stride)
        d[i] = v;
}

// ---- Sum UInt16 variants (mapping [0,1] -> pow2 range) ------------------------------------
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

template <int U, bool NT>
__global__ __launch_bounds__(256) void sumU(u32x4 const* __restrict__ a, u32x4 const* __restrict__ b,
                                            u32x4* __restrict__ d, uint64_t n, SumU16 f)
{
    uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride)
    {
        u32x4 va[U], vb[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            va[u] = a[i + u * stride];
            vb[u] = b[i + u * stride];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            u32x4 r = apply8(va[u], vb[u], f);
            if (NT)
                __builtin_nontemporal_store(r, d + i + u * stride);
            else
                d[i + u * stride] = r;
        }
    }
    for (; i < n; i += stride)
        d[i] = apply8(a[i], b[i], f);
}

// software-pipelined: prefetch the next item's loads before storing the current one
template <bool NT>
__global__ __launch_bounds__(256) void sumPipe(u32x4 const* __restrict__ a, u32x4 const* __restrict__ b,
                                               u32x4* __restrict__ d, uint64_t n, SumU16 f)
{
    uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x;
    if (i >= n)
        return;
    u32x4 ca = a[i], cb = b[i];
    for (;;)
    {
        uint64_t nx = i + stride;
        u32x4 na, nb;
        bool more = nx < n;
        if (more)
        {
            na = a[nx];
            nb = b[nx];
        }
        u32x4 r = apply8(ca, cb, f);
        if (NT)
            __builtin_nontemporal_store(r, d + i);
        else
            d[i] = r;
        if (!more)
            break;
        ca = na;
        cb = nb;
        i = nx;
    }
}

// contiguous-per-block chunking: each block owns a contiguous span (better DRAM page locality)
template <int U, bool NT>
__global__ __launch_bounds__(256) void sumChunk(u32x4 const* __restrict__ a, u32x4 const* __restrict__ b,
                                                u32x4* __restrict__ d, uint64_t n, SumU16 f)
{
    uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    uint64_t beg = blockIdx.x * per, end = beg + per < n ? beg + per : n;
    for (uint64_t i = beg + threadIdx.x; i < end; i += U * 256)
    {
        u32x4 va[U], vb[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < end)
            {
                va[u] = a[i + u * 256];
                vb[u] = b[i + u * 256];
            }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < end)
            {
                u32x4 r = apply8(va[u], vb[u], f);
                if (NT)
                    __builtin_nontemporal_store(r, d + i + u * 256);
                else
                    d[i + u * 256] = r;
            }
    }
}

// ---- Resample 2x replication variants (UInt16, identity codes) ---------------------------
// v1 (production r01): wave per source row, lane loads 8 src voxels, stores 2 x 16 B per dst row
__global__ __launch_bounds__(256) void rep2v1(uint16_t const* __restrict__ src, uint16_t* __restrict__ dst, int S)
{
    int lane = threadIdx.x & 63;
    uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), total = gridDim.x * 4;
    uint32_t tasks = uint32_t(S) * S;
    int E = 2 * S;
    for (uint32_t t = wave; t < tasks; t += total)
    {
        uint32_t sy = t % S, sz = t / S;
        uint16_t const* srow = src + (uint64_t(sz) * S + sy) * S;
        for (int c = lane; c < S / 8; c += 64)
        {
            u32x4 v = *reinterpret_cast<u32x4 const*>(srow + 8 * c);
            u32x4 g0, g1;
            g0.x = (v.x & 0xFFFF) * 0x10001u; g0.y = (v.x >> 16) * 0x10001u;
            g0.z = (v.y & 0xFFFF) * 0x10001u; g0.w = (v.y >> 16) * 0x10001u;
            g1.x = (v.z & 0xFFFF) * 0x10001u; g1.y = (v.z >> 16) * 0x10001u;
            g1.z = (v.w & 0xFFFF) * 0x10001u; g1.w = (v.w >> 16) * 0x10001u;
            for (int dz = 0; dz < 2; ++dz)
                for (int dy = 0; dy < 2; ++dy)
                {
                    uint16_t* drow = dst + (uint64_t(2 * sz + dz) * E + 2 * sy + dy) * E + 16 * c;
                    __builtin_nontemporal_store(g0, reinterpret_cast<u32x4*>(drow));
                    __builtin_nontemporal_store(g1, reinterpret_cast<u32x4*>(drow + 8));
                }
        }
    }
}

// v2: contiguous 1 KB per store instruction: lane l of store-instruction g writes dst voxels
// [512g + 8l, +8) from 4 source voxels (8-byte load); prefetch next task before storing.
template <bool NT, bool SWZ = true>
__global__ __launch_bounds__(256) void rep2v2(uint16_t const* __restrict__ src, uint16_t* __restrict__ dst, int S)
{
    int lane = threadIdx.x & 63;
    uint32_t wave = (SWZ ? xcdSwizzle(blockIdx.x, gridDim.x) : blockIdx.x) * 4 + (threadIdx.x >> 6), total = gridDim.x * 4;
    uint32_t tasks = uint32_t(S) * S;
    int E = 2 * S;
    int G = E / 512;   // store instructions per dst row (S multiple of 256 here)
    for (uint32_t t = wave; t < tasks; t += total)
    {
        uint32_t sy = t % S, sz = t / S;
        uint16_t const* srow = src + (uint64_t(sz) * S + sy) * S;
        u32x2 v[4];
        for (int g = 0; g < G && g < 4; ++g)
            v[g] = *reinterpret_cast<u32x2 const*>(srow + 256 * g + 4 * lane);
        for (int g = 0; g < G && g < 4; ++g)
        {
            u32x4 o;
            o.x = (v[g].x & 0xFFFF) * 0x10001u; o.y = (v[g].x >> 16) * 0x10001u;
            o.z = (v[g].y & 0xFFFF) * 0x10001u; o.w = (v[g].y >> 16) * 0x10001u;
            for (int dz = 0; dz < 2; ++dz)
                for (int dy = 0; dy < 2; ++dy)
                {
                    uint16_t* drow = dst + (uint64_t(2 * sz + dz) * E + 2 * sy + dy) * E + 512 * g + 8 * lane;
                    if (NT)
                        __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(drow));
                    else
                        *reinterpret_cast<u32x4*>(drow) = o;
                }
        }
    }
}

// v3: v2 + explicit prefetch of the next task's row
template <bool NT>
__global__ __launch_bounds__(256) void rep2v3(uint16_t const* __restrict__ src, uint16_t* __restrict__ dst, int S)
{
    int lane = threadIdx.x & 63;
    uint32_t wave = xcdSwizzle(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6), total = gridDim.x * 4;
    uint32_t tasks = uint32_t(S) * S;
    int E = 2 * S;
    constexpr int G = 2;   // S = 512
    uint32_t t = wave;
    if (t >= tasks)
        return;
    u32x2 cur[G];
    {
        uint16_t const* srow = src + (uint64_t(t / S) * S + t % S) * S;
#pragma unroll
        for (int g = 0; g < G; ++g)
            cur[g] = *reinterpret_cast<u32x2 const*>(srow + 256 * g + 4 * lane);
    }
    for (;;)
    {
        uint32_t nt = t + total;
        bool more = nt < tasks;
        u32x2 nxt[G];
        if (more)
        {
            uint16_t const* srow = src + (uint64_t(nt / S) * S + nt % S) * S;
#pragma unroll
            for (int g = 0; g < G; ++g)
                nxt[g] = *reinterpret_cast<u32x2 const*>(srow + 256 * g + 4 * lane);
        }
        uint32_t sy = t % S, sz = t / S;
#pragma unroll
        for (int g = 0; g < G; ++g)
        {
            u32x4 o;
            o.x = (cur[g].x & 0xFFFF) * 0x10001u; o.y = (cur[g].x >> 16) * 0x10001u;
            o.z = (cur[g].y & 0xFFFF) * 0x10001u; o.w = (cur[g].y >> 16) * 0x10001u;
#pragma unroll
            for (int dz = 0; dz < 2; ++dz)
#pragma unroll
                for (int dy = 0; dy < 2; ++dy)
                {
                    uint16_t* drow = dst + (uint64_t(2 * sz + dz) * E + 2 * sy + dy) * E + 512 * g + 8 * lane;
                    if (NT)
                        __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(drow));
                    else
                        *reinterpret_cast<u32x4*>(drow) = o;
                }
        }
        if (!more)
            break;
#pragma unroll
        for (int g = 0; g < G; ++g)
            cur[g] = nxt[g];
        t = nt;
    }
}

__global__ void randFill(uint32_t* p, uint64_t n)
{
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    {
        uint64_t x = i * 0x9E3779B97F4A7C15ull;
        x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
        p[i] = uint32_t(x);
    }
}

int main()
{
    const uint64_t E = 1024, S = 512;
    const uint64_t NV = E * E * E, NS = S * S * S;
    uint16_t *A, *B, *D, *Src;
    CHECK(hipMalloc(&A, NV * 2));
    CHECK(hipMalloc(&B, NV * 2));
    CHECK(hipMalloc(&D, NV * 2));
    CHECK(hipMalloc(&Src, NS * 2));
    CHECK(hipMemset(A, 0x11, NV * 2));
    CHECK(hipMemset(B, 0x22, NV * 2));
    CHECK(hipMemset(Src, 0x33, NS * 2));
    uint64_t n16 = NV * 2 / 16;
    double gb = 1e-9;
    auto report = [&](char const* name, float ms, double bytes) {
        std::printf("%-40s %8.4f ms  %8.1f GB/s\n", name, ms, bytes * gb / (ms * 1e-3));
    };
    double rb = 2.0 * NS + 2.0 * NV;
    for (int rep = 0; rep < 2; ++rep)
    {
        if (rep == 1)
        {
            hipLaunchKernelGGL(randFill, dim3(4096), dim3(256), 0, 0, (uint32_t*)Src, NS / 2);
            CHECK(hipDeviceSynchronize());
            std::printf("-- random source data --\n");
        }
    {
        report("rep2v2<nt,swz> grid=65536", timeIt([&] { hipLaunchKernelGGL((rep2v2<true, true>), dim3(65536), dim3(256), 0, 0, Src, D, (int)S); }), rb);
        report("rep2v2<nt,noswz> grid=65536", timeIt([&] { hipLaunchKernelGGL((rep2v2<true, false>), dim3(65536), dim3(256), 0, 0, Src, D, (int)S); }), rb);
        report("rep2v2<plain,swz> grid=65536", timeIt([&] { hipLaunchKernelGGL((rep2v2<false, true>), dim3(65536), dim3(256), 0, 0, Src, D, (int)S); }), rb);
        report("rep2v2<nt,swz> grid=8192", timeIt([&] { hipLaunchKernelGGL((rep2v2<true, true>), dim3(8192), dim3(256), 0, 0, Src, D, (int)S); }), rb);
        report("rep2v2<nt,noswz> grid=8192", timeIt([&] { hipLaunchKernelGGL((rep2v2<true, false>), dim3(8192), dim3(256), 0, 0, Src, D, (int)S); }), rb);
    }
    }
    CHECK(hipFree(A));
    CHECK(hipFree(B));
    CHECK(hipFree(D));
    CHECK(hipFree(Src));
    return 0;
}
