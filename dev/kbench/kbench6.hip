// kbench6.hip -- write-dominated 2x upsampling of a 1024^3 Float32 volume into 2048^3
// (BASELINE config 3 shape; development tool, not shipped).  Compares the pure 32 GiB write
// ceiling with task layouts for the replication:
//   fill      one workgroup per contiguous 16 KiB of dst, 16-B nt stores (write ceiling)
//   srcrow    one wave per source row, writes its 4 dst rows (library layout)
//   dstlin    one workgroup per contiguous dst chunk (linear dst order); lanes load the
//             source voxels of their 16 B from the (L2/MALL-resident) source row
//   dstlin2   as dstlin, but a workgroup covers the two dst rows (2y, 2y+1) of one source row
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -I../volkit_amd/csrc kbench6.hip -o kbench6
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "kernels/KernelCommon.hpp"

using namespace vkt::hipk;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); std::exit(1);} } while (0)

static float timeIt(std::function<void()> fn, int reps = 7)
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

constexpr int S = 1024, D = 2048;

// U instructions of 64 x 16 B per wave, 4 waves per workgroup: 16 KiB (U=4) per workgroup
template <int U, bool NT>
__global__ __launch_bounds__(256) void fill(u32x4* d, uint64_t n16)
{
    uint64_t base = (uint64_t(blockIdx.x) * 4 + threadIdx.x / 64) * 64 * U + (threadIdx.x & 63);
    u32x4 v = {1, 2, 3, 4};
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (base + 64 * u < n16)
        {
            if constexpr (NT) __builtin_nontemporal_store(v, d + base + 64 * u);
            else d[base + 64 * u] = v;
        }
}

// one wave per source row (y, z); dst row 2048 f32 = 8 instr of 64 x 16 B
__global__ __launch_bounds__(256) void srcrow(float const* s, float* d)
{
    uint32_t w = blockIdx.x * 4 + threadIdx.x / 64;
    int lane = threadIdx.x & 63;
    uint32_t y = w % S, z = w / S;
    if (z >= S) return;
    float const* sr = s + (uint64_t(z) * S + y) * S;
    u32x4 v[8];
#pragma unroll
    for (int g = 0; g < 8; ++g)
    {
        u32x2 q = *reinterpret_cast<u32x2 const*>(sr + 128 * g + 2 * lane);
        v[g] = u32x4{q.x, q.x, q.y, q.y};
    }
    for (int dz = 0; dz < 2; ++dz)
        for (int dy = 0; dy < 2; ++dy)
        {
            float* dr = d + (uint64_t(2 * z + dz) * D + 2 * y + dy) * D;
#pragma unroll
            for (int g = 0; g < 8; ++g)
                __builtin_nontemporal_store(v[g], reinterpret_cast<u32x4*>(dr + 256 * g + 4 * lane));
        }
}

// linear dst: workgroup b covers dst floats [b*RPW*2048, ...) i.e. RPW whole dst rows;
// wave w of the workgroup writes row (b*RPW + w / (4/RPW))... simplest: each wave one dst
// row half when RPW == 2 (4 waves x 1024 floats = 2 rows), one quarter row when RPW == 1.
template <int RPW>
__global__ __launch_bounds__(256) void dstlin(float const* s, float* d)
{
    constexpr int kWavesPerRow = 4 / RPW;            // 4 (RPW 1) or 2 (RPW 2)
    constexpr int kFloatsPerWave = D / kWavesPerRow;  // 512 or 1024
    constexpr int kInstr = kFloatsPerWave / 256;      // 2 or 4
    uint32_t const wave = threadIdx.x / 64;
    int const lane = threadIdx.x & 63;
    uint64_t const row = uint64_t(blockIdx.x) * RPW + wave / kWavesPerRow;   // dst row index
    uint32_t const part = wave % kWavesPerRow;
    uint32_t const yd = row % D, zd = row / D;
    float const* sr = s + (uint64_t(zd / 2) * S + yd / 2) * S + part * (kFloatsPerWave / 2);
    float* dr = d + row * D + part * kFloatsPerWave;
    u32x4 v[kInstr];
#pragma unroll
    for (int g = 0; g < kInstr; ++g)
    {
        u32x2 q = *reinterpret_cast<u32x2 const*>(sr + 128 * g + 2 * lane);
        v[g] = u32x4{q.x, q.x, q.y, q.y};
    }
#pragma unroll
    for (int g = 0; g < kInstr; ++g)
        __builtin_nontemporal_store(v[g], reinterpret_cast<u32x4*>(dr + 256 * g + 4 * lane));
}

// general linear-dst layout: each wave writes IPW consecutive 1-KiB instructions of one dst
// row, WPB waves per workgroup, workgroups in dst order
template <int IPW, int WPB>
__global__ __launch_bounds__(64 * WPB) void dstgen(float const* s, float* d)
{
    constexpr int kFloatsPerWave = 256 * IPW;
    constexpr int kWavesPerRow = D / kFloatsPerWave;
    uint64_t const gw = uint64_t(blockIdx.x) * WPB + threadIdx.x / 64;
    int const lane = threadIdx.x & 63;
    uint64_t const row = gw / kWavesPerRow;
    uint32_t const part = gw % kWavesPerRow;
    uint32_t const yd = row % D, zd = row / D;
    float const* sr = s + (uint64_t(zd / 2) * S + yd / 2) * S + part * (kFloatsPerWave / 2);
    float* dr = d + row * D + part * kFloatsPerWave;
    u32x4 v[IPW];
#pragma unroll
    for (int g = 0; g < IPW; ++g)
    {
        u32x2 q = *reinterpret_cast<u32x2 const*>(sr + 128 * g + 2 * lane);
        v[g] = u32x4{q.x, q.x, q.y, q.y};
    }
#pragma unroll
    for (int g = 0; g < IPW; ++g)
        __builtin_nontemporal_store(v[g], reinterpret_cast<u32x4*>(dr + 256 * g + 4 * lane));
}

// as dstgen, but each wave writes its part of the 2 dst rows (2y', 2y'+1) that read the same
// source row (one source load, two store streams 8 KiB apart)
template <int IPW, int WPB>
__global__ __launch_bounds__(64 * WPB) void dstpair(float const* s, float* d)
{
    constexpr int kFloatsPerWave = 256 * IPW;
    constexpr int kWavesPerRow = D / kFloatsPerWave;
    uint64_t const gw = uint64_t(blockIdx.x) * WPB + threadIdx.x / 64;
    int const lane = threadIdx.x & 63;
    uint64_t const pair = gw / kWavesPerRow;          // dst rows 2*pair, 2*pair+1
    uint32_t const part = gw % kWavesPerRow;
    uint64_t const row = 2 * pair;
    uint32_t const yd = row % D, zd = row / D;
    float const* sr = s + (uint64_t(zd / 2) * S + yd / 2) * S + part * (kFloatsPerWave / 2);
    float* dr = d + row * D + part * kFloatsPerWave;
    u32x4 v[IPW];
#pragma unroll
    for (int g = 0; g < IPW; ++g)
    {
        u32x2 q = *reinterpret_cast<u32x2 const*>(sr + 128 * g + 2 * lane);
        v[g] = u32x4{q.x, q.x, q.y, q.y};
    }
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int g = 0; g < IPW; ++g)
            __builtin_nontemporal_store(v[g], reinterpret_cast<u32x4*>(dr + r * D + 256 * g + 4 * lane));
}

// one wave per (source row, IPW-instruction x chunk): writes the chunk into all 4 dst rows
// (2 rows x 2 planes); chunks x-fastest, then y, then z
template <int IPW>
__global__ __launch_bounds__(64) void srcchunk(float const* s, float* d)
{
    constexpr int kChunks = D / (256 * IPW);
    uint64_t const gw = blockIdx.x;
    int const lane = threadIdx.x & 63;
    uint32_t const part = gw % kChunks;
    uint64_t const srow = gw / kChunks;
    uint32_t const y = srow % S, z = srow / S;
    float const* sr = s + srow * S + part * 128 * IPW;
    u32x4 v[IPW];
#pragma unroll
    for (int g = 0; g < IPW; ++g)
    {
        u32x2 q = *reinterpret_cast<u32x2 const*>(sr + 128 * g + 2 * lane);
        v[g] = u32x4{q.x, q.x, q.y, q.y};
    }
#pragma unroll
    for (int dz = 0; dz < 2; ++dz)
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
        {
            float* dr = d + (uint64_t(2 * z + dz) * D + 2 * y + dy) * D + part * 256 * IPW;
#pragma unroll
            for (int g = 0; g < IPW; ++g)
                __builtin_nontemporal_store(v[g], reinterpret_cast<u32x4*>(dr + 256 * g + 4 * lane));
        }
}

template <int U, int WPB>
__global__ __launch_bounds__(64 * WPB) void fillg(u32x4* d)
{
    uint64_t base = (uint64_t(blockIdx.x) * WPB + threadIdx.x / 64) * 64 * U + (threadIdx.x & 63);
    u32x4 v = {1, 2, 3, 4};
#pragma unroll
    for (int u = 0; u < U; ++u)
        __builtin_nontemporal_store(v, d + base + 64 * u);
}

// one workgroup per source row: 4 waves = the 4 dst rows (2y+dy, 2z+dz) of that row
__global__ __launch_bounds__(256) void srcrowWG(float const* s, float* d)
{
    uint32_t const r = blockIdx.x;
    uint32_t const wave = threadIdx.x / 64;
    int const lane = threadIdx.x & 63;
    uint32_t y = r % S, z = r / S;
    float const* sr = s + (uint64_t(z) * S + y) * S;
    float* dr = d + (uint64_t(2 * z + wave / 2) * D + 2 * y + wave % 2) * D;
    u32x4 v[8];
#pragma unroll
    for (int g = 0; g < 8; ++g)
    {
        u32x2 q = *reinterpret_cast<u32x2 const*>(sr + 128 * g + 2 * lane);
        v[g] = u32x4{q.x, q.x, q.y, q.y};
    }
#pragma unroll
    for (int g = 0; g < 8; ++g)
        __builtin_nontemporal_store(v[g], reinterpret_cast<u32x4*>(dr + 256 * g + 4 * lane));
}

// read-only pass over the source (the Linear pre-pass shape): 4 GiB
__global__ __launch_bounds__(256) void readAll(u32x4 const* s, uint64_t n16, uint32_t* out)
{
    uint64_t base = (uint64_t(blockIdx.x) * 4 + threadIdx.x / 64) * 256 + (threadIdx.x & 63);
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u)
    {
        u32x4 v = __builtin_nontemporal_load(s + base + 64 * u);
        acc |= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u)
        out[0] = acc;
}

int main()
{
    uint64_t const ns = uint64_t(S) * S * S, nd = uint64_t(D) * D * D;
    float *src, *dst;
    uint32_t* sink;
    CHECK(hipMalloc(&src, ns * 4));
    CHECK(hipMalloc(&dst, nd * 4));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(src, 0x3f, ns * 4));
    double const wbytes = nd * 4.0, rbytes = ns * 4.0;
    auto rep = [&](char const* name, float ms, double bytes) {
        std::printf("%-24s %8.4f ms %8.1f GB/s\n", name, ms, bytes * 1e-9 / (ms * 1e-3));
    };
    uint64_t n16 = nd * 4 / 16;
    for (int rr = 0; rr < 2; ++rr) {
    rep("fill U4 nt", timeIt([&] { hipLaunchKernelGGL((fill<4, true>), dim3(n16 / 1024), dim3(256), 0, 0, (u32x4*)dst, n16); }), wbytes);
    rep("fill U4 plain", timeIt([&] { hipLaunchKernelGGL((fill<4, false>), dim3(n16 / 1024), dim3(256), 0, 0, (u32x4*)dst, n16); }), wbytes);
    rep("fill U1 nt", timeIt([&] { hipLaunchKernelGGL((fill<1, true>), dim3(n16 / 256), dim3(256), 0, 0, (u32x4*)dst, n16); }), wbytes);
    rep("srcrow (wave/row)", timeIt([&] { hipLaunchKernelGGL(srcrow, dim3(S * S / 4), dim3(256), 0, 0, src, dst); }), wbytes + rbytes);
    rep("srcrowWG (wg/row)", timeIt([&] { hipLaunchKernelGGL(srcrowWG, dim3(S * S), dim3(256), 0, 0, src, dst); }), wbytes + rbytes);
    rep("dstlin RPW1", timeIt([&] { hipLaunchKernelGGL((dstlin<1>), dim3(D * D), dim3(256), 0, 0, src, dst); }), wbytes + rbytes);
    rep("dstlin RPW2", timeIt([&] { hipLaunchKernelGGL((dstlin<2>), dim3(D * D / 2), dim3(256), 0, 0, src, dst); }), wbytes + rbytes);
#define FG(U, W) rep("fill U" #U " WPB" #W, timeIt([&] { hipLaunchKernelGGL((fillg<U, W>), dim3(n16 / (64 * U * W)), dim3(64 * W), 0, 0, (u32x4*)dst); }), wbytes)
    FG(1, 4); FG(2, 2); FG(8, 1); FG(1, 16);
#define DG(I, W) rep("dstgen IPW" #I " WPB" #W, timeIt([&] { hipLaunchKernelGGL((dstgen<I, W>), dim3(nd / (256 * I * W)), dim3(64 * W), 0, 0, src, dst); }), wbytes + rbytes)
    DG(2, 2); DG(4, 1);
#define DP(I, W) rep("dstpair IPW" #I " WPB" #W, timeIt([&] { hipLaunchKernelGGL((dstpair<I, W>), dim3(nd / (512 * I * W)), dim3(64 * W), 0, 0, src, dst); }), wbytes + rbytes)
    DP(1, 1); DP(1, 4); DP(2, 1);
#define SC(I) rep("srcchunk IPW" #I, timeIt([&] { hipLaunchKernelGGL((srcchunk<I>), dim3(ns / (128 * I)), dim3(64), 0, 0, src, dst); }), wbytes + rbytes)
    SC(1); SC(2); SC(4);
    }
    uint64_t s16 = ns * 4 / 16;
    rep("read src 4 GiB", timeIt([&] { hipLaunchKernelGGL(readAll, dim3(s16 / 1024), dim3(256), 0, 0, (u32x4 const*)src, s16, sink); }), rbytes);
    return 0;
}
