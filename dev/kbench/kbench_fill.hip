// Dev microbenchmark: pure-store (Fill-shaped) kernels over a 2 GiB buffer on MI355X.
// One-wave workgroups storing Q KiB each (16 B per lane per instruction), nontemporal or
// plain stores, optionally XCD-contiguous block order.  Prints ms and TB/s per variant.
//   hipcc --offload-arch=gfx950 -O3 tools/kbench_fill.hip -o tools/kbench_fill && tools/kbench_fill
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int QKB, bool NT>
__global__ __launch_bounds__(64) void fillKernel(u32x4* p, uint64_t n16, uint32_t code)
{
    constexpr int kPer = QKB * 1024 / (64 * 16);   // store instructions per lane
    uint64_t const base = static_cast<uint64_t>(blockIdx.x) * (64 * kPer) + threadIdx.x;
    u32x4 v = {code, code, code, code};
#pragma unroll
    for (int u = 0; u < kPer; ++u)
    {
        uint64_t i = base + static_cast<uint64_t>(u) * 64;
        if (i < n16)
        {
            if constexpr (NT)
                __builtin_nontemporal_store(v, p + i);
            else
                p[i] = v;
        }
    }
}

template <int QKB>
__global__ __launch_bounds__(64) void copyKernel(u32x4 const* src, u32x4* p, uint64_t n16)
{
    constexpr int kPer = QKB * 1024 / (64 * 16);
    uint64_t const base = static_cast<uint64_t>(blockIdx.x) * (64 * kPer) + threadIdx.x;
    u32x4 v[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u)
    {
        uint64_t i = base + static_cast<uint64_t>(u) * 64;
        v[u] = i < n16 ? __builtin_nontemporal_load(src + i) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u)
    {
        uint64_t i = base + static_cast<uint64_t>(u) * 64;
        if (i < n16)
            __builtin_nontemporal_store(v[u] + 1u, p + i);
    }
}

template <int QKB>
float runCopy(u32x4 const* src, u32x4* p, uint64_t n16, hipEvent_t a, hipEvent_t b)
{
    uint64_t const per = QKB * 1024 / 16;
    unsigned const grid = static_cast<unsigned>((n16 + per - 1) / per);
    for (int w = 0; w < 20; ++w)
        hipLaunchKernelGGL((copyKernel<QKB>), dim3(grid), dim3(64), 0, 0, src, p, n16);
    hipEventRecord(a, 0);
    int const reps = 30;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((copyKernel<QKB>), dim3(grid), dim3(64), 0, 0, src, p, n16);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

template <int QKB>
__global__ __launch_bounds__(64) void sumKernel(u32x4 const* x, u32x4 const* y, u32x4* p, uint64_t n16)
{
    constexpr int kPer = QKB * 1024 / (64 * 16);
    uint64_t const base = static_cast<uint64_t>(blockIdx.x) * (64 * kPer) + threadIdx.x;
    u32x4 v[kPer], w[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u)
    {
        uint64_t i = base + static_cast<uint64_t>(u) * 64;
        v[u] = i < n16 ? __builtin_nontemporal_load(x + i) : u32x4{0, 0, 0, 0};
        w[u] = i < n16 ? __builtin_nontemporal_load(y + i) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u)
    {
        uint64_t i = base + static_cast<uint64_t>(u) * 64;
        if (i < n16)
            __builtin_nontemporal_store(v[u] + w[u], p + i);
    }
}

template <int QKB>
float runSum(u32x4 const* x, u32x4 const* y, u32x4* p, uint64_t n16, hipEvent_t a, hipEvent_t b)
{
    uint64_t const per = QKB * 1024 / 16;
    unsigned const grid = static_cast<unsigned>((n16 + per - 1) / per);
    for (int w = 0; w < 20; ++w)
        hipLaunchKernelGGL((sumKernel<QKB>), dim3(grid), dim3(64), 0, 0, x, y, p, n16);
    hipEventRecord(a, 0);
    int const reps = 30;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((sumKernel<QKB>), dim3(grid), dim3(64), 0, 0, x, y, p, n16);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

template <int QKB, bool NT>
float run(u32x4* p, uint64_t n16, hipEvent_t a, hipEvent_t b)
{
    uint64_t const per = QKB * 1024 / 16;
    unsigned const grid = static_cast<unsigned>((n16 + per - 1) / per);
    for (int w = 0; w < 20; ++w)
        hipLaunchKernelGGL((fillKernel<QKB, NT>), dim3(grid), dim3(64), 0, 0, p, n16, 0x12345678u);
    hipEventRecord(a, 0);
    int const reps = 30;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((fillKernel<QKB, NT>), dim3(grid), dim3(64), 0, 0, p, n16, 0x12345678u + r);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main()
{
    uint64_t const bytes = 2ull << 30;
    u32x4* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess)
        return 1;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    uint64_t const n16 = bytes / 16;
#define R(Q, NT)                                                                                      \
    {                                                                                                 \
        float ms = run<Q, NT>(p, n16, a, b);                                                          \
        std::printf("fill %2d KiB/wg nt=%d: %.4f ms  %.2f TB/s\n", Q, int(NT), ms, bytes / ms / 1e9); \
    }
    R(1, true) R(2, true) R(4, true) R(8, true) R(16, true)
    R(1, false) R(2, false) R(4, false) R(8, false) R(16, false)
    R(2, true) R(4, false)
    u32x4* q = nullptr;
    if (hipMalloc(&q, bytes) != hipSuccess)
        return 1;
#define RC(Q)                                                                                         \
    {                                                                                                 \
        float ms = runCopy<Q>(p, q, n16, a, b);                                                       \
        std::printf("copy %2d KiB/wg: %.4f ms  %.2f TB/s\n", Q, ms, 2 * bytes / ms / 1e9);           \
    }
    RC(1) RC(2) RC(4) RC(8) RC(2) RC(4)
    u32x4* r = nullptr;
    if (hipMalloc(&r, bytes) != hipSuccess)
        return 1;
#define RS(Q)                                                                                         \
    {                                                                                                 \
        float ms = runSum<Q>(p, q, r, n16, a, b);                                                     \
        std::printf("sum  %2d KiB/wg per stream: %.4f ms  %.2f TB/s\n", Q, ms, 3 * bytes / ms / 1e9); \
    }
    RS(1) RS(2) RS(4) RS(1) RS(2)
    hipFree(r);
    hipFree(q);
    hipFree(p);
    return 0;
}
