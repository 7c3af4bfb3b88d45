// Probe for DESIGN §4.6 (stale descriptor-table reads after a host-to-device table upload).
// Each experiment isolates one candidate mechanism; every kernel is bounded (fixed spin length,
// fixed grid), so the grid always drains.
//   E1 ordering: does hipMemcpyAsync(H2D) into a table wait for a kernel that is still going to
//      read it on the same stream?  A one-block kernel spins ~2 ms, then copies the table out;
//      the upload of new contents is enqueued right after the launch.  out == new => the copy
//      overtook the kernel.
//   E2 caches: a 1024-block kernel reads the table (warming every XCD's L2 and the scalar
//      caches), the new contents are uploaded by DMA, a second kernel reads it again through
//      scalar loads (uniform index, const __restrict__) and vector loads; any old word = stale.
//   E3 the round-1 pattern: per call hipMallocAsync a pool block, upload from pinned staging,
//      launch the reader, hipFreeAsync; results checked after all calls (a pool block is handed
//      back to the next call in stream order, before the previous reader has run).
//      Variants: one staging buffer reused by every call (host rewrites it while earlier
//      uploads may still be queued) vs one staging buffer per call.
// Build: hipcc --offload-arch=gfx950 -O2 tools/stale_probe.hip -o tools/stale_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                           \
    do                                                                                                  \
    {                                                                                                   \
        hipError_t e_ = (x);                                                                            \
        if (e_ != hipSuccess)                                                                           \
        {                                                                                               \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
            std::exit(1);                                                                               \
        }                                                                                               \
    } while (0)

// spin for `ticks` of the 100 MHz constant clock, then copy n words of the table to out
__global__ void delayedRead(uint32_t const* t, uint32_t* out, uint32_t n, uint64_t ticks)
{
    uint64_t const t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks)
        __builtin_amdgcn_s_sleep(8);
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
        out[i] = t[i];
}

// every block reads its descriptor word through the scalar path (uniform index) and the
// words w = lane + 64 k through the vector path; out[b] = scalar word, out2[...] = vector words
__global__ __launch_bounds__(64) void readTable(uint32_t const* __restrict__ t, uint32_t n, uint32_t* out,
                                                uint32_t* out2)
{
    uint32_t const b = blockIdx.x;
    uint32_t const s = t[b % n];   // uniform: s_load
    if (threadIdx.x == 0)
        out[b] = s;
    for (uint32_t w = threadIdx.x; w < 64; w += 64)
    {
        uint32_t i = (b * 64u + w) % n;
        out2[b * 64u + w] = __builtin_nontemporal_load(t + i) ^ 0u;   // vector load (per-lane index)
    }
}

static void fillPattern(uint32_t* h, uint32_t n, uint32_t stamp)
{
    for (uint32_t i = 0; i < n; ++i)
        h[i] = stamp * 0x9E3779B1u ^ i;
}

static void e1(bool pool, bool pinned, uint32_t bytes, hipStream_t s)
{
    uint32_t const n = bytes / 4;
    uint32_t *t, *out;
    if (pool)
        CK(hipMallocAsync(reinterpret_cast<void**>(&t), bytes, s));
    else
        CK(hipMalloc(&t, bytes));
    CK(hipMalloc(&out, bytes));
    uint32_t *hA, *hB;
    std::vector<uint32_t> pageA(n), pageB(n), got(n);
    if (pinned)
    {
        CK(hipHostMalloc(reinterpret_cast<void**>(&hA), bytes));
        CK(hipHostMalloc(reinterpret_cast<void**>(&hB), bytes));
    }
    else
    {
        hA = pageA.data();
        hB = pageB.data();
    }
    int overtaken = 0, torn = 0, ok = 0;
    int const reps = 8;
    for (int r = 0; r < reps; ++r)
    {
        fillPattern(hA, n, 2 * r + 1);
        fillPattern(hB, n, 2 * r + 2);
        CK(hipMemcpyAsync(t, hA, bytes, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        hipLaunchKernelGGL(delayedRead, dim3(1), dim3(256), 0, s, t, out, n, 200000ull);   // ~2 ms
        CK(hipGetLastError());
        CK(hipMemcpyAsync(t, hB, bytes, hipMemcpyHostToDevice, s));
        CK(hipMemcpyAsync(got.data(), out, bytes, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        uint32_t nA = 0, nB = 0;
        for (uint32_t i = 0; i < n; ++i)
        {
            uint32_t a = (2 * r + 1) * 0x9E3779B1u ^ i, b = (2 * r + 2) * 0x9E3779B1u ^ i;
            nA += got[i] == a;
            nB += got[i] == b;
        }
        if (nA == n)
            ++ok;
        else if (nB == n)
            ++overtaken;
        else
            ++torn;
    }
    std::printf("{\"exp\":\"E1\",\"alloc\":\"%s\",\"host\":\"%s\",\"bytes\":%u,\"reps\":%d,\"in_order\":%d,"
                "\"overtaken\":%d,\"torn\":%d}\n",
                pool ? "pool" : "hipMalloc", pinned ? "pinned" : "pageable", bytes, reps, ok, overtaken, torn);
    if (pinned)
    {
        CK(hipHostFree(hA));
        CK(hipHostFree(hB));
    }
    if (pool)
        CK(hipFreeAsync(t, s));
    else
        CK(hipFree(t));
    CK(hipStreamSynchronize(s));
    CK(hipFree(out));
}

static void e2(bool pool, uint32_t bytes, hipStream_t s)
{
    uint32_t const n = bytes / 4, blocks = 1024;
    uint32_t *t, *o1, *o2;
    if (pool)
        CK(hipMallocAsync(reinterpret_cast<void**>(&t), bytes, s));
    else
        CK(hipMalloc(&t, bytes));
    CK(hipMalloc(&o1, blocks * 4));
    CK(hipMalloc(&o2, blocks * 64 * 4));
    uint32_t* h;
    CK(hipHostMalloc(reinterpret_cast<void**>(&h), bytes));
    std::vector<uint32_t> g1(blocks), g2(blocks * 64);
    long staleS = 0, staleV = 0, checked = 0;
    int const reps = 200;
    for (int r = 0; r < reps; ++r)
    {
        fillPattern(h, n, r + 1);
        CK(hipMemcpyAsync(t, h, bytes, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(readTable, dim3(blocks), dim3(64), 0, s, t, n, o1, o2);   // warm caches
        CK(hipStreamSynchronize(s));
        fillPattern(h, n, r + 1 + 100000);
        CK(hipMemcpyAsync(t, h, bytes, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(readTable, dim3(blocks), dim3(64), 0, s, t, n, o1, o2);
        CK(hipGetLastError());
        CK(hipMemcpyAsync(g1.data(), o1, blocks * 4, hipMemcpyDeviceToHost, s));
        CK(hipMemcpyAsync(g2.data(), o2, blocks * 64 * 4, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        uint32_t const st = (r + 1 + 100000) * 0x9E3779B1u;
        for (uint32_t b = 0; b < blocks; ++b)
        {
            staleS += g1[b] != (st ^ (b % n));
            for (uint32_t w = 0; w < 64; ++w)
                staleV += g2[b * 64 + w] != (st ^ ((b * 64 + w) % n));
        }
        checked += blocks;
    }
    std::printf("{\"exp\":\"E2\",\"alloc\":\"%s\",\"bytes\":%u,\"reps\":%d,\"scalar_words\":%ld,\"scalar_stale\":%ld,"
                "\"vector_words\":%ld,\"vector_stale\":%ld}\n",
                pool ? "pool" : "hipMalloc", bytes, reps, checked, staleS, checked * 64, staleV);
    CK(hipHostFree(h));
    if (pool)
        CK(hipFreeAsync(t, s));
    else
        CK(hipFree(t));
    CK(hipStreamSynchronize(s));
    CK(hipFree(o1));
    CK(hipFree(o2));
}

static void e3(bool sharedStaging, bool syncAfterCopy, uint32_t bytes, hipStream_t s)
{
    uint32_t const n = bytes / 4, blocks = 1024;
    int const calls = 80;
    std::vector<uint32_t*> stg(sharedStaging ? 1 : calls);
    for (auto& p : stg)
        CK(hipHostMalloc(reinterpret_cast<void**>(&p), bytes));
    uint32_t *o1, *o2;
    CK(hipMalloc(&o1, size_t(calls) * blocks * 4));
    CK(hipMalloc(&o2, size_t(calls) * blocks * 64 * 4));
    for (int c = 0; c < calls; ++c)
    {
        uint32_t* h = stg[sharedStaging ? 0 : c];
        fillPattern(h, n, c + 7);
        uint32_t* t;
        CK(hipMallocAsync(reinterpret_cast<void**>(&t), bytes, s));
        CK(hipMemcpyAsync(t, h, bytes, hipMemcpyHostToDevice, s));
        if (syncAfterCopy)
            CK(hipStreamSynchronize(s));
        hipLaunchKernelGGL(readTable, dim3(blocks), dim3(64), 0, s, t, n, o1 + size_t(c) * blocks,
                           o2 + size_t(c) * blocks * 64);
        CK(hipGetLastError());
        CK(hipFreeAsync(t, s));
    }
    std::vector<uint32_t> g1(size_t(calls) * blocks), g2(size_t(calls) * blocks * 64);
    CK(hipMemcpyAsync(g1.data(), o1, g1.size() * 4, hipMemcpyDeviceToHost, s));
    CK(hipMemcpyAsync(g2.data(), o2, g2.size() * 4, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    int badCalls = 0;
    for (int c = 0; c < calls; ++c)
    {
        uint32_t const st = (c + 7) * 0x9E3779B1u;
        bool bad = false;
        for (uint32_t b = 0; b < blocks && !bad; ++b)
        {
            bad |= g1[size_t(c) * blocks + b] != (st ^ (b % n));
            for (uint32_t w = 0; w < 64; ++w)
                bad |= g2[(size_t(c) * blocks + b) * 64 + w] != (st ^ ((b * 64 + w) % n));
        }
        badCalls += bad;
    }
    std::printf("{\"exp\":\"E3\",\"staging\":\"%s\",\"sync_after_copy\":%s,\"bytes\":%u,\"calls\":%d,\"bad_calls\":%d}\n",
                sharedStaging ? "one buffer reused" : "one per call", syncAfterCopy ? "true" : "false", bytes, calls,
                badCalls);
    for (auto p : stg)
        CK(hipHostFree(p));
    CK(hipFree(o1));
    CK(hipFree(o2));
}

int main()
{
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t const sizes[] = {64, 1024, 4096, 65536, 1u << 20, 2u << 20};
    for (uint32_t b : sizes)
        for (int pool = 0; pool < 2; ++pool)
            for (int pinned = 1; pinned >= 0; --pinned)
                e1(pool, pinned, b, s);
    for (uint32_t b : sizes)
        for (int pool = 0; pool < 2; ++pool)
            e2(pool, b, s);
    for (uint32_t b : {4096u, 65536u, 1u << 20})
        for (int shared = 0; shared < 2; ++shared)
            for (int sync = 0; sync < 2; ++sync)
                e3(shared, sync, b, s);
    CK(hipStreamDestroy(s));
    std::printf("done\n");
    return 0;
}
