// libbench.cpp -- times the library's C-ABI SumRange / CopyRange at 1024^3 UInt16 from a plain
// C++ host (no Python, no torch), with HIP events on the backend's compute stream
// (development tool; separates library-path effects from the Python bench harness).
//   hipcc -O2 -std=c++17 -I../include libbench.cpp -L../volkit_amd/lib -lvolkit -Wl,-rpath,'$ORIGIN/../volkit_amd/lib' -o libbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <functional>
#include <vector>

#include "volkit_hip.h"

static float timeIt(hipStream_t s, std::function<void()> fn, int reps = 9)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    fn();
    hipDeviceSynchronize();
    std::vector<float> ts;
    for (int i = 0; i < reps; ++i)
    {
        hipEventRecord(a, s);
        fn();
        hipEventRecord(b, s);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main()
{
    int const e = 1024;
    size_t const n = size_t(e) * e * e * 2;
    void *pS, *pR, *pB, *pD;
    vktHipAllocate(&pS, size_t(512) * 512 * 512 * 2);
    vktHipAllocate(&pR, n);
    vktHipAllocate(&pB, n);
    vktHipAllocate(&pD, n);
    auto view = [&](void* p) { return vktHipVolumeView_t{static_cast<uint8_t*>(p), e, e, e, 5, 0.f, 1.f}; };
    vktHipVolumeView_t R = view(pR), B = view(pB), D = view(pD);
    vktHipSynthesize(R, 4);
    vktHipSynthesize(B, 5);
    void* sp;
    vktHipGetComputeStream(&sp);
    hipStream_t s = static_cast<hipStream_t>(sp);
    vktVec3i_t o{0, 0, 0}, l{e, e, e};
    for (int rep = 0; rep < 3; ++rep)
    {
        float ms = timeIt(s, [&] { vktHipArithmeticRange(vktHipOpSum, D, R, B, o, l, o); });
        std::printf("lib SumRange  %8.4f ms %8.1f GB/s\n", ms, 3.0 * n * 1e-6 / ms);
        ms = timeIt(s, [&] { vktHipCopyRange(D, B, o, l, o); });
        std::printf("lib CopyRange %8.4f ms %8.1f GB/s\n", ms, 2.0 * n * 1e-6 / ms);
    }
    return 0;
}
