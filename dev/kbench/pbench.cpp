// pbench.cpp -- times the product library's backend entry points (C ABI) in isolation and in
// the metric pipeline (development tool).  g++ -O2 -I../include pbench.cpp -L../volkit_amd/lib -lvolkit -lamdhip64
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "volkit_hip.h"

static float timeIt(std::function<void()> fn, int reps = 15)
{
    void* sp;
    vktHipGetComputeStream(&sp);
    hipStream_t s = (hipStream_t)sp;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    fn();
    hipStreamSynchronize(s);
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

static vktHipVolumeView_t vol(int x, int y, int z, int fmt, uint64_t seed)
{
    vktHipVolumeView_t v{};
    size_t bpv = fmt == vktDataFormatUInt8 ? 1 : fmt == vktDataFormatUInt16 ? 2 : 4;
    void* p = nullptr;
    if (vktHipAllocate(&p, size_t(x) * y * z * bpv) != vktNoError) { std::printf("alloc failed\n"); std::exit(1); }
    v.data = (uint8_t*)p; v.dimX = x; v.dimY = y; v.dimZ = z; v.dataFormat = fmt; v.mappingLo = 0.f; v.mappingHi = 1.f;
    vktHipSynthesize(v, seed);
    return v;
}

int main(int argc, char** argv)
{
    int E = argc > 1 ? std::atoi(argv[1]) : 1024, S = E / 2;
    auto U16 = vktDataFormatUInt16;
    vktHipVolumeView_t Sv = vol(S, S, S, U16, 1), R = vol(E, E, E, U16, 2), B = vol(E, E, E, U16, 3), D = vol(E, E, E, U16, 4);
    vktVec3i_t o{0, 0, 0}, l{E, E, E};
    double nv = double(E) * E * E, ns = double(S) * S * S;
    auto rep = [](char const* n, float ms, double bytes) { std::printf("%-44s %8.4f ms %8.1f GB/s\n", n, ms, bytes / (ms * 1e-3) * 1e-9); };
    rep("Resample alone", timeIt([&] { vktHipResample(R, Sv, vktFilterModeLinear); }), 2 * ns + 2 * nv);
    rep("SumRange alone", timeIt([&] { vktHipArithmeticRange(vktHipOpSum, D, R, B, o, l, o); }), 6 * nv);
    rep("SafeSum alone", timeIt([&] { vktHipArithmeticRange(vktHipOpSafeSum, D, R, B, o, l, o); }), 6 * nv);
    rep("pipeline Resample+SumRange", timeIt([&] { vktHipResample(R, Sv, vktFilterModeLinear); vktHipArithmeticRange(vktHipOpSum, D, R, B, o, l, o); }), 8 * nv + 2 * ns);
    rep("Fill 1024^3 u16", timeIt([&] { vktHipFillRange(D, o, l, 0.25f); }), 2 * nv);
    rep("Copy 1024^3 u16", timeIt([&] { vktHipCopyRange(D, R, o, l, o); }), 4 * nv);
    vktHipVolumeView_t Rm = R; Rm.mappingLo = -1.f; Rm.mappingHi = 3.f;
    rep("Sum mapped [-1,3] dst", timeIt([&] { vktHipArithmeticRange(vktHipOpSum, Rm, D, B, o, l, o); }), 6 * nv);
    vktHipVolumeView_t Bm = B; Bm.mappingLo = 0.25f; Bm.mappingHi = 7.5f;
    rep("SafeDiff mapped [.25,7.5] dst (IEEE div)", timeIt([&] { vktHipArithmeticRange(vktHipOpSafeDiff, Bm, D, R, o, l, o); }), 6 * nv);
    return 0;
}
