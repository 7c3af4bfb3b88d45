// Decompose.hip -- BrickDecompose on gfx950 (replaces BrickDecompose_cuda, an empty stub in
// the reference: src/vkt/Decompose_cuda.cu:8-26; semantics of BrickDecompose_serial,
// src/vkt/Decompose_serial.hpp:15-46).
//
// Semantics restated: brick (i,j,k) receives CopyRange(brick, source, first, last) with
//   first = (i,j,k)*brickSize - haloNeg,  last = min((i,j,k)*brickSize + brickSize, dims) + haloPos,
// dstOffset 0: brick[x-first] = source[clamp(x, 0, dims-1)] (Copy_serial.hpp:13-82), bytewise
// when format and mapping match, unmap->map otherwise.
//
// MI355X design: every brick is its own allocation, so a per-brick CopyRange would be one
// launch per brick (4096 launches for 64^3 bricks of a 1024^3 volume).  Instead one launch
// copies ALL bytewise bricks: a device table of brick descriptors, workgroup b handles
// chunk (b mod chunksPerBrick) of brick (b / chunksPerBrick) -- 1024 voxels, 4 per thread at
// a 256-voxel stride, so every wave-instruction reads and writes 64 consecutive voxels of a
// row.  Index decomposition uses precomputed 32-bit magic divisors; the clamp reproduces the
// halo semantics at the volume border.  HBM traffic = the algorithmic bytes of the copies
// (each brick voxel read once from the source -- halo voxels are re-reads of a neighbour's
// interior, counted as in SURVEY.md §8(d): b_src + b_dst per voxel in range).

#include "KernelCommon.hpp"
#include "../runtime/Runtime.hpp"
#include "volkit_hip.h"

#include <cstdlib>
#include <mutex>
#include <vector>

namespace vkt
{
namespace hipk
{
    bool validView(vktHipVolumeView_t const& v);
    bool overlaps(vktHipVolumeView_t const& a, vktHipVolumeView_t const& b);

    struct BrickDesc
    {
        uint8_t* dst;
        int32_t dimX, dimY;      // brick dims (dst row / plane pitch)
        int32_t fx, fy, fz;      // source voxel copied to brick (0,0,0); may be negative (halo)
        uint32_t nvox;           // voxels in the copy box (nx*ny*nz)
        FastDiv fdx, fdy;        // box nx, ny
    };

    constexpr int kDecompPerThread = 4;
    constexpr uint32_t kDecompChunk = kBlock * kDecompPerThread;   // voxels per workgroup

    __device__ __forceinline__ int32_t clampi(int32_t v, int32_t hi)
    {
        return v < 0 ? 0 : (v > hi ? hi : v);
    }

    template <int BPV>
    __global__ __launch_bounds__(kBlock) void brickCopyKernel(BrickDesc const* bricks, FastDiv chunksPerBrick,
                                                             uint8_t const* src, int32_t sdx, int32_t sdy,
                                                             int32_t sdz)
    {
        uint32_t const b = __builtin_amdgcn_readfirstlane(fdiv(blockIdx.x, chunksPerBrick));
        uint32_t const chunk = blockIdx.x - b * chunksPerBrick.d;
        BrickDesc const d = bricks[b];
        uint32_t const base = chunk * kDecompChunk;
        if (base >= d.nvox)
            return;   // border bricks are smaller than the largest one
        uint64_t const pitchY = static_cast<uint64_t>(d.dimX);
        uint64_t const pitchZ = pitchY * static_cast<uint64_t>(d.dimY);
        uint64_t const spY = static_cast<uint64_t>(sdx), spZ = spY * static_cast<uint64_t>(sdy);
        uint32_t codes[kDecompPerThread];
        uint64_t dsts[kDecompPerThread];
        bool live[kDecompPerThread];
#pragma unroll
        for (int u = 0; u < kDecompPerThread; ++u)
        {
            uint32_t const i = base + u * kBlock + threadIdx.x;
            live[u] = i < d.nvox;
            uint32_t const ii = live[u] ? i : 0;
            uint32_t const q = fdiv(ii, d.fdx);
            uint32_t const x = ii - q * d.fdx.d;
            uint32_t const z = fdiv(q, d.fdy);
            uint32_t const y = q - z * d.fdy.d;
            int32_t const sx = clampi(d.fx + static_cast<int32_t>(x), sdx - 1);
            int32_t const sy = clampi(d.fy + static_cast<int32_t>(y), sdy - 1);
            int32_t const sz = clampi(d.fz + static_cast<int32_t>(z), sdz - 1);
            codes[u] = loadCode<BPV>(src, static_cast<uint64_t>(sz) * spZ + static_cast<uint64_t>(sy) * spY +
                                              static_cast<uint64_t>(sx));
            dsts[u] = static_cast<uint64_t>(z) * pitchZ + static_cast<uint64_t>(y) * pitchY + x;
        }
#pragma unroll
        for (int u = 0; u < kDecompPerThread; ++u)
            if (live[u])
                storeCode<BPV>(d.dst, dsts[u], codes[u]);
    }

    // Descriptor table: pinned host staging + a grow-only device buffer, uploaded with a
    // stream-ordered H2D copy on the compute stream.  Both are reused only after the previous
    // decomposition's kernel finished (event recorded behind it), so a caller that switches
    // the compute stream between calls cannot race the table.
    struct DescTable
    {
        std::mutex m;
        BrickDesc* host = nullptr;
        BrickDesc* dev = nullptr;
        size_t cap = 0;
        hipEvent_t done = nullptr;
        bool pending = false;
    };

    DescTable& descTable()
    {
        static DescTable t;
        return t;
    }

} // hipk
} // vkt

using namespace vkt;
using namespace vkt::hipk;

extern "C" {

vktError vktHipBrickDecompose(vktHipVolumeView_t source, vktHipBrickRange_t const* bricks, int32_t numBricks)
{
    if (!validView(source))
        return rt::fail("vktHipBrickDecompose: invalid source view");
    if (numBricks < 0 || (numBricks > 0 && bricks == nullptr))
        return rt::fail("vktHipBrickDecompose: invalid brick list");
    if (numBricks == 0)
        return vktNoError;
    if (source.dimX <= 0 || source.dimY <= 0 || source.dimZ <= 0)
        return rt::fail("vktHipBrickDecompose: empty source volume");

    // validate everything before the first launch (reference: out-of-range writes are UB)
    std::vector<BrickDesc> fast;
    std::vector<int32_t> slow;
    fast.reserve(static_cast<size_t>(numBricks));
    uint32_t maxVox = 0;
    for (int32_t i = 0; i < numBricks; ++i)
    {
        vktHipBrickRange_t const& br = bricks[i];
        if (!validView(br.brick))
            return rt::fail("vktHipBrickDecompose: invalid brick view");
        int64_t nx = int64_t(br.last.x) - br.first.x, ny = int64_t(br.last.y) - br.first.y;
        int64_t nz = int64_t(br.last.z) - br.first.z;
        if (nx <= 0 || ny <= 0 || nz <= 0)
            continue;
        if (nx > br.brick.dimX || ny > br.brick.dimY || nz > br.brick.dimZ)
            return rt::fail("vktHipBrickDecompose: brick smaller than its range (reference writes out of bounds)");
        if (overlaps(br.brick, source))
            return rt::fail("vktHipBrickDecompose: brick aliases the source");
        bool bytewise = br.brick.dataFormat == source.dataFormat && br.brick.mappingLo == source.mappingLo &&
                        br.brick.mappingHi == source.mappingHi;   // Copy_serial.hpp:21-22
        uint64_t nv = static_cast<uint64_t>(nx) * static_cast<uint64_t>(ny) * static_cast<uint64_t>(nz);
        if (!bytewise || nv >= (1ull << 31))
        {
            slow.push_back(i);
            continue;
        }
        BrickDesc d{};
        d.dst = br.brick.data;
        d.dimX = br.brick.dimX;
        d.dimY = br.brick.dimY;
        d.fx = br.first.x;
        d.fy = br.first.y;
        d.fz = br.first.z;
        d.nvox = static_cast<uint32_t>(nv);
        d.fdx = makeFastDiv(static_cast<uint32_t>(nx));
        d.fdy = makeFastDiv(static_cast<uint32_t>(ny));
        maxVox = d.nvox > maxVox ? d.nvox : maxVox;
        fast.push_back(d);
    }

    hipStream_t s = rt::computeStream();
    if (!fast.empty())
    {
        uint32_t const bpv = codec::bytesPerVoxel(source.dataFormat);
        if (bpv != 1 && bpv != 2 && bpv != 4)
            return rt::fail("vktHipBrickDecompose: unsupported data format");
        uint64_t const chunks = (maxVox + kDecompChunk - 1) / kDecompChunk;
        uint64_t const blocks = chunks * fast.size();
        if (blocks >= (1ull << 32))
            return rt::fail("vktHipBrickDecompose: too many bricks for one launch");
        DescTable& st = descTable();
        std::lock_guard<std::mutex> lock(st.m);
        if (st.pending)
        {
            VKT_HIP_TRY(hipEventSynchronize(st.done));
            st.pending = false;
        }
        if (st.cap < fast.size())
        {
            if (st.host)
                VKT_HIP_TRY(hipHostFree(st.host));
            if (st.dev)
                VKT_HIP_TRY(hipFree(st.dev));
            st.host = nullptr;
            st.dev = nullptr;
            st.cap = 0;
            VKT_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&st.host), fast.size() * sizeof(BrickDesc)));
            VKT_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&st.dev), fast.size() * sizeof(BrickDesc)));
            st.cap = fast.size();
        }
        if (!st.done)
            VKT_HIP_TRY(hipEventCreateWithFlags(&st.done, hipEventDisableTiming));
        std::copy(fast.begin(), fast.end(), st.host);
        BrickDesc* dev = st.dev;
        VKT_HIP_TRY(hipMemcpyAsync(dev, st.host, fast.size() * sizeof(BrickDesc), hipMemcpyHostToDevice, s));
        FastDiv const fdc = makeFastDiv(static_cast<uint32_t>(chunks));
        unsigned const g = static_cast<unsigned>(blocks);
        if (bpv == 1)
            hipLaunchKernelGGL(brickCopyKernel<1>, dim3(g), dim3(kBlock), 0, s, dev, fdc, source.data, source.dimX,
                               source.dimY, source.dimZ);
        else if (bpv == 2)
            hipLaunchKernelGGL(brickCopyKernel<2>, dim3(g), dim3(kBlock), 0, s, dev, fdc, source.data, source.dimX,
                               source.dimY, source.dimZ);
        else
            hipLaunchKernelGGL(brickCopyKernel<4>, dim3(g), dim3(kBlock), 0, s, dev, fdc, source.data, source.dimX,
                               source.dimY, source.dimZ);
        VKT_HIP_TRY(hipGetLastError());
        VKT_HIP_TRY(hipEventRecord(st.done, s));
        st.pending = true;
    }
    // bricks that need the unmap -> map conversion: one CopyRange each
    for (int32_t i : slow)
    {
        vktHipBrickRange_t const& br = bricks[i];
        vktError e = vktHipCopyRange(br.brick, source, br.first, br.last, vktVec3i_t{0, 0, 0});
        if (e != vktNoError)
            return e;
    }
    return rt::finishLaunch("BrickDecompose_hip");
}

} // extern "C"
