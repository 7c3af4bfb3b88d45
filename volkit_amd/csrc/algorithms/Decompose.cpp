// Decompose.cpp -- BrickDecompose / BrickDecomposeResize front-ends and the C Array3D of
// StructuredVolume handles.
//
// Reference: src/vkt/Decompose.cpp:26-260 (C++ and C front-ends), src/vkt/Decompose_serial.hpp:
// 15-88 (the per-brick CopyRange loop), include/c/vkt/Array3D.h:18-237 (C array API).
// Under the GPU policy the whole decomposition is one vktHipBrickDecompose call
// (kernels/Decompose.hip); under the CPU policy it returns InvalidValue like every other
// algorithm of this GPU backend.

#include "../runtime/HostPool.hpp"
#include "../runtime/Runtime.hpp"
#include "../StructuredVolume_impl.hpp"
#include "volkit_hip.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <vector>

namespace vkt
{
namespace
{
    int32_t divUp(int32_t a, int32_t b) { return (a + b - 1) / b; }

    vktHipVolumeView_t brickView(StructuredVolume& v)
    {
        vktHipVolumeView_t out;
        out.data = rt::deviceData(v);
        Vec3i d = v.getDims();
        out.dimX = d.x;
        out.dimY = d.y;
        out.dimZ = d.z;
        out.dataFormat = static_cast<int32_t>(v.getDataFormat());
        Vec2f m = v.getVoxelMapping();
        out.mappingLo = m.x;
        out.mappingHi = m.y;
        return out;
    }

    bool validBrickSize(Vec3i b) { return b.x > 0 && b.y > 0 && b.z > 0; }

    // numBricks and the border brick size (reference Decompose.cpp:103-121)
    void brickGrid(Vec3i dims, Vec3i brick, Vec3i& numBricks, Vec3i& border)
    {
        numBricks = {divUp(dims.x, brick.x), divUp(dims.y, brick.y), divUp(dims.z, brick.z)};
        Vec3i ext{numBricks.x * brick.x, numBricks.y * brick.y, numBricks.z * brick.z};
        border = {dims.x % brick.x == 0 ? brick.x : brick.x - ext.x + dims.x,
                  dims.y % brick.y == 0 ? brick.y : brick.y - ext.y + dims.y,
                  dims.z % brick.z == 0 ? brick.z : brick.z - ext.z + dims.z};
    }

    std::vector<uint8_t*>& gridPointers()
    {
        thread_local std::vector<uint8_t*> p;
        return p;
    }

    // The usual decomposition -- the array has ceil(dims / brickSize) bricks per axis, each
    // allocated exactly at its box (cell +- halos, border cells cropped) in the source's format
    // and mapping, as BrickDecomposeResize builds it: one pass over the bricks that checks that
    // and collects their data pointers (gridPointers) for vktHipBrickDecomposeGrid, which derives
    // every brick's range from its index.  262 144 bricks of 16^3: the range list walk plus the
    // backend's validation of it took ~1.4 ms of host time per call on the MI355X box.  False
    // (and the range path runs) at the first brick that differs.
    template <class BrickAt, class Prefetch>
    bool uniformGrid(Vec3i arrDims, StructuredVolume& source, Vec3i brickSize, Vec3i haloNeg, Vec3i haloPos,
                     ExecutionPolicy const& ep, BrickAt& brickAt, Prefetch& prefetch, size_t total)
    {
        if (total == 0 || rt::knob(rt::Knob::DecomposeGrid) == 0)
            return false;
        Vec3i const dims = source.getDims();
        int32_t const sd[3] = {dims.x, dims.y, dims.z}, na[3] = {arrDims.x, arrDims.y, arrDims.z};
        int32_t const bs[3] = {brickSize.x, brickSize.y, brickSize.z};
        int32_t const hn[3] = {haloNeg.x, haloNeg.y, haloNeg.z}, hp[3] = {haloPos.x, haloPos.y, haloPos.z};
        int32_t ext[3][2];   // box extent of an axis' non-last / last bricks
        for (int a = 0; a < 3; ++a)
        {
            if (hn[a] < 0 || hp[a] < 0 || na[a] != divUp(sd[a], bs[a]))
                return false;
            ext[a][0] = hn[a] + bs[a] + hp[a];
            ext[a][1] = hn[a] + sd[a] - (na[a] - 1) * bs[a] + hp[a];
        }
        DataFormat const fmt = source.getDataFormat();
        Vec2f const map = source.getVoxelMapping();
        std::vector<uint8_t*>& ptrs = gridPointers();
        if (ptrs.size() < total)
            ptrs.resize(total);
        std::atomic<bool> ok{true};
        size_t const nx = static_cast<size_t>(na[0]), ny = static_cast<size_t>(na[1]);
        rt::parallelFor(total, 4096, [&](size_t b, size_t e) {
            ExecutionPolicy const saved = GetThreadExecutionPolicy();
            SetThreadExecutionPolicy(ep);
            constexpr size_t kAhead = 16;
            for (size_t i = b; i < std::min(e, b + kAhead); ++i)
                prefetch(i);
            size_t ix = b % nx, iy = (b / nx) % ny, iz = b / (nx * ny);
            bool good = true;
            for (size_t i = b; i < e && good; ++i)
            {
                if (i + kAhead < e)
                    prefetch(i + kAhead);
                StructuredVolume& v = brickAt(i);
                Vec3i const d = v.getDims();
                Vec2f const m = v.getVoxelMapping();
                good = d.x == ext[0][ix + 1 == nx] && d.y == ext[1][iy + 1 == ny] &&
                       d.z == ext[2][iz + 1 == static_cast<size_t>(na[2])] && v.getDataFormat() == fmt &&
                       m.x == map.x && m.y == map.y;
                ptrs[i] = v.getDataFor(ep);
                good = good && (ptrs[i] != nullptr || d.x * d.y * d.z == 0);   // (a failed migration: the range path reports it)
                if (++ix == nx)
                {
                    ix = 0;
                    if (++iy == ny)
                    {
                        iy = 0;
                        ++iz;
                    }
                }
            }
            if (!good)
                ok.store(false, std::memory_order_relaxed);
            SetThreadExecutionPolicy(saved);
        });
        return ok.load();
    }

    // The per-brick ranges of BrickDecompose_serial (Decompose_serial.hpp:24-44), then one
    // backend call.  `brickAt(i)` returns the StructuredVolume of brick linear index i.
    // `prefetch(i)` touches brick i's object ahead of its use (separately allocated C handles:
    // the walk is otherwise one DRAM latency per brick).
    template <class BrickAt, class Prefetch>
    Error decompose(Vec3i arrDims, StructuredVolume& source, Vec3i brickSize, Vec3i haloNeg, Vec3i haloPos,
                    BrickAt&& brickAt, Prefetch&& prefetch)
    {
        ExecutionPolicy ep = GetThreadExecutionPolicy();
        if (ep.device != ExecutionPolicy::Device::GPU)
        {
            rt::setLastError("BrickDecompose_hip: CPU execution policy");
            VKT_LOG(rt::LogLevel::Error) << "When calling algorithm: BrickDecompose_hip -- volkit-amd implements the "
                                            "GPU (HIP/gfx950) backend only; set ExecutionPolicy::Device::GPU";
            return InvalidValue;
        }
        if (!validBrickSize(brickSize))
        {
            rt::fail("BrickDecompose: brick size must be positive");
            return InvalidValue;
        }
        rt::ScopedKernelTimer timer("BrickDecompose_hip", ep.printPerformance != False);
        Vec3i const dims = source.getDims();
        size_t const nx = static_cast<size_t>(std::max(0, arrDims.x)), ny = static_cast<size_t>(std::max(0, arrDims.y));
        size_t const total = nx * ny * static_cast<size_t>(std::max(0, arrDims.z));
        // reused across calls (a fresh 15 MB vector for 16^3 bricks of 1024^3 cost ~0.8 ms of
        // page faults and zeroing per call); every element is overwritten below
        // (the workers below see the CALLER's buffer through `out`: naming a thread_local inside
        // the lambda would give each worker its own)
        if (uniformGrid(arrDims, source, brickSize, haloNeg, haloPos, ep, brickAt, prefetch, total))
            return static_cast<Error>(vktHipBrickDecomposeGrid(
                brickView(source),
                vktHipBrickGrid_t{{arrDims.x, arrDims.y, arrDims.z}, {brickSize.x, brickSize.y, brickSize.z},
                                  {haloNeg.x, haloNeg.y, haloNeg.z}, {haloPos.x, haloPos.y, haloPos.z}},
                gridPointers().data()));
        thread_local std::vector<vktHipBrickRange_t> ranges;
        if (ranges.size() < total)
            ranges.resize(total);
        vktHipBrickRange_t* const out = ranges.data();
        vktHipVolumeView_t const src = brickView(source);
        // Knob decompose.batch 1: the ranges are planned and handed to the backend in batches of
        // whole brick planes (~16 Ki bricks, at most kMaxBatches), so the host plans batch k + 1
        // while the GPU copies batch k.  Measured on MI355X (profiles/r04/decbatch.jsonl) it is
        // SLOWER: 16^3 bricks + halo 1 of 1024^3 UInt16 back-to-back 2.61 ms batched vs 1.54 ms
        // in one batch, incl. planning 2.80 vs 2.61 -- eight small copy launches fill the GPU
        // worse than one, and the per-call descriptor upload and grid inference repeat -- so the
        // default is one batch.
        constexpr size_t kBatchBricks = 16384, kMaxBatches = 8;
        size_t const nzb = static_cast<size_t>(std::max(0, arrDims.z)), plane = nx * ny;
        size_t batches = rt::knob(rt::Knob::DecomposeBatch) != 0
                             ? std::min(kMaxBatches, std::max<size_t>(1, total / kBatchBricks))
                             : 1;   // (knob decompose.batch 0: one batch, for the A/B)
        batches = std::min(batches, std::max<size_t>(1, nzb));
        size_t const planesPer = nzb > 0 ? (nzb + batches - 1) / batches : 0;
        // one view per brick (getData() migrates a brick that lives elsewhere): ~16 ns per brick,
        // 4 ms for the 262 144 bricks of 16^3 over 1024^3 serially -- split over the host pool,
        // each worker under the caller's policy (and device: HostPool)
        auto plan = [&](size_t b, size_t e) {
            ExecutionPolicy const saved = GetThreadExecutionPolicy();
            SetThreadExecutionPolicy(ep);
            constexpr size_t kAhead = 16;
            for (size_t i = b; i < std::min(e, b + kAhead); ++i)
                prefetch(i);
            for (size_t i = b; i < e; ++i)
            {
                if (i + kAhead < e)
                    prefetch(i + kAhead);
                int32_t const x = static_cast<int32_t>(i % nx), y = static_cast<int32_t>((i / nx) % ny);
                int32_t const z = static_cast<int32_t>(i / (nx * ny));
                vktHipBrickRange_t& r = out[i];
                vktVec3i_t first{x * brickSize.x, y * brickSize.y, z * brickSize.z};
                vktVec3i_t last{std::min(first.x + brickSize.x, dims.x), std::min(first.y + brickSize.y, dims.y),
                                std::min(first.z + brickSize.z, dims.z)};
                r.first = {first.x - haloNeg.x, first.y - haloNeg.y, first.z - haloNeg.z};
                r.last = {last.x + haloPos.x, last.y + haloPos.y, last.z + haloPos.z};
                r.brick = brickView(brickAt(i));
            }
            SetThreadExecutionPolicy(saved);
        };
        if (total == 0 || planesPer == 0)
            return static_cast<Error>(vktHipBrickDecompose(src, out, 0));
        for (size_t z0 = 0; z0 < nzb; z0 += planesPer)
        {
            size_t const b0 = z0 * plane, b1 = std::min(nzb, z0 + planesPer) * plane;
            rt::parallelFor(b1 - b0, 4096, [&](size_t b, size_t e) { plan(b0 + b, b0 + e); });
            vktError const e = vktHipBrickDecompose(src, out + b0, static_cast<int32_t>(b1 - b0));
            if (e != vktNoError)
                return static_cast<Error>(e);
        }
        return NoError;
    }
} // namespace

Error BrickDecompose(Array3D<StructuredVolume>& dest, StructuredVolume& source, int32_t bx, int32_t by, int32_t bz,
                     int32_t nx, int32_t ny, int32_t nz, int32_t px, int32_t py, int32_t pz)
{
    return BrickDecompose(dest, source, Vec3i{bx, by, bz}, Vec3i{nx, ny, nz}, Vec3i{px, py, pz});
}

Error BrickDecompose(Array3D<StructuredVolume>& dest, StructuredVolume& source, Vec3i brickSize, Vec3i haloSizeNeg,
                     Vec3i haloSizePos)
{
    StructuredVolume* bricks = dest.data();
    return decompose(dest.dims(), source, brickSize, haloSizeNeg, haloSizePos,
                     [&](size_t i) -> StructuredVolume& { return bricks[i]; }, [](size_t) {});
}

Error BrickDecomposeResize(Array3D<StructuredVolume>& dest, StructuredVolume& source, int32_t bx, int32_t by,
                           int32_t bz, int32_t nx, int32_t ny, int32_t nz, int32_t px, int32_t py, int32_t pz)
{
    return BrickDecomposeResize(dest, source, Vec3i{bx, by, bz}, Vec3i{nx, ny, nz}, Vec3i{px, py, pz});
}

// Reference Decompose.cpp:96-150: one brick per cell, border bricks cropped, halos added,
// same format / dist / mapping as the source.  Allocation happens on the calling thread's
// device (GPU policy: straight into HBM).
Error BrickDecomposeResize(Array3D<StructuredVolume>& dest, StructuredVolume& source, Vec3i brickSize,
                           Vec3i haloSizeNeg, Vec3i haloSizePos)
{
    if (!validBrickSize(brickSize))
    {
        rt::fail("BrickDecomposeResize: brick size must be positive");
        return InvalidValue;
    }
    Vec3i numBricks, border;
    brickGrid(source.getDims(), brickSize, numBricks, border);
    dest = Array3D<StructuredVolume>(numBricks);
    Vec3f dist = source.getDist();
    Vec2f map = source.getVoxelMapping();
    for (int32_t z = 0; z < numBricks.z; ++z)
        for (int32_t y = 0; y < numBricks.y; ++y)
            for (int32_t x = 0; x < numBricks.x; ++x)
            {
                Vec3i size{x < numBricks.x - 1 ? brickSize.x : border.x, y < numBricks.y - 1 ? brickSize.y : border.y,
                           z < numBricks.z - 1 ? brickSize.z : border.z};
                StructuredVolume brick(haloSizeNeg.x + size.x + haloSizePos.x, haloSizeNeg.y + size.y + haloSizePos.y,
                                       haloSizeNeg.z + size.z + haloSizePos.z, source.getDataFormat(), dist.x, dist.y,
                                       dist.z, map.x, map.y);
                dest[Vec3i{x, y, z}] = std::move(brick);
            }
    return NoError;
}

} // vkt

//--- C API ---------------------------------------------------------------------------------
struct vktArray3D_vktStructuredVolume_impl
{
    std::vector<vktStructuredVolume> handles;
    vktVec3i_t dims{0, 0, 0};
};

namespace
{
    size_t count(vktVec3i_t d)
    {
        return d.x > 0 && d.y > 0 && d.z > 0 ? static_cast<size_t>(d.x) * static_cast<size_t>(d.y) * static_cast<size_t>(d.z)
                                             : 0;
    }

    size_t linear(vktArray3D_vktStructuredVolume arr, vktVec3i_t i)
    {
        return (static_cast<size_t>(i.z) * static_cast<size_t>(arr->dims.y) + static_cast<size_t>(i.y)) *
                   static_cast<size_t>(arr->dims.x) +
               static_cast<size_t>(i.x);
    }
} // namespace

extern "C" {

void vktArray3D_vktStructuredVolume_CreateEmpty(vktArray3D_vktStructuredVolume* arr)
{
    *arr = new vktArray3D_vktStructuredVolume_impl;
}

void vktArray3D_vktStructuredVolume_Create(vktArray3D_vktStructuredVolume* arr, vktVec3i_t dims)
{
    *arr = new vktArray3D_vktStructuredVolume_impl;
    (*arr)->handles.assign(count(dims), nullptr);
    (*arr)->dims = dims;
}

// Copies the handle values (shallow, like the reference's byte copy of the handle buffer).
void vktArray3D_vktStructuredVolume_CreateCopy(vktArray3D_vktStructuredVolume* arr, vktArray3D_vktStructuredVolume rhs)
{
    *arr = new vktArray3D_vktStructuredVolume_impl(*rhs);
}

void vktArray3D_vktStructuredVolume_Destroy(vktArray3D_vktStructuredVolume arr)
{
    if (!arr)
        return;
    for (vktStructuredVolume h : arr->handles)
        if (h)
            vktStructuredVolumeDestroy(h);
    delete arr;
}

// Keeps the handles of the first min(old, new) slots (reference: ManagedBuffer resize keeps
// the leading bytes); new slots are NULL.
void vktArray3D_vktStructuredVolume_Resize(vktArray3D_vktStructuredVolume arr, vktVec3i_t dims)
{
    arr->handles.resize(count(dims), nullptr);
    arr->dims = dims;
}

void vktArray3D_vktStructuredVolume_Fill(vktArray3D_vktStructuredVolume arr, vktStructuredVolume value)
{
    std::fill(arr->handles.begin(), arr->handles.end(), value);
}

vktStructuredVolume* vktArray3D_vktStructuredVolume_Begin(vktArray3D_vktStructuredVolume arr)
{
    return arr->handles.data();
}

vktStructuredVolume const* vktArray3D_vktStructuredVolume_CBegin(vktArray3D_vktStructuredVolume arr)
{
    return arr->handles.data();
}

vktStructuredVolume* vktArray3D_vktStructuredVolume_End(vktArray3D_vktStructuredVolume arr)
{
    return arr->handles.data() + arr->handles.size();
}

vktStructuredVolume const* vktArray3D_vktStructuredVolume_CEnd(vktArray3D_vktStructuredVolume arr)
{
    return arr->handles.data() + arr->handles.size();
}

vktStructuredVolume* vktArray3D_vktStructuredVolume_Access(vktArray3D_vktStructuredVolume arr, vktVec3i_t index)
{
    return &arr->handles[linear(arr, index)];
}

vktStructuredVolume const* vktArray3D_vktStructuredVolume_CAccess(vktArray3D_vktStructuredVolume arr, vktVec3i_t index)
{
    return &arr->handles[linear(arr, index)];
}

vktBool_t vktArray3D_vktStructuredVolume_Empty(vktArray3D_vktStructuredVolume arr)
{
    return arr->handles.empty() ? VKT_TRUE : VKT_FALSE;
}

vktStructuredVolume* vktArray3D_vktStructuredVolume_Data(vktArray3D_vktStructuredVolume arr)
{
    return arr->handles.data();
}

vktStructuredVolume const* vktArray3D_vktStructuredVolume_CData(vktArray3D_vktStructuredVolume arr)
{
    return arr->handles.data();
}

vktVec3i_t vktArray3D_vktStructuredVolume_Dims(vktArray3D_vktStructuredVolume arr) { return arr->dims; }

size_t vktArray3D_vktStructuredVolume_NumElements(vktArray3D_vktStructuredVolume arr) { return arr->handles.size(); }

vktError vktBrickDecomposeSV(vktArray3D_vktStructuredVolume dest, vktStructuredVolume source, int32_t bx, int32_t by,
                             int32_t bz, int32_t nx, int32_t ny, int32_t nz, int32_t px, int32_t py, int32_t pz)
{
    if (!dest || !source)
        return vktInvalidValue;
    for (vktStructuredVolume h : dest->handles)
        if (!h)
            return vkt::rt::fail("vktBrickDecomposeSV: the array holds an unallocated brick (call vktBrickDecomposeResizeSV)");
    return static_cast<vktError>(vkt::decompose(vkt::Vec3i{dest->dims.x, dest->dims.y, dest->dims.z}, source->volume,
                                                vkt::Vec3i{bx, by, bz}, vkt::Vec3i{nx, ny, nz}, vkt::Vec3i{px, py, pz},
                                                [&](size_t i) -> vkt::StructuredVolume& {
                                                    return dest->handles[i]->volume;
                                                },
                                                [&](size_t i) {
                                                    char const* p = reinterpret_cast<char const*>(dest->handles[i]);
                                                    __builtin_prefetch(p);
                                                    __builtin_prefetch(p + 64);
                                                }));
}

// Reference Decompose.cpp:185-260; previously held handles are destroyed first (the
// reference overwrites and leaks them).
vktError vktBrickDecomposeResizeSV(vktArray3D_vktStructuredVolume dest, vktStructuredVolume source, int32_t bx,
                                   int32_t by, int32_t bz, int32_t nx, int32_t ny, int32_t nz, int32_t px, int32_t py,
                                   int32_t pz)
{
    if (!dest || !source)
        return vktInvalidValue;
    if (bx <= 0 || by <= 0 || bz <= 0)
        return vkt::rt::fail("vktBrickDecomposeResizeSV: brick size must be positive");
    vkt::Vec3i numBricks, border;
    vkt::brickGrid(source->volume.getDims(), vkt::Vec3i{bx, by, bz}, numBricks, border);
    for (vktStructuredVolume h : dest->handles)
        if (h)
            vktStructuredVolumeDestroy(h);
    dest->handles.assign(count(vktVec3i_t{numBricks.x, numBricks.y, numBricks.z}), nullptr);
    dest->dims = {numBricks.x, numBricks.y, numBricks.z};
    vkt::Vec3f dist = source->volume.getDist();
    vkt::Vec2f map = source->volume.getVoxelMapping();
    for (int32_t z = 0; z < numBricks.z; ++z)
        for (int32_t y = 0; y < numBricks.y; ++y)
            for (int32_t x = 0; x < numBricks.x; ++x)
            {
                int32_t sx = x < numBricks.x - 1 ? bx : border.x, sy = y < numBricks.y - 1 ? by : border.y;
                int32_t sz = z < numBricks.z - 1 ? bz : border.z;
                vktStructuredVolumeCreate(vktArray3D_vktStructuredVolume_Access(dest, vktVec3i_t{x, y, z}), nx + sx + px,
                                          ny + sy + py, nz + sz + pz,
                                          static_cast<vktDataFormat>(source->volume.getDataFormat()), dist.x, dist.y,
                                          dist.z, map.x, map.y);
            }
    return vktNoError;
}

} // extern "C"
