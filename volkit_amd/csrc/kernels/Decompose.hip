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
// copies ALL bytewise bricks: a device table of brick descriptors; a workgroup copies 1024
// 16-byte items (16 KiB) of one brick through an LDS tile (brickStaged), and workgroups are
// ordered (brick row, chunk, brick along x) per XCD so neighbouring bricks' shared source
// lines are fetched close together.
// Index decomposition uses precomputed 32-bit magic divisors; the clamp reproduces the
// halo semantics at the volume border.  HBM traffic = the algorithmic bytes of the copies
// (each brick voxel read once from the source -- halo voxels are re-reads of a neighbour's
// interior, counted as in SURVEY.md §8(d): b_src + b_dst per voxel in range).

#include "KernelCommon.hpp"
#include "../runtime/HostPool.hpp"
#include "../runtime/Runtime.hpp"
#include "volkit_hip.h"

#include <algorithm>
#include <atomic>
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
        int32_t nx;              // box row length
        uint32_t nitems;         // 16-B items (linear: ceil(nvox/V); rows: ny*nz*segsPerRow)
        uint32_t nvox;           // voxels in the copy box
        int32_t linear;          // brick rows/planes packed (dimX == nx, dimY == ny) and nx >= V
        FastDiv fseg, fdx, fdy;  // segments per row, box nx, box ny
        FastDiv fwpr;            // aligned 16-B source words per row (staged copy)
    };

    // One item = 16 bytes (16/BPV voxels).  Linear mode (the usual case: a brick allocated at
    // its box size is one contiguous run): item i is dst voxels [iV, iV+V) -- one aligned
    // 16-byte store out of the LDS tile the workgroup assembled (brickStaged).  Row mode (a
    // brick larger than its range): item = a 16-byte segment of one box row, one unaligned
    // 16-byte load and store, row tails and clamped segments voxel by voxel.
    constexpr uint32_t kBrickChunk = 1024;   // 16-B items (16 KiB) per workgroup
    // threads per workgroup NT (kBlock = 256, or 128 for small bricks: knob decompose.block) and
    // items per thread kBrickChunk / NT

    struct __attribute__((packed, aligned(1))) Unaligned16
    {
        u32x4 v;
    };

    __device__ __forceinline__ int32_t clampi(int32_t v, int32_t hi)
    {
        return v < 0 ? 0 : (v > hi ? hi : v);
    }

    template <int BPV>
    __device__ __forceinline__ uint32_t wordCode(u32x4 w, int k)
    {
        uint32_t const dw = k * BPV / 4 == 0 ? w.x : k * BPV / 4 == 1 ? w.y : k * BPV / 4 == 2 ? w.z : w.w;
        if constexpr (BPV == 4)
            return dw;
        else
            return (dw >> (8 * ((k * BPV) % 4))) & ((1u << (8 * BPV)) - 1u);
    }

    template <int BPV>
    __device__ __forceinline__ void ldsStoreCode(uint8_t* lds, int32_t voxel, uint32_t code)
    {
        if constexpr (BPV == 1)
            lds[voxel] = static_cast<uint8_t>(code);
        else if constexpr (BPV == 2)
            reinterpret_cast<uint16_t*>(lds)[voxel] = static_cast<uint16_t>(code);
        else
            reinterpret_cast<uint32_t*>(lds)[voxel] = code;
    }

    // Bytes [lo, hi) of the 16-B word v to LDS bytes [a, a + hi - lo) as naturally aligned
    // 1/2/4/8/16-B writes (leading pieces align the LDS address, trailing pieces finish): no
    // unaligned LDS write and no per-voxel loop.  (Knob decompose.aligned_lds: 1 for the partial
    // words at row ends, 2 for every word.)
    __device__ __forceinline__ void ldsStoreRange(uint8_t* lds, int32_t a, u32x4 v, int lo, int hi)
    {
        uint64_t const q0 = static_cast<uint64_t>(v.x) | static_cast<uint64_t>(v.y) << 32;
        uint64_t const q1 = static_cast<uint64_t>(v.z) | static_cast<uint64_t>(v.w) << 32;
        auto at = [&](int b) -> uint64_t {   // the (up to) 8 bytes of v starting at byte b
            uint64_t const l = (b & 8) ? q1 : q0, h = (b & 8) ? 0ull : q1;
            uint32_t const sh = static_cast<uint32_t>(b & 7) * 8u;
            return sh ? (l >> sh) | (h << (64u - sh)) : l;
        };
        int b = lo, n = hi - lo;
        if (n == 16 && (a & 15) == 0)
        {
            *reinterpret_cast<u32x4*>(lds + a) = v;
            return;
        }
        if ((a & 1) && n >= 1)
        {
            lds[a] = static_cast<uint8_t>(at(b));
            a += 1; b += 1; n -= 1;
        }
        if ((a & 2) && n >= 2)
        {
            *reinterpret_cast<uint16_t*>(lds + a) = static_cast<uint16_t>(at(b));
            a += 2; b += 2; n -= 2;
        }
        if ((a & 4) && n >= 4)
        {
            *reinterpret_cast<uint32_t*>(lds + a) = static_cast<uint32_t>(at(b));
            a += 4; b += 4; n -= 4;
        }
        if ((a & 8) && n >= 8)
        {
            *reinterpret_cast<uint64_t*>(lds + a) = at(b);
            a += 8; b += 8; n -= 8;
        }
        if (n >= 8)
        {
            *reinterpret_cast<uint64_t*>(lds + a) = at(b);
            a += 8; b += 8; n -= 8;
        }
        if (n >= 4)
        {
            *reinterpret_cast<uint32_t*>(lds + a) = static_cast<uint32_t>(at(b));
            a += 4; b += 4; n -= 4;
        }
        if (n >= 2)
        {
            *reinterpret_cast<uint16_t*>(lds + a) = static_cast<uint16_t>(at(b));
            a += 2; b += 2; n -= 2;
        }
        if (n >= 1)
            lds[a] = static_cast<uint8_t>(at(b));
    }

    // LDS-staged copy of one chunk (kBrickChunk 16-byte items = the dst voxels [vStart, vEnd)
    // of a brick stored contiguously).  Phase 1: the rows the chunk touches are read as
    // 16-byte-ALIGNED source words (the hot path: one global_load_dwordx4 per lane) and
    // written to LDS at their place in the brick layout (ds_write_b128 at any byte offset --
    // gfx950 LDS accepts unaligned b128); words cut by the row span or the chunk go voxel by
    // voxel, clamped halo voxels replicate the border voxel.  Phase 2: aligned 16-byte LDS
    // reads, one aligned 16-byte global store per item.  The byte shifting is done by LDS
    // addressing instead of VALU funnel shifts (a 128-bit shift per lane made the kernel VALU
    // bound: 256^3 bricks + halo 1 took 1.15 ms vs 0.75 ms without halo; staged: 0.83 ms).
    template <int BPV, int kStageWords, int NT, bool EDGE = false>
    __device__ __forceinline__ void brickStaged(BrickDesc const& d, uint32_t base, uint8_t const* src, int32_t sdx,
                                                int32_t sdy, int32_t sdz, int32_t alignedLds)
    {
        constexpr int32_t V = 16 / BPV;
        __shared__ u32x4 tile[kBrickChunk];   // 16 KiB
        uint8_t* const lds = reinterpret_cast<uint8_t*>(tile);
        uint64_t const spY = static_cast<uint64_t>(sdx), spZ = spY * static_cast<uint64_t>(sdy);
        uint64_t const srcBytes = spZ * static_cast<uint64_t>(sdz) * BPV;
        int32_t const vStart = static_cast<int32_t>(base) * V;
        int32_t const vEnd = min(vStart + static_cast<int32_t>(kBrickChunk) * V, static_cast<int32_t>(d.nvox));
        int32_t const chunkVox = vEnd - vStart;
        int32_t const rA = static_cast<int32_t>(fdiv(static_cast<uint32_t>(vStart), d.fdx));
        int32_t const rB = static_cast<int32_t>(fdiv(static_cast<uint32_t>(vEnd - 1), d.fdx));
        int32_t const nRows = rB - rA + 1;
        int32_t const lo = max(d.fx, 0), hi = min(d.fx + d.nx, sdx);   // in-volume x span of a row
        uint32_t const wpr = d.fwpr.d;
        auto rowBase = [&](int32_t r) -> uint64_t {
            uint32_t const z = fdiv(static_cast<uint32_t>(r), d.fdy);
            uint32_t const y = static_cast<uint32_t>(r) - z * d.fdy.d;
            return static_cast<uint64_t>(clampi(d.fz + static_cast<int32_t>(z), sdz - 1)) * spZ +
                   static_cast<uint64_t>(clampi(d.fy + static_cast<int32_t>(y), sdy - 1)) * spY;
        };
        uint32_t const total = static_cast<uint32_t>(nRows) * wpr;
        // alignedLds 4 (edge mode; host: one chunk per brick, 16-B row pitch): the words a row end
        // cuts are not placed word by word -- the <= V - 1 voxels at each end of a row's span are
        // copied voxel by voxel in a loop of their own, the same count for every row of the brick,
        // so no wave runs the per-voxel branches of a cut word
        // (a template parameter: the edge code in every instance cost the others 15 VGPRs --
        // brickCopyKernel<2, 6> 66 -> 81, 7 -> 5 waves per SIMD)
        constexpr bool edges = EDGE;
        // one aligned source word: where it comes from and where it lands in LDS
        struct Word
        {
            uint64_t rb;
            int32_t x0, li;
            bool live, whole;
            u32x4 v;
        };
        auto locate = [&](uint32_t t, Word& w) {
            w.live = t < total;
            uint32_t const tt = w.live ? t : 0u;
            uint32_t const q = fdiv(tt, d.fwpr);
            int32_t const r = rA + static_cast<int32_t>(q);
            w.rb = rowBase(r);
            uint64_t const startByte = (((w.rb + static_cast<uint64_t>(lo)) * BPV) & ~uint64_t(15)) + 16ull * (tt - q * wpr);
            w.live = w.live && startByte < (w.rb + static_cast<uint64_t>(hi)) * BPV;
            w.x0 = static_cast<int32_t>(startByte / BPV - w.rb);   // x of the word's first voxel
            w.li = r * d.nx + (w.x0 - d.fx) - vStart;              // its LDS voxel index
            w.whole = startByte + 16 <= srcBytes;
            w.v = u32x4{0u, 0u, 0u, 0u};
            // (edge mode: only the words inside the row span are loaded and placed)
            bool const need = !edges || (w.x0 >= lo && w.x0 + V <= hi);
            if (w.live && w.whole && need)
                w.v = *reinterpret_cast<u32x4 const*>(src + startByte);
        };
        // (knob decompose.aligned_lds 3) the tile's bytes past the chunk's voxels, when 16 of
        // them are free: a partial word writes its voxels outside the row span / chunk there
        int32_t const dumpB = chunkVox * BPV;
        bool const dumpable = alignedLds == 3 && dumpB + 16 <= static_cast<int32_t>(kBrickChunk) * 16;
        auto place = [&](Word const& w) {
            if (!w.live)
                return;
            if (w.whole && w.x0 >= lo && w.x0 + V <= hi && w.li >= 0 && w.li + V <= chunkVox)
            {
                if (alignedLds == 2)
                    ldsStoreRange(lds, w.li * BPV, w.v, 0, 16);
                else
                    reinterpret_cast<Unaligned16*>(lds + w.li * BPV)->v = w.v;
            }
            else if (edges)
                return;   // its voxels come from the edge loop
            else if (w.whole && dumpable)
            {
                // a word cut by a row end or the chunk: all V voxels written, the ones outside to
                // the dump bytes -- a select per voxel instead of a divergent branch (the
                // per-voxel ifs below cost ~30 scalar exec-mask instructions per word: SQ_INSTS_SALU
                // was as high as SQ_INSTS_VALU on 16^3 bricks, profiles/r04/dec16.pmc.jsonl)
#pragma unroll
                for (int k = 0; k < V; ++k)
                {
                    bool const in = w.x0 + k >= lo && w.x0 + k < hi && w.li + k >= 0 && w.li + k < chunkVox;
                    int32_t const b = in ? (w.li + k) * BPV : dumpB;
                    ldsStoreCode<BPV>(lds + b, 0, wordCode<BPV>(w.v, k));
                }
            }
            else if (w.whole && alignedLds == 1)
            {
                // the voxels of the word inside the row span and the chunk, as aligned pieces
                int32_t const k0 = max(max(lo - w.x0, -w.li), 0);
                int32_t const k1 = min(min(hi - w.x0, chunkVox - w.li), V);
                if (k1 > k0)
                    ldsStoreRange(lds, (w.li + k0) * BPV, w.v, k0 * BPV, k1 * BPV);
            }
            else
            {
#pragma unroll
                for (int k = 0; k < V; ++k)
                    if (w.x0 + k >= lo && w.x0 + k < hi && w.li + k >= 0 && w.li + k < chunkVox)
                        ldsStoreCode<BPV>(lds, w.li + k,
                                          w.whole ? wordCode<BPV>(w.v, k) : loadCode<BPV>(src, w.rb + w.x0 + k));
            }
        };
        // all loads of the first kStageWords rounds in flight before the first LDS write (a
        // load -> wait -> write loop serialises the memory latency per round; the words left
        // over after them cost the workgroup a second memory latency)
        Word words[kStageWords];
#pragma unroll
        for (int k = 0; k < kStageWords; ++k)
            locate(threadIdx.x + k * NT, words[k]);
        // edge mode: per row, h head voxels [lo, lo + h) before the first whole word and t tail
        // voxels [hi - t, hi) after the last (the row phase is the same for every row); their
        // first round of loads goes out right behind the word loads, so the two round trips
        // overlap
        int32_t eh = 0, et = 0;
        uint32_t en = 0;
        FastDiv fe{1u, 0u, 0u};
        if (edges && hi > lo)
        {
            int32_t const ph = (lo * BPV) & 15;
            int32_t const headB = (16 - ph) & 15, spanB = (hi - lo) * BPV;
            eh = spanB <= headB ? hi - lo : headB / BPV;
            et = spanB <= headB ? 0 : ((spanB - headB) & 15) / BPV;
            if (eh + et > 0)
            {
                fe = makeFastDiv(static_cast<uint32_t>(eh + et));
                en = static_cast<uint32_t>(nRows) * static_cast<uint32_t>(eh + et);
            }
        }
        auto edgeIssue = [&](uint32_t q0, uint32_t (&code)[4], int32_t (&at)[4]) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
            {
                uint32_t const q = q0 + static_cast<uint32_t>(u * NT) + threadIdx.x;
                uint32_t const qq = q < en ? q : 0u;
                uint32_t const rq = fdiv(qq, fe);
                int32_t const k = static_cast<int32_t>(qq - rq * fe.d);
                int32_t const x = k < eh ? lo + k : hi - et + (k - eh);
                int32_t const r = rA + static_cast<int32_t>(rq);
                at[u] = q < en ? r * d.nx + (x - d.fx) - vStart : -1;
                code[u] = q < en ? loadCode<BPV>(src, rowBase(r) + static_cast<uint64_t>(x)) : 0u;
            }
        };
        auto edgeWrite = [&](uint32_t const (&code)[4], int32_t const (&at)[4]) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (at[u] >= 0 && at[u] < chunkVox)
                    ldsStoreCode<BPV>(lds, at[u], code[u]);
        };
        uint32_t ecode[4] = {0u, 0u, 0u, 0u};
        int32_t eat[4] = {-1, -1, -1, -1};
        if (en > 0)
            edgeIssue(0u, ecode, eat);
#pragma unroll
        for (int k = 0; k < kStageWords; ++k)
            place(words[k]);
        for (uint32_t t = threadIdx.x + kStageWords * NT; t < total; t += NT)
        {
            Word w;
            locate(t, w);
            place(w);
        }
        if (en > 0)
        {
            edgeWrite(ecode, eat);
            for (uint32_t q0 = 4u * NT; q0 < en; q0 += 4u * NT)
            {
                edgeIssue(q0, ecode, eat);
                edgeWrite(ecode, eat);
            }
        }
        if (d.fx < 0 || d.fx + d.nx > sdx)   // clamped halo voxels (border bricks only)
        {
            for (int32_t q = threadIdx.x; q < nRows; q += NT)
            {
                int32_t const r = rA + q;
                uint64_t const rb = rowBase(r);
                int32_t const rowL = r * d.nx - d.fx - vStart;   // LDS index of x = 0
                if (d.fx < 0)
                {
                    uint32_t const c = loadCode<BPV>(src, rb);
                    for (int32_t x = d.fx; x < min(0, d.fx + d.nx); ++x)
                        if (rowL + x >= 0 && rowL + x < chunkVox)
                            ldsStoreCode<BPV>(lds, rowL + x, c);
                }
                if (d.fx + d.nx > sdx)
                {
                    uint32_t const c = loadCode<BPV>(src, rb + static_cast<uint64_t>(sdx - 1));
                    for (int32_t x = max(sdx, d.fx); x < d.fx + d.nx; ++x)
                        if (rowL + x >= 0 && rowL + x < chunkVox)
                            ldsStoreCode<BPV>(lds, rowL + x, c);
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < static_cast<int>(kBrickChunk) / NT; ++u)
        {
            int32_t const t = u * NT + static_cast<int32_t>(threadIdx.x);
            int32_t const lv = t * V;
            uint8_t* const out = d.dst + static_cast<uint64_t>(vStart + lv) * BPV;
            // global address space named (the brick pointer comes from the descriptor table; a
            // flat store would also count against the LDS wait counter), nontemporal
            if (lv + V <= chunkVox)
                __builtin_nontemporal_store(tile[t], (__attribute__((address_space(1))) u32x4*)(out));
            else
            {
                for (int32_t k = 0; k < V && lv + k < chunkVox; ++k)
                    storeCode<BPV>(out, k, loadCode<BPV>(lds, lv + k));
            }
        }
    }

    // Direct copy of one chunk (knob decompose.direct): the brick grid has no clamped voxel and
    // every box row is whole 16-B words at 16-B aligned source offsets (halo-free bricks whose x
    // size is a multiple of 16 / BPV), so dst word i of a brick is ONE aligned 16-B source word:
    // a load and a store per item, no LDS tile, no barrier.  Items past the brick load its last
    // word again (every address stays valid) and do not store.
    // NT threads of the workgroup (tid = 0 .. NT - 1) copy items [base, base + kPer NT) of the brick.
    template <int BPV, int NT, int kPer = 4>
    __device__ __forceinline__ void brickDirect(BrickDesc const& d, uint32_t base, uint8_t const* src, int32_t sdx,
                                                int32_t sdy, uint32_t tid)
    {
        constexpr int32_t V = 16 / BPV;
        uint64_t const spY = static_cast<uint64_t>(sdx), spZ = spY * static_cast<uint64_t>(sdy);
        uint32_t const end = min(base + static_cast<uint32_t>(kPer * NT), d.nitems);
        u32x4 v[kPer];
#pragma unroll
        for (int u = 0; u < kPer; ++u)
        {
            uint32_t const i = min(base + static_cast<uint32_t>(u * NT) + tid, end - 1u);
            uint32_t const vox = i * V;
            uint32_t const r = fdiv(vox, d.fdx);
            uint32_t const x = vox - r * d.fdx.d;
            uint32_t const z = fdiv(r, d.fdy);
            uint32_t const y = r - z * d.fdy.d;
            uint64_t const off = (static_cast<uint64_t>(d.fz + static_cast<int32_t>(z)) * spZ +
                                  static_cast<uint64_t>(d.fy + static_cast<int32_t>(y)) * spY +
                                  static_cast<uint64_t>(d.fx + static_cast<int32_t>(x))) * BPV;
            // a plain (cached) load: the 128-B line of a row is shared by the x-neighbour bricks
            // when rows are shorter than a line
            v[u] = *reinterpret_cast<u32x4 const*>(src + off);
        }
#pragma unroll
        for (int u = 0; u < kPer; ++u)
        {
            uint32_t const i = base + static_cast<uint32_t>(u * NT) + tid;
            if (i < end)
                __builtin_nontemporal_store(v[u], (__attribute__((address_space(1))) u32x4*)(d.dst + 16ull * i));
        }
    }

    // A uniform brick grid (what BrickDecompose builds: brick (ix, iy, iz) at index ix + nbx * (iy
    // + nby * iz), box = the grid cell extended by the halo, every brick linear): descriptors are
    // derived from the brick index and three classes per axis (first, interior, last brick), so a
    // workgroup loads only its brick's data pointer -- needed no earlier than its stores -- instead
    // of waiting for a 96-B descriptor before its first source load.
    struct BrickGrid
    {
        uint8_t* const* dst;                   // data pointer of brick b
        FastDiv fnbx, fnby;                    // bricks per grid row / per grid plane (y)
        int32_t nbx, nby, nbz;
        int32_t fx0, fy0, fz0;                 // box start of brick (0, 0, 0) (= -halo)
        int32_t bx, by, bz;                    // brick size (grid step)
        int32_t nx[3], ny[3], nz[3];           // box extent per class: 0 first, 1 interior, 2 last
        FastDiv fdx[3], fwpr[3], fdy[3];       // divisors of nx, the source words per row, ny
    };

    __device__ __forceinline__ int gridClass(int32_t i, int32_t n)
    {
        return i == n - 1 ? 2 : (i == 0 ? 0 : 1);
    }

    template <class T>
    __device__ __forceinline__ T pick3(T const (&a)[3], int c)
    {
        return c == 0 ? a[0] : (c == 1 ? a[1] : a[2]);
    }

    // The descriptor of brick b of a uniform grid (class per axis: first, interior, last brick).
    template <int BPV>
    __device__ __forceinline__ BrickDesc gridDesc(BrickGrid const& grid, uint32_t b)
    {
        constexpr int32_t V = 16 / BPV;
        BrickDesc d;
        {
            uint32_t const yz = fdiv(b, grid.fnbx);
            int32_t const ix = static_cast<int32_t>(b - yz * grid.fnbx.d);
            uint32_t const izu = fdiv(yz, grid.fnby);
            int32_t const iy = static_cast<int32_t>(yz - izu * grid.fnby.d), iz = static_cast<int32_t>(izu);
            int const cx = gridClass(ix, grid.nbx), cy = gridClass(iy, grid.nby), cz = gridClass(iz, grid.nbz);
            d.dst = grid.dst[b];
            d.fx = grid.fx0 + ix * grid.bx;
            d.fy = grid.fy0 + iy * grid.by;
            d.fz = grid.fz0 + iz * grid.bz;
            d.nx = pick3(grid.nx, cx);
            int32_t const ny = pick3(grid.ny, cy), nz = pick3(grid.nz, cz);
            d.dimX = d.nx;
            d.dimY = ny;
            d.nvox = static_cast<uint32_t>(d.nx) * static_cast<uint32_t>(ny) * static_cast<uint32_t>(nz);
            d.nitems = (d.nvox + V - 1) / V;
            d.linear = 1;
            d.fdx = pick3(grid.fdx, cx);
            d.fwpr = pick3(grid.fwpr, cx);
            d.fdy = pick3(grid.fdy, cy);
        }
        return d;
    }

    // Row mode (a brick larger than its range): one 16-B segment of a box row per item.
    template <int BPV, int NT>
    __device__ __forceinline__ void brickRows(BrickDesc const& d, uint32_t base, uint8_t const* src, int32_t sdx,
                                              int32_t sdy, int32_t sdz)
    {
        constexpr int32_t V = 16 / BPV;
        uint64_t const pitchY = static_cast<uint64_t>(d.dimX);
        uint64_t const pitchZ = pitchY * static_cast<uint64_t>(d.dimY);
        uint64_t const spY = static_cast<uint64_t>(sdx), spZ = spY * static_cast<uint64_t>(sdy);
        constexpr int kPer = static_cast<int>(kBrickChunk) / NT;
        u32x4 vals[kPer];
        uint64_t srow[kPer], drow[kPer];
        int32_t sx0[kPer], cnt[kPer];
        bool fast[kPer];
#pragma unroll
        for (int u = 0; u < kPer; ++u)
        {
            uint32_t const i = base + u * NT + threadIdx.x;
            bool const live = i < d.nitems;
            uint32_t const ii = live ? i : 0;
            uint32_t const row = fdiv(ii, d.fseg);
            uint32_t const seg = ii - row * d.fseg.d;
            uint32_t const z = fdiv(row, d.fdy);
            uint32_t const y = row - z * d.fdy.d;
            int32_t const x0 = static_cast<int32_t>(seg) * V;
            cnt[u] = live ? min(V, d.nx - x0) : 0;
            int32_t const sy = clampi(d.fy + static_cast<int32_t>(y), sdy - 1);
            int32_t const sz = clampi(d.fz + static_cast<int32_t>(z), sdz - 1);
            sx0[u] = d.fx + x0;
            srow[u] = static_cast<uint64_t>(sz) * spZ + static_cast<uint64_t>(sy) * spY;
            drow[u] = static_cast<uint64_t>(z) * pitchZ + static_cast<uint64_t>(y) * pitchY +
                      static_cast<uint64_t>(x0);
            fast[u] = cnt[u] == V && sx0[u] >= 0 && sx0[u] + V <= sdx;
            if (fast[u])
                vals[u] = reinterpret_cast<Unaligned16 const*>(src + (srow[u] + sx0[u]) * BPV)->v;
        }
#pragma unroll
        for (int u = 0; u < kPer; ++u)
        {
            if (fast[u])
            {
                reinterpret_cast<Unaligned16*>(d.dst + drow[u] * BPV)->v = vals[u];
            }
            else
            {
                // row tail or clamped border segment: voxel by voxel
#pragma unroll
                for (int32_t v = 0; v < V; ++v)
                    if (v < cnt[u])
                        storeCode<BPV>(d.dst, drow[u] + v,
                                       loadCode<BPV>(src, srow[u] + clampi(sx0[u] + v, sdx - 1)));
            }
        }
    }

    template <int BPV, int kStageWords, bool GRID, int NT = kBlock, bool DIRECT = false, bool EDGE = false>
    __global__ __launch_bounds__(NT) void brickCopyKernel(BrickDesc const* bricks, BrickGrid grid,
                                                             FastDiv chunksPerBrick, FastDiv groupSize,
                                                             uint8_t const* src, int32_t sdx, int32_t sdy, int32_t sdz,
                                                             int32_t alignedLds)
    {
        // blockIdx = (group, chunk, brick in group): consecutive workgroups copy the same rows
        // of neighbouring bricks along x, i.e. adjacent pieces of the same source rows, so the
        // 128-B lines two bricks share (unaligned brick starts, halos) are fetched from HBM once
        // and hit the Infinity Cache the second time.
        uint32_t const lb = xcdSwizzle(blockIdx.x, gridDim.x);
        uint32_t const rest = fdiv(lb, groupSize);
        uint32_t const ig = lb - rest * groupSize.d;
        uint32_t const grp = fdiv(rest, chunksPerBrick);
        uint32_t const chunk = __builtin_amdgcn_readfirstlane(rest - grp * chunksPerBrick.d);
        uint32_t const b = __builtin_amdgcn_readfirstlane(grp * groupSize.d + ig);
        BrickDesc d;
        if constexpr (GRID)
            d = gridDesc<BPV>(grid, b);
        else
            d = bricks[b];
        uint32_t const base = chunk * kBrickChunk;
        if (base >= d.nitems)
            return;   // border bricks are smaller than the largest one
        if constexpr (DIRECT)
        {
            static_assert(kBrickChunk == 4 * NT, "brickDirect: 4 items per thread");
            brickDirect<BPV, NT>(d, base, src, sdx, sdy, threadIdx.x);
            return;
        }
        if (GRID || d.linear)
        {
            brickStaged<BPV, kStageWords, NT, EDGE>(d, base, src, sdx, sdy, sdz, alignedLds);
            return;
        }
        brickRows<BPV, NT>(d, base, src, sdx, sdy, sdz);
    }

    // Direct copy of P small bricks per workgroup (every brick one chunk of <= 4 NT / P items):
    // NT / P threads -- whole waves -- per brick, the P bricks consecutive along x (a 16^3 UInt16
    // brick is 512 items: one workgroup per brick left half of its loads clamped duplicates).
    template <int BPV, int P, int KPER = 4, int NT = kBlock>
    __global__ __launch_bounds__(NT) void brickDirectKernel(BrickGrid grid, uint32_t nBricks, uint8_t const* src,
                                                            int32_t sdx, int32_t sdy)
    {
        constexpr int kTpb = NT / P;
        static_assert(kTpb % 64 == 0, "whole waves per brick");
        uint32_t const lb = xcdSwizzle(blockIdx.x, gridDim.x);
        uint32_t const sub = threadIdx.x / kTpb;
        uint32_t const b = __builtin_amdgcn_readfirstlane(lb * P + sub);
        if (b >= nBricks)
            return;
        BrickDesc const d = gridDesc<BPV>(grid, b);
        brickDirect<BPV, kTpb, KPER>(d, 0u, src, sdx, sdy, threadIdx.x - sub * kTpb);
    }


    // ---- Row-image copy of a uniform grid (round 6, knob decompose.row_image) ------------------
    // No cut words anywhere.  Phase 1: the 16-B ALIGNED source words covering each box row's
    // in-volume span go, coalesced (consecutive threads = consecutive words of a row, then the
    // next row), to ALIGNED places of a per-row LDS image (row r at r * IMG, IMG an odd number of
    // 16-B words so phase 2's per-row reads spread over the banks); border bricks then write
    // their clamped voxels next to the span.  Phase 2: one thread per destination row reads the
    // row's bytes from the image (unaligned ds_read_b128 at the row's phase, the same for every
    // row of the brick: source rows are 16-B multiples) and stores them as 16-B pieces at
    // r * rowBytes in the brick -- the last piece taken at rowBytes - 16, overlapping its
    // neighbour with the same bytes, so a row end costs one store, not per-voxel masks.  One brick
    // (<= 16 KiB, rows >= 16 B) per workgroup; dynamic LDS = rows * IMG.
    template <int BPV, int NT>
    __global__ __launch_bounds__(NT) void brickRowImageKernel(BrickGrid grid, uint8_t const* src, int32_t sdx,
                                                              int32_t sdy, int32_t sdz)
    {
        constexpr uint32_t kHead = 16;   // room for the left clamped halo voxels
        constexpr int kBatch = 4;
        extern __shared__ u32x4 imgRaw[];
        uint8_t* const img = reinterpret_cast<uint8_t*>(imgRaw);
        uint32_t const b = __builtin_amdgcn_readfirstlane(xcdSwizzle(blockIdx.x, gridDim.x));
        BrickDesc const d = gridDesc<BPV>(grid, b);
        int32_t const nRows = static_cast<int32_t>(fdiv(d.nvox, d.fdx));
        int32_t const lo = max(d.fx, 0), hi = min(d.fx + d.nx, sdx);
        uint64_t const spY = static_cast<uint64_t>(sdx), spZ = spY * static_cast<uint64_t>(sdy);
        uint64_t const srcBytes = spZ * static_cast<uint64_t>(sdz) * BPV;
        auto rowBase = [&](int32_t r) -> uint64_t {
            uint32_t const z = fdiv(static_cast<uint32_t>(r), d.fdy);
            uint32_t const y = static_cast<uint32_t>(r) - z * d.fdy.d;
            return static_cast<uint64_t>(clampi(d.fz + static_cast<int32_t>(z), sdz - 1)) * spZ +
                   static_cast<uint64_t>(clampi(d.fy + static_cast<int32_t>(y), sdy - 1)) * spY;
        };
        uint32_t const ph = (static_cast<uint32_t>(lo) * BPV) & 15u;
        uint32_t const alignLo = static_cast<uint32_t>(lo) * BPV - ph;   // in-row byte of word 0
        uint32_t const spanB = ph + static_cast<uint32_t>(hi - lo) * BPV;
        uint32_t const wpr = (spanB + 15u) / 16u;
        uint32_t const tailB = static_cast<uint32_t>(d.fx + d.nx - hi) * BPV;
        uint32_t const imgW = ((kHead + spanB + tailB + 15u) / 16u) | 1u;
        uint32_t const IMG = imgW * 16u;
        FastDiv const fw = makeFastDiv(wpr);
        uint32_t const total = static_cast<uint32_t>(nRows) * wpr;
        for (uint32_t t0 = threadIdx.x; t0 < total; t0 += kBatch * NT)
        {
            u32x4 w[kBatch];
            uint32_t at[kBatch];
#pragma unroll
            for (int u = 0; u < kBatch; ++u)
            {
                uint32_t const t = t0 + static_cast<uint32_t>(u * NT);
                uint32_t const tt = t < total ? t : 0u;
                uint32_t const r = fdiv(tt, fw);
                uint32_t const k = tt - r * wpr;
                uint64_t const byte = rowBase(static_cast<int32_t>(r)) * BPV + alignLo + 16ull * k;
                at[u] = t < total ? r * IMG + kHead + 16u * k : ~0u;
                if (byte + 16 <= srcBytes)
                    w[u] = *reinterpret_cast<u32x4 const*>(src + byte);
                else
                {
                    // the volume's last word: only the bytes inside the buffer
                    uint32_t q[4] = {0u, 0u, 0u, 0u};
                    for (uint32_t i = 0; i < 16u && byte + i < srcBytes; ++i)
                        q[i / 4] |= static_cast<uint32_t>(src[byte + i]) << (8 * (i % 4));
                    w[u] = u32x4{q[0], q[1], q[2], q[3]};
                }
            }
#pragma unroll
            for (int u = 0; u < kBatch; ++u)
                if (at[u] != ~0u)
                    *reinterpret_cast<u32x4*>(img + at[u]) = w[u];
        }
        if (d.fx < 0 || d.fx + d.nx > sdx)   // border brick: clamped voxels beside the span
        {
            __syncthreads();
            for (int32_t r = threadIdx.x; r < nRows; r += NT)
            {
                uint64_t const rb = rowBase(r);
                uint8_t* const row = img + static_cast<uint32_t>(r) * IMG + kHead + ph;   // x = lo
                if (d.fx < 0)
                {
                    uint32_t const c = loadCode<BPV>(src, rb);
                    for (int32_t x = d.fx; x < min(0, d.fx + d.nx); ++x)
                        storeCode<BPV>(row + (x - lo) * BPV, 0, c);
                }
                if (d.fx + d.nx > sdx)
                {
                    uint32_t const c = loadCode<BPV>(src, rb + static_cast<uint64_t>(sdx - 1));
                    for (int32_t x = max(sdx, d.fx); x < d.fx + d.nx; ++x)
                        storeCode<BPV>(row + (x - lo) * BPV, 0, c);
                }
            }
        }
        __syncthreads();
        uint32_t const rowB = static_cast<uint32_t>(d.nx) * BPV;
        uint32_t const pieces = (rowB + 15u) / 16u;
        int32_t const first = static_cast<int32_t>(kHead + ph) + (d.fx - lo) * BPV;   // image byte of x = fx
        for (int32_t r = threadIdx.x; r < nRows; r += NT)
        {
            uint8_t const* const in = img + static_cast<uint32_t>(r) * IMG + first;
            uint8_t* const out = d.dst + static_cast<uint64_t>(r) * rowB;
            for (uint32_t p = 0; p < pieces; ++p)
            {
                uint32_t const off = 16u * p + 16u <= rowB ? 16u * p : rowB - 16u;
                u32x4 const v = reinterpret_cast<Unaligned16 const*>(in + off)->v;
                // (global address space named: a flat store would also count on lgkmcnt and make the
                // next row's LDS reads wait for it)
                __builtin_nontemporal_store(v, (__attribute__((address_space(1))) u32x4*)(out + off));
            }
        }
    }

    // ---- Persistent, software-pipelined staged copy of a uniform grid (knob decompose.pipe) ----
    // The staged kernel above runs one workgroup per 16-KiB chunk: a small brick (16^3 + halo 1 =
    // 11.7 KB) is one short-lived workgroup whose loads, LDS pass and stores run back to back, so
    // the chip holds few bytes in flight (measured 4.2 TB/s of HBM traffic for 16^3 + halo).
    // Here a grid of resident workgroups walks the chunks (item = blockIdx + k * gridDim, the same
    // (brick row, chunk, brick) order and XCD grouping), with two LDS tiles: the source words of
    // chunk k + 1 are loaded while chunk k is stored from the other tile.
    template <int BPV, int W, int NT>
    __global__ __launch_bounds__(NT) void brickPipeKernel(BrickGrid grid, FastDiv chunksPerBrick, FastDiv groupSize,
                                                          uint32_t items, uint8_t const* src, int32_t sdx, int32_t sdy,
                                                          int32_t sdz, int32_t alignedLds)
    {
        constexpr int32_t V = 16 / BPV;
        __shared__ u32x4 tile[2][kBrickChunk];   // 32 KiB
        uint64_t const spY = static_cast<uint64_t>(sdx), spZ = spY * static_cast<uint64_t>(sdy);
        uint64_t const srcBytes = spZ * static_cast<uint64_t>(sdz) * BPV;
        struct Geom
        {
            uint8_t* dst;
            int32_t fx, fy, fz, nx, vStart, chunkVox, rA, nRows, lo, hi;
            uint32_t wpr, total;
            FastDiv fdx, fwpr, fdy;
            bool live;
        };
        auto geom = [&](uint32_t item) -> Geom {
            Geom g{};
            uint32_t const lb = xcdSwizzle(item, items);
            uint32_t const rest = fdiv(lb, groupSize);
            uint32_t const ig = lb - rest * groupSize.d;
            uint32_t const grp = fdiv(rest, chunksPerBrick);
            uint32_t const chunk = __builtin_amdgcn_readfirstlane(rest - grp * chunksPerBrick.d);
            uint32_t const b = __builtin_amdgcn_readfirstlane(grp * groupSize.d + ig);
            uint32_t const yz = fdiv(b, grid.fnbx);
            int32_t const ix = static_cast<int32_t>(b - yz * grid.fnbx.d);
            uint32_t const izu = fdiv(yz, grid.fnby);
            int32_t const iy = static_cast<int32_t>(yz - izu * grid.fnby.d), iz = static_cast<int32_t>(izu);
            int const cx = gridClass(ix, grid.nbx), cy = gridClass(iy, grid.nby), cz = gridClass(iz, grid.nbz);
            g.fx = grid.fx0 + ix * grid.bx;
            g.fy = grid.fy0 + iy * grid.by;
            g.fz = grid.fz0 + iz * grid.bz;
            g.nx = pick3(grid.nx, cx);
            int32_t const nvox = g.nx * pick3(grid.ny, cy) * pick3(grid.nz, cz);
            g.fdx = pick3(grid.fdx, cx);
            g.fwpr = pick3(grid.fwpr, cx);
            g.fdy = pick3(grid.fdy, cy);
            uint32_t const base = chunk * kBrickChunk;
            g.live = base < static_cast<uint32_t>((nvox + V - 1) / V);
            if (!g.live)
                return g;
            g.dst = grid.dst[b];
            g.vStart = static_cast<int32_t>(base) * V;
            int32_t const vEnd = min(g.vStart + static_cast<int32_t>(kBrickChunk) * V, nvox);
            g.chunkVox = vEnd - g.vStart;
            g.rA = static_cast<int32_t>(fdiv(static_cast<uint32_t>(g.vStart), g.fdx));
            g.nRows = static_cast<int32_t>(fdiv(static_cast<uint32_t>(vEnd - 1), g.fdx)) - g.rA + 1;
            g.lo = max(g.fx, 0);
            g.hi = min(g.fx + g.nx, sdx);
            g.wpr = g.fwpr.d;
            g.total = static_cast<uint32_t>(g.nRows) * g.wpr;
            return g;
        };
        auto rowBase = [&](Geom const& g, int32_t r) -> uint64_t {
            uint32_t const z = fdiv(static_cast<uint32_t>(r), g.fdy);
            uint32_t const y = static_cast<uint32_t>(r) - z * g.fdy.d;
            return static_cast<uint64_t>(clampi(g.fz + static_cast<int32_t>(z), sdz - 1)) * spZ +
                   static_cast<uint64_t>(clampi(g.fy + static_cast<int32_t>(y), sdy - 1)) * spY;
        };
        struct Word
        {
            uint64_t rb;
            int32_t x0, li;
            bool live, whole;
            u32x4 v;
        };
        auto locate = [&](Geom const& g, uint32_t t, Word& w) {
            w.live = t < g.total;
            uint32_t const tt = w.live ? t : 0u;
            uint32_t const q = fdiv(tt, g.fwpr);
            int32_t const r = g.rA + static_cast<int32_t>(q);
            w.rb = rowBase(g, r);
            uint64_t const startByte =
                (((w.rb + static_cast<uint64_t>(g.lo)) * BPV) & ~uint64_t(15)) + 16ull * (tt - q * g.wpr);
            w.live = w.live && startByte < (w.rb + static_cast<uint64_t>(g.hi)) * BPV;
            w.x0 = static_cast<int32_t>(startByte / BPV - w.rb);
            w.li = r * g.nx + (w.x0 - g.fx) - g.vStart;
            w.whole = startByte + 16 <= srcBytes;
            w.v = u32x4{0u, 0u, 0u, 0u};
            if (w.live && w.whole)
                w.v = *reinterpret_cast<u32x4 const*>(src + startByte);
        };
        auto place = [&](Geom const& g, uint8_t* lds, Word const& w) {
            if (!w.live)
                return;
            if (w.whole && w.x0 >= g.lo && w.x0 + V <= g.hi && w.li >= 0 && w.li + V <= g.chunkVox)
            {
                if (alignedLds == 2)
                    ldsStoreRange(lds, w.li * BPV, w.v, 0, 16);
                else
                    reinterpret_cast<Unaligned16*>(lds + w.li * BPV)->v = w.v;
            }
            else if (w.whole && (alignedLds == 1 || alignedLds == 2))
            {
                int32_t const k0 = max(max(g.lo - w.x0, -w.li), 0);
                int32_t const k1 = min(min(g.hi - w.x0, g.chunkVox - w.li), V);
                if (k1 > k0)
                    ldsStoreRange(lds, (w.li + k0) * BPV, w.v, k0 * BPV, k1 * BPV);
            }
            else
            {
#pragma unroll
                for (int k = 0; k < V; ++k)
                    if (w.x0 + k >= g.lo && w.x0 + k < g.hi && w.li + k >= 0 && w.li + k < g.chunkVox)
                        ldsStoreCode<BPV>(lds, w.li + k,
                                          w.whole ? wordCode<BPV>(w.v, k) : loadCode<BPV>(src, w.rb + w.x0 + k));
            }
        };
        // the words beyond the first W rounds, then the clamped x halo voxels (border bricks)
        auto stageRest = [&](Geom const& g, uint8_t* lds) {
            for (uint32_t t = threadIdx.x + W * NT; t < g.total; t += NT)
            {
                Word w;
                locate(g, t, w);
                place(g, lds, w);
            }
            if (g.fx < 0 || g.fx + g.nx > sdx)
            {
                for (int32_t q = threadIdx.x; q < g.nRows; q += NT)
                {
                    int32_t const r = g.rA + q;
                    uint64_t const rb = rowBase(g, r);
                    int32_t const rowL = r * g.nx - g.fx - g.vStart;
                    if (g.fx < 0)
                    {
                        uint32_t const c = loadCode<BPV>(src, rb);
                        for (int32_t x = g.fx; x < min(0, g.fx + g.nx); ++x)
                            if (rowL + x >= 0 && rowL + x < g.chunkVox)
                                ldsStoreCode<BPV>(lds, rowL + x, c);
                    }
                    if (g.fx + g.nx > sdx)
                    {
                        uint32_t const c = loadCode<BPV>(src, rb + static_cast<uint64_t>(sdx - 1));
                        for (int32_t x = max(sdx, g.fx); x < g.fx + g.nx; ++x)
                            if (rowL + x >= 0 && rowL + x < g.chunkVox)
                                ldsStoreCode<BPV>(lds, rowL + x, c);
                    }
                }
            }
        };
        auto storeOut = [&](Geom const& g, u32x4 const* t, uint8_t const* lds) {
#pragma unroll
            for (int u = 0; u < static_cast<int>(kBrickChunk) / NT; ++u)
            {
                int32_t const it = u * NT + static_cast<int32_t>(threadIdx.x);
                int32_t const lv = it * V;
                uint8_t* const out = g.dst + static_cast<uint64_t>(g.vStart + lv) * BPV;
                if (lv + V <= g.chunkVox)
                    __builtin_nontemporal_store(t[it], (__attribute__((address_space(1))) u32x4*)(out));
                else
                {
                    for (int32_t k = 0; k < V && lv + k < g.chunkVox; ++k)
                        storeCode<BPV>(out, k, loadCode<BPV>(lds, lv + k));
                }
            }
        };
        uint32_t item = blockIdx.x;
        if (item >= items)
            return;   // (whole workgroup)
        Geom cur = geom(item);
        Word words[W];
        int p = 0;
        if (cur.live)
        {
#pragma unroll
            for (int k = 0; k < W; ++k)
                locate(cur, threadIdx.x + k * NT, words[k]);
#pragma unroll
            for (int k = 0; k < W; ++k)
                place(cur, reinterpret_cast<uint8_t*>(tile[0]), words[k]);
            stageRest(cur, reinterpret_cast<uint8_t*>(tile[0]));
        }
        __syncthreads();
        while (true)   // item and every branch below are workgroup-uniform
        {
            uint32_t const nitem = item + gridDim.x;
            bool const more = nitem < items;
            Geom nxt{};
            if (more)
            {
                nxt = geom(nitem);
                if (nxt.live)
                {
#pragma unroll
                    for (int k = 0; k < W; ++k)
                        locate(nxt, threadIdx.x + k * NT, words[k]);
                }
            }
            if (cur.live)
                storeOut(cur, tile[p], reinterpret_cast<uint8_t const*>(tile[p]));
            if (!more)
                break;
            if (nxt.live)
            {
                uint8_t* const lds = reinterpret_cast<uint8_t*>(tile[p ^ 1]);
#pragma unroll
                for (int k = 0; k < W; ++k)
                    place(nxt, lds, words[k]);
                stageRest(nxt, lds);
            }
            __syncthreads();   // tile[p ^ 1] complete, and every wave is done reading tile[p]
            cur = nxt;
            p ^= 1;
            item = nitem;
        }
    }

    // ---- Two small bricks per workgroup (knob decompose.pair) --------------------------------
    // Bricks of one 16-KiB chunk or less (16^3 + halo 1 UInt16: 11.7 KB) made one short-lived
    // workgroup each: 262 144 workgroups whose load, LDS and store phases run back to back, and
    // whose rows (36 B, 4 source words of which 2 partial) re-read the neighbour's halo words.
    // Here a workgroup takes two x-neighbours of a brick row: it stages the UNION of their rows
    // (34 voxels: 5-6 words, the shared columns read once) into two LDS tiles -- a word lands in
    // each brick whose box it touches -- and stores both bricks: half the workgroups, ~30 % fewer
    // source words, twice the bytes per workgroup in flight.  An odd last brick of a row pairs
    // with nothing.  Pair types (pick by the pair index): 0 first, 1 interior, 2 last, 3 first and
    // last (one pair per row) -- the words per row of the union differ only by clamping.
    struct PairGeom
    {
        FastDiv fwpr[4];
        FastDiv fPairs;     // pairs per brick row
    };

    template <int BPV, int W, int NT>
    __global__ __launch_bounds__(NT) void brickPairKernel(BrickGrid grid, PairGeom pg, uint8_t const* src, int32_t sdx,
                                                          int32_t sdy, int32_t sdz, int32_t alignedLds)
    {
        constexpr int32_t V = 16 / BPV;
        __shared__ u32x4 tile[2][kBrickChunk];   // 32 KiB
        uint64_t const spY = static_cast<uint64_t>(sdx), spZ = spY * static_cast<uint64_t>(sdy);
        uint64_t const srcBytes = spZ * static_cast<uint64_t>(sdz) * BPV;
        uint32_t const lb = xcdSwizzle(blockIdx.x, gridDim.x);
        uint32_t const yz = __builtin_amdgcn_readfirstlane(fdiv(lb, pg.fPairs));
        uint32_t const px = __builtin_amdgcn_readfirstlane(lb - yz * pg.fPairs.d);
        uint32_t const izu = fdiv(yz, grid.fnby);
        int32_t const iy = static_cast<int32_t>(yz - izu * grid.fnby.d), iz = static_cast<int32_t>(izu);
        int32_t const ix0 = 2 * static_cast<int32_t>(px);
        bool const two = ix0 + 1 < grid.nbx;
        int const cy = gridClass(iy, grid.nby), cz = gridClass(iz, grid.nbz);
        int32_t const fy = grid.fy0 + iy * grid.by, fz = grid.fz0 + iz * grid.bz;
        int32_t const ny = pick3(grid.ny, cy), nz = pick3(grid.nz, cz);
        FastDiv const fdy = pick3(grid.fdy, cy);
        // the two bricks' geometry in scalars (arrays indexed by the brick number went to scratch)
        struct Brick
        {
            int32_t fx, nx, nvox, lo, hi;
            uint8_t* dst;
        };
        auto brick = [&](int32_t ix) -> Brick {
            Brick b;
            int const cx = gridClass(ix, grid.nbx);
            b.fx = grid.fx0 + ix * grid.bx;
            b.nx = pick3(grid.nx, cx);
            b.nvox = b.nx * ny * nz;
            b.lo = max(b.fx, 0);
            b.hi = min(b.fx + b.nx, sdx);
            b.dst = grid.dst[(static_cast<uint32_t>(iz) * grid.nby + static_cast<uint32_t>(iy)) * grid.nbx + ix];
            return b;
        };
        Brick const B0 = brick(ix0), B1 = brick(two ? ix0 + 1 : ix0);
        auto pickB = [&](int k) -> Brick const& { return k == 0 ? B0 : B1; };
        int const nb = two ? 2 : 1;
        int const type = px == 0 ? (px + 1 == pg.fPairs.d ? 3 : 0) : (px + 1 == pg.fPairs.d ? 2 : 1);
        // field-wise selects: a select of whole FastDivs became a dynamic index into a scratch copy
        auto sel4 = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
            return type == 0 ? a : type == 1 ? b : type == 2 ? c : d;
        };
        FastDiv const fwpr{sel4(pg.fwpr[0].d, pg.fwpr[1].d, pg.fwpr[2].d, pg.fwpr[3].d),
                           sel4(pg.fwpr[0].m, pg.fwpr[1].m, pg.fwpr[2].m, pg.fwpr[3].m),
                           sel4(pg.fwpr[0].l, pg.fwpr[1].l, pg.fwpr[2].l, pg.fwpr[3].l)};
        uint32_t const wpr = fwpr.d;
        int32_t const ulo = B0.lo, uhi = two ? B1.hi : B0.hi;   // the union's in-volume x span
        int32_t const nRows = ny * nz;
        uint32_t const total = static_cast<uint32_t>(nRows) * wpr;
        auto rowBase = [&](int32_t r) -> uint64_t {
            uint32_t const z = fdiv(static_cast<uint32_t>(r), fdy);
            uint32_t const y = static_cast<uint32_t>(r) - z * fdy.d;
            return static_cast<uint64_t>(clampi(fz + static_cast<int32_t>(z), sdz - 1)) * spZ +
                   static_cast<uint64_t>(clampi(fy + static_cast<int32_t>(y), sdy - 1)) * spY;
        };
        struct Word
        {
            uint64_t rb;
            int32_t x0, r;
            bool live, whole;
            u32x4 v;
        };
        auto locate = [&](uint32_t t, Word& w) {
            w.live = t < total;
            uint32_t const tt = w.live ? t : 0u;
            uint32_t const q = fdiv(tt, fwpr);
            w.r = static_cast<int32_t>(q);
            w.rb = rowBase(w.r);
            uint64_t const startByte =
                (((w.rb + static_cast<uint64_t>(ulo)) * BPV) & ~uint64_t(15)) + 16ull * (tt - q * wpr);
            w.live = w.live && startByte < (w.rb + static_cast<uint64_t>(uhi)) * BPV;
            w.x0 = static_cast<int32_t>(startByte / BPV - w.rb);
            w.whole = startByte + 16 <= srcBytes;
            w.v = u32x4{0u, 0u, 0u, 0u};
            if (w.live && w.whole)
                w.v = *reinterpret_cast<u32x4 const*>(src + startByte);
        };
        auto place = [&](Word const& w) {
            if (!w.live)
                return;
#pragma unroll
            for (int k = 0; k < 2; ++k)
            {
                Brick const& b = pickB(k);
                if (k >= nb || w.x0 + V <= b.lo || w.x0 >= b.hi)
                    continue;   // the word holds no voxel of brick k's in-volume span
                uint8_t* const lds = reinterpret_cast<uint8_t*>(tile[k]);
                int32_t const li = w.r * b.nx + (w.x0 - b.fx);   // brick-local voxel of the word's first
                if (w.whole && w.x0 >= b.lo && w.x0 + V <= b.hi)
                {
                    if (alignedLds == 2)
                        ldsStoreRange(lds, li * BPV, w.v, 0, 16);
                    else
                        reinterpret_cast<Unaligned16*>(lds + li * BPV)->v = w.v;
                }
                else if (w.whole && (alignedLds == 1 || alignedLds == 2))
                {
                    int32_t const k0 = max(b.lo - w.x0, 0), k1 = min(b.hi - w.x0, V);
                    ldsStoreRange(lds, (li + k0) * BPV, w.v, k0 * BPV, k1 * BPV);
                }
                else
                {
#pragma unroll
                    for (int j = 0; j < V; ++j)
                        if (w.x0 + j >= b.lo && w.x0 + j < b.hi)
                            ldsStoreCode<BPV>(lds, li + j,
                                              w.whole ? wordCode<BPV>(w.v, j) : loadCode<BPV>(src, w.rb + w.x0 + j));
                }
            }
        };
        {
            Word words[W];
#pragma unroll
            for (int k = 0; k < W; ++k)
                locate(threadIdx.x + k * NT, words[k]);
#pragma unroll
            for (int k = 0; k < W; ++k)
                place(words[k]);
        }
        for (uint32_t t = threadIdx.x + W * NT; t < total; t += NT)
        {
            Word w;
            locate(t, w);
            place(w);
        }
        // clamped x halo voxels (the border bricks of a row)
#pragma unroll
        for (int k = 0; k < 2; ++k)
        {
            Brick const& b = pickB(k);
            if (k >= nb || (b.fx >= 0 && b.fx + b.nx <= sdx))
                continue;
            uint8_t* const lds = reinterpret_cast<uint8_t*>(tile[k]);
            for (int32_t r = threadIdx.x; r < nRows; r += NT)
            {
                uint64_t const rb = rowBase(r);
                int32_t const rowL = r * b.nx - b.fx;   // LDS voxel of x = 0
                if (b.fx < 0)
                {
                    uint32_t const c = loadCode<BPV>(src, rb);
                    for (int32_t x = b.fx; x < min(0, b.fx + b.nx); ++x)
                        ldsStoreCode<BPV>(lds, rowL + x, c);
                }
                if (b.fx + b.nx > sdx)
                {
                    uint32_t const c = loadCode<BPV>(src, rb + static_cast<uint64_t>(sdx - 1));
                    for (int32_t x = max(sdx, b.fx); x < b.fx + b.nx; ++x)
                        ldsStoreCode<BPV>(lds, rowL + x, c);
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 2; ++k)
        {
            Brick const& b = pickB(k);
            if (k >= nb)
                continue;
            uint8_t const* const lds = reinterpret_cast<uint8_t const*>(tile[k]);
#pragma unroll
            for (int u = 0; u < static_cast<int>(kBrickChunk) / NT; ++u)
            {
                int32_t const it = u * NT + static_cast<int32_t>(threadIdx.x);
                int32_t const lv = it * V;
                if (lv >= b.nvox)
                    continue;
                uint8_t* const out = b.dst + static_cast<uint64_t>(lv) * BPV;
                if (lv + V <= b.nvox)
                    __builtin_nontemporal_store(tile[k][it], (__attribute__((address_space(1))) u32x4*)(out));
                else
                {
                    for (int32_t j = 0; j < V && lv + j < b.nvox; ++j)
                        storeCode<BPV>(out, j, loadCode<BPV>(lds, lv + j));
                }
            }
        }
    }

    // The pair kernel's per-type words per row (PairGeom), or false when the grid does not take
    // it: bricks of more than one chunk, a single brick per row.
    bool pairGeom(BrickGrid const& g, uint32_t bpv, uint32_t maxItems, int32_t sdx, PairGeom& pg, uint32_t& pairs)
    {
        if (maxItems > kBrickChunk || g.nbx < 2)
            return false;
        uint32_t const pp = static_cast<uint32_t>((g.nbx + 1) / 2);
        pg.fPairs = makeFastDiv(pp);
        auto cls = [&](int32_t ix) { return ix == g.nbx - 1 ? 2 : (ix == 0 ? 0 : 1); };
        auto words = [&](int32_t ix0) -> uint32_t {
            int32_t const ix1 = ix0 + 1 < g.nbx ? ix0 + 1 : ix0;
            int32_t const f0 = g.fx0 + ix0 * g.bx, f1 = g.fx0 + ix1 * g.bx;
            int64_t const span = std::min<int64_t>(f1 + g.nx[cls(ix1)], sdx) - std::max(f0, 0);
            return span > 0 ? static_cast<uint32_t>((span * bpv + 15) / 16 + 1) : 1u;
        };
        pg.fwpr[0] = makeFastDiv(words(0));
        pg.fwpr[1] = makeFastDiv(pp > 2 ? words(2) : words(0));
        pg.fwpr[2] = makeFastDiv(words(2 * static_cast<int32_t>(pp - 1)));
        pg.fwpr[3] = makeFastDiv(words(0));
        pairs = pp * static_cast<uint32_t>(g.nby) * static_cast<uint32_t>(g.nbz);
        return true;
    }

    // ---- Gather form of the uniform-grid copy (knob decompose.gather) ------------------------
    // Phase 1 stages the source rows a chunk touches in LDS as ALIGNED 16-B words -- row q of the
    // chunk at q * P bytes, P = the class's source words per row * 16 -- with aligned LDS writes
    // only; phase 2 assembles each 16-B output item with one unaligned ds_read_b128 from its row,
    // or two merged by a byte mask for an item that crosses a brick row end; only items with
    // clamped (x halo) voxels and a brick's last partial item go voxel by voxel.  The staged form
    // above scatters source words into the brick layout, the words cut by a row end voxel by
    // voxel: for 16^3 bricks + halo 1 (36-B rows: 2 of 4 words partial) that took ~550 VALU + ~560
    // SALU instructions per wave (profiles/r04/dec16.pmc.jsonl).  LDS: dynamic, (rows a chunk
    // touches) x P, sized on the host per launch.
    __device__ __forceinline__ u32x4 ldsRead16(uint8_t const* lds, uint32_t a)
    {
        return reinterpret_cast<Unaligned16 const*>(lds + a)->v;
    }

    // bytes [0, cb) from a, the rest from b (0 < cb < 16)
    __device__ __forceinline__ u32x4 mergeBytes(u32x4 a, u32x4 b, int32_t cb)
    {
        auto m = [&](int i) -> uint32_t {
            int32_t const n = min(max(cb - 4 * i, 0), 4);
            return n >= 4 ? ~0u : (1u << (8 * n)) - 1u;
        };
        uint32_t const m0 = m(0), m1 = m(1), m2 = m(2), m3 = m(3);
        return u32x4{(a.x & m0) | (b.x & ~m0), (a.y & m1) | (b.y & ~m1), (a.z & m2) | (b.z & ~m2),
                     (a.w & m3) | (b.w & ~m3)};
    }

    template <int BPV, int kStageWords, int NT>
    __global__ __launch_bounds__(NT) void brickGatherKernel(BrickGrid grid, FastDiv chunksPerBrick, FastDiv groupSize,
                                                            uint8_t const* src, int32_t sdx, int32_t sdy, int32_t sdz)
    {
        constexpr int32_t V = 16 / BPV;
        extern __shared__ u32x4 stage[];
        uint8_t* const lds = reinterpret_cast<uint8_t*>(stage);
        uint32_t const lb = xcdSwizzle(blockIdx.x, gridDim.x);
        uint32_t const rest = fdiv(lb, groupSize);
        uint32_t const ig = lb - rest * groupSize.d;
        uint32_t const grp = fdiv(rest, chunksPerBrick);
        uint32_t const chunk = __builtin_amdgcn_readfirstlane(rest - grp * chunksPerBrick.d);
        uint32_t const b = __builtin_amdgcn_readfirstlane(grp * groupSize.d + ig);
        uint32_t const yz = fdiv(b, grid.fnbx);
        int32_t const ix = static_cast<int32_t>(b - yz * grid.fnbx.d);
        uint32_t const izu = fdiv(yz, grid.fnby);
        int32_t const iy = static_cast<int32_t>(yz - izu * grid.fnby.d), iz = static_cast<int32_t>(izu);
        int const cx = gridClass(ix, grid.nbx), cy = gridClass(iy, grid.nby), cz = gridClass(iz, grid.nbz);
        int32_t const fx = grid.fx0 + ix * grid.bx, fy = grid.fy0 + iy * grid.by, fz = grid.fz0 + iz * grid.bz;
        int32_t const nx = pick3(grid.nx, cx), ny = pick3(grid.ny, cy), nz = pick3(grid.nz, cz);
        FastDiv const fdx = pick3(grid.fdx, cx), fwpr = pick3(grid.fwpr, cx), fdy = pick3(grid.fdy, cy);
        int32_t const nvox = nx * ny * nz;
        uint32_t const base = chunk * kBrickChunk;
        if (base >= static_cast<uint32_t>((nvox + V - 1) / V))
            return;   // border bricks are smaller than the largest one
        uint8_t* const dst = grid.dst[b];
        uint64_t const spY = static_cast<uint64_t>(sdx), spZ = spY * static_cast<uint64_t>(sdy);
        uint64_t const srcBytes = spZ * static_cast<uint64_t>(sdz) * BPV;
        int32_t const vStart = static_cast<int32_t>(base) * V;
        int32_t const vEnd = min(vStart + static_cast<int32_t>(kBrickChunk) * V, nvox);
        int32_t const chunkVox = vEnd - vStart;
        int32_t const rA = static_cast<int32_t>(fdiv(static_cast<uint32_t>(vStart), fdx));
        int32_t const rB = static_cast<int32_t>(fdiv(static_cast<uint32_t>(vEnd - 1), fdx));
        int32_t const nRows = rB - rA + 1;
        int32_t const lo = max(fx, 0), hi = min(fx + nx, sdx);   // in-volume x span of a row
        uint32_t const wpr = fwpr.d, P = wpr * 16u;
        auto rowBase = [&](int32_t r) -> uint64_t {   // source voxel index of x = 0 of brick row r
            uint32_t const z = fdiv(static_cast<uint32_t>(r), fdy);
            uint32_t const y = static_cast<uint32_t>(r) - z * fdy.d;
            return static_cast<uint64_t>(clampi(fz + static_cast<int32_t>(z), sdz - 1)) * spZ +
                   static_cast<uint64_t>(clampi(fy + static_cast<int32_t>(y), sdy - 1)) * spY;
        };
        // phase 1: word k of staged row q = the aligned source word k of the row's x span
        uint32_t const total = static_cast<uint32_t>(nRows) * wpr;
        // source byte offset of staged word t; ~0: nothing to load (past the row's span, where a
        // class's longest row has more words); the volume's last word, cut by the end of the
        // source allocation, is loaded byte by byte after the batch (cutWord)
        auto wordStart = [&](uint32_t t) -> uint64_t {
            uint32_t const q = fdiv(t, fwpr);
            uint32_t const k = t - q * wpr;
            uint64_t const rb = rowBase(rA + static_cast<int32_t>(q));
            uint64_t const start = (((rb + static_cast<uint64_t>(lo)) * BPV) & ~uint64_t(15)) + 16ull * k;
            return start < (rb + static_cast<uint64_t>(hi)) * BPV ? start : ~0ull;
        };
        auto cutWord = [&](uint32_t t, uint64_t start) {
            uint32_t w[4] = {0u, 0u, 0u, 0u};
            for (uint64_t i = start; i < srcBytes; ++i)
                w[(i - start) / 4] |= static_cast<uint32_t>(src[i]) << (8 * ((i - start) % 4));
            stage[t] = u32x4{w[0], w[1], w[2], w[3]};
        };
        for (uint32_t t0 = 0; t0 < total; t0 += kStageWords * NT)
        {
            u32x4 w[kStageWords];
            uint64_t at[kStageWords];
#pragma unroll
            for (int k = 0; k < kStageWords; ++k)
            {
                uint32_t const t = t0 + threadIdx.x + static_cast<uint32_t>(k * NT);
                at[k] = t < total ? wordStart(t) : ~0ull;
                w[k] = u32x4{0u, 0u, 0u, 0u};
                if (at[k] != ~0ull && at[k] + 16 <= srcBytes)
                    w[k] = *reinterpret_cast<u32x4 const*>(src + at[k]);
            }
#pragma unroll
            for (int k = 0; k < kStageWords; ++k)
            {
                uint32_t const t = t0 + threadIdx.x + static_cast<uint32_t>(k * NT);
                if (t < total)
                {
                    if (at[k] != ~0ull && at[k] + 16 > srcBytes)
                        cutWord(t, at[k]);
                    else
                        stage[t] = w[k];
                }
            }
        }
        __syncthreads();
        // LDS byte of source x (in [lo, hi)) in staged row q whose x = 0 is source voxel rb
        auto ldsAt = [&](int32_t q, uint64_t rb, int32_t sx) -> uint32_t {
            uint32_t const m = static_cast<uint32_t>(((rb + static_cast<uint64_t>(lo)) * BPV) & 15u);
            return static_cast<uint32_t>(q) * P + m + static_cast<uint32_t>((sx - lo) * BPV);
        };
#pragma unroll 1
        for (int u = 0; u < static_cast<int>(kBrickChunk) / NT; ++u)
        {
            int32_t const lv = (u * NT + static_cast<int32_t>(threadIdx.x)) * V;
            if (lv >= chunkVox)
                continue;
            int32_t const v = vStart + lv;
            int32_t const r = static_cast<int32_t>(fdiv(static_cast<uint32_t>(v), fdx));
            int32_t const x = v - r * nx;
            int32_t const q = r - rA;
            int32_t const c = nx - x;                 // voxels of the item left in row r
            uint64_t const rb = rowBase(r);
            uint8_t* const out = dst + static_cast<uint64_t>(v) * BPV;
            bool const whole = lv + V <= chunkVox;
            if (whole && c >= V && fx + x >= lo && fx + x + V <= hi)
            {
                __builtin_nontemporal_store(ldsRead16(lds, ldsAt(q, rb, fx + x)),
                                            (__attribute__((address_space(1))) u32x4*)(out));
                continue;
            }
            if (whole && c < V && fx + x >= lo && fx + nx <= hi && fx >= lo && fx + (V - c) <= hi)
            {
                // row r's tail, then row r + 1 from its x = 0 (read from V - c voxels before it)
                uint64_t const rb2 = rowBase(r + 1);
                u32x4 const a = ldsRead16(lds, ldsAt(q, rb, fx + x));
                u32x4 const bb = ldsRead16(lds, ldsAt(q + 1, rb2, fx) - static_cast<uint32_t>(c * BPV));
                __builtin_nontemporal_store(mergeBytes(a, bb, c * BPV), (__attribute__((address_space(1))) u32x4*)(out));
                continue;
            }
            // clamped x halo voxels, or the brick's last partial item: voxel by voxel
            int32_t const n = min(V, chunkVox - lv);
            int32_t rr = r, xx = x, qq = q;
            uint64_t rbb = rb;
            for (int32_t k = 0; k < n; ++k)
            {
                int32_t const sx = min(max(fx + xx, 0), sdx - 1);
                uint32_t const a = ldsAt(qq, rbb, sx);
                uint32_t code;
                if constexpr (BPV == 1)
                    code = lds[a];
                else if constexpr (BPV == 2)
                    code = static_cast<uint32_t>(lds[a]) | static_cast<uint32_t>(lds[a + 1]) << 8;
                else
                    code = static_cast<uint32_t>(lds[a]) | static_cast<uint32_t>(lds[a + 1]) << 8 |
                           static_cast<uint32_t>(lds[a + 2]) << 16 | static_cast<uint32_t>(lds[a + 3]) << 24;
                storeCode<BPV>(out, static_cast<uint64_t>(k), code);
                if (++xx == nx && k + 1 < n)
                {
                    xx = 0;
                    ++rr;
                    ++qq;
                    rbb = rowBase(rr);
                }
            }
        }
    }

    // Dynamic LDS bytes of brickGatherKernel for a grid (0: more than kGatherLdsMax -- the staged
    // kernel then runs): per class, the rows a 16-KiB chunk can touch x the words per row.
    constexpr uint32_t kGatherLdsMax = 64u * 1024u;

    uint32_t gatherLdsBytes(BrickGrid const& g, uint32_t bpv)
    {
        uint32_t const V = 16u / bpv;
        uint64_t need = 0;
        for (int cx = 0; cx < 3; ++cx)
            for (int cy = 0; cy < 3; ++cy)
                for (int cz = 0; cz < 3; ++cz)
                {
                    uint64_t const nvox = static_cast<uint64_t>(g.nx[cx]) * g.ny[cy] * g.nz[cz];
                    uint64_t const chunkVox = std::min<uint64_t>(static_cast<uint64_t>(kBrickChunk) * V, nvox);
                    uint64_t const rows = (chunkVox + g.nx[cx] - 1) / g.nx[cx] + 1;
                    need = std::max<uint64_t>(need, rows * g.fwpr[cx].d * 16ull);
                }
        return need <= kGatherLdsMax ? static_cast<uint32_t>(need) : 0u;
    }

    // Descriptor table: pinned host staging + a grow-only device buffer, uploaded with a
    // stream-ordered H2D copy on the compute stream.  Both are reused only after the previous
    // decomposition's kernel finished (event recorded behind it), so a caller that switches
    // the compute stream between calls cannot race the table.
    // A ring of kDescSlots tables: call n waits only for call n - kDescSlots, so the host
    // planning of the next decomposition (tens of thousands of descriptors for 32^3 bricks of
    // a 1024^3 volume) overlaps the kernel of the previous one instead of idling the GPU.
    struct DescTable
    {
        BrickDesc* host = nullptr;
        BrickDesc* dev = nullptr;
        uint8_t** hostPtr = nullptr;   // brick data pointers (uniform grids, BrickGrid::dst)
        uint8_t** devPtr = nullptr;
        size_t capDesc = 0, capPtr = 0;
        hipEvent_t done = nullptr;
        hipEvent_t copied = nullptr;   // the table's upload (copy stream) finished
        bool pending = false;
    };
    constexpr int kDescSlots = 3;

    struct DescRing
    {
        std::mutex m;
        DescTable slot[kDescSlots];
        int next = 0;
    };

    DescRing& descRing()
    {
        static DescRing r;
        return r;
    }

    // Uniform brick grid inferred from the range list (BrickGrid): nbx = the leading run of ranges
    // on one y/z box, nby = the rows of the first plane; the grid step from the neighbours of
    // range 0; the box extents of each axis class from one range each.  False when the list does
    // not factor into nbx * nby * nbz.  Each range is then checked against the pattern inside the
    // descriptor loop (gridMatches) -- one pass over the bricks, no second walk.
    struct GridGuess
    {
        BrickGrid g{};
        size_t pz = 0;
        bool ok = false;
    };

    GridGuess inferGrid(vktHipBrickRange_t const* r, size_t n)
    {
        GridGuess q;
        if (n == 0 || n >= (1ull << 31))
            return q;
        auto sameYZ = [&](size_t i) { return r[i].first.y == r[0].first.y && r[i].first.z == r[0].first.z; };
        size_t nbx = 1;
        while (nbx < n && sameYZ(nbx))
            ++nbx;
        size_t nby = 1;
        while ((nby + 1) * nbx <= n && r[nby * nbx].first.z == r[0].first.z && r[nby * nbx].first.y != r[(nby - 1) * nbx].first.y)
            ++nby;
        if (n % (nbx * nby) != 0)
            return q;
        size_t const nbz = n / (nbx * nby), pz = nbx * nby;
        BrickGrid& g = q.g;
        g.nbx = static_cast<int32_t>(nbx);
        g.nby = static_cast<int32_t>(nby);
        g.nbz = static_cast<int32_t>(nbz);
        g.fnbx = makeFastDiv(static_cast<uint32_t>(nbx));
        g.fnby = makeFastDiv(static_cast<uint32_t>(nby));
        g.fx0 = r[0].first.x;
        g.fy0 = r[0].first.y;
        g.fz0 = r[0].first.z;
        g.bx = nbx > 1 ? r[1].first.x - r[0].first.x : 0;
        g.by = nby > 1 ? r[nbx].first.y - r[0].first.y : 0;
        g.bz = nbz > 1 ? r[pz].first.z - r[0].first.z : 0;
        auto rep = [](int c, size_t nb) -> size_t { return c == 0 ? 0 : (c == 1 ? (nb > 2 ? 1 : 0) : nb - 1); };
        for (int c = 0; c < 3; ++c)
        {
            g.nx[c] = r[rep(c, nbx)].last.x - r[rep(c, nbx)].first.x;
            g.ny[c] = r[rep(c, nby) * nbx].last.y - r[rep(c, nby) * nbx].first.y;
            g.nz[c] = r[rep(c, nbz) * pz].last.z - r[rep(c, nbz) * pz].first.z;
        }
        q.pz = pz;
        q.ok = true;
        return q;
    }

    // range i (its descriptor d) at its place in the inferred grid, a linear brick.  Interior
    // bricks along x must not be clamped at the volume's x ends (a halo wider than a brick): their
    // source words per row (fwpr) would differ from the class representative's.
    bool gridMatches(GridGuess const& q, vktHipBrickRange_t const& r, BrickDesc const& d, size_t i, int32_t sdx)
    {
        BrickGrid const& g = q.g;
        int32_t const ix = static_cast<int32_t>(i % static_cast<size_t>(g.nbx));
        int32_t const iy = static_cast<int32_t>((i / static_cast<size_t>(g.nbx)) % static_cast<size_t>(g.nby));
        int32_t const iz = static_cast<int32_t>(i / q.pz);
        auto cls = [](int32_t k, int32_t nb) { return k == nb - 1 ? 2 : (k == 0 ? 0 : 1); };
        int32_t const nx = g.nx[cls(ix, g.nbx)], ny = g.ny[cls(iy, g.nby)], nz = g.nz[cls(iz, g.nbz)];
        if (cls(ix, g.nbx) == 1 && (r.first.x < 0 || r.first.x + nx > sdx))
            return false;
        return d.linear && r.first.x == g.fx0 + ix * g.bx && r.first.y == g.fy0 + iy * g.by &&
               r.first.z == g.fz0 + iz * g.bz && r.last.x - r.first.x == nx && r.last.y - r.first.y == ny &&
               r.last.z - r.first.z == nz;
    }

    // The class divisors from one descriptor of each class (every brick of a class has the same
    // box extent and source span, so the same divisors: gridMatches held for all of them).
    void gridDivisors(GridGuess& q, BrickDesc const* d)
    {
        BrickGrid& g = q.g;
        auto rep = [](int c, int32_t nb) -> size_t { return c == 0 ? 0 : (c == 1 ? (nb > 2 ? 1 : 0) : nb - 1); };
        for (int c = 0; c < 3; ++c)
        {
            g.fdx[c] = d[rep(c, g.nbx)].fdx;
            g.fwpr[c] = d[rep(c, g.nbx)].fwpr;
            g.fdy[c] = d[rep(c, g.nby) * static_cast<size_t>(g.nbx)].fdy;
        }
    }

    vktError prepareSlot(DescTable& st, size_t descs, size_t ptrs)
    {
        if (st.pending)
        {
            VKT_HIP_TRY(hipEventSynchronize(st.done));
            st.pending = false;
        }
        if (st.capDesc < descs)
        {
            if (st.host)
                VKT_HIP_TRY(hipHostFree(st.host));
            if (st.dev)
                VKT_HIP_TRY(hipFree(st.dev));
            st.host = nullptr;
            st.dev = nullptr;
            st.capDesc = 0;
            VKT_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&st.host), descs * sizeof(BrickDesc)));
            VKT_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&st.dev), descs * sizeof(BrickDesc)));
            st.capDesc = descs;
        }
        if (st.capPtr < ptrs)
        {
            if (st.hostPtr)
                VKT_HIP_TRY(hipHostFree(st.hostPtr));
            if (st.devPtr)
                VKT_HIP_TRY(hipFree(st.devPtr));
            st.hostPtr = nullptr;
            st.devPtr = nullptr;
            st.capPtr = 0;
            VKT_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&st.hostPtr), ptrs * sizeof(uint8_t*)));
            VKT_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&st.devPtr), ptrs * sizeof(uint8_t*)));
            st.capPtr = ptrs;
        }
        if (!st.done)
            VKT_HIP_TRY(hipEventCreateWithFlags(&st.done, hipEventDisableTiming));
        if (!st.copied)
            VKT_HIP_TRY(hipEventCreateWithFlags(&st.copied, hipEventDisableTiming));
        return vktNoError;
    }

    // Upload the slot's table (descriptors, or the brick pointers of a uniform grid) on the copy
    // stream and launch the copy of nFast bricks (groups of `run` bricks along x, chunks of up to
    // maxItems 16-B items).  Caller holds the ring lock.
    vktError launchBricks(DescRing& ring, DescTable& st, bool useGrid, BrickGrid grid, size_t nFast, size_t run,
                          uint32_t maxItems, vktHipVolumeView_t const& source, uint32_t bpv)
    {
        hipStream_t s = rt::computeStream();
        uint64_t const chunks = (maxItems + kBrickChunk - 1) / kBrickChunk;
        uint64_t const blocks = chunks * nFast;
        if (blocks >= (1ull << 32))
            return rt::fail("BrickDecompose: too many bricks for one launch");
        ring.next = (ring.next + 1) % kDescSlots;
        BrickDesc* dev = st.dev;
        // the table goes up on the copy stream, so it overlaps the previous call's kernel
        // (262 144 descriptors of 16^3 bricks are 25 MB, 0.59 ms of PCIe; their data pointers
        // 2 MB); the kernel waits for it.  The slot's previous kernel has finished (st.done
        // above), so its buffers are free.
        hipStream_t const cs = rt::copyStream();
        if (useGrid)
        {
            VKT_HIP_TRY(hipMemcpyAsync(st.devPtr, st.hostPtr, nFast * sizeof(uint8_t*), hipMemcpyHostToDevice, cs));
            grid.dst = st.devPtr;
        }
        else
            VKT_HIP_TRY(hipMemcpyAsync(dev, st.host, nFast * sizeof(BrickDesc), hipMemcpyHostToDevice, cs));
        VKT_HIP_TRY(hipEventRecord(st.copied, cs));
        VKT_HIP_TRY(hipStreamWaitEvent(s, st.copied, 0));
        FastDiv const fdc = makeFastDiv(static_cast<uint32_t>(chunks));
        FastDiv const fdg = makeFastDiv(static_cast<uint32_t>(nFast % run == 0 ? run : 1));
        unsigned const g = static_cast<unsigned>(blocks);
        // (knob value 4, the edge mode of brickStaged, needs one chunk per brick and a 16-B row
        // pitch; elsewhere it runs as 0)
        // 5 (default): the edge mode for UInt8 -- a cut word is up to 15 voxels of per-voxel
        // branches there (16^3 + halo 1 back-to-back 1.38-1.50 -> 1.30 ms), the per-voxel loop for
        // the wider formats (UInt16 16^3 + halo 1.52-1.68 -> 1.82 ms in the edge mode;
        // profiles/r05/decedge.jsonl, decedge_u8.jsonl)
        int32_t alignedLds = static_cast<int32_t>(rt::knob(rt::Knob::DecomposeAlignedLds));
        if (alignedLds == 5)
            alignedLds = bpv == 1 ? 4 : 0;
        if (alignedLds == 4 && (chunks != 1 || (static_cast<int64_t>(source.dimX) * bpv) % 16 != 0))
            alignedLds = 0;
        // words staged per thread: enough that a chunk's source words are all in flight at once
        // (one memory latency per workgroup): a 16-KiB chunk of 32^3 bricks + halo 1 (68-B rows)
        // reads ~1450 aligned words = 5.7 per thread.  In-process A/B (profiles/r03/decompose_ab.jsonl,
        // back-to-back calls): 32^3 + halo 1.256 -> 1.211 ms with 6, 1.218 ms with 8; 64^3 + halo,
        // 128^3 and 256^3 + halo unchanged within 1 %
        int64_t const sw = rt::knob(rt::Knob::DecomposeStageWords);
        // threads per workgroup (knob decompose.block): 128 gives each thread twice the items and
        // staged words of a 256-thread workgroup over the same 16-KiB chunk
        bool const half = rt::knob(rt::Knob::DecomposeBlock) == 128;
        uint32_t const gatherLds =
            useGrid && rt::knob(rt::Knob::DecomposeGather) != 0 ? gatherLdsBytes(grid, bpv) : 0u;
        bool const pipe = useGrid && gatherLds == 0 && !half && rt::knob(rt::Knob::DecomposePipe) != 0;
        PairGeom pg{};
        uint32_t pairs = 0;
        bool const pair = useGrid && gatherLds == 0 && !pipe && !half && rt::knob(rt::Knob::DecomposePair) != 0 &&
                          pairGeom(grid, bpv, maxItems, source.dimX, pg, pairs);
        // direct copy (brickDirect): no clamped voxel anywhere in the grid, every box row whole
        // 16-B words at 16-B aligned source offsets
        auto directGrid = [&] {
            if (!useGrid || rt::knob(rt::Knob::DecomposeDirect) == 0 || (source.dimX * bpv) % 16 != 0 ||
                (static_cast<int64_t>(grid.fx0) * bpv) % 16 != 0 || (static_cast<int64_t>(grid.bx) * bpv) % 16 != 0 ||
                grid.fx0 < 0 || grid.fy0 < 0 || grid.fz0 < 0)
                return false;
            int32_t const sdim[3] = {source.dimX, source.dimY, source.dimZ};
            int32_t const f0[3] = {grid.fx0, grid.fy0, grid.fz0}, step[3] = {grid.bx, grid.by, grid.bz};
            int32_t const nb[3] = {grid.nbx, grid.nby, grid.nbz};
            int32_t const* ext[3] = {grid.nx, grid.ny, grid.nz};
            for (int a = 0; a < 3; ++a)
                for (int c = 0; c < 3; ++c)
                {
                    // classes in use (gridClass): 0 with >= 2 bricks, 1 with >= 3, 2 always; the
                    // last brick of class c: brick 0, nb - 2, nb - 1
                    if ((c == 0 && nb[a] < 2) || (c == 1 && nb[a] < 3))
                        continue;
                    int64_t const i = c == 0 ? 0 : (c == 1 ? nb[a] - 2 : nb[a] - 1);
                    if (f0[a] + i * step[a] + ext[a][c] > sdim[a])
                        return false;
                    if (a == 0 && (static_cast<int64_t>(ext[0][c]) * bpv) % 16 != 0)
                        return false;
                }
            return true;
        };
        bool const direct = !half && gatherLds == 0 && !pipe && !pair && directGrid();
        // row-image copy (knob decompose.row_image: 2 (default) UInt8, 1 every format, 0 off): one
        // brick of <= 16 KiB per workgroup, rows >= 16 B, 16-B multiple source rows, halos <= 16 B.
        // Measured (profiles/r06/decrow.jsonl, 1024^3 -> 16^3 bricks + halo 1, back-to-back): UInt8
        // 1.27-1.32 -> 1.04 ms, UInt16 1.46-1.60 -> 2.55 ms (a 36-B row's three 16-B pieces per lane
        // scatter each store instruction over ~2.3 KB), UInt16 8^3 + halo 5.85-6.32 -> 5.05 ms
        int64_t const rowImageKnob = rt::knob(rt::Knob::DecomposeRowImage);
        uint32_t rowImageLds = 0;
        if (!direct && useGrid && chunks == 1 && gatherLds == 0 && !pipe && !pair && !half &&
            (rowImageKnob == 1 || (rowImageKnob == 2 && bpv == 1)) &&
            (static_cast<int64_t>(source.dimX) * bpv) % 16 == 0)
        {
            int32_t minNx = grid.nx[2], maxNx = grid.nx[2], maxRows = 0;
            for (int c = 0; c < 3; ++c)
            {
                if ((c == 0 && grid.nbx < 2) || (c == 1 && grid.nbx < 3))
                    continue;
                minNx = std::min(minNx, grid.nx[c]);
                maxNx = std::max(maxNx, grid.nx[c]);
            }
            for (int cy = 0; cy < 3; ++cy)
                for (int cz = 0; cz < 3; ++cz)
                    maxRows = std::max(maxRows, grid.ny[cy] * grid.nz[cz]);
            int64_t const img = ((16 + 15 + static_cast<int64_t>(maxNx) * bpv + 16 + 15) / 16 | 1) * 16;
            if (static_cast<int64_t>(minNx) * bpv >= 16 && -grid.fx0 * static_cast<int64_t>(bpv) <= 16 &&
                img * maxRows <= 65536)
                rowImageLds = static_cast<uint32_t>(img * maxRows);
        }
        // small bricks: P per workgroup (knob decompose.direct 1; 2 keeps one per workgroup).
        // Measured and rejected: 4 bricks of <= 512 items per workgroup at 8 items per thread
        // (16^3 UInt16 0.858 vs 0.862 ms, within the spread)
        uint32_t const perWg = !direct || chunks != 1 || rt::knob(rt::Knob::DecomposeDirect) != 1
                                   ? 1u
                                   : (maxItems <= kBrickChunk / 4 ? 4u : (maxItems <= kBrickChunk / 2 ? 2u : 1u));
        auto launch = [&](auto bpvC, auto swC) {
            constexpr int B = decltype(bpvC)::value, W = decltype(swC)::value;
            if (rowImageLds != 0)
                hipLaunchKernelGGL((brickRowImageKernel<B, kBlock>), dim3(static_cast<unsigned>(nFast)), dim3(kBlock),
                                   rowImageLds, s, grid, source.data, source.dimX, source.dimY, source.dimZ);
            else if (direct && perWg > 1)
            {
                unsigned const gw = static_cast<unsigned>((nFast + perWg - 1) / perWg);
                if (perWg == 4)
                    hipLaunchKernelGGL((brickDirectKernel<B, 4>), dim3(gw), dim3(kBlock), 0, s, grid,
                                       static_cast<uint32_t>(nFast), source.data, source.dimX, source.dimY);
                else
                    hipLaunchKernelGGL((brickDirectKernel<B, 2>), dim3(gw), dim3(kBlock), 0, s, grid,
                                       static_cast<uint32_t>(nFast), source.data, source.dimX, source.dimY);
            }
            else if (direct)
                hipLaunchKernelGGL((brickCopyKernel<B, W, true, kBlock, true>), dim3(g), dim3(kBlock), 0, s, dev, grid,
                                   fdc, fdg, source.data, source.dimX, source.dimY, source.dimZ, alignedLds);
            else if (pair)
                hipLaunchKernelGGL((brickPairKernel<B, W + 2, kBlock>), dim3(pairs), dim3(kBlock), 0, s, grid, pg,
                                   source.data, source.dimX, source.dimY, source.dimZ, alignedLds);
            else if (pipe)
            {
                // resident workgroups only (a persistent walk), a multiple of 8 (XCD grouping)
                static unsigned const perCU = [] {
                    int n = 0;
                    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
                            &n, reinterpret_cast<void const*>(brickPipeKernel<B, W, kBlock>), kBlock, 0) != hipSuccess ||
                        n < 1)
                    {
                        (void)hipGetLastError();
                        n = 2;
                    }
                    return static_cast<unsigned>(std::min(n, 8));
                }();
                unsigned G = std::min<unsigned>(g, kNumCUs * perCU);
                if (G >= 8)
                    G &= ~7u;
                hipLaunchKernelGGL((brickPipeKernel<B, W, kBlock>), dim3(G), dim3(kBlock), 0, s, grid, fdc, fdg, g,
                                   source.data, source.dimX, source.dimY, source.dimZ, alignedLds);
            }
            else if (gatherLds != 0)
                hipLaunchKernelGGL((brickGatherKernel<B, W, kBlock>), dim3(g), dim3(kBlock), gatherLds, s, grid, fdc, fdg,
                                   source.data, source.dimX, source.dimY, source.dimZ);
            else if (half)
            {
                if (useGrid)
                    hipLaunchKernelGGL((brickCopyKernel<B, 2 * W, true, 128>), dim3(g), dim3(128), 0, s, dev, grid, fdc,
                                       fdg, source.data, source.dimX, source.dimY, source.dimZ, alignedLds);
                else
                    hipLaunchKernelGGL((brickCopyKernel<B, 2 * W, false, 128>), dim3(g), dim3(128), 0, s, dev, grid, fdc,
                                       fdg, source.data, source.dimX, source.dimY, source.dimZ, alignedLds);
            }
            else if (useGrid && alignedLds == 4)
                hipLaunchKernelGGL((brickCopyKernel<B, W, true, kBlock, false, true>), dim3(g), dim3(kBlock), 0, s, dev,
                                   grid, fdc, fdg, source.data, source.dimX, source.dimY, source.dimZ, alignedLds);
            else if (useGrid)
                hipLaunchKernelGGL((brickCopyKernel<B, W, true>), dim3(g), dim3(kBlock), 0, s, dev, grid, fdc, fdg,
                                   source.data, source.dimX, source.dimY, source.dimZ, alignedLds);
            else if (alignedLds == 4)
                hipLaunchKernelGGL((brickCopyKernel<B, W, false, kBlock, false, true>), dim3(g), dim3(kBlock), 0, s, dev,
                                   grid, fdc, fdg, source.data, source.dimX, source.dimY, source.dimZ, alignedLds);
            else
                hipLaunchKernelGGL((brickCopyKernel<B, W, false>), dim3(g), dim3(kBlock), 0, s, dev, grid, fdc, fdg,
                                   source.data, source.dimX, source.dimY, source.dimZ, alignedLds);
        };
        auto bySw = [&](auto bpvC) {
            if (sw <= 5)
                launch(bpvC, std::integral_constant<int, 5>{});
            else if (sw == 6)
                launch(bpvC, std::integral_constant<int, 6>{});
            else
                launch(bpvC, std::integral_constant<int, 8>{});
        };
        if (bpv == 1)
            bySw(std::integral_constant<int, 1>{});
        else if (bpv == 2)
            bySw(std::integral_constant<int, 2>{});
        else
            bySw(std::integral_constant<int, 4>{});
        VKT_HIP_TRY(hipGetLastError());
        VKT_HIP_TRY(hipEventRecord(st.done, s));
        st.pending = true;
        return vktNoError;
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

    uint32_t const bpv = codec::bytesPerVoxel(source.dataFormat);
    if (bpv != 1 && bpv != 2 && bpv != 4)
        return rt::fail("vktHipBrickDecompose: unsupported data format");
    // The descriptors are written straight into the pinned staging table of the next ring
    // slot (held under the ring lock until the launch), validating everything before the first
    // launch (reference: out-of-range writes are UB).
    DescRing& ring = descRing();
    std::unique_lock<std::mutex> lock(ring.m);
    DescTable& st = ring.slot[ring.next];
    size_t const need = static_cast<size_t>(numBricks);
    if (vktError const e = prepareSlot(st, need, need); e != vktNoError)
        return e;
    BrickDesc* const fast = st.host;
    int64_t const V = 16 / bpv;                            // voxels per 16-B segment
    uint32_t const vShift = bpv == 1 ? 4u : bpv == 2 ? 3u : 2u;
    bool const srcAligned = source.dimX >= V && reinterpret_cast<uintptr_t>(source.data) % 16 == 0;
    // One descriptor per brick, at the brick's own index (a brick with an empty range or one that
    // needs unmap -> map gets nitems = 0 and its workgroups return at once), built in parallel
    // chunks on the host pool: 262 144 bricks of 16^3 cost ~9 ns each serially.
    // uniform grid (BrickGrid): inferred from the ranges, each range checked in the loop below
    GridGuess guess = rt::knob(rt::Knob::DecomposeGrid) != 0 ? inferGrid(bricks, static_cast<size_t>(numBricks))
                                                            : GridGuess{};
    std::atomic<bool> gridOk{guess.ok};
    uint8_t** const ptrs = st.hostPtr;
    std::mutex merge;
    std::vector<int32_t> slow;
    uint32_t maxItems = 0;
    int32_t errBrick = numBricks;
    char const* errWhat = nullptr;
    // A uniform grid (the usual BrickDecompose list) uploads only the brick pointers: the pass
    // validates every range and builds its descriptor on the stack, storing no table (262 144
    // descriptors of 16^3 bricks are 25 MB of host writes per call).  When the grid does not hold
    // (or was not guessed), a second pass -- or the only one -- writes the table.
    auto pass = [&](bool writeTable) {
        rt::parallelFor(static_cast<size_t>(numBricks), 4096, [&](size_t b, size_t e) {
            // bricks of a decomposition share a few sizes: reuse the last divisor of each kind
            // (each makeFastDiv costs a 64-bit division)
            struct LastDiv
            {
                FastDiv f{0u, 0u, 0u};
                bool valid = false;
                FastDiv operator()(uint32_t d)
                {
                    if (!valid || f.d != d)
                    {
                        f = makeFastDiv(d);
                        valid = true;
                    }
                    return f;
                }
            } divSeg, divX, divWpr, divY;
            std::vector<int32_t> mySlow;
            bool myGrid = !writeTable && guess.ok && gridOk.load(std::memory_order_relaxed);
            uint32_t myMax = 0;
            int32_t myErr = numBricks;
            char const* myWhat = nullptr;
            BrickDesc local;
            for (size_t ii = b; ii < e; ++ii)
            {
                int32_t const i = static_cast<int32_t>(ii);
                vktHipBrickRange_t const& br = bricks[i];
                BrickDesc& d = writeTable ? fast[i] : local;
                d = BrickDesc{};
                d.fx = br.first.x;
                d.fy = br.first.y;
                d.fz = br.first.z;
                if (!validView(br.brick))
                {
                    myErr = i;
                    myWhat = "vktHipBrickDecompose: invalid brick view";
                    break;
                }
                int64_t nx = int64_t(br.last.x) - br.first.x, ny = int64_t(br.last.y) - br.first.y;
                int64_t nz = int64_t(br.last.z) - br.first.z;
                if (nx <= 0 || ny <= 0 || nz <= 0)
                {
                    myGrid = false;   // (the grid kernel would copy a box for it)
                    continue;
                }
                if (nx > br.brick.dimX || ny > br.brick.dimY || nz > br.brick.dimZ)
                {
                    myErr = i;
                    myWhat = "vktHipBrickDecompose: brick smaller than its range (reference writes out of bounds)";
                    break;
                }
                if (overlaps(br.brick, source))
                {
                    myErr = i;
                    myWhat = "vktHipBrickDecompose: brick aliases the source";
                    break;
                }
                bool bytewise = br.brick.dataFormat == source.dataFormat && br.brick.mappingLo == source.mappingLo &&
                                br.brick.mappingHi == source.mappingHi;   // Copy_serial.hpp:21-22
                uint64_t nv = static_cast<uint64_t>(nx) * static_cast<uint64_t>(ny) * static_cast<uint64_t>(nz);
                if (!bytewise || nv >= (1ull << 31))
                {
                    mySlow.push_back(i);
                    myGrid = false;
                    continue;
                }
                d.dst = br.brick.data;
                d.dimX = br.brick.dimX;
                d.dimY = br.brick.dimY;
                uint32_t const seg = static_cast<uint32_t>((nx + V - 1) >> vShift);   // 16-B segments per row
                d.nx = static_cast<int32_t>(nx);
                d.nvox = static_cast<uint32_t>(nv);
                d.linear = nx == br.brick.dimX && ny == br.brick.dimY && nx >= V && srcAligned &&
                           reinterpret_cast<uintptr_t>(br.brick.data) % 16 == 0;
                d.nitems = d.linear ? static_cast<uint32_t>((nv + V - 1) >> vShift) : static_cast<uint32_t>(ny * nz) * seg;
                d.fseg = divSeg(seg);
                d.fdx = divX(static_cast<uint32_t>(nx));
                {
                    int64_t const span = std::min<int64_t>(br.first.x + nx, source.dimX) - std::max<int32_t>(br.first.x, 0);
                    d.fwpr = divWpr(span > 0 ? static_cast<uint32_t>((span * bpv + 15) / 16 + 1) : 0u);
                }
                d.fdy = divY(static_cast<uint32_t>(ny));
                myMax = d.nitems > myMax ? d.nitems : myMax;
                if (myGrid)
                {
                    myGrid = gridMatches(guess, br, d, ii, source.dimX);
                    ptrs[i] = d.dst;
                }
            }
            if (!myGrid)
                gridOk.store(false, std::memory_order_relaxed);
            std::lock_guard<std::mutex> g(merge);
            if (writeTable || !guess.ok)
                slow.insert(slow.end(), mySlow.begin(), mySlow.end());
            maxItems = std::max(maxItems, myMax);
            if (myErr < errBrick)
            {
                errBrick = myErr;
                errWhat = myWhat;
            }
        });
    };
    if (guess.ok)
    {
        pass(false);
        if (errWhat == nullptr && !gridOk.load())
        {
            maxItems = 0;
            pass(true);   // the grid failed somewhere: the descriptor table after all
        }
        else if (errWhat == nullptr)
        {
            // the class representatives' descriptors (gridDivisors) and the brick-row run below
            auto rep = [](int c, int32_t nb) -> size_t { return c == 0 ? 0 : (c == 1 ? (nb > 2 ? 1 : 0) : nb - 1); };
            std::vector<size_t> reps;
            for (int c = 0; c < 3; ++c)
            {
                reps.push_back(rep(c, guess.g.nbx));
                reps.push_back(rep(c, guess.g.nby) * static_cast<size_t>(guess.g.nbx));
            }
            for (size_t r : reps)
            {
                vktHipBrickRange_t const& br = bricks[r];
                BrickDesc& d = fast[r];
                d = BrickDesc{};
                int64_t const nx = int64_t(br.last.x) - br.first.x, ny = int64_t(br.last.y) - br.first.y;
                int64_t const span = std::min<int64_t>(br.first.x + nx, source.dimX) - std::max<int32_t>(br.first.x, 0);
                d.fdx = makeFastDiv(static_cast<uint32_t>(nx));
                d.fwpr = makeFastDiv(span > 0 ? static_cast<uint32_t>((span * bpv + 15) / 16 + 1) : 0u);
                d.fdy = makeFastDiv(static_cast<uint32_t>(ny));
            }
        }
    }
    else
        pass(true);
    if (errWhat != nullptr)   // the first bad brick in list order, before anything launched
        return rt::fail(errWhat);
    std::sort(slow.begin(), slow.end());
    size_t const nFast = maxItems > 0 ? static_cast<size_t>(numBricks) : 0;
    if (nFast > 0)
    {
        // group = the run of leading bricks with the same y/z box (one brick row of an
        // Array3D).  Any group size dividing the brick count maps blocks 1:1 onto (brick,
        // chunk); it only changes the order in which bricks are visited.
        size_t run = 1;
        while (run < nFast && bricks[run].first.y == bricks[0].first.y && bricks[run].first.z == bricks[0].first.z)
            ++run;
        bool const useGrid = slow.empty() && guess.ok && gridOk.load() && nFast == static_cast<size_t>(numBricks);
        if (useGrid)
            gridDivisors(guess, fast);
        if (vktError const e = launchBricks(ring, st, useGrid, guess.g, nFast, run, maxItems, source, bpv);
            e != vktNoError)
            return e;
    }
    lock.unlock();
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

vktError vktHipBrickDecomposeGrid(vktHipVolumeView_t source, vktHipBrickGrid_t grid, uint8_t* const* brickData)
{
    if (!validView(source) || source.dimX <= 0 || source.dimY <= 0 || source.dimZ <= 0)
        return rt::fail("vktHipBrickDecomposeGrid: invalid source view");
    uint32_t const bpv = codec::bytesPerVoxel(source.dataFormat);
    if (bpv != 1 && bpv != 2 && bpv != 4)
        return rt::fail("vktHipBrickDecomposeGrid: unsupported data format");
    int32_t const sd[3] = {source.dimX, source.dimY, source.dimZ};
    int32_t const nb[3] = {grid.numBricks.x, grid.numBricks.y, grid.numBricks.z};
    int32_t const bs[3] = {grid.brickSize.x, grid.brickSize.y, grid.brickSize.z};
    int32_t const hn[3] = {grid.haloNeg.x, grid.haloNeg.y, grid.haloNeg.z};
    int32_t const hp[3] = {grid.haloPos.x, grid.haloPos.y, grid.haloPos.z};
    // box extent per axis and class (0 first brick, 1 interior, 2 last -- gridClass; a single
    // brick is class 2), and the x of the representative brick of each class
    int32_t ext[3][3], fxc[3];
    for (int a = 0; a < 3; ++a)
    {
        if (bs[a] <= 0 || hn[a] < 0 || hp[a] < 0 || nb[a] != (sd[a] + bs[a] - 1) / bs[a])
            return rt::fail("vktHipBrickDecomposeGrid: grid does not match the source (numBricks = ceil(dims / "
                            "brickSize), halos >= 0)");
        int32_t const border = sd[a] - (nb[a] - 1) * bs[a];
        ext[a][0] = hn[a] + (nb[a] > 1 ? bs[a] : border) + hp[a];
        ext[a][1] = hn[a] + bs[a] + hp[a];
        ext[a][2] = hn[a] + border + hp[a];
    }
    if (brickData == nullptr)
        return rt::fail("vktHipBrickDecomposeGrid: null brick pointer list");
    size_t const n = static_cast<size_t>(nb[0]) * static_cast<size_t>(nb[1]) * static_cast<size_t>(nb[2]);
    if (n >= (1ull << 31))
        return rt::fail("vktHipBrickDecomposeGrid: too many bricks");
    fxc[0] = -hn[0];
    fxc[1] = bs[0] - hn[0];
    fxc[2] = (nb[0] - 1) * bs[0] - hn[0];
    int32_t const V = 16 / static_cast<int32_t>(bpv);
    int64_t const maxVox = static_cast<int64_t>(std::max({ext[0][0], ext[0][1], ext[0][2]})) *
                           std::max({ext[1][0], ext[1][1], ext[1][2]}) * std::max({ext[2][0], ext[2][1], ext[2][2]});
    // what the index-derived (grid) kernel needs: linear bricks (rows of >= 16 B, 16-B aligned
    // source), interior bricks along x never clamped (one source span per class), boxes < 2^31
    bool ok = source.dimX >= V && reinterpret_cast<uintptr_t>(source.data) % 16 == 0 && maxVox < (1ll << 31) &&
              rt::knob(rt::Knob::DecomposeGrid) != 0;
    for (int c = 0; c < 3; ++c)
        ok = ok && ext[0][c] >= V;
    if (nb[0] > 2)
        ok = ok && fxc[1] >= 0 && (nb[0] - 2) * bs[0] - hn[0] + ext[0][1] <= sd[0];
    auto boxOf = [&](size_t i, vktHipBrickRange_t& r) {
        int32_t const ix = static_cast<int32_t>(i % static_cast<size_t>(nb[0]));
        int32_t const iy = static_cast<int32_t>((i / static_cast<size_t>(nb[0])) % static_cast<size_t>(nb[1]));
        int32_t const iz = static_cast<int32_t>(i / (static_cast<size_t>(nb[0]) * static_cast<size_t>(nb[1])));
        int32_t const c[3] = {ix * bs[0], iy * bs[1], iz * bs[2]};
        r.first = {c[0] - hn[0], c[1] - hn[1], c[2] - hn[2]};
        r.last = {std::min(c[0] + bs[0], sd[0]) + hp[0], std::min(c[1] + bs[1], sd[1]) + hp[1],
                  std::min(c[2] + bs[2], sd[2]) + hp[2]};
        r.brick = source;
        r.brick.data = brickData[i];
        r.brick.dimX = r.last.x - r.first.x;
        r.brick.dimY = r.last.y - r.first.y;
        r.brick.dimZ = r.last.z - r.first.z;
    };
    if (!ok)
    {
        // the general path on the equivalent range list
        thread_local std::vector<vktHipBrickRange_t> ranges;
        ranges.resize(n);
        rt::parallelFor(n, 4096, [&](size_t b, size_t e) {
            for (size_t i = b; i < e; ++i)
                boxOf(i, ranges[i]);
        });
        return vktHipBrickDecompose(source, ranges.data(), static_cast<int32_t>(n));
    }
    DescRing& ring = descRing();
    std::unique_lock<std::mutex> lock(ring.m);
    DescTable& st = ring.slot[ring.next];
    if (vktError const e = prepareSlot(st, 0, n); e != vktNoError)
        return e;
    // the pointers into the pinned table; each checked: non-null, not inside the source
    uint8_t const* const s0 = source.data;
    uint8_t const* const s1 = s0 + static_cast<uint64_t>(sd[0]) * sd[1] * sd[2] * bpv;
    std::atomic<int64_t> bad{-1};
    uint8_t** const ptrs = st.hostPtr;
    rt::parallelFor(n, 8192, [&](size_t b, size_t e) {
        auto cls = [](size_t k, int32_t nbk) { return k == static_cast<size_t>(nbk - 1) ? 2 : (k == 0 ? 0 : 1); };
        for (size_t i = b; i < e; ++i)
        {
            uint8_t* const p = brickData[i];
            ptrs[i] = p;
            size_t const ix = i % static_cast<size_t>(nb[0]), yz = i / static_cast<size_t>(nb[0]);
            size_t const iy = yz % static_cast<size_t>(nb[1]), iz = yz / static_cast<size_t>(nb[1]);
            uint64_t const bytes = static_cast<uint64_t>(ext[0][cls(ix, nb[0])]) * ext[1][cls(iy, nb[1])] *
                                   ext[2][cls(iz, nb[2])] * bpv;
            if (p == nullptr || (p < s1 && p + bytes > s0))
            {
                int64_t expect = -1;
                bad.compare_exchange_strong(expect, static_cast<int64_t>(i));
            }
        }
    });
    if (bad.load() >= 0)
        return rt::fail("vktHipBrickDecomposeGrid: a brick pointer is null or inside the source");
    BrickGrid g{};
    g.nbx = nb[0];
    g.nby = nb[1];
    g.nbz = nb[2];
    g.fnbx = makeFastDiv(static_cast<uint32_t>(nb[0]));
    g.fnby = makeFastDiv(static_cast<uint32_t>(nb[1]));
    g.fx0 = -hn[0];
    g.fy0 = -hn[1];
    g.fz0 = -hn[2];
    g.bx = nb[0] > 1 ? bs[0] : 0;
    g.by = nb[1] > 1 ? bs[1] : 0;
    g.bz = nb[2] > 1 ? bs[2] : 0;
    for (int c = 0; c < 3; ++c)
    {
        g.nx[c] = ext[0][c];
        g.ny[c] = ext[1][c];
        g.nz[c] = ext[2][c];
        g.fdx[c] = makeFastDiv(static_cast<uint32_t>(ext[0][c]));
        g.fdy[c] = makeFastDiv(static_cast<uint32_t>(ext[1][c]));
        int64_t const span = std::min<int64_t>(fxc[c] + ext[0][c], sd[0]) - std::max<int32_t>(fxc[c], 0);
        g.fwpr[c] = makeFastDiv(span > 0 ? static_cast<uint32_t>((span * bpv + 15) / 16 + 1) : 1u);
    }
    uint32_t const maxItems = static_cast<uint32_t>((maxVox + V - 1) / V);
    if (vktError const e = launchBricks(ring, st, true, g, n, static_cast<size_t>(nb[0]), maxItems, source, bpv);
        e != vktNoError)
        return e;
    lock.unlock();
    return rt::finishLaunch("BrickDecompose_hip");
}

} // extern "C"
