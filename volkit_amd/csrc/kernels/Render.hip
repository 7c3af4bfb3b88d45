// Render.hip -- the reference's three volume renderers as gfx950 kernels (SURVEY.md §8(f) F4,
// BASELINE config 5: 1024^3 UInt8 multi-scattering, 1024^2 viewport).
//
// Restated from reference src/vkt/Render_kernel.hpp:
//  * RayMarchingKernel (:80-158): front-to-back emission/absorption, opacity correction
//    1 - (1 - a)^dt, premultiplied colour, step dt in object space.  The reference's
//    early-termination test reads result.color (never written) and so never fires; stopping
//    once dst.w == 1 exactly is bit-identical (every later contribution is exactly 0).
//  * ImplicitIsoKernel (:164-268): iso crossings between consecutive samples, gradient by
//    central differences of raw texels at +-0.01 in texture space, shading .2 + albedo *
//    max(0, N.-dir) * voxel.
//  * MultiScatteringKernel (:276-418): Woodcock (delta) tracking against the majorant,
//    albedo = LUT.rgb or voxel, Russian roulette below throughput 0.2, isotropic phase
//    function (Henyey-Greenstein g = 0), at most 1024 bounces, sky gradient
//    (1-t)*(1,1,1) + t*(.5,.7,1) with t = y / height.
// Camera rays, random numbers and the transcendental functions are this project's own
// (common/RenderMath.hpp): visionaray is not vendored, so those sequences are unpinned; the
// CPU oracle restates the same sequences and the GPU image is compared with it bit for bit.
//
// MI355X design: one thread per pixel, 8x8-pixel tiles per wave (neighbouring rays walk
// neighbouring voxels -> the texel loads of a wave share cache lines), all frames of a call
// accumulated in registers (one launch, one read-modify-write of the accumulation buffer).
// The texel fetch is a plain global load of the dense volume (L2/MALL resident neighbourhood);
// nearest filtering and clamp addressing are integer index math.

#include "KernelCommon.hpp"
#include "../common/RenderMath.hpp"
#include "../runtime/Runtime.hpp"
#include "volkit_hip.h"

namespace vkt
{
namespace hipk
{
    bool validView(vktHipVolumeView_t const& v);

    struct V3
    {
        float x, y, z;
    };

    __device__ __forceinline__ V3 v3(float const* a) { return V3{a[0], a[1], a[2]}; }
    __device__ __forceinline__ V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
    __device__ __forceinline__ V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
    __device__ __forceinline__ V3 operator*(V3 a, float s) { return V3{a.x * s, a.y * s, a.z * s}; }
    __device__ __forceinline__ V3 mul(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }
    __device__ __forceinline__ V3 div(V3 a, V3 b) { return V3{a.x / b.x, a.y / b.y, a.z / b.z}; }
    __device__ __forceinline__ float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
    __device__ __forceinline__ V3 normalize(V3 a) { return a * (1.f / sqrtf(dot(a, a))); }

    struct Hit
    {
        float tnear, tfar;
        bool hit;
    };

    // slab test against [0, box]
    __device__ __forceinline__ Hit intersectBox(V3 ori, V3 dir, V3 box)
    {
        V3 const inv{1.f / dir.x, 1.f / dir.y, 1.f / dir.z};
        V3 const t1 = mul(V3{0.f - ori.x, 0.f - ori.y, 0.f - ori.z}, inv);
        V3 const t2 = mul(box - ori, inv);
        float const tn = fmaxf(fmaxf(fminf(t1.x, t2.x), fminf(t1.y, t2.y)), fminf(t1.z, t2.z));
        float const tf = fminf(fminf(fmaxf(t1.x, t2.x), fmaxf(t1.y, t2.y)), fmaxf(t1.z, t2.z));
        return Hit{tn, tf, tn <= tf};
    }

    // nearest texel index with clamp addressing: floor(c * n) clamped to [0, n - 1]
    __device__ __forceinline__ int32_t texIndex(float c, int32_t n)
    {
        float f = c * static_cast<float>(n);
        if (!(f >= 0.f))
            f = 0.f;
        float const hi = static_cast<float>(n - 1);
        if (f > hi)
            f = hi;
        return static_cast<int32_t>(floorf(f));
    }

    struct Tex
    {
        uint8_t const* data;
        int32_t nx, ny, nz;
        int32_t fmt;
        float lo, hi;
        int32_t nbx, nby;   // bricked copy: bricks per row / per column (8^3 voxels each)
    };

    // texel offset of voxel (x, y, z): dense x-fastest, or the 8^3-brick copy
    template <bool BRICK>
    __device__ __forceinline__ uint64_t texOffset(Tex const& t, uint32_t x, uint32_t y, uint32_t z)
    {
        if constexpr (BRICK)
            return ((static_cast<uint64_t>(z >> 3) * static_cast<uint32_t>(t.nby) + (y >> 3)) *
                        static_cast<uint64_t>(static_cast<uint32_t>(t.nbx)) +
                    (x >> 3)) * 512u +
                   (((z & 7u) << 6) | ((y & 7u) << 3) | (x & 7u));
        else
            return (static_cast<uint64_t>(z) * static_cast<uint64_t>(t.ny) + y) * static_cast<uint64_t>(t.nx) + x;
    }

    constexpr uint64_t kMaxBrickBytes = 8ull << 30;

    // dense -> 8^3 bricks, edge bricks clamp-replicated.  A workgroup converts the 16 / BPV
    // consecutive bricks along x of one brick row: 64 source rows (8 planes x 8 rows) of 128 B
    // each, read as aligned 16-B pieces into an LDS tile (rows padded to 136 B: the brick-order
    // reads of rows ly and ly + 1 then fall on different banks), written out as the bricks'
    // contiguous 8 KiB with 16-B stores (two brick rows per store).  Rows off the 16-B grid or
    // pieces past the volume go voxel by voxel with the clamp.  (One thread per 8-voxel brick row
    // with byte loads and stores took 3.3 ms for a 1024^3 UInt8 volume, longer than a
    // multi-scattering frame.)
    constexpr int kBrickRowPitch = 136;
    template <int BPV>
    __global__ __launch_bounds__(256) void brickKernel(uint8_t const* src, uint8_t* dst, int32_t nx, int32_t ny,
                                                      int32_t nz, int32_t nbx, int32_t nby, uint32_t groupsX)
    {
        constexpr int32_t NB = 16 / BPV;          // bricks per workgroup
        constexpr int32_t VPP = 16 / BPV;         // voxels per 16-B piece
        __shared__ uint8_t tile[64 * kBrickRowPitch];
        uint32_t const gx = blockIdx.x % groupsX, byz = blockIdx.x / groupsX;
        int32_t const by = static_cast<int32_t>(byz % static_cast<uint32_t>(nby));
        int32_t const bz = static_cast<int32_t>(byz / static_cast<uint32_t>(nby));
        int32_t const bx0 = static_cast<int32_t>(gx) * NB;
        int32_t const x0 = bx0 * 8;
        bool const alignedRows = (static_cast<int64_t>(nx) * BPV) % 16 == 0 && (reinterpret_cast<uintptr_t>(src) & 15u) == 0;
        // 512 pieces of 16 B: row q = p / 8 (lz = q / 8, ly = q % 8), piece c = p % 8
        for (int32_t p = threadIdx.x; p < 512; p += 256)
        {
            int32_t const q = p >> 3, c = p & 7;
            int32_t const z = min(bz * 8 + (q >> 3), nz - 1), y = min(by * 8 + (q & 7), ny - 1);
            uint64_t const row = (static_cast<uint64_t>(z) * static_cast<uint64_t>(ny) + static_cast<uint64_t>(y)) *
                                 static_cast<uint64_t>(nx);
            int32_t const xa = x0 + c * VPP;
            uint8_t* const t = tile + q * kBrickRowPitch + c * 16;
            if (alignedRows && xa + VPP <= nx)
            {
                u32x4 const v = *reinterpret_cast<u32x4 const*>(src + (row + static_cast<uint64_t>(xa)) * BPV);
                uint32_t* const tw = reinterpret_cast<uint32_t*>(t);   // (136-B rows: 8-B aligned)
                tw[0] = v.x;
                tw[1] = v.y;
                tw[2] = v.z;
                tw[3] = v.w;
            }
            else
            {
                for (int32_t i = 0; i < VPP; ++i)
                {
                    int32_t const x = min(xa + i, nx - 1);
                    for (int k = 0; k < BPV; ++k)
                        t[i * BPV + k] = src[(row + static_cast<uint64_t>(x)) * BPV + k];
                }
            }
        }
        __syncthreads();
        // out piece o (16 B): brick k = o / (32 BPV), brick rows (lz, ly) and (lz, ly + 1) for BPV 1;
        // for BPV 2 / 4 one piece holds one / half a brick row
        int32_t const nb = min(NB, nbx - bx0);
        uint8_t* const out = dst + ((static_cast<uint64_t>(bz) * static_cast<uint64_t>(nby) + static_cast<uint64_t>(by)) *
                                        static_cast<uint64_t>(nbx) +
                                    static_cast<uint64_t>(bx0)) *
                                       (512u * BPV);
        for (int32_t o = threadIdx.x; o < nb * 32 * BPV; o += 256)
        {
            int32_t const k = o / (32 * BPV), w = o % (32 * BPV);   // brick, piece inside it
            int32_t const v0 = w * VPP;                              // first voxel (lz*64 + ly*8 + lx)
            u32x4 r;
            if constexpr (BPV == 1)
            {
                int32_t const q = v0 >> 3;   // (lz, ly) row of the first 8 voxels; the next row follows
                uint2 const a = *reinterpret_cast<uint2 const*>(tile + q * kBrickRowPitch + k * 8);
                uint2 const b = *reinterpret_cast<uint2 const*>(tile + (q + 1) * kBrickRowPitch + k * 8);
                r = u32x4{a.x, a.y, b.x, b.y};
            }
            else
            {
                // one brick row (BPV 2) or half of one (BPV 4); 8-B aligned in the tile: two b64
                int32_t const q = v0 >> 3, lx = v0 & 7;
                uint8_t const* const t = tile + q * kBrickRowPitch + k * 8 * BPV + lx * BPV;
                uint2 const a = *reinterpret_cast<uint2 const*>(t);
                uint2 const b = *reinterpret_cast<uint2 const*>(t + 8);
                r = u32x4{a.x, a.y, b.x, b.y};
            }
            __builtin_nontemporal_store(r, reinterpret_cast<u32x4*>(out + static_cast<uint64_t>(o) * 16u));
        }
    }

    // code / D for an integer code, correctly rounded, in three instructions instead of the
    // IEEE division sequence: q0 = code * RN(1/D), one fma residual, one fma correction.
    // Checked with exact rational arithmetic for every code of both texel formats (D = 255:
    // 256 codes, D = 65535: 65 536 codes; tests/test_render.py) -- the plain product alone is
    // off by one ulp for 126 and 512 of them.
    template <int D>
    __device__ __forceinline__ float unormDiv(uint32_t code)
    {
        constexpr float kD = static_cast<float>(D);
        constexpr float kR = D == 255 ? 0x1.010102p-8f : 0x1.000100p-16f;   // RN(1 / D)
        float const c = static_cast<float>(code);
        float const q0 = c * kR;
        float const e = __builtin_fmaf(-q0, kD, c);
        return __builtin_fmaf(e, kR, q0);
    }

    // raw texel value as the reference's texture returns it: unorm for integer formats
    template <int FMT, bool BRICK>
    __device__ __forceinline__ float texel(Tex const& t, V3 c)
    {
        uint64_t const i = texOffset<BRICK>(t, static_cast<uint32_t>(texIndex(c.x, t.nx)),
                                     static_cast<uint32_t>(texIndex(c.y, t.ny)), static_cast<uint32_t>(texIndex(c.z, t.nz)));
        if constexpr (FMT == codec::FmtUInt8)
            return unormDiv<255>(t.data[i]);   // == float(code) / 255.f
        else if constexpr (FMT == codec::FmtUInt16)
            return unormDiv<65535>(reinterpret_cast<uint16_t const*>(t.data)[i]);   // == float(code) / 65535.f
        else
            return (reinterpret_cast<float const*>(t.data)[i] - t.lo) / (t.hi - t.lo);
    }

    struct Lut
    {
        float const* rgba;
        int32_t n;
    };

    __device__ __forceinline__ void lutLookup(Lut const& l, float v, float (&out)[4])
    {
        int32_t const i = texIndex(v, l.n);
        for (int k = 0; k < 4; ++k)
            out[k] = l.rgba[4 * i + k];
    }

    __device__ __forceinline__ float linearToSrgb(float x)
    {
        return x <= 0.0031308f ? 12.92f * x : 1.055f * rmath::pow(x, 1.f / 2.4f) - 0.055f;
    }

    // primary ray of pixel (x, y): jittered pixel position, thin lens (4 draws, always)
    __device__ __forceinline__ void primaryRay(vktHipRenderParams_t const& p, rmath::Rng& gen, int32_t x, int32_t y,
                                               V3& ori, V3& dir)
    {
        float const jx = gen.next(), jy = gen.next();
        float const sx = 2.f * (static_cast<float>(x) + jx) / static_cast<float>(p.width) - 1.f;
        float const sy = 2.f * (static_cast<float>(y) + jy) / static_cast<float>(p.height) - 1.f;
        V3 const W = v3(p.W);
        dir = normalize(W + v3(p.U) * sx + v3(p.V) * sy);
        ori = v3(p.eye);
        float const lu = gen.next(), lv = gen.next();
        if (p.lensRadius > 0.f)
        {
            V3 const focus = ori + dir * (p.focalDistance / dot(dir, W));
            float const r = p.lensRadius * sqrtf(lu);
            float s, c;
            rmath::sincos(6.28318531f * lv, s, c);
            ori = ori + v3(p.right) * (r * c) + v3(p.up) * (r * s);
            dir = normalize(focus - ori);
        }
    }

    // sky gradient of the reference (1 - t) * (1,1,1) + t * (.5,.7,1), t = y / height
    __device__ __forceinline__ void skyTimes(vktHipRenderParams_t const& p, int32_t y, V3 thr, float (&out)[4])
    {
        float const ty = static_cast<float>(y) / static_cast<float>(p.height);
        out[0] = ((1.f - ty) * 1.f + ty * 0.5f) * thr.x;
        out[1] = ((1.f - ty) * 1.f + ty * 0.7f) * thr.y;
        out[2] = ((1.f - ty) * 1.f + ty * 1.0f) * thr.z;
        out[3] = 1.f;
    }

    template <int FMT, int ALGO, bool BRICK>
    __device__ void samplePixel(vktHipRenderParams_t const& p, Tex const& tex, Lut const& lut, int32_t x, int32_t y,
                                uint32_t frame, float (&out)[4])
    {
        rmath::Rng gen(static_cast<uint32_t>(y) * static_cast<uint32_t>(p.width) + static_cast<uint32_t>(x), frame);
        V3 ori, dir;
        primaryRay(p, gen, x, y, ori, dir);
        V3 const box = v3(p.bbox);
        Hit h = intersectBox(ori, dir, box);
        float const v0 = 0.f;
        out[0] = out[1] = out[2] = out[3] = v0;

        if constexpr (ALGO == 0)   // ray marching
        {
            float t = h.tnear;
            V3 tc = div(ori + dir * t, box);
            V3 const inc = div(dir * p.dtRayMarching, box);
            float dst[4] = {0.f, 0.f, 0.f, 0.f};
            while (t < h.tfar)
            {
                float const voxel = texel<FMT, BRICK>(tex, tc);
                float col[4];
                if (lut.rgba)
                    lutLookup(lut, voxel, col);
                else
                    col[0] = col[1] = col[2] = col[3] = voxel;
                col[3] = 1.f - rmath::pow(1.f - col[3], p.dtRayMarching);
                col[0] *= col[3];
                col[1] *= col[3];
                col[2] *= col[3];
                float const rem = 1.f - dst[3];
                for (int k = 0; k < 4; ++k)
                    dst[k] += col[k] * rem;
                if (dst[3] == 1.f)
                    break;   // every further term is exactly 0 (see header)
                tc = tc + inc;
                t += p.dtRayMarching;
            }
            for (int k = 0; k < 4; ++k)
                out[k] = dst[k];
            return;
        }
        if constexpr (ALGO == 1)   // implicit iso
        {
            float t = h.tnear;
            V3 tc = div(ori + dir * t, box);
            V3 const inc = div(dir * p.dtImplicitIso, box);
            float last = -1e20f, isoT = -1e20f;
            float dst[4] = {0.f, 0.f, 0.f, 0.f};
            while (t < h.tfar)
            {
                float const voxel = texel<FMT, BRICK>(tex, tc);
                if (last >= -1e10f)
                {
                    for (int32_t i = 0; i < p.numIsoSurfaces; ++i)
                    {
                        float const iso = p.isoSurfaces[i];
                        if ((last <= iso && voxel >= iso) || (last >= iso && voxel <= iso))
                        {
                            float col[4];
                            if (lut.rgba)
                                lutLookup(lut, voxel, col);
                            else
                                col[0] = col[1] = col[2] = col[3] = voxel;
                            isoT = t;
                            float const d = 0.01f;
                            V3 s1{texel<FMT, BRICK>(tex, tc + V3{d, 0.f, 0.f}), texel<FMT, BRICK>(tex, tc + V3{0.f, d, 0.f}),
                                  texel<FMT, BRICK>(tex, tc + V3{0.f, 0.f, d})};
                            V3 s2{texel<FMT, BRICK>(tex, tc - V3{d, 0.f, 0.f}), texel<FMT, BRICK>(tex, tc - V3{0.f, d, 0.f}),
                                  texel<FMT, BRICK>(tex, tc - V3{0.f, 0.f, d})};
                            V3 const N = normalize(s2 - s1);
                            float const kd = fmaxf(0.f, dot(N, V3{-dir.x, -dir.y, -dir.z})) * voxel;
                            dst[0] = 0.2f + col[0] * kd;
                            dst[1] = 0.2f + col[1] * kd;
                            dst[2] = 0.2f + col[2] * kd;
                            dst[3] = 1.f;
                        }
                    }
                }
                if (isoT >= -1e10f)
                    break;
                tc = tc + inc;
                t += p.dtImplicitIso;
                last = voxel;
            }
            for (int k = 0; k < 4; ++k)
                out[k] = dst[k];
            return;
        }
        // multi-scattering
        V3 thr{1.f, 1.f, 1.f};
        float const mu_ = p.majorant;
        if (h.hit)
        {
            ori = ori + dir * h.tnear;
            h.tfar -= h.tnear;
            uint32_t bounce = 0;
            for (;;)
            {
                // sample_interaction: Woodcock tracking (:320-341)
                float t = 0.f;
                V3 pos;
                bool interact;
                for (;;)
                {
                    t -= rmath::ln(1.f - gen.next()) / mu_;
                    pos = ori + dir * t;
                    if (t >= h.tfar)
                    {
                        interact = false;
                        break;
                    }
                    float const voxel = texel<FMT, BRICK>(tex, div(pos, box));
                    float mu;
                    if (lut.rgba)
                    {
                        float col[4];
                        lutLookup(lut, voxel, col);
                        mu = col[3];
                    }
                    else
                        mu = voxel;
                    if (!(mu < gen.next() * mu_))
                    {
                        interact = true;
                        break;
                    }
                }
                if (!interact)
                    break;
                ori = pos;
                if (bounce++ >= 1024)
                {
                    thr = V3{0.f, 0.f, 0.f};
                    break;
                }
                float const voxel = texel<FMT, BRICK>(tex, div(ori, box));
                V3 alb;
                if (lut.rgba)
                {
                    float col[4];
                    lutLookup(lut, voxel, col);
                    alb = V3{col[0], col[1], col[2]};
                }
                else
                    alb = V3{voxel, voxel, voxel};
                thr = mul(thr, alb);
                float const prob = fmaxf(fmaxf(thr.x, thr.y), thr.z);
                if (prob < 0.2f)
                {
                    if (gen.next() > prob)
                    {
                        thr = V3{0.f, 0.f, 0.f};
                        break;
                    }
                    thr = V3{thr.x / prob, thr.y / prob, thr.z / prob};
                }
                // isotropic phase function
                float const cz = 1.f - 2.f * gen.next();
                float const sr = sqrtf(fmaxf(0.f, 1.f - cz * cz));
                float s, c;
                rmath::sincos(6.28318531f * gen.next(), s, c);
                dir = V3{sr * c, sr * s, cz};
                h = intersectBox(ori, dir, box);
            }
        }
        skyTimes(p, y, thr, out);
    }

    // 8x8-pixel tile per wave; a 256-thread workgroup covers 16x16 pixels
    template <int FMT, int ALGO, bool BRICK>
    __device__ __forceinline__ void renderPixel(vktHipRenderParams_t const& p, Tex const& tex, Lut const& lut,
                                                float* accum, float* color, int32_t numFrames)
    {
        int const t = threadIdx.x;
        int const wave = t >> 6, lane = t & 63;
        int32_t const x = static_cast<int32_t>(blockIdx.x) * 16 + (wave & 1) * 8 + (lane & 7);
        int32_t const y = static_cast<int32_t>(blockIdx.y) * 16 + (wave >> 1) * 8 + (lane >> 3);
        if (x >= p.width || y >= p.height)
            return;
        uint64_t const pix = static_cast<uint64_t>(y) * static_cast<uint64_t>(p.width) + static_cast<uint64_t>(x);
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        if (p.frameBegin > 0)
            for (int k = 0; k < 4; ++k)
                acc[k] = accum[4 * pix + k];
        for (int32_t f = 1; f <= numFrames; ++f)
        {
            uint32_t const frame = p.frameBegin + static_cast<uint32_t>(f);
            float s[4];
            samplePixel<FMT, ALGO, BRICK>(p, tex, lut, x, y, frame, s);
            float const alpha = 1.f / static_cast<float>(frame);
            for (int k = 0; k < 4; ++k)
                acc[k] = (1.f - alpha) * acc[k] + alpha * s[k];
        }
        for (int k = 0; k < 4; ++k)
            accum[4 * pix + k] = acc[k];
        if (color)
        {
            for (int k = 0; k < 3; ++k)
                color[4 * pix + k] = p.sRGB ? linearToSrgb(acc[k]) : acc[k];
            color[4 * pix + 3] = acc[3];
        }
    }

    // One kernel per algorithm, so each gets its own register allocation and occupancy.
    // Capping ray marching and multi-scattering at 4 waves per SIMD (amdgpu_waves_per_eu) keeps
    // the texel working set of the resident waves in the caches (config 5, 1024^3 UInt8:
    // RayMarching 2.50 -> 2.23 ms, MultiScattering 3.47 -> 3.29 ms per frame); ImplicitIso
    // runs best uncapped.
    template <int FMT>
    __global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 4))) void renderRayMarchingKernel(
        vktHipRenderParams_t p, Tex tex, Lut lut, float* accum, float* color, int32_t numFrames)
    {
        renderPixel<FMT, 0, false>(p, tex, lut, accum, color, numFrames);
    }

    template <int FMT>
    __global__ __launch_bounds__(kBlock) void renderImplicitIsoKernel(vktHipRenderParams_t p, Tex tex, Lut lut,
                                                                     float* accum, float* color, int32_t numFrames)
    {
        renderPixel<FMT, 1, false>(p, tex, lut, accum, color, numFrames);
    }

    template <int FMT, bool BRICK>
    __global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 4))) void renderMultiScatteringKernel(
        vktHipRenderParams_t p, Tex tex, Lut lut, float* accum, float* color, int32_t numFrames)
    {
        renderPixel<FMT, 2, BRICK>(p, tex, lut, accum, color, numFrames);
    }

} // hipk
} // vkt

using namespace vkt;
using namespace vkt::hipk;

extern "C" {

vktError vktHipRender(vktHipVolumeView_t volume, vktHipRenderParams_t const* params, float* accum, float* color,
                      int32_t numFrames)
{
    if (!params || !validView(volume))
        return rt::fail("vktHipRender: invalid arguments");
    vktHipRenderParams_t const& p = *params;
    if (p.width <= 0 || p.height <= 0 || numFrames < 0 || !accum)
        return rt::fail("vktHipRender: invalid viewport / buffers");
    if (p.algo < 0 || p.algo > 2)
        return rt::fail("vktHipRender: unknown render algorithm");
    if (p.numIsoSurfaces < 0 || p.numIsoSurfaces > 10 || (p.lut && p.lutSize <= 0))
        return rt::fail("vktHipRender: invalid iso surfaces / lookup table");
    if (volume.dimX <= 0 || volume.dimY <= 0 || volume.dimZ <= 0)
        return rt::fail("vktHipRender: empty volume");
    int32_t const fmt = volume.dataFormat;
    if (fmt != codec::FmtUInt8 && fmt != codec::FmtUInt16 && fmt != codec::FmtFloat32)
        return rt::fail("vktHipRender: volume format must be UInt8, UInt16 or Float32 (reference texel types)");
    if (numFrames == 0)
        return vktNoError;
    Tex tex{volume.data, volume.dimX, volume.dimY, volume.dimZ, fmt, volume.mappingLo, volume.mappingHi, 0, 0};
    hipStream_t s = rt::computeStream();
    Lut lut{p.lut, p.lutSize};
    dim3 grid(static_cast<unsigned>((p.width + 15) / 16), static_cast<unsigned>((p.height + 15) / 16));
    if (p.algo == 0 || p.algo == 1)
    {
#define VKT_RENDER(KERNEL)                                                                                          \
    do {                                                                                                            \
        if (fmt == codec::FmtUInt8)                                                                                 \
            hipLaunchKernelGGL(KERNEL<codec::FmtUInt8>, grid, dim3(kBlock), 0, s, p, tex, lut, accum, color, numFrames);   \
        else if (fmt == codec::FmtUInt16)                                                                           \
            hipLaunchKernelGGL(KERNEL<codec::FmtUInt16>, grid, dim3(kBlock), 0, s, p, tex, lut, accum, color, numFrames);  \
        else                                                                                                        \
            hipLaunchKernelGGL(KERNEL<codec::FmtFloat32>, grid, dim3(kBlock), 0, s, p, tex, lut, accum, color, numFrames); \
    } while (0)
        if (p.algo == 0)
            VKT_RENDER(renderRayMarchingKernel);
        else
            VKT_RENDER(renderImplicitIsoKernel);
#undef VKT_RENDER
        return rt::finishLaunch("Render_hip");
    }
    // Multi-scattering samples the volume at scattered, isotropic positions: it reads an 8^3-
    // brick copy made for the call (one streaming pass; config 5: 3.29 -> 2.92 ms per frame
    // over 8 frames), when the copy fits kMaxBrickBytes; else the dense volume.
    static rt::StreamScratch bricks;
    int32_t const nbx = (volume.dimX + 7) / 8, nby = (volume.dimY + 7) / 8, nbz = (volume.dimZ + 7) / 8;
    uint32_t const bpv = codec::bytesPerVoxel(fmt);
    uint64_t const brickRows = static_cast<uint64_t>(nbx) * static_cast<uint64_t>(nby) * static_cast<uint64_t>(nbz) * 64;
    uint8_t* b = brickRows * 8 * bpv <= kMaxBrickBytes && rt::knob(rt::Knob::RenderBricks) != 0
                     ? static_cast<uint8_t*>(bricks.acquire(brickRows * 8 * bpv, s))
                     : nullptr;
    if (!b)
        (void)hipGetLastError();   // a failed scratch allocation only means: render the dense volume
    if (b)
    {
        uint32_t const groupsX = static_cast<uint32_t>((nbx + 16 / bpv - 1) / (16 / bpv));
        unsigned const g = static_cast<unsigned>(static_cast<uint64_t>(groupsX) * nby * nbz);
#define VKT_BRICK(BPV)                                                                                           \
    hipLaunchKernelGGL(brickKernel<BPV>, dim3(g), dim3(256), 0, s, volume.data, b, volume.dimX, volume.dimY,     \
                       volume.dimZ, nbx, nby, groupsX)
        if (bpv == 1)
            VKT_BRICK(1);
        else if (bpv == 2)
            VKT_BRICK(2);
        else
            VKT_BRICK(4);
#undef VKT_BRICK
        tex.data = b;
        tex.nbx = nbx;
        tex.nby = nby;
    }
#define VKT_RENDER_MS(BRICK)                                                                                      \
    do {                                                                                                          \
        if (fmt == codec::FmtUInt8)                                                                               \
            hipLaunchKernelGGL((renderMultiScatteringKernel<codec::FmtUInt8, BRICK>), grid, dim3(kBlock), 0, s, p, tex, lut, accum, color, numFrames); \
        else if (fmt == codec::FmtUInt16)                                                                         \
            hipLaunchKernelGGL((renderMultiScatteringKernel<codec::FmtUInt16, BRICK>), grid, dim3(kBlock), 0, s, p, tex, lut, accum, color, numFrames); \
        else                                                                                                      \
            hipLaunchKernelGGL((renderMultiScatteringKernel<codec::FmtFloat32, BRICK>), grid, dim3(kBlock), 0, s, p, tex, lut, accum, color, numFrames); \
    } while (0)
    if (b)
    {
        VKT_RENDER_MS(true);
        bricks.release(s);
    }
    else
        VKT_RENDER_MS(false);
#undef VKT_RENDER_MS
    return rt::finishLaunch("Render_hip");
}

} // extern "C"
