// Pointwise.hip -- gfx950 kernels and backend entry points for FillRange, CopyRange, the
// ten arithmetic ops, format conversion, MemsetRange and the synthetic-input generator.
//
// Replaces the reference's FillRange_cuda (src/vkt/Fill_cuda.cu:22-55, which is never
// reached for SV because Call() has no GPU branch, src/vkt/Callable.cpp:53-66),
// CopyRange_cuda (src/vkt/Copy_cuda.cu:12-111), ArithmeticOp_kernel x10
// (src/vkt/Arithmetic_cuda.cu:12-296) and MemsetRange_cuda (src/vkt/Memory_cuda.cu:15-49).
// Semantics follow the SERIAL path, not the CUDA path:
// arithmetic writes dst[x + dstOffset] at absolute x; CopyRange clamps source indices.
//
// Roofline: every op here is HBM-bound.  Algorithmic bytes per voxel of the range:
// Fill b_dst; Copy b_src + b_dst; arithmetic b_s1 + b_s2 + b_dst (6 B for UInt16).

#include "PointwiseOps.hpp"
#include "../runtime/Runtime.hpp"
#include "volkit_hip.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace vkt
{
namespace hipk
{
    // ---- planning --------------------------------------------------------------------
    PwPlan planPointwise(int ns, Operand d, Operand s1, Operand s2, int64_t nx, int64_t ny, int64_t nz)
    {
        PwPlan p;
        p.d = d;
        p.s1 = s1;
        p.s2 = s2;
        p.g.nx = nx;
        p.g.ny = ny;
        p.g.nz = nz;
        Operand* ops[3] = {&p.d, &p.s1, &p.s2};
        int nops = ns + 1;

        bool vec = true, uniform = true, anyClamp = false, gen = true;
        uint32_t bpv = p.d.bpv;
        for (int i = 0; i < nops; ++i)
        {
            Operand& o = *ops[i];
            int64_t dx = o.dims[0], dy = o.dims[1];
            o.base = (static_cast<int64_t>(o.origin[2]) * dy + o.origin[1]) * dx + o.origin[0];
            o.sy = dx;
            o.sz = dx * dy;
            if (o.clamp || o.bpv != bpv)
                vec = false;
            uniform = uniform && o.bpv == bpv;
            anyClamp = anyClamp || o.clamp;
            // general path: 1/2/4-byte voxels at voxel-aligned addresses
            gen = gen && (o.bpv == 1 || o.bpv == 2 || o.bpv == 4) &&
                  reinterpret_cast<uintptr_t>(o.data) % o.bpv == 0;
        }

        // collapse rows that are contiguous in every operand (not when a source clamps: its
        // rows repeat at the border)
        int64_t vnx = nx, vny = ny, vnz = nz;
        bool mergeY = vny > 1 && !anyClamp;
        for (int i = 0; i < nops && mergeY; ++i)
            mergeY = ops[i]->sy == vnx;
        if (mergeY)
        {
            vnx *= vny;
            vny = 1;
        }
        if (vny == 1 && vnz > 1 && !anyClamp)
        {
            bool mergeZ = true;
            for (int i = 0; i < nops && mergeZ; ++i)
                mergeZ = ops[i]->sz == vnx;
            if (mergeZ)
            {
                vnx *= vnz;
                vnz = 1;
            }
        }
        p.g.vnx = vnx;
        p.g.vny = vny;
        p.g.vnz = vnz;
        // common misalignment phase of the row starts: a scalar head of (8 - phase) % 8 voxels
        // brings every operand to an 8-voxel boundary at the same x
        int64_t const phase = ops[0]->base & 7;
        for (int i = 1; i < nops; ++i)
            if ((ops[i]->base & 7) != phase)
                vec = false;
        int64_t head = (8 - phase) & 7;
        if (head > vnx)
            head = vnx;
        p.g.vhead = head;
        p.g.vnx8 = head + ((vnx - head) & ~int64_t(7));
        // Several rows: no scalar row edges.  Each row is covered by whole items from the
        // 8-aligned voxel at or below its start (vhead = -phase); items straddling a row end load
        // whole vectors and store only the row's voxels.  The straddling loads stay inside each
        // operand's allocation: the vector path needs sy and sz multiples of 8 for several rows
        // (checked below), so 8-aligned row supersets never leave the row's plane.  A separate
        // scalar edge pass over every row cost ~20 % (800^3 sub-box of 1024^3 at x0 = 100:
        // 0.666 ms vs 0.533 ms at x0 = 96, where rows have no edges).
        p.g.padded = 0;
        p.g.merge = 0;
        p.g.vhead0 = p.g.vend0 = 0;
        if (vny * vnz > 1 && rt::knob(rt::Knob::PointwisePaddedRows) != 0)
        {
            p.g.padded = 1;
            p.g.vhead = -phase;
            p.g.vnx8 = -phase + ((phase + vnx + 7) & ~int64_t(7));
        }
        uint64_t const vecItems = static_cast<uint64_t>((p.g.vnx8 - p.g.vhead) / 8) * static_cast<uint64_t>(vny) * vnz;
        uint64_t const total = static_cast<uint64_t>(nx) * ny * nz;
        p.g.fast32 = vecItems < (1ull << 32) && total < (1ull << 32) ? 1 : 0;
        p.g.divCpr = makeFastDiv(static_cast<uint32_t>((p.g.vnx8 - p.g.vhead) / 8 > 0 ? (p.g.vnx8 - p.g.vhead) / 8 : 1));
        p.g.divVny = makeFastDiv(static_cast<uint32_t>(vny));
        p.g.divNx = makeFastDiv(static_cast<uint32_t>(nx));
        p.g.divNy = makeFastDiv(static_cast<uint32_t>(ny));

        // 8-voxel chunks must start aligned in every operand
        uint64_t needAlign = bpv == 1 ? 8u : 16u;
        for (int i = 0; i < nops && vec; ++i)
        {
            Operand const& o = *ops[i];
            if ((reinterpret_cast<uintptr_t>(o.data) % needAlign) != 0)
                vec = false;
            if (vny > 1 && (o.sy & 7) != 0)
                vec = false;
            if (vnz > 1 && (o.sz & 7) != 0)
                vec = false;
        }
        if (!(bpv == 1 || bpv == 2 || bpv == 4))
            vec = false;
        p.vec = vec;
        p.bpv = bpv;

        // Padded rows with 64-B sector completion (a partly written sector costs HBM a
        // read-modify-write): the items extend to the destination's sector
        // boundaries; chunks outside the box are its own bytes, loaded and stored back whole;
        // sources are read only inside the original 8-aligned row items.  Needs one sector phase
        // for every row, >= 64-B gaps between box rows and planes (no sector holds two rows'
        // voxels) and a 64-B aligned destination (every sector inside it).  Copies, conversions
        // and fills only: in-process A/B on an 800^3 sub-box of 1024^3 at x0 = 100, CopyRange
        // 0.480 -> 0.422 ms, SafeSumRange 0.627 -> 0.649 ms (its partly read source sectors stay).
        // Not for UInt8 here: its per-item loop (8 B per lane) lost the batching of its loads to
        // the conditional destination-chunk loads -- 800^3 sub-box copy x 0..800 0.250 -> 0.378
        // ms; UInt8 rows complete their sectors on the 16-voxel pair grid below.
        // (3-stream ops: 4-byte voxels on the contiguous-lane halves only -- 800^3 sub-box of
        // 1024^3 at x0 = 100, Float32 SumRange 1.218 -> 1.147 ms, while UInt16 lost again, 0.624 ->
        // 0.645 ms, profiles/r03/merge3_ab.jsonl; knob value 2 forces it for A/B)
        bool const merge3 = rt::knob(rt::Knob::PointwiseMergeSectors) == 2 ||
                            (bpv == 4 && rt::knob(rt::Knob::PointwiseF32Halves) != 0);
        if (vec && p.g.padded && (ns <= 1 || merge3) && bpv != 1)
        {
            int64_t const bd = bpv;
            int64_t const sv = 64 / bd;
            uint64_t const dBytes = static_cast<uint64_t>(p.d.dims[0]) * static_cast<uint64_t>(p.d.dims[1]) *
                                    static_cast<uint64_t>(p.d.dims[2]) * bpv;
            bool const ok = rt::knob(rt::Knob::PointwiseMergeSectors) != 0 &&
                            reinterpret_cast<uintptr_t>(p.d.data) % 64 == 0 && dBytes % 64 == 0 &&
                            (vny <= 1 || ((p.d.sy * bd) % 64 == 0 && (p.d.sy - vnx) * bd >= 64)) &&
                            (vnz <= 1 || ((p.d.sz * bd) % 64 == 0 && (p.d.sz - (vny - 1) * p.d.sy - vnx) * bd >= 64));
            int64_t const ph = static_cast<int64_t>(static_cast<uint64_t>(p.d.base) % static_cast<uint64_t>(sv));
            if (ok && (ph != 0 || (ph + vnx) % sv != 0))
            {
                p.g.merge = 1;
                p.g.vhead0 = p.g.vhead;
                p.g.vend0 = p.g.vnx8;
                p.g.vhead = -ph;
                p.g.vnx8 = -ph + (ph + vnx + sv - 1) / sv * sv;
                uint64_t const items = static_cast<uint64_t>((p.g.vnx8 - p.g.vhead) / 8) * static_cast<uint64_t>(vny) * vnz;
                p.g.fast32 = items < (1ull << 32) && total < (1ull << 32) ? 1 : 0;
                p.g.divCpr = makeFastDiv(static_cast<uint32_t>((p.g.vnx8 - p.g.vhead) / 8));
            }
        }
        // Rows that start and end on the 8-voxel grid and need no sector completion have no
        // edges: the padded form covers them with the same items, but the flag kept 4-byte
        // multi-row boxes off the contiguous-lane shape (Pointwise.hpp) -- 800^3 sub-box of
        // 1024^3 Float32 Copy x 0..800 0.853 -> 0.753 ms with the flag off (u8_f32 probe, r02).
        if (p.g.padded && !p.g.merge && phase == 0 && vnx % 8 == 0)
            p.g.padded = 0;
        // UInt8 rows on a 16-voxel grid (pair16, Pointwise.hpp): one 16-B access per lane for
        // two items instead of one 8-B access per item, byte-range stores at the row ends.
        // Needs every operand's rows at one phase mod 16 and 16-B aligned row supersets (the
        // superset stays inside the volume's row: pitches are multiples of 16).
        p.g.pair16 = 0;
        p.g.f32halves = bpv == 4 && rt::knob(rt::Knob::PointwiseF32Halves) != 0 ? 1 : 0;
        if (vec && bpv == 1 && vny * vnz > 1 && rt::knob(rt::Knob::PointwisePaddedRows) != 0 &&
            rt::knob(rt::Knob::PointwiseU8Pairs) != 0)
        {
            int64_t const ph16 = ops[0]->base & 15;
            bool ok = true;
            for (int i = 0; i < nops && ok; ++i)
            {
                Operand const& o = *ops[i];
                ok = (o.base & 15) == ph16 && reinterpret_cast<uintptr_t>(o.data) % 16 == 0 &&
                     (vny <= 1 || (o.sy & 15) == 0) && (vnz <= 1 || (o.sz & 15) == 0);
            }
            // Measured (800^3 sub-boxes of 1024^3, profiles/r03/subrows_*): copies gain everywhere
            // (x0 = 100 0.422 -> 0.295 ms, x 0..800 0.239 -> 0.205 ms); the 3-stream ops gain only
            // where row ends need masked stores (SumRange x0 = 100 0.425 -> 0.389 ms) and lost on
            // whole-x planes (0.328 -> 0.375 ms), so edge-free 3-stream boxes keep the per-item
            // loop (knob value 2 forces pairs for A/B)
            bool const edges16 = ph16 != 0 || vnx % 16 != 0;
            if (ok && (ns <= 1 || edges16 || rt::knob(rt::Knob::PointwiseU8Pairs) == 2))
            {
                p.g.pair16 = 1;
                p.g.padded = edges16 ? 1 : 0;
                p.g.vhead = -ph16;
                p.g.vnx8 = -ph16 + ((ph16 + vnx + 15) & ~int64_t(15));
                // 64-B sector completion for the pairs (as the aligned path above for 2- and
                // 4-byte voxels): rows extended to whole destination sectors, sources read inside
                // the 16-voxel row grid only.  Every op: in-process A/B on an 800^3 sub-box of
                // 1024^3 at x0 = 100 (profiles/r03/u8_merge_ab.jsonl), CopyRange 0.297 -> 0.275 ms,
                // SumRange 0.424 -> 0.376 ms (unlike UInt16, where the 3-stream ops lost).
                int64_t const ph64 = static_cast<int64_t>(static_cast<uint64_t>(p.d.base) % 64u);
                uint64_t const dBytes = static_cast<uint64_t>(p.d.dims[0]) * static_cast<uint64_t>(p.d.dims[1]) *
                                        static_cast<uint64_t>(p.d.dims[2]);
                int64_t const mk = rt::knob(rt::Knob::PointwiseMergeSectors);
                bool const merge = edges16 && mk != 0 &&
                                   reinterpret_cast<uintptr_t>(p.d.data) % 64 == 0 && dBytes % 64 == 0 &&
                                   (vny <= 1 || (p.d.sy % 64 == 0 && p.d.sy - vnx >= 64)) &&
                                   (vnz <= 1 || (p.d.sz % 64 == 0 && p.d.sz - (vny - 1) * p.d.sy - vnx >= 64)) &&
                                   (ph64 != 0 || (ph64 + vnx) % 64 != 0);
                if (merge)
                {
                    p.g.merge = 1;
                    p.g.vhead0 = p.g.vhead;
                    p.g.vend0 = p.g.vnx8;
                    p.g.vhead = -ph64;
                    p.g.vnx8 = -ph64 + (ph64 + vnx + 63) / 64 * 64;
                }
                uint64_t const items = static_cast<uint64_t>((p.g.vnx8 - p.g.vhead) / 8) * static_cast<uint64_t>(vny) * vnz;
                p.g.fast32 = items < (1ull << 32) && total < (1ull << 32) ? 1 : 0;
                p.g.divCpr = makeFastDiv(static_cast<uint32_t>((p.g.vnx8 - p.g.vhead) / 8));
            }
        }

        // general vector path (Pointwise.hpp): any phase, pitch or clamp; voxel sizes may differ
        // (launchPointwise takes it for uniform sizes, convertBox for mixed ones)
        GenGeom& gg = p.gg;
        gg.vnx = vnx;
        gg.vny = vny;
        gg.vnz = vnz;
        gg.cpr = static_cast<uint64_t>((vnx + 14) / 8);
        uint64_t const rows = static_cast<uint64_t>(vny) * static_cast<uint64_t>(vnz);
        gg.items = rows * gg.cpr;
        gg.dph = static_cast<int32_t>((reinterpret_cast<uintptr_t>(p.d.data) / p.d.bpv) & 7);
        gg.fast32 = gg.items < (1ull << 32) ? 1 : 0;
        gg.anyClamp = anyClamp ? 1 : 0;
        // 32-bit addressing: every byte of each operand at an offset < 2^32 from its 16-B aligned
        // base (the window words, merged chunks and stores address only valid voxels' words; voxel
        // indices times B stay < 2^32), pitches and box extents fit the 24-bit multiplies, items
        // < 2^32.  A 4 GiB operand (1024^3 Float32) qualifies when 16-B aligned: it had been sent to
        // the 64-bit path (~2.5x the VALU, per-voxel row-end stores, no sector completion) by a
        // 64-B margin no access needs.
        {
            bool fast = gg.items < (1ull << 32) && vny < (1ll << 24) && vnz < (1ll << 24);
            for (int i = 0; i < nops && fast; ++i)
            {
                Operand const& o = *ops[i];
                uint64_t const bytes = static_cast<uint64_t>(o.dims[0]) * static_cast<uint64_t>(o.dims[1]) *
                                       static_cast<uint64_t>(o.dims[2]) * o.bpv;
                uint64_t const mis = reinterpret_cast<uintptr_t>(o.data) & 15u;
                fast = mis + bytes <= (1ull << 32) && (o.clamp || o.base >= 0) &&
                       (vny <= 1 || (o.sy < (1ll << 24) && o.dims[0] < (1 << 24))) &&
                       (vnz <= 1 || o.sz < (1ll << 24)) && (!o.clamp || static_cast<int64_t>(o.dims[0]) * o.dims[1] < (1ll << 24));
            }
            gg.fast = fast && rt::knob(rt::Knob::PointwiseGeneral32) != 0 ? 1 : 0;
        }
        // 64-B sector completion at the row ends (measured on MI355X: a copy of 1024^2 rows of
        // 896 UInt16 voxels takes 0.61 ms when the rows end on a 64-B boundary and 0.78 ms when
        // they end one voxel short -- a partly written 64-B sector costs HBM a read-modify-write).
        // Items then cover whole sectors: the voxels outside the box are rewritten with the
        // destination's own bytes.  Only where no sector holds box voxels of two rows (gaps of
        // >= 64 B between consecutive box rows and planes) and every sector lies inside the
        // destination volume (64-B aligned start and size).
        {
            uint32_t const bd = p.d.bpv;
            int64_t const sv = 64 / bd;
            uint64_t const dBytes = static_cast<uint64_t>(p.d.dims[0]) * static_cast<uint64_t>(p.d.dims[1]) *
                                    static_cast<uint64_t>(p.d.dims[2]) * bd;
            // The 3-stream ops complete their sectors too (round 4, with one store statement per
            // item; round 3 had measured them slower here): 800^3 sub-box at x0 = 100, SumRange
            // dstOffset -97 Float32 1.271 -> 1.232 ms, UInt16 0.684 -> 0.632 ms, UInt8 0.435 ->
            // 0.426 ms (profiles/r04/f32m3.jsonl, m3ab.jsonl).  (The aligned path's 3-stream
            // completion, merge3 above, still loses for UInt16: 0.623 -> 0.644 ms.)
            bool merge = gg.fast &&
                         rt::knob(rt::Knob::PointwiseMergeSectors) != 0 &&
                         reinterpret_cast<uintptr_t>(p.d.data) % 64 == 0 && dBytes % 64 == 0;
            if (merge && vny > 1)
                merge = (p.d.sy - vnx) * static_cast<int64_t>(bd) >= 64;
            if (merge && vnz > 1)
                merge = (p.d.sz - (vny - 1) * p.d.sy - vnx) * static_cast<int64_t>(bd) >= 64;
            gg.merge = merge ? 1 : 0;
            gg.sv = static_cast<int32_t>(sv);
            gg.dph64 = static_cast<int32_t>((reinterpret_cast<uintptr_t>(p.d.data) / bd) % static_cast<uint64_t>(sv));
            if (merge)
            {
                gg.cpr = static_cast<uint64_t>(((vnx + sv - 1 + sv - 1) / sv) * sv / 8);
                gg.items = rows * gg.cpr;
                gg.fast32 = gg.items < (1ull << 32) ? 1 : 0;
                gg.fast = gg.fast && gg.fast32;
                gg.merge = gg.fast;
                gg.divCpr = makeFastDiv(static_cast<uint32_t>(gg.cpr));
            }
        }
        // 1- or 4-byte voxels in every operand on the 32-bit path: 16-B items of 16 / B voxels
        // (Pointwise.hpp pointwiseGenSpanFast16); the same row cover and sector completion in
        // units of 16 / B voxels
        gg.wide = 0;
        {
            uint32_t const B = p.d.bpv;
            bool const same = (ns < 1 || p.s1.bpv == B) && (ns < 2 || p.s2.bpv == B);
            // Float32 (knob pointwise.f32_wide: 1 every op, 2 ops of at most one source): after the
            // round-4 single store statement the 16-B items win for copies (800^3 at x0 = 100 ->
            // dst 0 0.821 -> 0.768 ms, -> dst x0 = 3 0.884 -> 0.803 ms, 1021 x 1024^2 x0 = 3 -> 0
            // 1.722 -> 1.470 ms) and still lose for SumRange dstOffset -97 (1.239 -> 1.257 ms),
            // profiles/r04/configs_bench.jsonl f32gen / f32dw
            int64_t const f32w = rt::knob(rt::Knob::PointwiseF32Wide);
            bool const on = B == 1 ? rt::knob(rt::Knob::PointwiseU8Wide) != 0
                                   : B == 4 && (f32w == 1 || (f32w == 2 && ns < 2));
            if (gg.fast && same && on)
            {
                int64_t const V = 16 / B, sv = 64 / B;
                uint64_t const cpr = gg.merge ? static_cast<uint64_t>(((vnx + sv - 1 + sv - 1) / sv) * sv / V)
                                              : static_cast<uint64_t>((vnx + 2 * V - 2) / V);
                uint64_t const items = rows * cpr;
                if (items < (1ull << 32))
                {
                    gg.wide = 1;
                    gg.cpr = cpr;
                    gg.items = items;
                    gg.dph = static_cast<int32_t>((reinterpret_cast<uintptr_t>(p.d.data) / B) & static_cast<uint64_t>(V - 1));
                }
            }
        }
        gg.divCpr = makeFastDiv(static_cast<uint32_t>(gg.cpr));
        gg.divVny = makeFastDiv(static_cast<uint32_t>(vny));
        // whole-dword window offsets (4-byte voxels at 4-B aligned addresses; knob pointwise.dword_shift)
        {
            bool dw = p.d.bpv == 4 && rt::knob(rt::Knob::PointwiseDwordShift) != 0;
            for (int i = 0; i < nops && dw; ++i)
                dw = ops[i]->bpv == 4 && reinterpret_cast<uintptr_t>(ops[i]->data) % 4 == 0;
            gg.dword = dw ? 1 : 0;
        }
        // UInt8 copies / fills over multi-row boxes of long rows without row edges (e.g. whole-x
        // planes of a y sub-range) run faster on the general path's wide items than on the pair
        // grid: 800 planes of 1024 x 800 voxels 0.254 -> 0.226 ms, while 800-voxel rows lost 3 %
        // and rows with edges tied (profiles/r03/u8_general_ab.jsonl; the 3-stream ops lost on the
        // general path everywhere).  Knob pointwise.u8_pairs = 3 sends every UInt8 multi-row box there (A/B).
        {
            int64_t const k = rt::knob(rt::Knob::PointwiseU8Pairs);
            bool const edgeFreeLong = ns <= 1 && (ops[0]->base & 15) == 0 && vnx % 16 == 0 && vnx >= 4096;
            if (vec && bpv == 1 && vny * vnz > 1 && gg.wide && (k == 3 || (k == 1 && edgeFreeLong)))
                vec = false;
        }
        p.vec = vec;
        p.gen = gen && !vec && rt::knob(rt::Knob::PointwiseGeneral) != 0;
        p.uniform = uniform;
        static bool const debugPlan = std::getenv("VKT_DEBUG_PLAN") != nullptr;   // diagnostics: the chosen path
        if (debugPlan)
            std::fprintf(stderr,
                         "VKT_PLAN ns=%d bpv=%u box=%lldx%lldx%lld rows=%lldx%lldx%lld bases=%lld/%lld/%lld vec=%d "
                         "padded=%d merge=%d pair16=%d gen=%d gg.fast=%d gg.merge=%d gg.wide=%d gg.dword=%d "
                         "gg.cpr=%llu gg.items=%llu\n",
                         ns, bpv, static_cast<long long>(nx), static_cast<long long>(ny), static_cast<long long>(nz),
                         static_cast<long long>(vnx), static_cast<long long>(vny), static_cast<long long>(vnz),
                         static_cast<long long>(p.d.base), static_cast<long long>(p.s1.base),
                         static_cast<long long>(p.s2.base), p.vec ? 1 : 0, p.g.padded, p.g.merge, p.g.pair16,
                         p.gen ? 1 : 0, gg.fast, gg.merge, gg.wide, gg.dword, static_cast<unsigned long long>(gg.cpr),
                         static_cast<unsigned long long>(gg.items));
        return p;
    }

    // ---- validation helpers ------------------------------------------------------------
    bool validView(vktHipVolumeView_t const& v)
    {
        if (v.dimX < 0 || v.dimY < 0 || v.dimZ < 0)
            return false;
        uint32_t b = codec::bytesPerVoxel(v.dataFormat);
        if (b == 255u)
            return false;
        if (v.data == nullptr && static_cast<int64_t>(v.dimX) * v.dimY * v.dimZ > 0)
            return false;
        return true;
    }

    uint64_t viewBytes(vktHipVolumeView_t const& v)
    {
        return static_cast<uint64_t>(v.dimX) * static_cast<uint64_t>(v.dimY) * static_cast<uint64_t>(v.dimZ) *
               codec::bytesPerVoxel(v.dataFormat);
    }

    bool boxInside(vktHipVolumeView_t const& v, vktVec3i_t o, int64_t nx, int64_t ny, int64_t nz)
    {
        return o.x >= 0 && o.y >= 0 && o.z >= 0 && o.x + nx <= v.dimX && o.y + ny <= v.dimY && o.z + nz <= v.dimZ;
    }

    bool overlaps(vktHipVolumeView_t const& a, vktHipVolumeView_t const& b)
    {
        uintptr_t a0 = reinterpret_cast<uintptr_t>(a.data), a1 = a0 + viewBytes(a);
        uintptr_t b0 = reinterpret_cast<uintptr_t>(b.data), b1 = b0 + viewBytes(b);
        return a0 < b1 && b0 < a1;
    }

    Operand makeOperand(vktHipVolumeView_t const& v, vktVec3i_t origin, bool clamp)
    {
        Operand o{};
        o.data = v.data;
        o.dims[0] = v.dimX;
        o.dims[1] = v.dimY;
        o.dims[2] = v.dimZ;
        o.origin[0] = origin.x;
        o.origin[1] = origin.y;
        o.origin[2] = origin.z;
        o.clamp = clamp ? 1 : 0;
        o.fmt = v.dataFormat;
        o.bpv = codec::bytesPerVoxel(v.dataFormat);
        o.lo = v.mappingLo;
        o.hi = v.mappingHi;
        return o;
    }

    // Formats whose encode writes nothing (reference MapVoxelImpl switch has no case).
    bool encodeWrites(int32_t fmt)
    {
        return fmt == codec::FmtInt16 || fmt == codec::FmtUInt8 || fmt == codec::FmtUInt16 ||
               fmt == codec::FmtUInt32 || fmt == codec::FmtFloat32;
    }

    // ---- conversion (shared with Resample's same-dims branch) ---------------------------
    // Source and destination voxel sizes differ: general vector path, formats fixed at compile
    // time for the UInt8 / UInt16 / Float32 pairs, run-time formats otherwise.
    template <int FS, int FD, int BS, int BD>
    vktError convertFixed(PwPlan const& p, float slo, float shi, MapParams const& dm, hipStream_t s)
    {
        return dm.rangeIsPow2 ? launchGen<1, BD, BS, BS>(p, ConvertF<FS, FD, 1>{FS, FD, slo, shi, dm}, s)
                              : launchGen<1, BD, BS, BS>(p, ConvertF<FS, FD, 2>{FS, FD, slo, shi, dm}, s);
    }

    template <int BS, int BD>
    vktError convertDyn(PwPlan const& p, int32_t fs, int32_t fd, float slo, float shi, MapParams const& dm,
                        hipStream_t s)
    {
        return launchGen<1, BD, BS, BS>(p, ConvertF<kDyn, kDyn>{fs, fd, slo, shi, dm}, s);
    }

    vktError convertMixed(PwPlan const& p, int32_t fs, int32_t fd, float slo, float shi, MapParams const& dm,
                          hipStream_t s)
    {
        constexpr int U8 = codec::FmtUInt8, U16 = codec::FmtUInt16, F32 = codec::FmtFloat32;
        if (fs == U8 && fd == U16) return convertFixed<U8, U16, 1, 2>(p, slo, shi, dm, s);
        if (fs == U8 && fd == F32) return convertFixed<U8, F32, 1, 4>(p, slo, shi, dm, s);
        if (fs == U16 && fd == U8) return convertFixed<U16, U8, 2, 1>(p, slo, shi, dm, s);
        if (fs == U16 && fd == F32) return convertFixed<U16, F32, 2, 4>(p, slo, shi, dm, s);
        if (fs == F32 && fd == U8) return convertFixed<F32, U8, 4, 1>(p, slo, shi, dm, s);
        if (fs == F32 && fd == U16) return convertFixed<F32, U16, 4, 2>(p, slo, shi, dm, s);
        uint32_t const bs = p.s1.bpv, bd = p.d.bpv;
        if (bs == 1 && bd == 2) return convertDyn<1, 2>(p, fs, fd, slo, shi, dm, s);
        if (bs == 1 && bd == 4) return convertDyn<1, 4>(p, fs, fd, slo, shi, dm, s);
        if (bs == 2 && bd == 1) return convertDyn<2, 1>(p, fs, fd, slo, shi, dm, s);
        if (bs == 2 && bd == 4) return convertDyn<2, 4>(p, fs, fd, slo, shi, dm, s);
        if (bs == 4 && bd == 1) return convertDyn<4, 1>(p, fs, fd, slo, shi, dm, s);
        return convertDyn<4, 2>(p, fs, fd, slo, shi, dm, s);
    }

    vktError convertBox(vktHipVolumeView_t dst, vktHipVolumeView_t src, vktVec3i_t srcOrigin, bool clampSrc,
                        vktVec3i_t dstOrigin, int64_t nx, int64_t ny, int64_t nz)
    {
        hipStream_t s = rt::computeStream();
        Operand od = makeOperand(dst, dstOrigin, false);
        Operand os = makeOperand(src, srcOrigin, clampSrc);
        PwPlan p = planPointwise(1, od, os, os, nx, ny, nz);
        MapParams dm = codec::makeMapParams(dst.mappingLo, dst.mappingHi);
        int32_t fs = src.dataFormat, fd = dst.dataFormat;
        if ((p.vec || (p.gen && p.uniform)) && fs == fd)
        {
            if (fs == codec::FmtUInt8)
                return dm.rangeIsPow2 ? launchPointwise<1, 1>(p, ConvertF<codec::FmtUInt8, codec::FmtUInt8, 1>{fs, fd, src.mappingLo, src.mappingHi, dm}, s)
                                      : launchPointwise<1, 1>(p, ConvertF<codec::FmtUInt8, codec::FmtUInt8, 2>{fs, fd, src.mappingLo, src.mappingHi, dm}, s);
            if (fs == codec::FmtUInt16)
                return dm.rangeIsPow2 ? launchPointwise<1, 2>(p, ConvertF<codec::FmtUInt16, codec::FmtUInt16, 1>{fs, fd, src.mappingLo, src.mappingHi, dm}, s)
                                      : launchPointwise<1, 2>(p, ConvertF<codec::FmtUInt16, codec::FmtUInt16, 2>{fs, fd, src.mappingLo, src.mappingHi, dm}, s);
            if (fs == codec::FmtFloat32)
                return dm.rangeIsPow2 ? launchPointwise<1, 4>(p, ConvertF<codec::FmtFloat32, codec::FmtFloat32, 1>{fs, fd, src.mappingLo, src.mappingHi, dm}, s)
                                      : launchPointwise<1, 4>(p, ConvertF<codec::FmtFloat32, codec::FmtFloat32, 2>{fs, fd, src.mappingLo, src.mappingHi, dm}, s);
        }
        if (p.gen && !p.uniform)
            return convertMixed(p, fs, fd, src.mappingLo, src.mappingHi, dm, s);
        return launchByBpv<1>(p, ConvertF<kDyn, kDyn>{fs, fd, src.mappingLo, src.mappingHi, dm}, s);
    }

    // ---- MemsetRange ---------------------------------------------------------------
    // dst byte k (k < nbytes = whole patterns only) = pattern[k % psize] (reference
    // MemsetRange_serial, src/vkt/Memory_serial.hpp:24-37).  One kernel for every pattern size
    // and alignment: the bytes before dst's first 128-byte line and after the last whole
    // 16-byte vector go byte by byte; every 16-byte vector in between is ONE aligned store of
    // bytes [phase, phase + 16) of the *extended* pattern E (E[k] = pattern[k % psize], length
    // psize + 15, staged in LDS), phase = (vector offset) % psize -- no per-byte modulo.  One
    // 256-lane workgroup per 4 KiB (the pure-store quantum of §4.1).  Patterns whose E fits the
    // kernel argument (psize <= 241) need no device copy; larger ones are uploaded once per
    // call into the call site's grow-only scratch and staged into LDS (psize + 15 <= 48 KiB)
    // or read from it (L2-resident) beyond that.
    constexpr uint32_t kPatArgBytes = 256;
    constexpr uint32_t kPatLdsBytes = 48 * 1024;
    constexpr uint64_t kMemsetBlocksPerLaunch = 1ull << 20;

    struct PatternArg
    {
        uint8_t e[kPatArgBytes];
    };

    // SRC: 0 E in the kernel argument, 1 E in global memory staged to LDS, 2 E read from global
    template <int SRC>
    __global__ __launch_bounds__(kBlock) void memsetPatternKernel(uint8_t* dst, uint64_t nbytes, uint64_t head,
                                                                  uint64_t nvec, uint64_t vbase, uint32_t psize,
                                                                  uint32_t elen, PatternArg arg,
                                                                  uint8_t const* gpat)
    {
        extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
        uint8_t const* e = lds;
        if constexpr (SRC == 2)
            e = gpat;
        else
        {
            for (uint32_t k = threadIdx.x; k < elen; k += kBlock)
                lds[k] = SRC == 0 ? arg.e[k] : gpat[k];
            __syncthreads();
        }
        uint64_t const v = vbase + blockIdx.x * static_cast<uint64_t>(kBlock) + threadIdx.x;
        if (v < nvec)
        {
            uint64_t const off = head + 16 * v;
            uint32_t const ph = static_cast<uint32_t>(off % psize);
            u32x4 w;
            if constexpr (SRC == 2)
            {
                uint8_t b[16];
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    b[i] = e[ph + i];
                __builtin_memcpy(&w, b, 16);
            }
            else
                w = *reinterpret_cast<u32x4 const*>(e + ph);   // unaligned ds_read_b128 (gfx950 LDS)
            __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(dst + off));
        }
        // the bytes outside the vector span: the first block's lanes take the head, the last
        // launch's last block the tail
        if (vbase == 0 && blockIdx.x == 0 && threadIdx.x < head)
            dst[threadIdx.x] = e[threadIdx.x % psize];
        uint64_t const tail0 = head + 16 * nvec;
        if (vbase + (static_cast<uint64_t>(blockIdx.x) + 1) * kBlock >= nvec &&
            vbase + static_cast<uint64_t>(blockIdx.x) * kBlock <= (nvec > 0 ? nvec - 1 : 0))
            for (uint64_t k = tail0 + threadIdx.x; k < nbytes; k += kBlock)
                dst[k] = e[k % psize];
    }

    vktError memsetRange(void* dst, void const* pattern, std::size_t dstSize, std::size_t patternSize)
    {
        if (patternSize == 0 || dstSize < patternSize)
            return vktNoError;
        if (dst == nullptr || pattern == nullptr)
            return rt::fail("MemsetRange: null pointer");
        if (patternSize > (1u << 30))
            return rt::fail("MemsetRange: pattern larger than 1 GiB");
        uint64_t const nbytes = (dstSize / patternSize) * patternSize;   // whole patterns only
        // a pageable host destination would fault the kernel (no XNACK): refused, nothing launched
        vktError const where = rt::requireDevicePointer(dst, nbytes, "MemsetRange: destination is not device memory");
        if (where != vktNoError)
            return where;
        hipStream_t s = rt::computeStream();
        uint8_t const* pb = static_cast<uint8_t const*>(pattern);
        uint32_t const psize = static_cast<uint32_t>(patternSize);
        uint32_t const elen = psize + 15;
        // vectors start on a 128-byte line: with a merely 16-byte-aligned start every 4 KiB
        // workgroup shares its first and last line with a neighbour (2 GiB, 4-byte pattern at
        // dst + 1: 4.9 TB/s, vs 6.7 TB/s line-aligned)
        uint64_t head = (128 - reinterpret_cast<uintptr_t>(dst) % 128) % 128;
        if (head > nbytes)
            head = nbytes;
        uint64_t const nvec = (nbytes - head) / 16;

        PatternArg arg{};
        uint8_t* big = nullptr;
        int src = 0;
        static rt::StreamScratch bigScratch;   // grow-only, not a pool block
        if (elen <= kPatArgBytes)
        {
            for (uint32_t k = 0; k < elen; ++k)
                arg.e[k] = pb[k % psize];
        }
        else
        {
            big = static_cast<uint8_t*>(bigScratch.acquire(elen, s));
            if (big == nullptr)
                return vktInvalidValue;
            // E = pattern followed by its first 15 bytes; the pageable source is consumed
            // before returning
            vktError e = rt::check(hipMemcpyAsync(big, pb, psize, hipMemcpyHostToDevice, s), "MemsetRange: upload");
            if (e == vktNoError)
                e = rt::check(hipMemcpyAsync(big + psize, pb, 15 < psize ? 15 : psize, hipMemcpyHostToDevice, s),
                              "MemsetRange: upload");
            if (e == vktNoError)
                e = rt::check(hipStreamSynchronize(s), "MemsetRange: upload");
            if (e != vktNoError)
            {
                bigScratch.release(s);
                return e;
            }
            src = elen <= kPatLdsBytes ? 1 : 2;
        }
        uint64_t const blocks = nvec > 0 ? (nvec + kBlock - 1) / kBlock : 1;   // >= 1: head/tail bytes
        size_t const shmem = src == 2 ? 0 : (elen + 15) / 16 * 16;
        for (uint64_t b0 = 0; b0 < blocks; b0 += kMemsetBlocksPerLaunch)
        {
            uint64_t nb = blocks - b0 < kMemsetBlocksPerLaunch ? blocks - b0 : kMemsetBlocksPerLaunch;
            uint64_t vbase = b0 * kBlock;
            auto* d = static_cast<uint8_t*>(dst);
            if (src == 0)
                hipLaunchKernelGGL(memsetPatternKernel<0>, dim3(static_cast<uint32_t>(nb)), dim3(kBlock), shmem, s, d,
                                   nbytes, head, nvec, vbase, psize, elen, arg, big);
            else if (src == 1)
                hipLaunchKernelGGL(memsetPatternKernel<1>, dim3(static_cast<uint32_t>(nb)), dim3(kBlock), shmem, s, d,
                                   nbytes, head, nvec, vbase, psize, elen, arg, big);
            else
                hipLaunchKernelGGL(memsetPatternKernel<2>, dim3(static_cast<uint32_t>(nb)), dim3(kBlock), shmem, s, d,
                                   nbytes, head, nvec, vbase, psize, elen, arg, big);
        }
        if (big != nullptr)
            bigScratch.release(s);
        return rt::finishLaunch("MemsetRange");
    }

    // ---- synthetic input -------------------------------------------------------------
    __device__ __forceinline__ uint64_t splitmix64(uint64_t x)
    {
        x += 0x9E3779B97F4A7C15ull;
        x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
        x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
        return x ^ (x >> 31);
    }

    __global__ __launch_bounds__(kBlock) void synthKernel(uint8_t* data, uint64_t nbytes, uint64_t seed)
    {
        uint64_t const stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
        uint64_t const words = nbytes / 8;
        for (uint64_t w = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; w <= words; w += stride)
        {
            uint64_t r = splitmix64(seed + w);
            if (w < words)
                __builtin_nontemporal_store(r, reinterpret_cast<uint64_t*>(data) + w);
            else
                for (uint64_t b = 0; b < nbytes % 8; ++b)
                    data[8 * w + b] = static_cast<uint8_t>(r >> (8 * b));
        }
    }

} // hipk
} // vkt

using namespace vkt;
using namespace vkt::hipk;

extern "C" {

vktError vktHipFillRange(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last, float value)
{
    if (!validView(volume))
        return rt::fail("vktHipFillRange: invalid volume view");
    int64_t nx = int64_t(last.x) - first.x, ny = int64_t(last.y) - first.y, nz = int64_t(last.z) - first.z;
    if (nx <= 0 || ny <= 0 || nz <= 0)
        return vktNoError;
    if (!boxInside(volume, first, nx, ny, nz))
        return rt::fail("vktHipFillRange: range outside the volume");
    if (!encodeWrites(volume.dataFormat))
        return vktNoError;   // reference MapVoxelImpl writes nothing for Int8/Int32
    bool w;
    uint32_t code = codec::encode(value, volume.dataFormat, codec::makeMapParams(volume.mappingLo, volume.mappingHi), w);
    Operand od = makeOperand(volume, first, false);
    PwPlan p = planPointwise(0, od, od, od, nx, ny, nz);
    vktError e = launchByBpv<0>(p, FillF{code}, rt::computeStream());
    return e != vktNoError ? e : rt::finishLaunch("FillRange_hip");
}

vktError vktHipCopyRange(vktHipVolumeView_t dst, vktHipVolumeView_t src, vktVec3i_t first, vktVec3i_t last,
                         vktVec3i_t dstOffset)
{
    if (!validView(dst) || !validView(src))
        return rt::fail("vktHipCopyRange: invalid volume view");
    int64_t nx = int64_t(last.x) - first.x, ny = int64_t(last.y) - first.y, nz = int64_t(last.z) - first.z;
    if (nx <= 0 || ny <= 0 || nz <= 0)
        return vktNoError;
    if (src.dimX <= 0 || src.dimY <= 0 || src.dimZ <= 0)
        return rt::fail("vktHipCopyRange: empty source volume");
    if (!boxInside(dst, dstOffset, nx, ny, nz))
        return rt::fail("vktHipCopyRange: destination range outside the volume");
    bool clamp = !boxInside(src, first, nx, ny, nz);
    if (overlaps(dst, src) && !(dst.data == src.data && first.x == dstOffset.x && first.y == dstOffset.y &&
                                first.z == dstOffset.z && !clamp))
        return rt::fail("vktHipCopyRange: overlapping source and destination are not supported");
    bool bytewise = dst.dataFormat == src.dataFormat && dst.mappingLo == src.mappingLo &&
                    dst.mappingHi == src.mappingHi;   // Copy_serial.hpp:21-22
    hipStream_t s = rt::computeStream();
    vktError e;
    if (bytewise)
    {
        Operand od = makeOperand(dst, dstOffset, false);
        Operand os = makeOperand(src, first, clamp);
        PwPlan p = planPointwise(1, od, os, os, nx, ny, nz);
        e = launchByBpv<1>(p, PassF{}, s);
    }
    else
    {
        if (!encodeWrites(dst.dataFormat))
            return vktNoError;
        e = convertBox(dst, src, first, clamp, dstOffset, nx, ny, nz);
    }
    return e != vktNoError ? e : rt::finishLaunch("CopyRange_hip");
}

vktError vktHipArithmeticRange(vktHipArithmeticOp op, vktHipVolumeView_t dest, vktHipVolumeView_t source1,
                               vktHipVolumeView_t source2, vktVec3i_t first, vktVec3i_t last, vktVec3i_t dstOffset)
{
    if (!validView(dest) || !validView(source1) || !validView(source2))
        return rt::fail("vktHipArithmeticRange: invalid volume view");
    if (op < 0 || op >= vktHipOpCount)
        return rt::fail("vktHipArithmeticRange: unknown op");
    int64_t nx = int64_t(last.x) - first.x, ny = int64_t(last.y) - first.y, nz = int64_t(last.z) - first.z;
    if (nx <= 0 || ny <= 0 || nz <= 0)
        return vktNoError;
    vktVec3i_t dOrigin{first.x + dstOffset.x, first.y + dstOffset.y, first.z + dstOffset.z};
    if (!boxInside(source1, first, nx, ny, nz) || !boxInside(source2, first, nx, ny, nz) ||
        !boxInside(dest, dOrigin, nx, ny, nz))
        return rt::fail("vktHipArithmeticRange: range outside a volume");
    bool shifted = dstOffset.x != 0 || dstOffset.y != 0 || dstOffset.z != 0;
    if (shifted && (overlaps(dest, source1) || overlaps(dest, source2)))
        return rt::fail("vktHipArithmeticRange: dest aliases a source with a non-zero dstOffset");
    if (!encodeWrites(dest.dataFormat))
        return vktNoError;
    Operand od = makeOperand(dest, dOrigin, false);
    Operand o1 = makeOperand(source1, first, false);
    Operand o2 = makeOperand(source2, first, false);
    PwPlan p = planPointwise(2, od, o1, o2, nx, ny, nz);
    hipStream_t s = rt::computeStream();
    vktError e = vktNoError;
    switch (op / 2)
    {
    case 0: e = arithmeticPair0(op, p, dest, source1, source2, s); break;
    case 1: e = arithmeticPair1(op, p, dest, source1, source2, s); break;
    case 2: e = arithmeticPair2(op, p, dest, source1, source2, s); break;
    case 3: e = arithmeticPair3(op, p, dest, source1, source2, s); break;
    default: e = arithmeticPair4(op, p, dest, source1, source2, s); break;
    }
    return e != vktNoError ? e : rt::finishLaunch("ArithmeticRange_hip");
}

vktError vktHipSynthesize(vktHipVolumeView_t volume, uint64_t seed)
{
    if (!validView(volume))
        return rt::fail("vktHipSynthesize: invalid volume view");
    uint64_t nbytes = viewBytes(volume);
    if (nbytes == 0)
        return vktNoError;
    if (reinterpret_cast<uintptr_t>(volume.data) % 8 != 0)
        return rt::fail("vktHipSynthesize: data must be 8-byte aligned");
    hipLaunchKernelGGL(synthKernel, dim3(streamingGrid(nbytes / 8 + 1, kBlock)), dim3(kBlock), 0,
                       rt::computeStream(), volume.data, nbytes, seed);
    return rt::finishLaunch("Synthesize_hip");
}

} // extern "C"
