// Slab.cpp -- FillRange / CopyRange / arithmetic Range calls over Z-slab partitioned volumes
// ("Range variants intersect [first, last) with each slab; a dstOffset.z that
// moves voxels across slab boundaries sends the affected planes to their owner").
//
// The reference is single-volume: FillRange_serial writes dst[x] for x in [first, last)
// (src/vkt/Fill_serial.hpp:20-26), CopyRange_serial writes dst[x - first + dstOffset] =
// src[clamp(x, 0, dims - 1)] (src/vkt/Copy_serial.hpp:38-47), ArithmeticOp writes
// dst[x + dstOffset] = f(s1[x], s2[x]) at absolute x (src/vkt/Arithmetic_serial.hpp:25-41).
// Over slabs every rank computes the dst planes it owns.  The reference's z loop variable maps
// to the dst plane z + shift (shift = 0 Fill, dstOffset.z - first.z Copy, dstOffset.z
// arithmetic), so rank r's loop planes are [first.z, last.z) intersected with its owned dst
// planes minus shift.  That range is cut where the owner of a source plane changes (and, for
// Copy, where the clamp starts and ends); each piece reads each source either from the own
// slab or from a gather buffer that the source's owner fills (one move per remote piece and
// source).  Every rank derives every rank's pieces from the global arguments, so the moves are
// enumerated in one global order and pair up in order on both sides (RCCL group semantics);
// with every slab in this process the moves are device copies.  Then the local op -- the same
// backend entry points as for whole volumes -- runs piece by piece on views of the own slab or
// of the gather buffer.  Equal results to one call on the whole volume, by construction: each
// dst voxel is written once, by its owner, from the same source values.

#include "Comm.hpp"
#include "volkit_codec.hpp"

#include <algorithm>
#include <string>
#include <vector>

namespace vkt
{
namespace hipk
{
    vktError transformRange1Shifted(vktHipVolumeView_t volume, vktVec3i_t first, vktVec3i_t last,
                                    vktTransformUnaryOp unaryOp, int32_t zShift);
}
namespace
{
    struct Move
    {
        int32_t from, to, source, z0, z1, bufPlane;
    };

    int32_t ownerOf(int32_t z, int32_t G, int32_t W)
    {
        int64_t const size = (static_cast<int64_t>(G) + W - 1) / W;
        return static_cast<int32_t>(z / size);
    }

    int32_t clampZ(int32_t z, int32_t G) { return z < 0 ? 0 : (z > G - 1 ? G - 1 : z); }

    struct Args
    {
        vktHipSlabOpKind kind;
        int32_t W;
        int32_t dstG;
        int32_t srcG[2];
        int32_t f, l, o;   // first.z, last.z, dstOffset.z
        int nsrc() const { return kind == vktHipSlabFill ? 0 : kind == vktHipSlabCopy ? 1 : 2; }
        int32_t shift() const { return kind == vktHipSlabCopy ? o - f : kind == vktHipSlabArithmetic ? o : 0; }
    };

    // global checks, identical on every rank (before anything moves)
    vktError validate(Args const& a, char const* what)
    {
        auto bad = [&](char const* why) { return rt::fail((std::string(what) + ": " + why).c_str()); };
        if (a.W <= 0)
            return bad("invalid number of ranks");
        if (a.dstG < 0 || (a.nsrc() >= 1 && a.srcG[0] < 0) || (a.nsrc() == 2 && a.srcG[1] < 0))
            return bad("negative global depth");
        if (a.l <= a.f)
            return vktNoError;
        switch (a.kind)
        {
        case vktHipSlabFill:
            if (a.f < 0 || a.l > a.dstG)
                return bad("range outside the volume");
            break;
        case vktHipSlabCopy:
            if (a.srcG[0] <= 0)
                return bad("empty source volume");
            if (a.o < 0 || static_cast<int64_t>(a.o) + (a.l - a.f) > a.dstG)
                return bad("destination range outside the volume");
            break;
        default:
            if (a.f < 0 || a.l > a.srcG[0] || a.l > a.srcG[1] || static_cast<int64_t>(a.f) + a.o < 0 ||
                static_cast<int64_t>(a.l) + a.o > a.dstG)
                return bad("range outside a volume");
            break;
        }
        return vktNoError;
    }

    // source plane range [z0, z0 + n) that loop planes [zb, ze) read from source k
    void sourcePlanes(Args const& a, int k, int32_t zb, int32_t ze, int32_t& z0, int32_t& n)
    {
        if (a.kind == vktHipSlabCopy)
        {
            z0 = clampZ(zb, a.srcG[0]);
            n = clampZ(ze - 1, a.srcG[0]) - z0 + 1;
        }
        else
        {
            z0 = zb;
            n = ze - zb;
        }
        (void)k;
    }

    // pieces of rank r (gather-buffer offsets filled in); bufPlanes[k] = buffer sizes
    void planRank(Args const& a, int32_t r, std::vector<vktHipSlabPiece_t>& pieces, int32_t bufPlanes[2])
    {
        pieces.clear();
        bufPlanes[0] = bufPlanes[1] = 0;
        if (a.l <= a.f)
            return;
        int32_t d0, d1;
        comm::slabBounds(a.dstG, a.W, r, d0, d1);
        int32_t const sh = a.shift();
        int64_t const zb64 = std::max<int64_t>(a.f, static_cast<int64_t>(d0) - sh);
        int64_t const ze64 = std::min<int64_t>(a.l, static_cast<int64_t>(d1) - sh);
        if (ze64 <= zb64)
            return;
        int32_t const zb = static_cast<int32_t>(zb64), ze = static_cast<int32_t>(ze64);
        // cut points: source ownership changes (and the clamp borders of a Copy)
        std::vector<int32_t> cuts{zb, ze};
        for (int k = 0; k < a.nsrc(); ++k)
        {
            int32_t const G = a.srcG[k];
            int64_t const size = (static_cast<int64_t>(G) + a.W - 1) / a.W;
            for (int64_t c = 0; c <= G; c += size > 0 ? size : 1)
                if (c > zb && c < ze)
                    cuts.push_back(static_cast<int32_t>(c));
            if (a.kind == vktHipSlabCopy && G > zb && G < ze)
                cuts.push_back(G);
            if (size <= 0)
                break;
        }
        std::sort(cuts.begin(), cuts.end());
        cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
        for (size_t i = 0; i + 1 < cuts.size(); ++i)
        {
            vktHipSlabPiece_t p{};
            p.zBegin = cuts[i];
            p.zEnd = cuts[i + 1];
            p.dstZ = p.zBegin + sh;
            for (int k = 0; k < 2; ++k)
            {
                p.srcZ[k] = p.srcPlanes[k] = 0;
                p.bufPlane[k] = -1;
                if (k >= a.nsrc())
                    continue;
                sourcePlanes(a, k, p.zBegin, p.zEnd, p.srcZ[k], p.srcPlanes[k]);
                if (ownerOf(p.srcZ[k], a.srcG[k], a.W) != r)
                {
                    p.bufPlane[k] = bufPlanes[k];
                    bufPlanes[k] += p.srcPlanes[k];
                }
            }
            pieces.push_back(p);
        }
    }

    // every rank's remote pieces as moves, in the one global order (receiver, piece, source)
    void allMoves(Args const& a, std::vector<Move>& moves)
    {
        moves.clear();
        std::vector<vktHipSlabPiece_t> ps;
        int32_t bp[2];
        for (int32_t r = 0; r < a.W; ++r)
        {
            planRank(a, r, ps, bp);
            for (vktHipSlabPiece_t const& p : ps)
                for (int k = 0; k < a.nsrc(); ++k)
                    if (p.bufPlane[k] >= 0)
                        moves.push_back(Move{ownerOf(p.srcZ[k], a.srcG[k], a.W), r, k, p.srcZ[k],
                                             p.srcZ[k] + p.srcPlanes[k], p.bufPlane[k]});
        }
    }

    vktHipVolumeView_t subView(vktHipVolumeView_t v, uint8_t* data, int32_t planes)
    {
        v.data = data;
        v.dimZ = planes;
        return v;
    }

    vktError checkSlab(vktHipSlab_t const& s, Args const& a, int32_t rank, int32_t G, char const* what)
    {
        auto bad = [&](char const* why) { return rt::fail((std::string(what) + ": " + why).c_str()); };
        if (s.globalDimZ != G)
            return bad("slab globalDimZ differs from the partitioned volume's depth");
        int32_t o0, o1;
        comm::slabBounds(G, a.W, rank, o0, o1);
        if (s.z0 < 0 || static_cast<int64_t>(s.z0) + s.view.dimZ > G)
            return bad("slab planes outside the global volume");
        if (o1 > o0 && (s.z0 > o0 || s.z0 + s.view.dimZ < o1))
            return bad("slab does not hold the planes its rank owns");
        if (comm::planeBytes(s.view) == 0 && static_cast<int64_t>(s.view.dimX) * s.view.dimY > 0)
            return bad("invalid slab view");
        return vktNoError;
    }

    // The local op of one piece of rank r.
    vktError runPiece(Args const& a, vktHipArithmeticOp op, vktHipSlab_t const& dst, vktHipSlab_t const* src,
                      uint8_t* const* buf, vktHipSlabPiece_t const& p, vktVec3i_t first, vktVec3i_t last,
                      vktVec3i_t off, float value)
    {
        if (a.kind == vktHipSlabFill)
            return vktHipFillRange(dst.view, vktVec3i_t{first.x, first.y, p.zBegin - dst.z0},
                                   vktVec3i_t{last.x, last.y, p.zEnd - dst.z0}, value);
        // source views: the own slab whole (local plane = global - z0; keeps in-place calls in
        // place) when every source is own and they share z0, else exactly the piece's planes
        bool const own = p.bufPlane[0] < 0 && (a.nsrc() < 2 || (p.bufPlane[1] < 0 && src[0].z0 == src[1].z0));
        vktHipVolumeView_t v[2];
        int32_t base = 0;   // global plane of local source plane 0
        for (int k = 0; k < a.nsrc(); ++k)
        {
            size_t const plane = comm::planeBytes(src[k].view);
            if (own)
            {
                v[k] = src[k].view;
                base = src[k].z0;
            }
            else if (p.bufPlane[k] < 0)
            {
                v[k] = subView(src[k].view, src[k].view.data + static_cast<size_t>(p.srcZ[k] - src[k].z0) * plane,
                               p.srcPlanes[k]);
                base = p.srcZ[k];
            }
            else
            {
                v[k] = subView(src[k].view, buf[k] + static_cast<size_t>(p.bufPlane[k]) * plane, p.srcPlanes[k]);
                base = p.srcZ[k];
            }
        }
        int32_t const dz = p.dstZ - dst.z0;   // local dst plane of loop plane zBegin
        if (a.kind == vktHipSlabCopy)
            return vktHipCopyRange(dst.view, v[0], vktVec3i_t{first.x, first.y, p.zBegin - base},
                                   vktVec3i_t{last.x, last.y, p.zEnd - base}, vktVec3i_t{off.x, off.y, dz});
        // arithmetic: both sources share the loop origin (same base: both own with one z0, or
        // both sub-views of exactly the piece's planes)
        int32_t const lz = p.zBegin - base;
        return vktHipArithmeticRange(op, dst.view, v[0], v[1], vktVec3i_t{first.x, first.y, lz},
                                     vktVec3i_t{last.x, last.y, lz + (p.zEnd - p.zBegin)},
                                     vktVec3i_t{off.x, off.y, dz - lz});
    }

    vktError runPieces(Args const& a, vktHipArithmeticOp op, vktHipSlab_t const& dst, vktHipSlab_t const* src,
                       uint8_t* const* buf, std::vector<vktHipSlabPiece_t> const& pieces, vktVec3i_t first,
                       vktVec3i_t last, vktVec3i_t off, float value)
    {
        for (vktHipSlabPiece_t const& p : pieces)
        {
            vktError const e = runPiece(a, op, dst, src, buf, p, first, last, off, value);
            if (e != vktNoError)
                return e;
        }
        return vktNoError;
    }

    // slab arrays checked against the partition (rank0 + i is slab i's rank)
    vktError checkSlabs(Args const& a, int32_t rank0, int32_t numSlabs, vktHipSlab_t const* dst,
                        vktHipSlab_t const* const* srcs, char const* what)
    {
        for (int32_t i = 0; i < numSlabs; ++i)
        {
            vktError e = checkSlab(dst[i], a, rank0 + i, a.dstG, what);
            for (int k = 0; k < a.nsrc() && e == vktNoError; ++k)
                e = checkSlab(srcs[k][i], a, rank0 + i, a.srcG[k], what);
            if (e != vktNoError)
                return e;
        }
        return vktNoError;
    }

    vktError slabRange(char const* what, vktHipSlabOpKind kind, vktHipArithmeticOp op, vktHipComm_t comm,
                       int32_t numSlabs, vktHipSlab_t const* dst, vktHipSlab_t const* s1, vktHipSlab_t const* s2,
                       vktVec3i_t first, vktVec3i_t last, vktVec3i_t off, float value)
    {
        auto bad = [&](char const* why) { return rt::fail((std::string(what) + ": " + why).c_str()); };
        if (dst == nullptr || (kind != vktHipSlabFill && s1 == nullptr) || (kind == vktHipSlabArithmetic && s2 == nullptr))
            return bad("null slab array");
        if (comm != nullptr && numSlabs != 1)
            return bad("with a communicator, pass this rank's slab only (numSlabs = 1)");
        if (numSlabs <= 0)
            return bad("numSlabs must be positive");
        Args a{kind, comm ? comm->nranks : numSlabs, dst[0].globalDimZ,
               {s1 ? s1[0].globalDimZ : 0, s2 ? s2[0].globalDimZ : 0}, first.z, last.z, off.z};
        vktError e = validate(a, what);
        if (e != vktNoError)
            return e;
        if (last.x <= first.x || last.y <= first.y || last.z <= first.z)
            return vktNoError;   // empty (or reversed) ranges: nothing, like the backend calls
        int32_t const rank0 = comm ? comm->rank : 0;
        vktHipSlab_t const* srcs[2] = {s1, s2};
        if ((e = checkSlabs(a, rank0, numSlabs, dst, srcs, what)) != vktNoError)
            return e;
        // gather buffers of every rank handled here, one scratch allocation
        std::vector<std::vector<vktHipSlabPiece_t>> pieces(numSlabs);
        std::vector<size_t> bufOff(static_cast<size_t>(numSlabs) * 2, 0);
        size_t total = 0;
        for (int32_t i = 0; i < numSlabs; ++i)
        {
            int32_t bp[2];
            planRank(a, rank0 + i, pieces[i], bp);
            for (int k = 0; k < a.nsrc(); ++k)
            {
                bufOff[2 * i + k] = total;
                total += (static_cast<size_t>(bp[k]) * comm::planeBytes(srcs[k][i].view) + 255) / 256 * 256;
            }
        }
        hipStream_t const s = rt::computeStream();
        static rt::StreamScratch scratch;
        uint8_t* sp = nullptr;
        if (total > 0 && (sp = static_cast<uint8_t*>(scratch.acquire(total, s))) == nullptr)
            return rt::fail((std::string(what) + ": gather buffer allocation failed").c_str());
        auto release = [&] {
            if (sp)
                scratch.release(s);
        };
        std::vector<Move> moves;
        allMoves(a, moves);
        if (comm != nullptr)
        {
            std::vector<comm::Xfer> xs;
            for (Move const& m : moves)
            {
                if (m.from != rank0 && m.to != rank0)
                    continue;
                comm::Xfer x{m.from == rank0 ? m.to : m.from, m.from == rank0 ? 1 : 0, nullptr, 0};
                vktHipSlab_t const& sl = srcs[m.source][0];
                if (x.send)
                    e = comm::planeSpan(sl.view, sl.z0, m.z0, m.z1, what, x.ptr, x.bytes);
                else
                {
                    x.ptr = sp + bufOff[m.source] + static_cast<size_t>(m.bufPlane) * comm::planeBytes(sl.view);
                    x.bytes = static_cast<size_t>(m.z1 - m.z0) * comm::planeBytes(sl.view);
                }
                if (e != vktNoError)
                {
                    release();
                    return e;
                }
                xs.push_back(x);
            }
            e = comm::rcclRound(comm, xs, s, what);
        }
        else
        {
            for (Move const& m : moves)
            {
                vktHipSlab_t const& from = srcs[m.source][m.from];
                vktHipSlab_t const& to = srcs[m.source][m.to];
                uint8_t* p;
                size_t n;
                e = comm::planeSpan(from.view, from.z0, m.z0, m.z1, what, p, n);
                if (e == vktNoError && comm::planeBytes(from.view) != comm::planeBytes(to.view))
                    e = bad("slabs of one volume with different plane sizes");
                if (e == vktNoError)
                    e = comm::localMove(sp + bufOff[2 * m.to + m.source] +
                                            static_cast<size_t>(m.bufPlane) * comm::planeBytes(to.view),
                                        p, n, s, what);
                if (e != vktNoError)
                    break;
            }
        }
        for (int32_t i = 0; i < numSlabs && e == vktNoError; ++i)
        {
            vktHipSlab_t src[2];
            uint8_t* buf[2] = {nullptr, nullptr};
            for (int k = 0; k < a.nsrc(); ++k)
            {
                src[k] = srcs[k][i];
                buf[k] = sp ? sp + bufOff[2 * i + k] : nullptr;
            }
            e = runPieces(a, op, dst[i], src, buf, pieces[i], first, last, off, value);
        }
        release();
        if (e != vktNoError)
            return e;
        return comm != nullptr ? comm::finishRound(comm, what) : rt::finishLaunch(what);
    }
} // namespace
} // namespace vkt

using namespace vkt;

extern "C" {

vktError vktHipSlabRangePlan(vktHipSlabOpKind kind, int32_t nranks, int32_t rank, int32_t dstGlobalDimZ,
                             int32_t src1GlobalDimZ, int32_t src2GlobalDimZ, vktVec3i_t first, vktVec3i_t last,
                             vktVec3i_t dstOffset, vktHipSlabPiece_t* pieces, int32_t pieceCapacity,
                             int32_t* numPieces, vktHipSlabMove_t* moves, int32_t moveCapacity, int32_t* numMoves,
                             int32_t* bufPlanes)
{
    char const* what = "vktHipSlabRangePlan";
    if (numPieces == nullptr || numMoves == nullptr || bufPlanes == nullptr)
        return rt::fail("vktHipSlabRangePlan: null pointer");
    if (kind < vktHipSlabFill || kind > vktHipSlabArithmetic)
        return rt::fail("vktHipSlabRangePlan: unknown op kind");
    if (nranks <= 0 || rank < 0 || rank >= nranks)
        return rt::fail("vktHipSlabRangePlan: invalid rank / nranks");
    Args a{kind, nranks, dstGlobalDimZ, {src1GlobalDimZ, src2GlobalDimZ}, first.z, last.z, dstOffset.z};
    vktError e = validate(a, what);
    if (e != vktNoError)
        return e;
    std::vector<vktHipSlabPiece_t> ps;
    int32_t bp[2] = {0, 0};
    std::vector<Move> ms;
    if (last.x > first.x && last.y > first.y)
    {
        planRank(a, rank, ps, bp);
        allMoves(a, ms);
    }
    std::vector<vktHipSlabMove_t> mine;
    for (Move const& m : ms)
        if (m.from == rank || m.to == rank)
            mine.push_back(vktHipSlabMove_t{m.from == rank ? m.to : m.from, m.from == rank ? 1 : 0, m.source, m.z0,
                                            m.z1, m.bufPlane});
    *numPieces = static_cast<int32_t>(ps.size());
    *numMoves = static_cast<int32_t>(mine.size());
    bufPlanes[0] = bp[0];
    bufPlanes[1] = bp[1];
    if (pieces != nullptr)
    {
        if (pieceCapacity < *numPieces)
            return rt::fail("vktHipSlabRangePlan: piece array too small");
        std::copy(ps.begin(), ps.end(), pieces);
    }
    if (moves != nullptr)
    {
        if (moveCapacity < *numMoves)
            return rt::fail("vktHipSlabRangePlan: move array too small");
        std::copy(mine.begin(), mine.end(), moves);
    }
    return vktNoError;
}

vktError vktHipSlabRangePieces(vktHipSlabOpKind kind, vktHipArithmeticOp op, int32_t nranks, int32_t rank,
                               vktHipSlab_t dst, vktHipSlab_t const* source1, vktHipSlab_t const* source2,
                               vktVec3i_t first, vktVec3i_t last, vktVec3i_t dstOffset, float value,
                               void* gather1, void* gather2)
{
    char const* what = "vktHipSlabRangePieces";
    if (kind < vktHipSlabFill || kind > vktHipSlabArithmetic || op < 0 || op >= vktHipOpCount)
        return rt::fail("vktHipSlabRangePieces: unknown op");
    if (nranks <= 0 || rank < 0 || rank >= nranks)
        return rt::fail("vktHipSlabRangePieces: invalid rank / nranks");
    if ((kind != vktHipSlabFill && source1 == nullptr) || (kind == vktHipSlabArithmetic && source2 == nullptr))
        return rt::fail("vktHipSlabRangePieces: null source slab");
    Args a{kind, nranks, dst.globalDimZ, {source1 ? source1->globalDimZ : 0, source2 ? source2->globalDimZ : 0},
           first.z, last.z, dstOffset.z};
    vktError e = validate(a, what);
    if (e != vktNoError || last.x <= first.x || last.y <= first.y || last.z <= first.z)
        return e;
    vktHipSlab_t const* srcs[2] = {source1, source2};
    if ((e = checkSlabs(a, rank, 1, &dst, srcs, what)) != vktNoError)
        return e;
    std::vector<vktHipSlabPiece_t> ps;
    int32_t bp[2];
    planRank(a, rank, ps, bp);
    uint8_t* buf[2] = {static_cast<uint8_t*>(gather1), static_cast<uint8_t*>(gather2)};
    for (int k = 0; k < a.nsrc(); ++k)
        if (bp[k] > 0 && buf[k] == nullptr)
            return rt::fail("vktHipSlabRangePieces: the plan reads a gather buffer that was not passed");
    vktHipSlab_t src[2];
    for (int k = 0; k < a.nsrc(); ++k)
        src[k] = *srcs[k];
    e = runPieces(a, op, dst, src, buf, ps, first, last, dstOffset, value);
    return e != vktNoError ? e : rt::finishLaunch(what);
}

vktError vktHipSlabTransformRange1(int32_t nranks, int32_t rank, vktHipSlab_t slab, vktVec3i_t first, vktVec3i_t last,
                                   vktTransformUnaryOp unaryOp)
{
    char const* what = "vktHipSlabTransformRange1";
    if (unaryOp == nullptr)
        return rt::fail("vktHipSlabTransformRange1: null operation");
    if (nranks <= 0 || rank < 0 || rank >= nranks)
        return rt::fail("vktHipSlabTransformRange1: invalid rank / nranks");
    // the owned planes of the range: the Fill plan (no sources, nothing moves)
    Args a{vktHipSlabFill, nranks, slab.globalDimZ, {0, 0}, first.z, last.z, 0};
    vktError e = validate(a, what);
    if (e != vktNoError || last.x <= first.x || last.y <= first.y || last.z <= first.z)
        return e;
    if ((e = checkSlabs(a, rank, 1, &slab, nullptr, what)) != vktNoError)
        return e;
    std::vector<vktHipSlabPiece_t> ps;
    int32_t bp[2];
    planRank(a, rank, ps, bp);
    for (vktHipSlabPiece_t const& p : ps)
        if ((e = hipk::transformRange1Shifted(slab.view, vktVec3i_t{first.x, first.y, p.zBegin - slab.z0},
                                              vktVec3i_t{last.x, last.y, p.zEnd - slab.z0}, unaryOp, slab.z0)) !=
            vktNoError)
            return e;
    return vktNoError;
}

vktError vktHipSlabFillRange(vktHipComm_t comm, int32_t numSlabs, vktHipSlab_t const* dst, vktVec3i_t first,
                             vktVec3i_t last, float value)
{
    return slabRange("vktHipSlabFillRange", vktHipSlabFill, vktHipOpSum, comm, numSlabs, dst, nullptr, nullptr, first,
                     last, vktVec3i_t{0, 0, 0}, value);
}

vktError vktHipSlabCopyRange(vktHipComm_t comm, int32_t numSlabs, vktHipSlab_t const* dst, vktHipSlab_t const* src,
                             vktVec3i_t first, vktVec3i_t last, vktVec3i_t dstOffset)
{
    return slabRange("vktHipSlabCopyRange", vktHipSlabCopy, vktHipOpSum, comm, numSlabs, dst, src, nullptr, first,
                     last, dstOffset, 0.f);
}

vktError vktHipSlabArithmeticRange(vktHipComm_t comm, vktHipArithmeticOp op, int32_t numSlabs,
                                   vktHipSlab_t const* dest, vktHipSlab_t const* source1,
                                   vktHipSlab_t const* source2, vktVec3i_t first, vktVec3i_t last,
                                   vktVec3i_t dstOffset)
{
    if (op < 0 || op >= vktHipOpCount)
        return rt::fail("vktHipSlabArithmeticRange: unknown op");
    return slabRange("vktHipSlabArithmeticRange", vktHipSlabArithmetic, op, comm, numSlabs, dest, source1, source2,
                     first, last, dstOffset, 0.f);
}

} // extern "C"
