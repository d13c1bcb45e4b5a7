/*! @file sx_traverse.hpp
 * @brief wave-cooperative breadth-first octree traversal (gfx950 wave64), shared by the neighbor search and the
 *        halo discovery.
 *
 * The linked octree is the reference's OctreeData layout (childOffsets[node] = first of 8 children, 0 = leaf).
 * One wavefront expands up to 8 queued internal nodes per step, one child per lane (8 nodes x 8 octants = 64
 * lanes); passing leaves and internal nodes are compacted with ballot + popcount into LDS lists.  Control flow
 * is wave-uniform; the overlap predicate is evaluated per lane.
 */
#pragma once

#include "sx_device.hpp"

namespace sx
{

constexpr int kQCap = 512;  //!< internal-node ring per wave (power of 2)

/*! Collect every leaf node passing `overlaps` (whose ancestors all pass) into cand[0..return), at most CCap leaves.
 *  Sets `overflow` if the queue or the candidate list ran out of space (the caller reports an error).  The capacity
 *  is a template parameter: the search builds (sx_neighbors.hip) and the halo discovery (sx_sim.cpp) size it
 *  differently, each in its own translation unit.
 *  The queue holds the FIRST CHILD of every passing internal node (childOffsets[node], loaded with the node's own
 *  leaf test), so a step's chain of dependent global loads is one deep: the children's boxes and child offsets.
 *  Leaves come out in the order of the level-by-level expansion (deterministic). */
template<int CCap, class Overlaps>
__device__ __forceinline__ int waveCollectLeaves(const int32_t* __restrict__ childOffsets, Overlaps&& overlaps,
                                                 int* queue, int* cand, int lane, bool& overflow)
{
    const uint64_t ltMask  = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int            numCand = 0, qh = 0, qt = 0;
    overflow               = false;
    if (overlaps(0))
    {
        const int c0 = childOffsets[0];
        if (c0 == 0) { numCand = 1, cand[0] = 0; }
        else { queue[0] = c0, qt = 1; }
    }
    __builtin_amdgcn_wave_barrier();
    // up to 16 queued nodes per step, two children per lane (queue items qh..qh+7 in the first half, qh+8..qh+15 in
    // the second): both halves' loads are in flight together.  Items produced by this step are appended behind every
    // item already queued, so the FIFO order -- and the order of the collected leaves -- is that of 8-node steps.
    while (qh < qt)
    {
        const int  take  = min(16, qt - qh);
        const int  slot  = lane >> 3, oct = lane & 7;
        const bool okA   = slot < take, okB = slot + 8 < take;
        const int  cA    = okA ? queue[(qh + slot) & (kQCap - 1)] + oct : 0;
        const int  cB    = okB ? queue[(qh + slot + 8) & (kQCap - 1)] + oct : 0;
        const int  gA    = childOffsets[cA]; // issued with the box loads of overlaps(): independent of them
        const int  gB    = childOffsets[cB];
        const bool pA    = okA && overlaps(cA);
        const bool pB    = okB && overlaps(cB);
        const bool leafA = pA && gA == 0, innerA = pA && gA != 0;
        const bool leafB = pB && gB == 0, innerB = pB && gB != 0;
        const uint64_t blA = __ballot(leafA), biA = __ballot(innerA);
        const uint64_t blB = __ballot(leafB), biB = __ballot(innerB);
        if (leafA)
        {
            const int pos = numCand + __popcll(blA & ltMask);
            if (pos < CCap) cand[pos] = cA;
        }
        if (leafB)
        {
            const int pos = numCand + __popcll(blA) + __popcll(blB & ltMask);
            if (pos < CCap) cand[pos] = cB;
        }
        if (innerA) queue[(qt + __popcll(biA & ltMask)) & (kQCap - 1)] = gA;
        if (innerB) queue[(qt + __popcll(biA) + __popcll(biB & ltMask)) & (kQCap - 1)] = gB;
        numCand += __popcll(blA) + __popcll(blB);
        qt += __popcll(biA) + __popcll(biB);
        qh += take;
        if (qt - qh > kQCap) overflow = true;
        __builtin_amdgcn_wave_barrier();
    }
    if (numCand > CCap)
    {
        overflow = true;
        numCand  = CCap;
    }
    return numCand;
}

//! minimum-image folding of a coordinate difference on periodic axes (box.hpp:193-205 applyPbc)
__device__ __forceinline__ double foldPbc(double d, const DevBox& b, int k)
{
    return d - (double)b.pbc[k] * b.l[k] * rint(d * b.il[k]);
}

//! squared minimum distance between an axis-aligned box (center c, half-size s) and a point/box (center p,
//! half-size q), with minimum-image folding
__device__ __forceinline__ double boxDist2(const double* c, const double* s, double px, double py, double pz,
                                           double qx, double qy, double qz, const DevBox& b)
{
    double d0 = fabs(foldPbc(c[0] - px, b, 0)) - s[0] - qx;
    double d1 = fabs(foldPbc(c[1] - py, b, 1)) - s[1] - qy;
    double d2 = fabs(foldPbc(c[2] - pz, b, 2)) - s[2] - qz;
    d0        = d0 > 0 ? d0 : 0;
    d1        = d1 > 0 ? d1 : 0;
    d2        = d2 > 0 ? d2 : 0;
    return d0 * d0 + d1 * d1 + d2 * d2;
}

} // namespace sx
