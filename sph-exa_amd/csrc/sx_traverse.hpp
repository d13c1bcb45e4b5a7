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
 *  differently, each in its own translation unit. */
template<int CCap, class Overlaps>
__device__ __forceinline__ int waveCollectLeaves(const int32_t* __restrict__ childOffsets, Overlaps&& overlaps,
                                                 int* queue, int* cand, int lane, bool& overflow)
{
    const uint64_t ltMask  = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int            numCand = 0, qh = 0, qt = 0;
    overflow               = false;
    if (overlaps(0))
    {
        if (childOffsets[0] == 0) { numCand = 1, cand[0] = 0; }
        else { queue[0] = 0, qt = 1; }
    }
    __builtin_amdgcn_wave_barrier();
    while (qh < qt)
    {
        const int  take  = min(8, qt - qh);
        const int  slot  = lane >> 3, oct = lane & 7;
        const bool ok    = slot < take;
        const int  node  = ok ? queue[(qh + slot) & (kQCap - 1)] : 0;
        const int  child = ok ? childOffsets[node] + oct : 0;
        const bool pass  = ok && overlaps(child);
        const bool leaf  = pass && childOffsets[child] == 0;
        const bool inner = pass && !leaf;
        const uint64_t bl = __ballot(leaf), bi = __ballot(inner);
        if (leaf)
        {
            int pos = numCand + __popcll(bl & ltMask);
            if (pos < CCap) cand[pos] = child;
        }
        if (inner) { queue[(qt + __popcll(bi & ltMask)) & (kQCap - 1)] = child; }
        numCand += __popcll(bl);
        qt += __popcll(bi);
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
