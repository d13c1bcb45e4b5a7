/*! @file sx_neighbors.hip
 * @brief Neighbor search with the coupled h-nc iteration, one wavefront per 64-particle SFC block (gfx950).
 *
 * Replaces cstone::findNeighbors + sph::findNeighborsSph (cstone/findneighbors.hpp:95-188,
 * sph/find_neighbors.hpp:10-44) and the traversal inside xmassGpu (hydro_ve/xmass_gpu.cu:56-101).
 *
 * Per block (wave):
 *   1. wave reductions give the block's bounding box and max h;
 *   2. waveCollectLeaves (sx_traverse.hpp) gathers every leaf whose geometric box comes within 2*hmax of the
 *      block box (minimum image on periodic axes, inflated by the key-quantisation margin);
 *   3. each candidate leaf's particles (a contiguous SFC range) are loaded coalesced, one per lane, and broadcast
 *      lane by lane with v_readlane: every lane tests the candidate against its own particle with the reference CPU
 *      criterion, in double, without FMA contraction (this file is compiled -ffp-contract=off):
 *          d2 = dx*dx + dy*dy + dz*dz  <  (double)(4.0f*h*h),   j != i,
 *      dx folded with rint() on periodic axes when the particle is within 2h of the box edge (findneighbors.hpp:118);
 *      hits are appended to the lane-interleaved list nidx[(block*ngmax + k)*64 + lane] (k < ngmax, counting on);
 *   4. lanes with nc = count+1 outside [ng0/4, ngmax+1] update h (updateH) and the block repeats, at most 10
 *      updates per lane (the CPU loop's `iteration++ < 10`), so h, nc and the neighbor SET are identical to the
 *      CPU reference.
 */
#include "sx_traverse.hpp"
#include "sx_tree.hpp"

namespace sx
{

constexpr int kNsWaves = 4; // waves per workgroup

__global__ __launch_bounds__(kNsWaves * 64) void findNeighborsKernel(NsArgs a)
{
    __shared__ int s_queue[kNsWaves][kQCap];
    __shared__ int s_cand[kNsWaves][kCCap];

    const int      wave = threadIdx.x >> 6;
    const int      lane = threadIdx.x & 63;
    const uint32_t g    = xcdBlock(blockIdx.x, gridDim.x) * kNsWaves + wave;
    if (g >= a.numGroups) return; // whole wave, no block barrier in this kernel
    int* queue = s_queue[wave];
    int* cand  = s_cand[wave];

    const uint32_t i     = a.first + g * kGroupSize + lane;
    const bool     valid = i < a.last;
    const uint32_t iSafe = valid ? i : a.first + g * kGroupSize; // lane 0 of the block is always valid
    const double   xi = a.x[iSafe], yi = a.y[iSafe], zi = a.z[iSafe];
    float          hi = a.h[iSafe];

    uint32_t* nlist = a.nidx + (size_t)g * a.ngmax * kWave + lane;

    const unsigned     ngmin      = a.ng0 / 4;
    int                iteration  = 0;
    bool               active     = valid;
    unsigned           count      = 0;
    unsigned long long candTested = 0;

    // block bounding box (positions do not change between iterations)
    const double bx0 = waveMin(xi), bx1 = waveMax(xi);
    const double by0 = waveMin(yi), by1 = waveMax(yi);
    const double bz0 = waveMin(zi), bz1 = waveMax(zi);
    const double gcx = 0.5 * (bx0 + bx1), gcy = 0.5 * (by0 + by1), gcz = 0.5 * (bz0 + bz1);
    const double gsx = 0.5 * (bx1 - bx0), gsy = 0.5 * (by1 - by0), gsz = 0.5 * (bz1 - bz0);

    while (true)
    {
        // ---- 2. candidate leaves for radius 2*hmax ----------------------------------------------------
        const float  hmax = waveMax(valid ? hi : 0.0f);
        const double R    = 2.0 * (double)hmax * (1.0 + 1e-6) + a.margin;
        const double R2   = R * R;
        bool         overflow;
        const int    numCand = waveCollectLeaves(
            a.childOffsets,
            [&](int node) {
                return boxDist2(a.centers + 3 * (size_t)node, a.sizes + 3 * (size_t)node, gcx, gcy, gcz, gsx, gsy, gsz,
                                a.box) < R2;
            },
            queue, cand, lane, overflow);
        if (overflow && lane == 0) atomicOr(&a.stats[0], 1u);

        // ---- 3. test candidates against each lane's own particle --------------------------------------
        const float  r2f       = 4.0f * hi * hi;
        const double radSq     = (double)r2f;
        const double tw        = 2.0 * (double)hi;
        const bool   inside    = (xi - tw >= a.box.lim[0]) && (yi - tw >= a.box.lim[2]) &&
                            (zi - tw >= a.box.lim[4]) && (xi + tw <= a.box.lim[1]) &&
                            (yi + tw <= a.box.lim[3]) && (zi + tw <= a.box.lim[5]);
        const bool   usePbc    = a.box.anyPbc && !inside;
        const bool   anyPbcUse = __ballot(usePbc && valid) != 0;
        const double rr        = 2.0 * (double)(valid ? hi : 0.0f) * (1.0 + 1e-6) + a.margin;

        count = 0;
        for (int c = 0; c < numCand; ++c)
        {
            const int      node = __builtin_amdgcn_readfirstlane(cand[c]);
            const int      leaf = a.internalToLeaf[node];
            const uint32_t p0 = a.layout[leaf], p1 = a.layout[leaf + 1];
            if (p0 == p1) continue;
            // per-lane sphere-vs-leaf prune (conservative): skip the leaf if no lane can reach it
            const bool reach = valid && boxDist2(a.centers + 3 * (size_t)node, a.sizes + 3 * (size_t)node, xi, yi, zi,
                                                 0.0, 0.0, 0.0, a.box) < rr * rr;
            if (__ballot(reach) == 0) continue;
            for (uint32_t s0 = p0; s0 < p1; s0 += kWave)
            {
                const uint32_t jl = s0 + lane;
                double         xj = 0, yj = 0, zj = 0;
                if (jl < p1)
                {
                    xj = a.x[jl];
                    yj = a.y[jl];
                    zj = a.z[jl];
                }
                const int m = (int)min<uint32_t>(kWave, p1 - s0);
                candTested += m;
                if (anyPbcUse)
                {
                    for (int k = 0; k < m; ++k)
                    {
                        double dx = readlaneD(xj, k) - xi;
                        double dy = readlaneD(yj, k) - yi;
                        double dz = readlaneD(zj, k) - zi;
                        if (usePbc)
                        {
                            dx = foldPbc(dx, a.box, 0);
                            dy = foldPbc(dy, a.box, 1);
                            dz = foldPbc(dz, a.box, 2);
                        }
                        const uint32_t j   = s0 + k;
                        const bool     hit = valid && (dx * dx + dy * dy + dz * dz < radSq) && j != i;
                        if (hit)
                        {
                            if (count < a.ngmax) nlist[(size_t)count * kWave] = j;
                            count++;
                        }
                    }
                }
                else
                {
                    for (int k = 0; k < m; ++k)
                    {
                        double         dx  = readlaneD(xj, k) - xi;
                        double         dy  = readlaneD(yj, k) - yi;
                        double         dz  = readlaneD(zj, k) - zi;
                        const uint32_t j   = s0 + k;
                        const bool     hit = valid && (dx * dx + dy * dy + dz * dz < radSq) && j != i;
                        if (hit)
                        {
                            if (count < a.ngmax) nlist[(size_t)count * kWave] = j;
                            count++;
                        }
                    }
                }
            }
        }

        // ---- 4. h-nc iteration (sph/find_neighbors.hpp:28-33) ----------------------------------------
        if (!a.iterateH) break;
        const unsigned ncSph = count + 1;
        const bool     bad   = active && (ngmin > ncSph || (ncSph - 1) > a.ngmax);
        bool           again = false;
        if (bad)
        {
            if (iteration < 10)
            {
                iteration++;
                hi    = updateH(a.ng0, ncSph, hi, a.powTab);
                again = true;
            }
            else { iteration = 11; }
        }
        active = again;
        if (__ballot(again) == 0) break;
    }

    if (valid)
    {
        a.nc[i] = count + 1;
        if (a.iterateH) a.h[i] = hi;
    }
    // statistics (NcStats-like)
    const unsigned           failed = (valid && a.iterateH && iteration >= 10) ? 1u : 0u;
    const unsigned           nfail  = waveSum(failed);
    const unsigned           maxCnt = waveMax(valid ? count : 0u);
    const unsigned long long stored = waveSum((unsigned long long)(valid ? min(count, a.ngmax) : 0u));
    const unsigned long long tested = waveSum(valid ? candTested : 0ull);
    if (lane == 0)
    {
        if (nfail) atomicAdd(&a.stats[1], nfail);
        atomicMax(&a.stats[2], maxCnt);
        atomicAdd(reinterpret_cast<unsigned long long*>(a.stats + 4), stored);
        atomicAdd(reinterpret_cast<unsigned long long*>(a.stats + 6), tested);
    }
}

__global__ void exportKernel(const uint32_t* nidx, const uint32_t* nc, uint32_t first, uint32_t last, uint32_t ngmax,
                             uint32_t* out)
{
    uint32_t i = first + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= last) return;
    uint32_t ni = i - first, g = ni / kGroupSize, lane = ni % kGroupSize;
    uint32_t c  = nc[i] - 1;
    c           = c < ngmax ? c : ngmax;
    for (uint32_t k = 0; k < ngmax; ++k)
        out[(size_t)ni * ngmax + k] = k < c ? nidx[((size_t)g * ngmax + k) * kWave + lane] : 0u;
}

__global__ void importKernel(uint32_t* nidx, uint32_t first, uint32_t last, uint32_t ngmax, const uint32_t* in)
{
    uint32_t i = first + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= last) return;
    uint32_t ni = i - first, g = ni / kGroupSize, lane = ni % kGroupSize;
    for (uint32_t k = 0; k < ngmax; ++k)
        nidx[((size_t)g * ngmax + k) * kWave + lane] = in[(size_t)ni * ngmax + k];
}

hipError_t findNeighbors(const NsArgs& a, hipStream_t s)
{
    if (a.numGroups == 0) return hipSuccess;
    unsigned blocks = (a.numGroups + kNsWaves - 1) / kNsWaves;
    findNeighborsKernel<<<blocks, kNsWaves * 64, 0, s>>>(a);
    return hipGetLastError();
}

hipError_t exportNeighbors(const uint32_t* nidx, const uint32_t* nc, uint32_t first, uint32_t last, uint32_t ngmax,
                           uint32_t* out, hipStream_t s)
{
    uint32_t n = last - first;
    if (n) exportKernel<<<(n + 255) / 256, 256, 0, s>>>(nidx, nc, first, last, ngmax, out);
    return hipGetLastError();
}

hipError_t importNeighbors(uint32_t* nidx, uint32_t first, uint32_t last, uint32_t ngmax, const uint32_t* in,
                           hipStream_t s)
{
    uint32_t n = last - first;
    if (n) importKernel<<<(n + 255) / 256, 256, 0, s>>>(nidx, first, last, ngmax, in);
    return hipGetLastError();
}

} // namespace sx
