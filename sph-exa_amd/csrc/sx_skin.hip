/*! @file sx_skin.hip
 * @brief Skin-list reuse of the neighbor search on gfx950 (see sx_skin.hpp): displacement grid, node-box refresh,
 *        and the filter that turns the last build's skin lists into the step's exact lists.
 *
 * The filter replaces the step's search (cstone::findNeighbors + sph::findNeighborsSph, findneighbors.hpp:95-188,
 * find_neighbors.hpp:10-44) for every cluster whose skin is still valid.  One 256-thread workgroup per cluster:
 *   1. validity: each target's drift bound against its skin (sx_skin.hpp); the region's per-step displacement maximum
 *      comes from the grid cells around the wave boxes;
 *   2. the cluster's skin union U_s is staged in LDS as float positions relative to the cluster origin (minimum image,
 *      folded in double) with |p|^2, and the global indices;
 *   3. every lane walks its skin list (two u16 positions per word, prefetched) and tests each entry with the packed
 *      form of the search, t = |p|^2 + (|r|^2 - 4h^2) - 2 p.r in float, an error bound deciding when the reference's
 *      double criterion d2 < (double)(4h^2) must be evaluated (x, y, z from global memory) -- so the neighbor set is
 *      bit-identical to findNeighbors; j != i by global index;
 *   4. lanes with nc outside [ng0/4, ngmax+1] update h and walk again (at most 10 updates, the CPU loop's bound); an
 *      updated h must stay within the skin, else the cluster is stale;
 *   5. h, nc, the targets' RecX and the exact lists (ascending positions into U_s, first ngmax in stream order) are
 *      written only by a cluster that completes;
 *   4b. (round 6) a walk whose hit bits equal one of the cluster's two recorded list sets keeps that set (no 5), and a
 *      cluster whose freeze reference proves its hits unchanged is not walked (1b: the XMass over its exact lists).
 * This file is compiled with -ffp-contract=off (the double criterion must round like the reference).
 */
#include "sx_kernel_poly.hpp"
#include "sx_skin.hpp"
#include "sx_traverse.hpp"

namespace sx
{

namespace
{

constexpr int kWalkPF  = 8;    //!< skin-list words per walk block (16 entries: one u16 of hit bits per lane)
//! walk blocks per lane at the largest skin-list capacity (256 entries)
constexpr int kWalkBlocks = (nlocWords(256) + kWalkPF - 1) / kWalkPF;
constexpr int kB       = kCluster;

__device__ __forceinline__ int cellIndex(double v, const SkinGrid& g, int d) { return gridCell(v, g, d); }

//! v if k, else +0 (an AND of the bits: no select the compiler could turn into a branch)
__device__ __forceinline__ float keepOrZero(float v, bool k)
{
    return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, v) & (0u - (uint32_t)k));
}

//! |(x, y, z)| of float differences, rounded upwards (an upper bound of the exact length of the exact differences:
//! each float difference is within 2^-24 relative, the sum of squares and the root within a few ulp more)
__device__ __forceinline__ float norm3up(float x, float y, float z)
{
    return sqrtf(fmaf(x, x, fmaf(y, y, z * z))) * (1.0f + 0x1p-18f) + 1e-30f;
}

//! leaf boxes from their particles (relative to the geometric center, minimum image), one wave per leaf node
__global__ void leafBoxKernel(const int32_t* childOffsets, const int32_t* internalToLeaf, const uint32_t* layout,
                              int numNodes, const double* gc, const double* gs, const double* x, const double* y,
                              const double* z, DevBox box, double* centers, double* sizes, int withCells)
{
    // 16 lanes per node (a leaf holds at most the bucket size, 64 on the path; four nodes per wave)
    constexpr int G    = 16;
    const int     node = blockIdx.x * (blockDim.x / G) + (int)(threadIdx.x / G);
    const int     sub  = threadIdx.x & (G - 1);
    const bool    leafNode = node < numNodes && childOffsets[node] == 0;
    const int      leaf = leafNode ? internalToLeaf[node] : 0;
    const uint32_t p0 = leafNode ? layout[leaf] : 0u, p1 = leafNode ? layout[leaf + 1] : 0u;
    const double   c[3] = {leafNode ? gc[3 * node] : 0.0, leafNode ? gc[3 * node + 1] : 0.0,
                           leafNode ? gc[3 * node + 2] : 0.0};
    double         lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t j = p0 + sub; j < p1; j += G)
    {
        const double q[3] = {x[j], y[j], z[j]};
        for (int d = 0; d < 3; ++d)
        {
            const double r = foldPbc(q[d] - c[d], box, d);
            lo[d]          = fmin(lo[d], r);
            hi[d]          = fmax(hi[d], r);
        }
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1)
        for (int d = 0; d < 3; ++d)
        {
            lo[d] = fmin(lo[d], __shfl_xor(lo[d], o, G));
            hi[d] = fmax(hi[d], __shfl_xor(hi[d], o, G));
        }
    if (leafNode && sub == 0)
    {
        for (int d = 0; d < 3; ++d)
        {
            if (withCells) // the box of the particles and the leaf's cell together
            {
                lo[d] = fmin(lo[d], -gs[3 * node + d]);
                hi[d] = fmax(hi[d], gs[3 * node + d]);
            }
            // an empty leaf keeps its cell (it contributes no candidates either way)
            const bool   empty = p1 <= p0;
            const double m     = empty ? 0.0 : 0.5 * (lo[d] + hi[d]);
            const double s     = empty ? gs[3 * node + d] : 0.5 * (hi[d] - lo[d]);
            centers[3 * node + d] = c[d] + m;
            sizes[3 * node + d]   = s;
        }
    }
}

//! inner boxes of one level from their eight children (folded relative to the node's geometric center)
__global__ void innerBoxKernel(const int32_t* childOffsets, int b, int e, const double* gc, DevBox box, double* centers,
                               double* sizes)
{
    const int node = b + blockIdx.x * blockDim.x + threadIdx.x;
    if (node >= e) return;
    const int c0 = childOffsets[node];
    if (c0 == 0) return;
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int k = c0; k < c0 + 8; ++k)
        for (int d = 0; d < 3; ++d)
        {
            const double r = foldPbc(centers[3 * k + d] - gc[3 * node + d], box, d);
            lo[d]          = fmin(lo[d], r - sizes[3 * k + d]);
            hi[d]          = fmax(hi[d], r + sizes[3 * k + d]);
        }
    for (int d = 0; d < 3; ++d)
    {
        centers[3 * node + d] = gc[3 * node + d] + 0.5 * (lo[d] + hi[d]);
        sizes[3 * node + d]   = 0.5 * (hi[d] - lo[d]);
    }
}

__global__ void markStaleKernel(const uint32_t* list, uint32_t numClusters, float* acc)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < list[0] && k < numClusters) acc[list[1 + k]] = INFINITY;
}

__global__ __launch_bounds__(1024) void reduceClusterStatsKernel(const uint4* cl, uint32_t n, uint32_t* stats)
{
    __shared__ uint32_t           s_max[4][16];
    __shared__ unsigned long long s_sum[3][16];
    uint32_t                      mx = 0, mu = 0, kp = 0, fz = 0; // clusters whose exact lists the filter kept, frozen
    unsigned long long            st = 0, te = 0, un = 0;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
    {
        const uint4 v = cl[i];
        mx = max(mx, v.x), st += v.y & 0x3fffffffu, te += v.z, un += v.w, mu = max(mu, v.w), kp += v.y >> 31,
        fz += (v.y >> 30) & 1u;
    }
    mx = waveMax(mx), mu = waveMax(mu), st = waveSum(st), te = waveSum(te), un = waveSum(un), kp = waveSum(kp), fz = waveSum(fz);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
        s_max[0][w] = mx, s_max[1][w] = mu, s_max[2][w] = kp, s_max[3][w] = fz, s_sum[0][w] = st, s_sum[1][w] = te, s_sum[2][w] = un;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        for (int k = 1; k < (int)(blockDim.x >> 6); ++k)
            mx = max(mx, s_max[0][k]), mu = max(mu, s_max[1][k]), kp += s_max[2][k], fz += s_max[3][k], st += s_sum[0][k],
            te += s_sum[1][k], un += s_sum[2][k];
        stats[2]                                          = mx;
        stats[18]                                         = kp;
        stats[19]                                         = fz;
        stats[12]                                         = mu;
        *reinterpret_cast<unsigned long long*>(stats + 4) = st;
        *reinterpret_cast<unsigned long long*>(stats + 6) = te;
        *reinterpret_cast<unsigned long long*>(stats + 8) = un;
    }
}

//! a stale cluster goes to the rebuild list, or -- stale again on the step after its rebuild (a region whose relative
//! motion outruns any skin: a shock, a convergent flow) -- straight to the exact-search list (a.direct)
__device__ __forceinline__ void pushStale(const SkinArgs& a, uint32_t c)
{
    uint32_t* L = (a.direct && a.streak && a.streak[c]) ? a.direct : a.stale;
    L[1 + atomicAdd(&L[0], 1u)] = c;
    if (a.streak) a.streak[c] = 1;
    if (a.same) a.same[c] = 0; // its lists are rewritten by a rebuild or the exact search (into set A)
}
static_assert((kWalkBlocks + 1) / 2 <= (int)kSkinMaskWords, "hit-mask words per target");

//! four workgroups per CU by LDS: at most 128 VGPRs keep them all
__global__ __launch_bounds__(kB) __attribute__((amdgpu_waves_per_eu(4))) void skinFilterKernel(SkinArgs a,
                                                                                              uint32_t numClusters)
{
    // LDS: 40960 B, exactly a quarter of the CU's 160 KB: four workgroups per CU (one more byte leaves three)
    __shared__ float4   s_rec[kSkinCap]; // U_s positions relative to the cluster origin, |p|^2; then the exact-union
                                         // ranks (u16) of the U_s entries, once pass A is done with the positions
    __shared__ uint8_t  s_hit[kSkinCap + 4]; // U_s entry hit by some target (exact union); [kSkinCap]: spare
    __shared__ uint16_t s_bm[kWalkBlocks][kB]; // pass A's stored hits per walk block and lane (bit e: entry e)
    uint16_t* const     s_rank = reinterpret_cast<uint16_t*>(s_rec);
    __shared__ float    s_red[kClusterWaves];
    __shared__ int      s_vote[kClusterWaves];
    __shared__ uint32_t s_wsum[kClusterWaves];
    __shared__ uint4    s_cst[kClusterWaves]; // .w: the wave's freeze minimum K + 2h (s_wsum: K - 2h) at the end

    const uint32_t nWork = a.list ? __builtin_amdgcn_readfirstlane(a.list[0]) : numClusters;
    if (blockIdx.x >= nWork) return;
    const uint32_t blk  = a.list ? blockIdx.x : xcdBlock(blockIdx.x, gridDim.x);
    const uint32_t c    = __builtin_amdgcn_readfirstlane(a.list ? a.list[1 + blk] : blk);
    const int      wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t gw   = c * kClusterWaves + wave;
    const uint32_t c0   = a.first + c * kCluster;
    const uint32_t i    = c0 + threadIdx.x;
    const bool     valid = gw < a.numGroups && i < a.last;
    const uint32_t iS    = valid ? i : c0;
    const double   xi = a.x[iS], yi = a.y[iS], zi = a.z[iS];
    const double   ox = a.x[c0], oy = a.y[c0], oz = a.z[c0];
    float          hi   = a.h[iS];
    const float    h0   = hi;
    const float    hbi  = a.fresh ? hi : a.hb[iS];
    // the last step's displacement relative to the cluster's reference particle (its first): this target's relative
    // path since the build, d_i (rounding of the float displacements pushed upwards)
    const float    ux = a.dispX[c0], uy = a.dispY[c0], uz = a.dispZ[c0];
    const float    di = a.fresh ? 0.0f
                                : a.rel[iS] + norm3up(a.dispX[iS] - ux, a.dispY[iS] - uy, a.dispZ[iS] - uz);
    const float    Ri = 2.0f * (hbi * a.skin1);
    const uint32_t scount = valid ? a.scnt[i] - 1u : 0u;
    const uint32_t U      = __builtin_amdgcn_readfirstlane(a.ucountS[c]);
    const float    kEps   = 0x1p-16f;
    // the freeze reference (1b), loaded with the target's state: its latency off the vote's chain
    // the cluster's list sets (SkinArgs::same): the current one (B with a second set and its bit), which hold lists
    const uint32_t lstate    = (a.same && a.keepLists && !a.fresh) ? (uint32_t)a.same[c] : 0u;
    const uint32_t lcur      = (a.nlocB && (lstate & kListsBSel)) ? 1u : 0u;
    const bool     curValid  = ((lstate >> lcur) & 1u) != 0;
    const bool     mayFreeze = a.frz && curValid;
    const float2   fref      = mayFreeze ? a.frz[c] : make_float2(-INFINITY, -INFINITY);
    //! per bit k of v: whether any thread of the workgroup set it (one vote round for several decisions)
    auto           blockBits = [&](uint32_t v) -> uint32_t {
        uint32_t w = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k)
            w |= __ballot((v >> k) & 1u) != 0 ? 1u << k : 0u;
        if (lane == 0) s_vote[wave] = (int)w;
        __syncthreads();
        uint32_t any = 0;
        for (int k = 0; k < kClusterWaves; ++k)
            any |= (uint32_t)s_vote[k];
        __syncthreads();
        return any;
    };
    auto blockAny = [&](bool v) -> bool { return blockBits(v ? 1u : 0u) != 0; };

    // ---- 1. the region's displacement since the build: A = acc + this step's maximum over the grid cells around
    //         the wave boxes grown by the largest skin radius
    float A = 0.0f;
    if (!a.fresh)
    {
        const double rx = foldPbc(xi - ox, a.box, 0), ry = foldPbc(yi - oy, a.box, 1), rz = foldPbc(zi - oz, a.box, 2);
        double       lo[3]  = {valid ? rx : INFINITY, valid ? ry : INFINITY, valid ? rz : INFINITY};
        double       hb3[3] = {valid ? rx : -INFINITY, valid ? ry : -INFINITY, valid ? rz : -INFINITY};
        float        rmax   = valid ? Ri : 0.0f;
        for (int d = 0; d < 3; ++d)
        {
            lo[d]  = -waveMax(-lo[d]);
            hb3[d] = waveMax(hb3[d]);
        }
        rmax      = waveMax(rmax);
        float gmx = 0.0f;
        if (rmax > 0.0f)
        {
            const double o[3] = {ox, oy, oz};
            int          k0[3], nk[3];
            uint32_t     total = 1; // at most grid.n^3 (each nk within [1, grid.n]): 32-bit division below
            for (int d = 0; d < 3; ++d)
            {
                k0[d]  = cellIndex(o[d] + lo[d] - (double)rmax, a.grid, d);
                int k1 = cellIndex(o[d] + hb3[d] + (double)rmax, a.grid, d);
                nk[d]  = k1 - k0[d] + 1;
                if (a.grid.pbc[d] && nk[d] >= a.grid.n) k0[d] = 0, nk[d] = a.grid.n;
                total *= nk[d];
            }
            // a region of many cells (a wave spanning an SFC seam across the box) scans them all: rare
            for (uint32_t q = lane; q < total; q += kWave)
            {
                int      k[3];
                uint32_t r = q;
                for (int d = 0; d < 3; ++d)
                {
                    const uint32_t rq = r / (uint32_t)nk[d];
                    k[d]              = k0[d] + (int)(r - rq * (uint32_t)nk[d]);
                    r                 = rq;
                    if (a.grid.pbc[d]) k[d] = wrapCell(k[d], a.grid.n);
                }
                const size_t nc   = (size_t)a.grid.n * a.grid.n * a.grid.n;
                const size_t cell = ((size_t)k[2] * a.grid.n + k[1]) * a.grid.n + k[0];
                const uint32_t lx = a.cells[cell], ly = a.cells[nc + cell], lz = a.cells[2 * nc + cell];
                if (lx != 0xffffffffu) // a cell without particles has no range
                {
                    // the largest |d - u| over the cell's component ranges
                    const float ex = fmaxf(fabsf(orderedFloat(lx) - ux), fabsf(orderedFloat(a.cells[3 * nc + cell]) - ux));
                    const float ey = fmaxf(fabsf(orderedFloat(ly) - uy), fabsf(orderedFloat(a.cells[4 * nc + cell]) - uy));
                    const float ez = fmaxf(fabsf(orderedFloat(lz) - uz), fabsf(orderedFloat(a.cells[5 * nc + cell]) - uz));
                    gmx = fmaxf(gmx, norm3up(ex, ey, ez));
                }
            }
        }
        gmx = waveMax(gmx);
        if (lane == 0) s_red[wave] = gmx;
        __syncthreads();
        float g = s_red[0];
        for (int w = 1; w < kClusterWaves; ++w)
            g = fmaxf(g, s_red[w]);
        A = a.acc[c] + g;
        __syncthreads();
    }
    // a target's skin holds every current neighbor while 2h + d + A <= R (1 - eps); a build that overflowed a capacity
    // (skin list beyond ngmaxS, union beyond the slot) never serves, nor a union beyond the LDS capacity
    auto withinSkin = [&](float h) { return 2.0f * h + di + A <= Ri * (1.0f - kEps); };
    // ---- 1b. frozen: since the last pass that walked this cluster (its reference: per target the smallest distance
    //          g of a skin entry to the 2h sphere, and d_i + A_C, h then) no target and no entry has moved, nor has
    //          2h changed, by enough for any entry to cross the sphere -- the relative motion of i and an entry is at
    //          most the growth of d_i + A_C since (sx_skin.hpp's bound, also for entries outside the ball), so
    //          2 |h - h_ref| + (d_i + A_C) - (d_i + A_C)_ref < g keeps every hit and miss.  The exact lists in place
    //          are then this step's: no walk of the skin lists, the fused XMass over the exact lists
    //          Per cluster the reference pass left fref = min over its targets of K_i + 2 h_i and of K_i - 2 h_i,
    //          K_i = g_i + (d_i + A_C) then (-inf: never frozen); d_i + A_C + 2h_i below the first and d_i + A_C - 2h_i
    //          below the second give 2 |h_i - h_i,ref| + (d_i + A_C) < K_i for every target.  One vote with 1.
    bool frozen = false;
    {
        const bool bad  = valid && (scount > a.ngmaxS || !withinSkin(hi));
        // one more drift like the one since the build would make the cluster stale (stats[13]: the host stops using
        // skins that cannot outlast two steps, sx_sim.cpp)
        const bool thin = !a.fresh && valid && 2.0f * hi + 2.0f * (di + A) > Ri * (1.0f - kEps);
        const float e    = di + A + kEps * Ri;
        const bool  melt = valid && !(e + 2.0f * hi < fref.x && e - 2.0f * hi < fref.y);
        const uint32_t v = blockBits((bad ? 1u : 0u) | (thin ? 2u : 0u) | (melt ? 4u : 0u));
        if ((v & 1u) || U > (uint32_t)kSkinCap || U > a.ucap - a.uoff)
        {
            if (threadIdx.x == 0) pushStale(a, c);
            return;
        }
        if ((v & 2u) && threadIdx.x == 0) atomicAdd(&a.stats[13], 1u);
        frozen = mayFreeze && !(v & 4u);
    }
    int      iteration = 0;
    unsigned count = 0, stored = 0;
    const float mi   = a.m[iS];
    float    rho0    = mi; // fused XMass (xmassJLoop, hydro_ve/xmass_kern.hpp:50-79) of the final pass
    bool     kept    = frozen;
    uint32_t ue      = 0;
    float    frzK    = -INFINITY; // this pass's freeze reference (1b)
    const float xr = (float)foldPbc(xi - ox, a.box, 0), yr = (float)foldPbc(yi - oy, a.box, 1),
                zr = (float)foldPbc(zi - oz, a.box, 2);
    //! set k's lists of this lane, union of this cluster, union count
    auto setLists = [&](uint32_t k) { return (k ? a.nlocB : a.nloc) + (size_t)gw * nlocWords(a.ngmax) * kWave + lane; };
    auto setUnion = [&](uint32_t k) { return a.uni + (size_t)c * a.ucap + (k ? a.uoffB : 0u); };
    auto setCount = [&](uint32_t k) { return k ? a.ucountB + c : a.ucount + c; };
    auto setMask  = [&](uint32_t k) {
        uint32_t* m = k ? a.hitMaskB : a.hitMask;
        return m ? m + (size_t)gw * kSkinMaskWords * kWave + lane : nullptr;
    };
    const uint32_t* const ll = setLists(lcur); // the current set's lists (the frozen path's XMass)
    //! stages n union entries (global indices list[0 .. n)) as float positions relative to the cluster origin and
    //! masses; returns the largest |p|_1 over them (all loads of a thread in flight together)
    auto stage = [&](const uint32_t* list, uint32_t n) -> float {
        constexpr int S = (kSkinCap + kB - 1) / kB; // every entry of a union up to kSkinCap
        uint32_t      js[S];
#pragma unroll
        for (int q = 0; q < S; ++q)
        {
            // unconditional (clamped): a load under a condition is waited for at the branch merge
            js[q] = list[min(threadIdx.x + q * kB, n ? n - 1u : 0u)];
        }
        double px[S], py[S], pz[S];
        float  mq[S];
#pragma unroll
        for (int q = 0; q < S; ++q)
            px[q] = a.x[js[q]], py[q] = a.y[js[q]], pz[q] = a.z[js[q]], mq[q] = a.m[js[q]];
        float pm = 0.0f;
#pragma unroll
        for (int q = 0; q < S; ++q)
        {
            const uint32_t u = threadIdx.x + q * kB;
            if (u < n)
            {
                const float fx = (float)foldPbc(px[q] - ox, a.box, 0);
                const float fy = (float)foldPbc(py[q] - oy, a.box, 1);
                const float fz = (float)foldPbc(pz[q] - oz, a.box, 2);
                s_rec[u]       = make_float4(fx, fy, fz, mq[q]);
                pm             = fmaxf(pm, fabsf(fx) + fabsf(fy) + fabsf(fz));
            }
        }
        pm = waveMax(pm);
        if (lane == 0) s_red[wave] = pm;
        __syncthreads();
        float r = s_red[0];
        for (int w = 1; w < kClusterWaves; ++w)
            r = fmaxf(r, s_red[w]);
        return r;
    };

    if (frozen)
    {
        // ---- 2'/3'. the exact union staged, the fused XMass over the exact lists (count, h, lists unchanged)
        ue = __builtin_amdgcn_readfirstlane(*setCount(lcur));
        (void)stage(setUnion(lcur), ue);
        count  = valid ? a.nc[i] - 1u : 0u;
        stored = min(count, a.ngmax);
        if (a.xmOut && valid)
        {
            const float    hInv = 1.0f / hi, hInv2 = hInv * hInv;
            const uint32_t nw = (stored + 1) >> 1, last = nw ? nw - 1 : 0u;
            constexpr int  PF = kWalkPF;
            uint32_t       nx[PF];
#pragma unroll
            for (int u = 0; u < PF; ++u)
                nx[u] = ll[(size_t)min((uint32_t)u, last) * kWave];
            for (uint32_t w0 = 0; w0 < nw; w0 += PF)
            {
                uint32_t cw[PF];
#pragma unroll
                for (int u = 0; u < PF; ++u)
                {
                    cw[u] = nx[u];
                    nx[u] = ll[(size_t)min(w0 + PF + u, last) * kWave];
                }
#pragma unroll
                for (int u = 0; u < PF; ++u)
                {
                    const uint32_t w = w0 + u;
#pragma unroll
                    for (int h2 = 0; h2 < 2; ++h2)
                    {
                        const float4 q  = s_rec[min(h2 ? cw[u] >> 16 : cw[u] & 0xffffu, (uint32_t)kSkinCap - 1u)];
                        const float  dx = q.x - xr, dy = q.y - yr, dz = q.z - zr;
                        const float  r2 = fmaf(dx, dx, fmaf(dy, dy, dz * dz));
                        rho0 += keepOrZero(kernelWt(r2 * hInv2) * q.w, 2 * w + h2 < stored);
                    }
                }
            }
        }
    }
    else
    {

    // ---- 2. stage U_s
    const uint32_t* un   = a.uni + (size_t)c * a.ucap + a.uoff;
    const float     pmax = stage(un, U);

    // ---- 3. walk the skin lists: count, mark the exact union, store the hits' U_s positions (rewritten in step 5)
    const uint32_t  WS = nlocWords(a.ngmaxS);
    const uint32_t* sl = a.sloc + (size_t)gw * WS * kWave + lane;
    const unsigned  ngmin     = a.ng0 / 4;
    bool            active    = valid;
    //! one pass over this lane's skin list in blocks of kWalkPF words (16 entries): begin(b) starts block b,
    //! visit(p, e, inr) takes entry e of the block (U_s position p; inr: the entry is in the list, else p is a valid
    //! position of no meaning), end(b) closes the block.  Every entry of a block is visited without a branch (a wave's
    //! lanes take the hit and the miss paths of one entry together anyway; the branches only cost exec-mask traffic).
    //! List words are loaded a block ahead, every load unconditional (clamped to the lane's last word, word 0 for an
    //! empty list): a load under a condition is waited for at the branch merge
    auto walk = [&](auto&& begin, auto&& visit, auto&& end) {
        if (!valid) return;
        const uint32_t nw   = (scount + 1) >> 1;
        const uint32_t last = nw ? nw - 1 : 0u;
        constexpr int  PF   = kWalkPF;
        uint32_t       nx[PF];
#pragma unroll
        for (int u = 0; u < PF; ++u)
            nx[u] = sl[(size_t)min((uint32_t)u, last) * kWave];
        for (uint32_t w0 = 0, b = 0; w0 < nw; w0 += PF, ++b)
        {
            uint32_t cw[PF];
#pragma unroll
            for (int u = 0; u < PF; ++u)
            {
                cw[u] = nx[u];
                nx[u] = sl[(size_t)min(w0 + PF + u, last) * kWave];
            }
            begin(b);
#pragma unroll
            for (int u = 0; u < PF; ++u)
            {
                // words past the list repeat its last word (valid positions); the upper half past an odd count is
                // clamped into the staged range
                const uint32_t w = w0 + u;
                visit(cw[u] & 0xffffu, 2 * u, 2 * w < scount);
                visit(min(cw[u] >> 16, (uint32_t)kSkinCap - 1u), 2 * u + 1, 2 * w + 1 < scount);
            }
            end(b);
        }
    };
    float          r2f = 0, tol = 0;
    double         radSq = 0;
    bool           safe = true, usePbc = false;
    //! t = |p - r|^2 - 4h^2 in float (p, r relative to the cluster origin), with the reference's double criterion
    //! where |t| may be rounding (the bound of sx_neighbors.hip's |p|^2 + |r|^2 - 2p.r form, which covers this one);
    //! r2 becomes the pair's r^2 (the fused XMass)
    auto test = [&](uint32_t p, float4 q, bool inr, float& r2, float& t) -> bool {
        const float dx = q.x - xr, dy = q.y - yr, dz = q.z - zr;
        r2             = fmaf(dx, dx, fmaf(dy, dy, dz * dz));
        t              = r2 - r2f;
        bool        hit = t < 0.0f;
        // bitwise, not short-circuit: one branch per entry, around the (rare) double criterion
        if (inr & ((!safe) | (fabsf(t) <= tol)))
        {
            const uint32_t j  = un[p];
            double         ex = a.x[j] - xi, ey = a.y[j] - yi, ez = a.z[j] - zi;
            if (usePbc)
            {
                ex = foldPbc(ex, a.box, 0);
                ey = foldPbc(ey, a.box, 1);
                ez = foldPbc(ez, a.box, 2);
            }
            const double d2 = ex * ex + ey * ey + ez * ez;
            hit             = d2 < radSq;
            r2              = (float)d2;
        }
        return inr & hit; // j != i: the build's skin list never holds the target itself
    };
    float hInv2 = 0;
    float tmin = INFINITY; // the final pass's smallest |t| over the walked entries (1b)
    while (true)
    {
        for (uint32_t u = threadIdx.x; u < U; u += kB)
            s_hit[u] = 0;
        __syncthreads();
        r2f              = 4.0f * hi * hi;
        radSq            = (double)r2f;
        const float hInv = 1.0f / hi;
        hInv2            = hInv * hInv;
        rho0             = mi;
        const double tw  = 2.0 * (double)hi;
        const bool inside = (xi - tw >= a.box.lim[0]) && (yi - tw >= a.box.lim[2]) && (zi - tw >= a.box.lim[4]) &&
                            (xi + tw <= a.box.lim[1]) && (yi + tw <= a.box.lim[3]) && (zi + tw <= a.box.lim[5]);
        usePbc = a.box.anyPbc && !inside;
        // the float test is exact only where the minimum image relative to the cluster origin is the pair's minimum
        // image (|r| + 2h < L/2 on periodic axes); other lanes test every entry in double
        safe = true;
        for (int d = 0; d < 3; ++d)
        {
            const float rd = d == 0 ? xr : (d == 1 ? yr : zr);
            if (a.box.pbc[d] && (fabsf(rd) + 2.05f * hi) >= 0.49f * (float)a.box.l[d]) safe = false;
        }
        // |t| below tol may be rounding: those entries take the double criterion (sx_neighbors.hip's bound, with
        // E >= |p| + |r| over the staged entries)
        const float E = pmax + fabsf(xr) + fabsf(yr) + fabsf(zr);
        tol           = 0x1p-19f * fmaf(E, E, r2f);
        // every valid lane walks (a converged lane marks the same union entries again); no global store in the walk:
        // vmcnt counts stores too, in order, so a store between the prefetch and its use would be waited for as well
        unsigned cnt = 0, st = 0;
        uint32_t bits = 0;
        tmin = INFINITY;
        walk([&](uint32_t) { bits = 0; },
             [&](uint32_t p, int e, bool inr) {
                 const float4 q = s_rec[p];
                 float        r2, t;
                 const bool   hit  = test(p, q, inr, r2, t);
                 tmin = fminf(tmin, fabsf(t)); // entries past the list (repeated or clamped) only lower it
                 const bool   keep = hit & (cnt < a.ngmax); // the first ngmax hits in list order
                 // no branch: a miss marks the spare byte; rho0 + (+0) == rho0
                 s_hit[keep ? p : (uint32_t)kSkinCap] = 1;
                 bits |= (uint32_t)keep << e;
                 st += (uint32_t)keep;
                 cnt += (uint32_t)hit;
                 if (a.xmOut) rho0 += keepOrZero(kernelWt(r2 * hInv2) * q.w, keep);
             },
             [&](uint32_t b) { s_bm[b][threadIdx.x] = (uint16_t)bits; });
        count  = cnt;
        stored = st;
        // ---- 4. h-nc iteration (sph/find_neighbors.hpp:28-33); a grown h must stay within the skin
        bool again = false, outgrown = false;
        if (a.iterateH && active)
        {
            const unsigned ncSph = count + 1;
            if (ngmin > ncSph || (ncSph - 1) > a.ngmax)
            {
                if (iteration < 10)
                {
                    iteration++;
                    hi       = updateH(a.ng0, ncSph, hi, a.powTab);
                    again    = true;
                    outgrown = !withinSkin(hi);
                }
                else iteration = 11;
            }
        }
        active = again;
        if (blockAny(outgrown))
        {
            if (threadIdx.x == 0) pushStale(a, c);
            return; // h, nc untouched; lists and union are rewritten by the rebuild
        }
        if (!blockAny(again)) break;
    }
    // the freeze reference of this pass (1b): g = min((min |t| - tol) / (R + 2h), R - 2h) bounds every entry's
    // distance to the 2h sphere from below -- |r - 2h| = |r^2 - 4h^2| / (r + 2h) for an entry within the skin radius R
    // (|t| is within tol of |r^2 - 4h^2|), at least R - 2h beyond it; only lanes whose test was the float one (safe)
    // and whose h did not iterate
    if (valid && safe && iteration == 0)
    {
        const float g = fminf(fmaxf(0.0f, tmin - tol) / ((Ri + 2.0f * hi) * (1.0f + 0x1p-20f)), Ri - 2.0f * hi);
        frzK          = (g * (1.0f - 0x1p-20f) + di + A) * (1.0f - 0x1p-22f);
    }

    // ---- 4b. every target kept the same hits as the pass that wrote one of this cluster's list sets: that set is
    //          this step's (the skin lists are fixed between builds, so equal bits are equal sets) -- the current one
    //          (kept), or the other (the set becomes current: a lattice's h moving back to the last shell)
    const uint32_t nbl = valid ? (((scount + 1) >> 1) + kWalkPF - 1) / kWalkPF : 0u; // walk blocks of this lane
    auto           maskWord = [&](uint32_t k) {
        const uint32_t lo = s_bm[2 * k][threadIdx.x];
        return 2 * k + 1 < nbl ? lo | ((uint32_t)s_bm[2 * k + 1][threadIdx.x] << 16) : lo;
    };
    auto sameBits = [&](const uint32_t* hm) -> bool {
        constexpr int MW = (kWalkBlocks + 1) / 2;
        const uint32_t nmw = (nbl + 1) >> 1;
        uint32_t       prev[MW];
#pragma unroll
        for (int k = 0; k < MW; ++k)
            prev[k] = hm[(size_t)min((uint32_t)k, nmw ? nmw - 1 : 0u) * kWave]; // unconditional (clamped)
        bool diff = false;
#pragma unroll
        for (int k = 0; k < MW; ++k)
            if ((uint32_t)k < nmw) diff |= prev[k] != maskWord(k);
        return !blockAny(diff);
    };
    uint32_t lnew = lstate; // the cluster's list sets after this pass
    uint32_t ltgt = lcur;   // the set this pass's lists are in
    // the other set first: a walked (not frozen) step of a cluster that holds two sets mostly moves back to the other
    // (a lattice's h crossing a shell: two such steps, then frozen ones); each comparison reads 32 B per target
    const bool otherValid = a.nlocB && a.hitMask && ((lstate >> (1u - lcur)) & 1u);
    if (otherValid && sameBits(setMask(1u - lcur)))
    {
        kept = true, ltgt = 1u - lcur;
        lnew = (lstate & 3u) | (ltgt ? kListsBSel : 0u);
    }
    if (!kept && a.hitMask && curValid) kept = sameBits(setMask(lcur));
    if (!kept)
    {
        // written into the other set (with a second one: the current set stays valid), or set A
        ltgt = a.nlocB ? 1u - lcur : 0u;
        lnew = (curValid && ltgt != lcur ? 1u << lcur : 0u) | (1u << ltgt) | (ltgt ? kListsBSel : 0u);
    }

    // ---- 5. exact union: ranks of the hit U_s entries (U_s order), the union at the set's start, lists rewritten
    ue = kept ? __builtin_amdgcn_readfirstlane(*setCount(ltgt)) : 0u;
    if (!kept)
    {
        // every thread a run of consecutive entries
        const uint32_t B  = (U + kB - 1) / kB;
        const uint32_t b0 = min(U, threadIdx.x * B), b1 = min(U, b0 + B);
        uint32_t       sum = 0;
        for (uint32_t u = b0; u < b1; ++u)
            sum += s_hit[u];
        uint32_t incl = sum;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1)
        {
            const uint32_t t = __shfl_up(incl, o, kWave);
            if (lane >= o) incl += t;
        }
        if (lane == kWave - 1) s_wsum[wave] = incl;
        __syncthreads();
        uint32_t run = incl - sum;
        for (int w = 0; w < wave; ++w)
            run += s_wsum[w];
        for (int w = 0; w < kClusterWaves; ++w)
            ue += s_wsum[w];
        uint32_t* ux = setUnion(ltgt);
        for (uint32_t u0 = b0; u0 < b1; u0 += 8)
        {
            uint32_t jj[8];
#pragma unroll
            for (int q = 0; q < 8; ++q)
                jj[q] = un[min(u0 + q, U - 1u)];
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (u0 + q < b1)
                {
                    s_rank[u0 + q] = (uint16_t)run;
                    if (s_hit[u0 + q]) ux[run++] = jj[q];
                }
        }
        __syncthreads();
    }
    // pass B: the same walk, the first ngmax hits written as exact-union ranks (two per word); the hit bits recorded
    if (!kept)
    {
        uint32_t* const lw = setLists(ltgt);
        unsigned st = 0;
        uint32_t pend = 0, bits = 0;
        walk([&](uint32_t b) { bits = s_bm[b][threadIdx.x]; },
             [&](uint32_t p, int e, bool) {
                 const bool     keep = ((bits >> e) & 1u) != 0;
                 const uint32_t r    = s_rank[p];
                 const bool     odd  = (st & 1u) != 0;
                 if (keep && odd) lw[(size_t)(st >> 1) * kWave] = pend | (r << 16);
                 pend = (keep && !odd) ? r : pend;
                 st += keep ? 1u : 0u;
             },
             [](uint32_t) {});
        if (st & 1u) lw[(size_t)(st >> 1) * kWave] = pend;
        if (uint32_t* const hm = setMask(ltgt))
            for (uint32_t k = 0; 2 * k < nbl; ++k)
                hm[(size_t)k * kWave] = maskWord(k);
        if (threadIdx.x == 0) *setCount(ltgt) = ue;
    }
    if (threadIdx.x == 0 && a.same && lnew != lstate) a.same[c] = (uint8_t)lnew;
    } // not frozen

    // ---- 6. outputs
    if (valid)
    {
        if (!frozen)
        {
            a.nc[i] = count + 1; // (a frozen cluster's count is the one in place)
        }
        if (a.iterateH && iteration > 0) a.h[i] = hi; // (h changes only by the iteration)
        if (a.rxOut) a.rxOut[i] = RecX{xi, yi, zi, hi, a.m[i]};
        if (a.fresh) a.hb[i] = h0;
        a.rel[i] = di; // 0 for a fresh cluster
        if (a.xmOut)
        {
            const float hInv  = 1.0f / hi;
            const float h3Inv = hInv * hInv * hInv;
            const float xm    = (float)((double)mi / ((double)rho0 * a.K * (double)h3Inv));
            a.xmOut[i]        = xm;
            if (a.rtXm) a.rtXm[i] = RecT{xm, 0.0f, 0.0f, 0.0f};
        }
    }
    if (threadIdx.x == 0)
    {
        a.acc[c]    = a.fresh ? 0.0f : A;
        if (a.streak && !a.fresh) a.streak[c] = 0; // served by its skin: a later stale step rebuilds it again
    }
    const unsigned           failed = (valid && a.iterateH && iteration >= 10) ? 1u : 0u;
    const unsigned           nfail  = waveSum(failed);
    const unsigned           maxCnt = waveMax(valid ? count : 0u);
    const unsigned long long nst    = waveSum((unsigned long long)(valid ? stored : 0u));
    const unsigned long long walked = waveSum((unsigned long long)scount);
    // the freeze reference of a walked pass (1b): the cluster's minima of K_i +- 2h_i
    const float kp = waveMin(valid ? frzK + 2.0f * hi : INFINITY), km = waveMin(valid ? frzK - 2.0f * hi : INFINITY);
    if (lane == 0)
    {
        if (nfail) atomicAdd(&a.stats[1], nfail);
        // (LDS: 40960 B is exactly a quarter of the CU's, four workgroups; no byte more)
        s_cst[wave]  = make_uint4(maxCnt, (uint32_t)nst, (uint32_t)walked, __float_as_uint(kp));
        s_wsum[wave] = __float_as_uint(km);
    }
    __syncthreads();
    if (threadIdx.x == 0)
    {
        if (a.frz && !frozen)
        {
            float2 f = make_float2(__uint_as_float(s_cst[0].w), __uint_as_float(s_wsum[0]));
            for (int w = 1; w < kClusterWaves; ++w)
                f.x = fminf(f.x, __uint_as_float(s_cst[w].w)), f.y = fminf(f.y, __uint_as_float(s_wsum[w]));
            a.frz[c] = f;
        }
        uint4 t = s_cst[0];
        for (int w = 1; w < kClusterWaves; ++w)
            t.x = max(t.x, s_cst[w].x), t.y += s_cst[w].y, t.z += s_cst[w].z;
        t.y |= (kept ? 0x80000000u : 0u) | (frozen ? 0x40000000u : 0u); // (stored entries < 2^30)
        t.w          = ue; // (replaces the freeze minimum)
        a.clStats[c] = t;
    }
}

inline unsigned grid1(size_t n, int b = 256) { return (unsigned)((n + b - 1) / b); }

} // namespace

hipError_t skinFilter(const SkinArgs& a, uint32_t numClusters, hipStream_t s)
{
    if (numClusters) skinFilterKernel<<<numClusters, kB, 0, s>>>(a, numClusters);
    return hipGetLastError();
}

hipError_t skinRefreshBoxes(const DevTree& t, const double* x, const double* y, const double* z, const DevBox& box,
                            double* centers, double* sizes, hipStream_t s, bool withCells)
{
    if (t.numNodes <= 0) return hipSuccess;
    // leaves first (any level), then the inner nodes level by level from the deepest
    leafBoxKernel<<<grid1(t.numNodes, 16), 256, 0, s>>>(t.childOffsets, t.internalToLeaf, t.layout, t.numNodes,
                                                          t.centers, t.sizes, x, y, z, box, centers, sizes,
                                                          withCells ? 1 : 0);
    for (int level = kMaxLevel; level >= 0; --level)
    {
        const int b = t.levelRangeHost[level], e = t.levelRangeHost[level + 1];
        if (e > b) innerBoxKernel<<<grid1(e - b), 256, 0, s>>>(t.childOffsets, b, e, t.centers, box, centers, sizes);
    }
    return hipGetLastError();
}

hipError_t skinMarkStale(const uint32_t* list, uint32_t numClusters, float* acc, hipStream_t s)
{
    if (numClusters) markStaleKernel<<<grid1(numClusters), 256, 0, s>>>(list, numClusters, acc);
    return hipGetLastError();
}

hipError_t reduceClusterStats(const uint4* clStats, uint32_t numClusters, uint32_t* stats, hipStream_t s)
{
    reduceClusterStatsKernel<<<1, 1024, 0, s>>>(clStats, numClusters, stats);
    return hipGetLastError();
}

} // namespace sx
