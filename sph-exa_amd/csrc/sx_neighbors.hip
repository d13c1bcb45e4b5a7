/*! @file sx_neighbors.hip
 * @brief Neighbor search with the coupled h-nc iteration, one 256-thread workgroup per 256-particle SFC cluster
 *        (four wave64 groups) on gfx950.
 *
 * Replaces cstone::findNeighbors + sph::findNeighborsSph (cstone/findneighbors.hpp:95-188,
 * sph/find_neighbors.hpp:10-44) and the traversal inside xmassGpu (hydro_ve/xmass_gpu.cu:56-101).
 *
 * Per cluster (workgroup):
 *   1. search regions in registers (wave / 16-particle sub-group boxes, particle spheres where the SFC range jumps);
 *   2. the four waves together collect every leaf whose geometric box comes within 2*h*ext of some region
 *      (clusterCollectLeaves: one breadth-first walk per cluster, each wave testing 8 nodes x 8 octants per step;
 *      minimum image on periodic axes, inflated by the key-quantisation margin) and number the particles of those
 *      leaves consecutively: the cluster's CANDIDATE SPACE (leaf cc's particles start at s_cOff[cc]);
 *   3. each wave streams the candidate leaves one of its lanes can reach in blocks of 64 particles, culls them
 *      against the wave box grown by 2 hmax and stages the survivors into 64-slot CHUNKS (records in LDS, the
 *      slot's candidate index in the wave's chunk table); every lane tests a chunk against its own particle with a
 *      packed f32 test whose ambiguous chunks go to the reference CPU criterion in double
 *          d2 = dx*dx + dy*dy + dz*dz  <  (double)(4.0f*h*h),   j != i
 *      (dx minimum-image on periodic axes, findneighbors.hpp:118-158); a lane's hits in a chunk are one 64-bit
 *      HIT MASK, capped to the first ngmax hits in stream order like the reference's list;
 *   4. lanes with nc = count+1 outside [ng0/4, ngmax+1] update h (updateH) and the cluster repeats, at most 10
 *      updates per lane (the CPU loop's `iteration++ < 10`), so h, nc and the neighbor SET are identical to the
 *      CPU reference;
 *   5. cluster lists: the union bitmap over the candidate space (OR-ed per chunk) is numbered by a prefix popcount:
 *      the UNION of the cluster's neighbors (uni[], candidate order = leaf runs); the chunk tables are translated to
 *      union positions and every lane expands its hit masks into its u16 list (ascending, which the chunked LDS
 *      staging of sx_hydro_cluster.hip relies on).
 *
 * Deferred list expansion (step 5).  Appending a chunk's hits right after its test walks the chunk's hit masks in a
 * divergent loop whose trip count is the MAX over the wave's lanes of the hits in that chunk; a chunk is a compact
 * region, so the lanes near it have many hits and the others few, and the sum of these maxima was ~3.9x a lane's
 * own hit count (Sedov lattice: 180 iterations per wave against 46).  The masks of the last h pass are therefore
 * kept (global scratch per resident workgroup, only the nonzero ones, compacted per lane: zero masks, about half
 * of them, cost no traffic; the chunk tables in LDS) and expanded once after the pass, each
 * lane walking its own nonzero masks: trip count = max over lanes of its own hits / 2.  A wave with more chunks
 * than its table holds expands the full batch early with candidate indices, which the final pass rewrites to union
 * positions.
 *
 * Work distribution: a persistent grid (the occupancy's worth of workgroups) takes clusters from eight work
 * counters, one per XCD range of the SFC order (blocks are dealt round-robin to the XCDs, so workgroup b serves XCD
 * range b % 8 and steals from the other ranges when its own is done): consecutive clusters share neighbors in the
 * XCD's L2, and every workgroup owns a fixed slot of the hit-mask scratch.
 */
#include "sx_skin.hpp"
#include "sx_traverse.hpp"
#include "sx_tree.hpp"

// Two builds of this file: the default one (large capacities: 2048 candidate leaves, 2^16 candidate particles per
// cluster, 53 KB of LDS, three workgroups per CU) and, with SX_NS_SMALL, a compact one in namespace sx::small
// (1024 leaves, 2^14 particles, 36 KB, four workgroups per CU; Makefile).  findNeighbors runs the compact one;
// a cluster that exceeds its capacities is left unwritten and listed, and the large one redoes the listed clusters.
#ifdef SX_NS_SMALL
namespace sx
{
namespace small
{
#else
namespace sx
{
#endif

#ifndef SX_NS_CCAP
#define SX_NS_CCAP 2048
#endif
constexpr int kCCap = SX_NS_CCAP; //!< candidate leaves per cluster (this build's namespace: sx or sx::small)

#ifndef SX_NS_CAND_LOG2
#define SX_NS_CAND_LOG2 16
#endif
constexpr int kCandSpace = 1 << SX_NS_CAND_LOG2; //!< candidate particles per cluster (u16 list entries)
constexpr int kMaxRegions = 128;           //!< search regions per cluster (boxes or particle spheres)
constexpr int kCandWords = kCandSpace / 32;
#ifndef SX_NS_BATCH
#define SX_NS_BATCH 8
#endif
constexpr int kBatch = SX_NS_BATCH; //!< chunks whose hit masks a wave keeps before expanding them into its lists
static_assert(kBatch <= 32, "nonzero-chunk bits per lane");

#ifndef SX_NS_NT_LIST
#define SX_NS_NT_LIST 0
#endif
//! a u16-pair list word: the lists are read only by later kernels, a streaming store keeps them from evicting the
//! hit-mask rows and candidate coordinates this kernel re-reads from L2 (variant SX_NS_NT_LIST)
__device__ __forceinline__ void storeList(uint32_t* p, uint32_t w)
{
    if constexpr (SX_NS_NT_LIST) __builtin_nontemporal_store(w, p);
    else *p = w;
}


__device__ __forceinline__ uint32_t bitRank(const uint32_t* bits, const uint32_t* pre, uint32_t idx)
{
    const uint32_t w = idx >> 5;
    return pre[w] + __popc(bits[w] & ((1u << (idx & 31)) - 1u));
}

typedef float v2f __attribute__((ext_vector_type(2)));


#ifndef SX_NS_WAVES_PER_EU
#define SX_NS_WAVES_PER_EU 3
#endif

//! per-wave LDS of the stream: 64 staged candidate records (pair layout) and the batch's chunk tables (candidate
//! index, later union position, of every slot).  The search regions alias it (they are only used before the stream).
struct NsWaveLds
{
    float4   rec[kWave];
    uint16_t tab[kBatch][kWave];
};
constexpr int kRegionBytes = 2 * kMaxRegions * (int)sizeof(double4);
constexpr int kWaveLdsBytes = (int)sizeof(NsWaveLds) * kClusterWaves;
union NsStreamLds
{
    NsWaveLds w[kClusterWaves];
    double4   reg[2 * kMaxRegions];
};

//! the cluster's candidate space and union bitmap: dead once the final list expansion starts, whose hit masks then
//! take the same bytes (kMaskSlots nonzero-chunk masks per thread, thread-interleaved)
struct NsCandLds
{
    int      queue[kQCap];
    int      cand[kCCap];
    uint32_t cOff[kCCap + 1];
    uint32_t p0[kCCap];    // first particle of candidate leaf cc
    uint8_t  reach[kCCap]; // bit w: some lane of wave w may reach leaf cc
    uint32_t bits[kCandWords];
    uint32_t pre[kCandWords];
};
constexpr int kMaskSlots = (int)(sizeof(NsCandLds) / (sizeof(uint64_t) * kCluster));
union NsCandOrMasks
{
    NsCandLds c;
    uint64_t  mk[kMaskSlots][kCluster];
};
//! masks per thread in the final expansion: the candidate-space bytes plus the two of each wave's staging records
constexpr int kMaskLds = kMaskSlots + 2;
static_assert(sizeof(float4) * kWave >= 2 * sizeof(uint64_t) * kWave, "two mask slots per lane in the records");

//! clusters [lo, hi) of XCD range x
__device__ __forceinline__ uint32_t rangeLo(uint32_t numClusters, uint32_t x)
{
    return (uint32_t)((uint64_t)numClusters * x / 8);
}

//! next cluster of this workgroup: the XCD range of blockIdx % 8 from the ticket `own` already drawn there (or a
//! new one when own == ~0u), then the other ranges (work stealing); numClusters when every range is done
__device__ __forceinline__ uint32_t grabCluster(uint32_t* work, uint32_t numClusters, uint32_t own = ~0u)
{
    const uint32_t x0 = blockIdx.x & 7;
    if (own != ~0u)
    {
        const uint32_t lo = rangeLo(numClusters, x0), hi = rangeLo(numClusters, x0 + 1);
        if (lo + own < hi) return lo + own;
    }
    for (uint32_t t = own != ~0u ? 1u : 0u; t < 8; ++t)
    {
        const uint32_t x  = (x0 + t) & 7;
        const uint32_t lo = (uint32_t)((uint64_t)numClusters * x / 8), hi = (uint32_t)((uint64_t)numClusters * (x + 1) / 8);
        if (__hip_atomic_load(&work[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= hi - lo) continue;
        const uint32_t k = atomicAdd(&work[x], 1u);
        if (lo + k < hi) return lo + k;
    }
    return numClusters;
}

/*! Every leaf passing `overlaps` (all ancestors passing) into cand[0..return), by all four waves of the workgroup
 *  (called by every thread).  FIFO breadth-first expansion as waveCollectLeaves (sx_traverse.hpp; the queue holds
 *  first-child indices), 32 queued nodes per step, 8 per wave: wave w takes items qh+8w..qh+8w+7, and the
 *  passing leaves and inner nodes of a step are appended in wave order, then lane order -- the order a single wave
 *  taking 8 items per step produces, so the collected leaves are the same list.  Two barriers per step. */
template<class Overlaps>
__device__ __forceinline__ int clusterCollectLeaves(const int32_t* __restrict__ childOffsets, Overlaps&& overlaps,
                                                    int* queue, int* cand, uint2* s_cnt, int wave, int lane,
                                                    unsigned& overflow)
{
    const uint64_t ltMask  = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int            numCand = 0, qh = 0, qt = 0;
    overflow               = 0u; // bit 64: traversal queue, bit 32: candidate leaves (stats[0] bits)
    if (overlaps(0))
    {
        const int c0 = childOffsets[0];
        if (c0 == 0) numCand = 1;
        else qt = 1;
        if (threadIdx.x == 0)
        {
            if (c0 == 0) cand[0] = 0;
            else queue[0] = c0;
        }
    }
    __syncthreads();
    while (qh < qt)
    {
        const int  base  = qh + 8 * wave;
        const int  take  = min(8, qt - base); // <= 0: this wave has no item this step
        const int  slot  = lane >> 3, oct = lane & 7;
        const bool ok    = slot < take;
        const int  child = ok ? queue[(base + slot) & (kQCap - 1)] + oct : 0;
        const int  gc    = childOffsets[child]; // issued with the box loads of overlaps(): independent of them
        const bool pass  = ok && overlaps(child);
        const bool leaf  = pass && gc == 0;
        const bool inner = pass && !leaf;
        const uint64_t bl = __ballot(leaf), bi = __ballot(inner);
        if (lane == 0) s_cnt[wave] = make_uint2(__popcll(bl), __popcll(bi));
        __syncthreads();
        uint32_t offL = 0, offI = 0, totL = 0, totI = 0;
#pragma unroll
        for (int w = 0; w < kClusterWaves; ++w)
        {
            const uint2 cw = s_cnt[w];
            if (w < wave) offL += cw.x, offI += cw.y;
            totL += cw.x, totI += cw.y;
        }
        if (leaf)
        {
            const int pos = numCand + (int)offL + __popcll(bl & ltMask);
            if (pos < kCCap) cand[pos] = child;
        }
        if (inner) queue[(qt + (int)offI + __popcll(bi & ltMask)) & (kQCap - 1)] = gc;
        const int consumed = min(8 * kClusterWaves, qt - qh);
        numCand += (int)totL;
        qt += (int)totI;
        qh += consumed;
        if (qt - qh > kQCap) overflow |= 64u;
        __syncthreads(); // the queue and cand writes are visible; s_cnt is rewritten by the next step
    }
    if (numCand > kCCap)
    {
        overflow |= 32u;
        numCand = kCCap;
    }
    return numCand;
}

__global__ __launch_bounds__(kCluster) __attribute__((amdgpu_waves_per_eu(SX_NS_WAVES_PER_EU))) void
findNeighborsKernel(NsArgs a)
{
    __shared__ NsCandOrMasks s_cm;
    int* const               s_queue = s_cm.c.queue;
    int* const               s_cand  = s_cm.c.cand;
    uint32_t* const          s_cOff  = s_cm.c.cOff;
    uint32_t* const          s_p0    = s_cm.c.p0;
    uint8_t* const           s_reach = s_cm.c.reach;
    uint32_t* const          s_bits  = s_cm.c.bits;
    uint32_t* const          s_pre   = s_cm.c.pre;
    __shared__ int         s_nreg;
    __shared__ int         s_again[kClusterWaves];
    __shared__ uint32_t    s_wsum[kClusterWaves];
    __shared__ NsStreamLds s_str;
    __shared__ int         s_numCand;
    __shared__ int         s_abandon; // the compact build gives this cluster up (capacity): the large build redoes it
    __shared__ uint4       s_cst[kClusterWaves]; // per-wave statistics
    __shared__ uint32_t    s_next;               // the cluster this workgroup takes next
    __shared__ uint2       s_bfsCnt[kClusterWaves];
    double4* const s_reg = s_str.reg;            // search regions: pairs {cx, cy, cz, R}, {hx, hy, hz, owner wave}

    // the fallback launch (a.redoList) redoes the clusters the compact build gave up: redoList[0] of them, ids at
    // redoList[1..]; it exits at once when there are none
    const uint32_t numClusters =
        a.redoList ? __builtin_amdgcn_readfirstlane(a.redoList[0]) : (a.numGroups + kClusterWaves - 1) / kClusterWaves;
    if (numClusters == 0) return;
#ifdef SX_NS_SMALL
    if (a.redo && blockIdx.x == 0 && threadIdx.x == 0) a.stats[11] = 1u; // the compact build ran first
#endif
    const int      wave        = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); // wave-uniform: scalar
    const int      lane        = threadIdx.x & 63;
    NsWaveLds&     wl          = s_str.w[wave];
    // this wave's hit-mask rows (kBatch x 64 lanes), one slot per workgroup of the persistent grid
    uint64_t* const maskRow = a.hitMasks + ((size_t)blockIdx.x * kClusterWaves + wave) * kBatch * kWave + lane;
    if (threadIdx.x == 0) s_next = grabCluster(a.work, numClusters);
    __syncthreads();
    // this workgroup's work item: a cluster, or a position in the redo list (uniform: the cluster's origin, list and
    // scratch addresses are then scalar)
    uint32_t ci = __builtin_amdgcn_readfirstlane(s_next);
    while (ci < numClusters)
    {
    const uint32_t c = a.redoList ? __builtin_amdgcn_readfirstlane(a.redoList[1 + ci]) : ci;
    __syncthreads(); // every thread has read s_next
    // the next ticket of this workgroup's XCD range is drawn now and read at the end of the cluster, so the atomic's
    // round trip overlaps the search instead of stalling wave 0 before its first barrier
    uint32_t ticket = 0;
    if (threadIdx.x == 0) ticket = atomicAdd(&a.work[blockIdx.x & 7], 1u);
    const uint32_t g     = c * kClusterWaves + wave;
    const uint32_t c0    = a.first + c * kCluster;
    const uint32_t i     = c0 + threadIdx.x;
    const bool     valid = g < a.numGroups && i < a.last && (!a.active || a.active[i]);
    const uint32_t iSafe = valid ? i : c0; // positions only: the cluster's first particle is always in range
    const double   xi = a.x[iSafe], yi = a.y[iSafe], zi = a.z[iSafe];
    const double   ox = a.x[c0], oy = a.y[c0], oz = a.z[c0]; // cluster origin of the float prefilter
    // skin builds (sx_skin.hpp) search within 2 h (1 + s): every radius of this kernel scales with hi, and a skin
    // build neither iterates h nor writes it
    float          hi = a.skin1 > 0.0f ? a.h[iSafe] * a.skin1 : a.h[iSafe];

    const bool     local = a.localLists != 0;
    uint32_t*      gl    = a.nidx + (size_t)g * a.ngmax * kWave + lane;
    uint32_t*      ll    = local ? a.nloc + (size_t)g * nlocWords(a.ngmax) * kWave + lane : nullptr;
    const uint64_t ltMask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

    const unsigned     ngmin      = a.ng0 / 4;
    int                iteration  = 0;
    bool               active     = valid;
    unsigned           count      = 0;
    unsigned           stored     = 0;
    uint32_t           pend       = 0; // low half of the next u16-pair word
    unsigned long long candTested = 0;
    int                nq         = 0; // chunks of the current batch (wave-uniform)
    uint32_t           nzq        = 0; // bit q: this lane hit something in chunk q of the batch
    uint32_t           nEarly     = 0; // list entries written as candidate indices by early batch expansions

    // expand the batch's hit masks into this lane's list: candidate indices (early, the union is not known yet) or
    // union positions (final: the chunk tables translated first).  Per lane, its nonzero chunks in order, two hits
    // per iteration; the next nonzero chunk's mask is loaded while the current one is expanded.
    auto expandBatch = [&](bool final) {
        // the mask stores of this wave precede their loads; the translated tables have landed
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
        // the next mask is loaded unconditionally (row 0 when there is none, then discarded by hn): a load under a
        // divergent condition makes the compiler copy its result at the branch merge, i.e. wait for it at once
        uint32_t nz = nzq;
        int      q  = nz ? __builtin_ctz(nz) : 0;
        nz &= nz - 1u;
        uint64_t m  = __builtin_nontemporal_load(maskRow);
        bool     hn = nz != 0u;
        int      qn = hn ? __builtin_ctz(nz) : 0;
        int      kn = 1; // row of the next nonzero chunk
        uint64_t mn = __builtin_nontemporal_load(maskRow + (size_t)(hn ? kn : 0) * kWave);
        nz &= nz - 1u;
        if (!nzq) m = 0ull;
        while (m)
        {
            const uint16_t* tq = wl.tab[q];
            const uint32_t  e1 = tq[__builtin_ctzll(m)];
            m &= m - 1ull;
            const bool     two = m != 0ull;
            const uint32_t e2  = two ? tq[__builtin_ctzll(m)] : 0u;
            if (two) m &= m - 1ull;
            // one store site: odd parity completes the pending word, even parity writes a fresh pair
            const bool     odd = stored & 1u;
            const uint32_t w   = odd ? (pend | (e1 << 16)) : (e1 | (e2 << 16));
            if (odd || two) storeList(ll + (size_t)(stored >> 1) * kWave, w);
            pend = odd ? e2 : e1;
            stored += two ? 2u : 1u;
            if (!m)
            {
                m  = hn ? mn : 0ull, q = qn;
                hn = nz != 0u;
                qn = hn ? __builtin_ctz(nz) : 0;
                kn += hn ? 1 : 0;
                mn = __builtin_nontemporal_load(maskRow + (size_t)(hn ? kn : 0) * kWave);
                nz &= nz - 1u;
            }
        }
        if (!final) nEarly = stored;
        nq  = 0;
        nzq = 0;
        // the last (unused) next-mask load completes here: left outstanding, its registers are reused by the stream's
        // staging code, and the wait the compiler must then put there (vmcnt(0), on every path through the merge)
        // would also wait for the next block's prefetched coordinates
        __builtin_amdgcn_s_waitcnt(0x0f70); // vmcnt(0)
        __builtin_amdgcn_wave_barrier(); // table reads precede the next chunk's staging writes
    };

    /*! the final expansion with the masks in LDS: every thread's nonzero-chunk masks are loaded in bursts (all loads
     *  of a burst in flight together) and parked in the candidate-space bytes and its wave's record slots (kMaskLds
     *  per thread), then walked by a per-lane cursor that reads only LDS.  No global load may sit inside the walk:
     *  vmcnt counts the list stores too, in order, so any load there (even one only a few lanes take, or a flat
     *  access the compiler cannot place in LDS) makes every iteration wait for the previous iteration's stores to
     *  complete.  A lane with more nonzero chunks than slots is served in further rounds of kMaskLds masks.  Called
     *  by every thread of the workgroup after the union and the early-entry rewrite, when the candidate space is
     *  dead. */
    auto expandFinal = [&]() {
        uint64_t* const slotsRec = reinterpret_cast<uint64_t*>(wl.rec); // [2][64] of this wave
        auto slot = [&](int k) -> uint64_t& {
            return k < kMaskSlots ? s_cm.mk[k][threadIdx.x] : slotsRec[(k - kMaskSlots) * kWave + lane];
        };
        const int nnz = __popc(nzq);
        uint32_t  nz  = nzq; // chunks of the masks not yet walked (bit q: chunk q of the batch)
        for (int r0 = 0; __ballot(r0 < nnz) != 0ull; r0 += kMaskLds)
        {
            // this round's rows r0 .. r0 + rn - 1 (the lane's nonzero masks, compacted) -> slots 0 .. rn - 1, groups
            // of 8 loads in flight (16 VGPRs)
            const int rn = max(0, min(nnz - r0, kMaskLds));
            for (int k0 = 0; k0 < rn; k0 += 8)
            {
                uint64_t v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    v[u] = k0 + u < rn ? __builtin_nontemporal_load(maskRow + (size_t)(r0 + k0 + u) * kWave) : 0ull;
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (k0 + u < rn) slot(k0 + u) = v[u];
            }
            __builtin_amdgcn_s_waitcnt(0xc07f); // lgkmcnt(0): this thread's slots have landed (only it reads them)
            int q = rn > 0 ? __builtin_ctz(nz) : 0;
            if (rn > 0) nz &= nz - 1u;
            int      k = 0;
            uint64_t m = rn > 0 ? slot(0) : 0ull;
            while (m)
            {
                const uint16_t* tq = wl.tab[q];
                const uint32_t  e1 = tq[__builtin_ctzll(m)];
                m &= m - 1ull;
                const bool     two = m != 0ull;
                const uint32_t e2  = two ? tq[__builtin_ctzll(m)] : 0u;
                if (two) m &= m - 1ull;
                // one store site: odd parity completes the pending word, even parity writes a fresh pair
                const bool     odd = stored & 1u;
                const uint32_t w   = odd ? (pend | (e1 << 16)) : (e1 | (e2 << 16));
                if (odd || two) storeList(ll + (size_t)(stored >> 1) * kWave, w);
                pend = odd ? e2 : e1;
                stored += two ? 2u : 1u;
                if (!m && k + 1 < rn)
                {
                    q = __builtin_ctz(nz);
                    nz &= nz - 1u;
                    ++k;
                    m = slot(k);
                }
            }
        }
        nq  = 0;
        nzq = 0;
    };

    int  numCand   = 0;
    bool abandoned = false;
    while (true)
    {
        // ---- 1./2. search regions, then the candidate leaves within reach of one, numbered into the candidate space
        if (threadIdx.x == 0) s_nreg = 0;
        __syncthreads();
        {
            // regions: the wave box when it is coherent, else its coherent 16-particle sub-group boxes and, for
            // incoherent sub-groups, the spheres of their particles (all in registers: 16-lane then 64-lane shuffles
            // over the valid lanes).  Coherent: the box grown by the largest search radius is no wider than 20 of the
            // group's smallest h (16 search radii for a uniform h) -- the box's candidates scale with the densest
            // part's particles per volume, so a group spanning a density gradient (a collapsing core and its
            // envelope) takes smaller boxes.  An SFC range can jump across empty space (the curve leaves and
            // re-enters a sphere's surface), so a wave box may span a gap.
            double lo[3] = {valid ? xi : INFINITY, valid ? yi : INFINITY, valid ? zi : INFINITY};
            double hb[3] = {valid ? xi : -INFINITY, valid ? yi : -INFINITY, valid ? zi : -INFINITY};
            float  hq    = valid ? hi : 0.0f;
            float  hqMin = valid ? hi : INFINITY;
#pragma unroll
            for (int o = 8; o > 0; o >>= 1)
            {
                for (int d = 0; d < 3; ++d)
                {
                    lo[d] = fmin(lo[d], __shfl_xor(lo[d], o, 16));
                    hb[d] = fmax(hb[d], __shfl_xor(hb[d], o, 16));
                }
                hq    = fmaxf(hq, __shfl_xor(hq, o, 16));
                hqMin = fminf(hqMin, __shfl_xor(hqMin, o, 16));
            }
            double wlo[3] = {lo[0], lo[1], lo[2]}, whi[3] = {hb[0], hb[1], hb[2]};
            float  hw     = hq, hwMin = hqMin;
#pragma unroll
            for (int o = 16; o < 64; o <<= 1)
            {
                for (int d = 0; d < 3; ++d)
                {
                    wlo[d] = fmin(wlo[d], __shfl_xor(wlo[d], o, 64));
                    whi[d] = fmax(whi[d], __shfl_xor(whi[d], o, 64));
                }
                hw    = fmaxf(hw, __shfl_xor(hw, o, 64));
                hwMin = fminf(hwMin, __shfl_xor(hwMin, o, 64));
            }
            auto addRegion = [&](double x0, double x1, double y0, double y1, double z0, double z1, float h) {
                const int k = atomicAdd(&s_nreg, 1);
                if (k < kMaxRegions)
                {
                    const double ext = a.extFactor > 1.0 ? a.extFactor : 1.0;
                    s_reg[2 * k]     = make_double4(0.5 * (x0 + x1), 0.5 * (y0 + y1), 0.5 * (z0 + z1),
                                                2.0 * (double)h * ext * (1.0 + 1e-6) + a.margin);
                    s_reg[2 * k + 1] = make_double4(0.5 * (x1 - x0), 0.5 * (y1 - y0), 0.5 * (z1 - z0), (double)wave);
                }
            };
            const double coh  = a.coherence > 0.0f ? (double)a.coherence : 20.0;
            const double extW = fmax(whi[0] - wlo[0], fmax(whi[1] - wlo[1], whi[2] - wlo[2]));
            if (extW + 4.0 * (double)hw <= coh * (double)hwMin)
            {
                if (lane == 0 && hw > 0.0f) addRegion(wlo[0], whi[0], wlo[1], whi[1], wlo[2], whi[2], hw);
            }
            else
            {
                const double ext = fmax(hb[0] - lo[0], fmax(hb[1] - lo[1], hb[2] - lo[2]));
                if (ext + 4.0 * (double)hq <= coh * (double)hqMin)
                {
                    if ((lane & 15) == 0 && hq > 0.0f) addRegion(lo[0], hb[0], lo[1], hb[1], lo[2], hb[2], hq);
                }
                else if (valid) addRegion(xi, xi, yi, yi, zi, zi, hi);
            }
        }
        __syncthreads();
        const int nreg = min(s_nreg, kMaxRegions);
        // waves whose regions reach node (bit w)
        auto reachMask = [&](int node, bool any) -> unsigned {
            const double* nc_  = a.centers + 3 * (size_t)node;
            const double* ns_  = a.sizes + 3 * (size_t)node;
            unsigned      bits = 0;
            for (int k = 0; k < nreg; ++k)
            {
                const double4 rc = s_reg[2 * k], rh = s_reg[2 * k + 1];
                if (boxDist2(nc_, ns_, rc.x, rc.y, rc.z, rh.x, rh.y, rh.z, a.box) < rc.w * rc.w)
                {
                    bits |= 1u << (int)rh.w;
                    if (any) break;
                }
            }
            return bits;
        };
        unsigned  overflow = 0u;
        const int nCand    = clusterCollectLeaves(
            a.childOffsets, [&](int node) { return reachMask(node, true) != 0u; }, s_queue, s_cand, s_bfsCnt, wave,
            lane, overflow);
        if (wave == 0)
        {
            if (lane == 0 && s_nreg > kMaxRegions) overflow |= 16u; // regions dropped: the candidates may be short
            // exclusive scan of the candidate leaf sizes
            uint32_t run = 0;
            for (int b = 0; b < nCand; b += kWave)
            {
                uint32_t sz = 0;
                if (b + lane < nCand)
                {
                    const int      leaf = a.internalToLeaf[s_cand[b + lane]];
                    const uint32_t q0   = a.layout[leaf];
                    sz                  = a.layout[leaf + 1] - q0;
                    s_p0[b + lane]      = q0;
                }
                uint32_t incl = sz;
#pragma unroll
                for (int o = 1; o < kWave; o <<= 1)
                {
                    uint32_t t = __shfl_up(incl, o, kWave);
                    if (lane >= o) incl += t;
                }
                if (b + lane < nCand) s_cOff[b + lane] = run + incl - sz;
                run += __shfl(incl, kWave - 1, kWave);
            }
            if (lane == 0)
            {
                s_cOff[nCand] = run;
                // error bits: 2 = traversal queue / candidate-leaf list full / regions dropped (which: 64 / 32 /
                // 16), 4 = candidate space beyond u16
                unsigned f = (overflow ? 2u | overflow : 0u) | ((local && run > (uint32_t)kCandSpace) ? 4u : 0u);
#ifdef SX_NS_SMALL
                if (a.forceOverflow) f |= 4u; // test hook (sx_set_search_mode 3): exercise the device-side fallback
#endif
                // with a redo list (compact build first) an over-capacity cluster is handed to the large build; a
                // skin build's cluster over the large build's capacities is left unbuilt with an over-capacity union
                // count (the filter sends it to the exact search); otherwise it is an error of the search
                const bool skinB = a.skin1 > 0.0f;
                s_abandon        = f && (a.redo || skinB) ? 1 : 0;
                if (f && a.redo)
                {
                    a.redo[1 + atomicAdd(&a.redo[0], 1u)] = c;
#ifdef SX_NS_SMALL
                    atomicAdd(&a.stats[10], 1u); // compact -> large
#else
                    atomicAdd(&a.stats[17], 1u); // large -> large with smaller search regions
#endif
                }
                else if (f && skinB) a.ucount[c] = 0xffffffffu;
                else if (f)
                {
                    atomicOr(&a.stats[0], 1u | f);
                    // a failing cluster for the error report: its index, candidate leaves and search regions
                    if (atomicCAS(&a.stats[14], 0u, c + 1u) == 0u) a.stats[15] = (uint32_t)nCand, a.stats[16] = s_nreg;
                }
                s_numCand = f ? 0 : nCand;
            }
        }
        __syncthreads();
        numCand = s_numCand;
        if (s_abandon)
        {
            abandoned = true; // nothing of this cluster is written: h, nc, lists and union stay for the redo
            break;
        }
        // which waves may reach which candidate leaf: leaf box vs wave box grown by the wave's search radius
        // (conservative; replaces a per-lane test inside the stream, so the stream touches no tree data)
        for (int cc = threadIdx.x; cc < numCand; cc += kCluster)
        {
            const int node = s_cand[cc];
            s_reach[cc]    = (uint8_t)reachMask(node, false);
        }
        if (local)
        {
            const uint32_t nw = (s_cOff[numCand] + 31) / 32;
            for (uint32_t w = threadIdx.x; w < nw; w += kCluster)
                s_bits[w] = 0;
        }
        __syncthreads(); // the regions (aliasing the stream LDS) are no longer read

        // ---- 3. stream candidates, test against each lane's own particle ------------------------------
        const float  r2f    = 4.0f * hi * hi;
        const double radSq  = (double)r2f;
        const double tw     = 2.0 * (double)hi;
        const bool   inside = (xi - tw >= a.box.lim[0]) && (yi - tw >= a.box.lim[2]) && (zi - tw >= a.box.lim[4]) &&
                            (xi + tw <= a.box.lim[1]) && (yi + tw <= a.box.lim[3]) && (zi + tw <= a.box.lim[5]);
        const bool   usePbc = a.box.anyPbc && !inside;
        // float prefilter in the cluster frame: p = fold(x - o) (minimum image relative to the cluster origin).  For
        // a lane with |r| + 2h < L/2 on the periodic axes (r = its own p) every neighbor closer than 2h sits at
        // p_j = r + d with d the minimum-image displacement, and any other image is farther: |p_j - r| >= distance
        const float xr = (float)foldPbc(xi - ox, a.box, 0), yr = (float)foldPbc(yi - oy, a.box, 1),
                    zr = (float)foldPbc(zi - oz, a.box, 2);
        bool safe = true;
        for (int d = 0; d < 3; ++d)
        {
            const float rd = d == 0 ? xr : (d == 1 ? yr : zr);
            if (a.box.pbc[d] && (fabsf(rd) + 2.05f * hi) >= 0.49f * (float)a.box.l[d]) safe = false;
        }
        const bool  fastWave = a.prefilter != 0 && __ballot(valid && !safe) == 0;
        const float thr      = valid ? r2f : -1e30f; // invalid lanes: t ~ +1e30, never a hit, never ambiguous
        // per-candidate cull against the wave's box of r grown by 2 hmax (exact displacement argument above, with a
        // relative margin for the f32 rounding of p and r); a culled candidate is farther than 2h from every lane
        float blo[3] = {valid ? xr : 3e38f, valid ? yr : 3e38f, valid ? zr : 3e38f};
        float bhi[3] = {valid ? xr : -3e38f, valid ? yr : -3e38f, valid ? zr : -3e38f};
        float hw     = valid ? hi : 0.0f;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1)
        {
            for (int d = 0; d < 3; ++d)
            {
                blo[d] = fminf(blo[d], __shfl_xor(blo[d], o, kWave));
                bhi[d] = fmaxf(bhi[d], __shfl_xor(bhi[d], o, kWave));
            }
            hw = fmaxf(hw, __shfl_xor(hw, o, kWave));
        }
        // the wave box (identical in every lane after the butterfly): scalar registers
        auto        rfl = [](float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
        const float bcx = rfl(0.5f * (blo[0] + bhi[0])), bcy = rfl(0.5f * (blo[1] + bhi[1])),
                    bcz = rfl(0.5f * (blo[2] + bhi[2]));
        const float bsx = rfl(0.5f * (bhi[0] - blo[0])), bsy = rfl(0.5f * (bhi[1] - blo[1])),
                    bsz = rfl(0.5f * (bhi[2] - blo[2]));
        const float bmag  = fmaxf(fabsf(blo[0]), fabsf(bhi[0])) + fmaxf(fabsf(blo[1]), fabsf(bhi[1])) +
                           fmaxf(fabsf(blo[2]), fabsf(bhi[2]));
        const float cullR = 2.0f * hw * (1.0f + 0x1p-12f) + 0x1p-16f * (bmag + 2.0f * hw);
        const float cullR2 = rfl((fastWave && hw > 0.0f) ? cullR * cullR : 3e38f);
        // bound on |p| + |r| over every staged candidate and lane: the error scale of the packed test
        const float E   = bmag + cullR + sqrtf(xr * xr + yr * yr + zr * zr);
        const float tol = valid ? 0x1p-19f * fmaf(E, E, thr) : 0.0f;
        const float cr  = fmaf(xr, xr, fmaf(yr, yr, fmaf(zr, zr, -thr))); // |r|^2 - 4h^2
        const v2f   mrx = {-2.0f * xr, -2.0f * xr}, mry = {-2.0f * yr, -2.0f * yr}, mrz = {-2.0f * zr, -2.0f * zr},
                  c2 = {cr, cr};
        float*         srec   = reinterpret_cast<float*>(wl.rec); // 64 slots, pair layout

        // candidate index -> global particle index (s_cOff ascending in cc): the exact chunks and global lists
        auto globalOf = [&](uint32_t ci) -> uint32_t {
            int lo = 0, hi2 = numCand - 1;
            while (lo < hi2)
            {
                const int mid = (lo + hi2 + 1) >> 1;
                if (s_cOff[mid] <= ci) lo = mid;
                else hi2 = mid - 1;
            }
            return s_p0[lo] + (ci - s_cOff[lo]);
        };
        // the reference criterion in double for the m staged slots of table row tq: this lane's hits as slot bits
        auto exactChunk = [&](int m, const uint16_t* tq) -> uint64_t {
            double xj = 0, yj = 0, zj = 0;
            if (lane < m)
            {
                const uint32_t j = globalOf(tq[lane]);
                xj = a.x[j], yj = a.y[j], zj = a.z[j];
            }
            uint64_t hm = 0;
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
                if (valid && (dx * dx + dy * dy + dz * dz < radSq)) hm |= 1ull << k;
            }
            // the coordinate loads complete inside this rare path (m = 0 skips the loop): otherwise their registers,
            // reused by the common path, make it wait for every outstanding load, the next block's prefetch included
            __builtin_amdgcn_s_waitcnt(0x0f70); // vmcnt(0)
            return hm;
        };

        count         = 0;
        stored        = 0;
        nEarly        = 0;
        nq            = 0;
        nzq           = 0;
        uint32_t seq     = 0;           // candidates tested before the current chunk (wave-uniform)
        uint32_t selfSeq = 0xffffffffu; // stream sequence number of this lane's own particle once staged
        int      fill    = 0;

        // test the fill staged slots of table row nq: hit mask -> count, union bitmap, the batch (or global lists)
        auto testChunk = [&]() {
            const int m = fill;
            candTested += m;
            uint16_t* tq = wl.tab[nq];
            // pad the group of 8 with far-away records (t ~ 1e36: no hit, not ambiguous)
            const int mp = (m + 7) & ~7;
            if (lane >= m && lane < mp)
            {
                float* P = srec + (lane >> 1) * 8 + (lane & 1);
                P[0] = 1e18f, P[2] = 1e18f, P[4] = 1e18f, P[6] = 3e36f;
            }
            __builtin_amdgcn_s_waitcnt(0xc07f); // lgkmcnt(0): staged and padded slots have landed
            __builtin_amdgcn_wave_barrier();
            uint64_t hm    = 0;
            bool     exact = !fastWave;
            if (!exact)
            {
                // t = |p - r|^2 - 4h^2 = pw + (|r|^2 - 4h^2) - 2 p.r per candidate pair (packed f32, p from LDS);
                // hit = sign bit of t, gathered by v_alignbit; |t| < tol defers the chunk to the exact double test
                const float4* sc  = reinterpret_cast<const float4*>(srec);
                const int     ng  = mp >> 3; // groups of 8 candidates (4 pairs)
                uint32_t      acc = 0, wlo = 0, whi = 0;
                float         am  = 3.0e38f;
                for (int g = 0; g < ng; ++g)
                {
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                    {
                        const float4 A = sc[(g * 4 + u) * 2], B = sc[(g * 4 + u) * 2 + 1];
                        const v2f    qx = {A.x, A.y}, qy = {A.z, A.w}, qz = {B.x, B.y}, qw = {B.z, B.w};
                        v2f          t  = qw + c2;
                        t               = __builtin_elementwise_fma(qz, mrz, t);
                        t               = __builtin_elementwise_fma(qy, mry, t);
                        t               = __builtin_elementwise_fma(qx, mrx, t);
                        acc             = __builtin_amdgcn_alignbit(acc, __float_as_uint(t.x), 31);
                        acc             = __builtin_amdgcn_alignbit(acc, __float_as_uint(t.y), 31);
                        am              = fminf(am, fminf(fabsf(t.x), fabsf(t.y)));
                    }
                    if (g == 3) wlo = __builtin_bitreverse32(acc), acc = 0;
                }
                // candidate k of a half sits at bit (n-1-k) of acc: reverse, then drop the unused low bits
                if (ng < 4) wlo = __builtin_bitreverse32(acc) >> (32 - 8 * ng);
                else if (ng > 4) whi = __builtin_bitreverse32(acc) >> (32 - 8 * (ng - 4));
                if (__ballot(am < tol)) exact = true;
                else
                {
                    hm = (uint64_t)wlo | ((uint64_t)whi << 32);
                    if (m < 64) hm &= (1ull << m) - 1ull;
                }
            }
            if (exact) hm = exactChunk(m, tq);
            const uint32_t sd = selfSeq - seq;
            if (sd < (uint32_t)m) hm &= ~(1ull << sd); // j != i
            const unsigned nh = __popcll(hm);
            if (count + nh > a.ngmax)
            {
                // keep the first (ngmax - count) hits in stream order, like the capped CPU list
                unsigned keep = count < a.ngmax ? a.ngmax - count : 0u;
                uint64_t kept = 0;
                while (keep--)
                {
                    const uint64_t low = hm & (~hm + 1ull);
                    kept |= low;
                    hm ^= low;
                }
                hm = kept;
            }
            count += nh;
            if (local)
            {
                // union bitmap: slot k hit by some lane -> its candidate bit
                const uint64_t wm = waveOr64(hm);
                if (lane < m && ((wm >> lane) & 1ull))
                {
                    const uint32_t ci = tq[lane];
                    atomicOr(&s_bits[ci >> 5], 1u << (ci & 31));
                }
                // the chunk joins the batch: a nonzero mask goes to the lane's next row (rows compacted per lane: the
                // k-th nonzero chunk of the batch, bit k of nzq, sits in row k; zero masks cost no traffic)
                if (hm) maskRow[(size_t)__popc(nzq) * kWave] = hm;
                nzq |= (hm != 0ull ? 1u : 0u) << nq;
                if (++nq == kBatch) expandBatch(false);
            }
            else
            {
                while (hm)
                {
                    const int k = __builtin_ctzll(hm);
                    hm &= hm - 1ull;
                    gl[(size_t)stored * kWave] = globalOf(tq[k]);
                    stored++;
                }
            }
            seq += m;
            fill = 0;
            __builtin_amdgcn_wave_barrier(); // every lane's slot reads precede the next staging writes
        };

        // blocks of up to 64 consecutive particles of the reachable candidate leaves, in candidate order; the next
        // block's coordinates are loaded while the current one is culled, staged and (when the chunk fills) tested.
        // Reachable non-empty leaves are found 64 at a time: lane l of the window holds leaf wb + l, a ballot gives
        // the window's reachable set (wave-uniform scalar iteration).
        const uint32_t wbit = 1u << wave;
        struct Blk
        {
            int      cc;
            uint32_t s, p1, base;
        };
        int      wb  = -kWave;
        uint64_t rm  = 0;
        uint32_t wp0 = 0, wcnt = 0, wco = 0;
        auto     advance = [&](Blk& q) {
            if (q.cc >= 0 && q.cc < numCand && q.s + kWave < q.p1)
            {
                q.s += kWave;
                return;
            }
            while (rm == 0)
            {
                wb += kWave;
                if (wb >= numCand)
                {
                    q.cc = numCand;
                    return;
                }
                const int l = wb + lane;
                wp0 = 0, wcnt = 0, wco = 0;
                bool r = false;
                if (l < numCand)
                {
                    wp0  = s_p0[l];
                    wco  = s_cOff[l];
                    wcnt = s_cOff[l + 1] - wco;
                    r    = (s_reach[l] & wbit) && wcnt > 0;
                }
                rm = __ballot(r);
            }
            int k = __builtin_ctzll(rm);
            rm &= rm - 1ull;
            q.cc   = wb + k;
            q.s    = __builtin_amdgcn_readlane(wp0, k);
            q.p1   = q.s + __builtin_amdgcn_readlane(wcnt, k);
            q.base = __builtin_amdgcn_readlane(wco, k) - q.s;
            // the next reachable candidate leaves of the window whose particles continue this range (SFC-adjacent
            // leaves) join the block span: their candidate numbers continue it too (same base), so the stream and
            // its order are unchanged, only fewer and fuller 64-particle blocks
            while (k + 1 < kWave && ((rm >> (k + 1)) & 1ull))
            {
                if ((uint32_t)__builtin_amdgcn_readlane(wp0, k + 1) != q.p1) break;
                ++k;
                rm &= rm - 1ull;
                q.p1 += __builtin_amdgcn_readlane(wcnt, k);
            }
        };
        auto load = [&](const Blk& q, double& X, double& Y, double& Z) {
            if (q.cc < numCand && q.s + lane < q.p1)
            {
                const uint32_t j = q.s + lane;
                X = a.x[j], Y = a.y[j], Z = a.z[j];
            }
        };
        // cull, stage and (when the chunk fills, or after the last block) test one block; `last`: no block follows
        auto block = [&](const Blk& cur, double cx, double cy, double cz, bool last) {
            const uint32_t j  = cur.s + lane;
            const bool     in = j < cur.p1;
            float          px = 0, py = 0, pz = 0;
            bool           pass = in;
            if (in && fastWave)
            {
                px = (float)foldPbc(cx - ox, a.box, 0);
                py = (float)foldPbc(cy - oy, a.box, 1);
                pz = (float)foldPbc(cz - oz, a.box, 2);
                const float dx = fmaxf(fabsf(px - bcx) - bsx, 0.0f), dy = fmaxf(fabsf(py - bcy) - bsy, 0.0f),
                            dz = fmaxf(fabsf(pz - bcz) - bsz, 0.0f);
                pass = fmaf(dx, dx, fmaf(dy, dy, dz * dz)) <= cullR2;
            }
            const uint64_t bm = __ballot(pass);
            const int      n  = __popcll(bm);
            if (fill + n > kWave) testChunk();
            if (pass)
            {
                const int slot = fill + __popcll(bm & ltMask);
                float*    P    = srec + (slot >> 1) * 8 + (slot & 1);
                P[0] = px, P[2] = py, P[4] = pz, P[6] = fmaf(px, px, fmaf(py, py, pz * pz));
                wl.tab[nq][slot] = (uint16_t)(cur.base + j);
            }
            // this lane's own particle in the block (it always passes: it lies in the wave box); this block only, a
            // span of merged leaves holds several blocks
            if (valid && i >= cur.s && i - cur.s < (uint32_t)kWave && i < cur.p1)
                selfSeq = seq + (uint32_t)(fill + __popcll(bm & ((1ull << (i - cur.s)) - 1ull)));
            fill += n;
            if (fill == kWave || (last && fill > 0)) testChunk();
        };
        Blk cur{-1, 0, 0, 0};
        advance(cur);
        double cx = 0, cy = 0, cz = 0;
        load(cur, cx, cy, cz);
        while (cur.cc < numCand)
        {
            Blk nxt = cur;
            advance(nxt);
            double nx = 0, ny = 0, nz = 0;
            load(nxt, nx, ny, nz);
            block(cur, cx, cy, cz, nxt.cc >= numCand);
            cur = nxt, cx = nx, cy = ny, cz = nz;
        }

        // ---- 4. h-nc iteration (sph/find_neighbors.hpp:28-33) ----------------------------------------
        bool again = false;
        if (a.iterateH)
        {
            const unsigned ncSph = count + 1;
            const bool     bad   = active && (ngmin > ncSph || (ncSph - 1) > a.ngmax);
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
        }
        const bool waveAgain = __ballot(again) != 0; // full-wave ballot, then one lane publishes it
        if (lane == 0) s_again[wave] = waveAgain;
        __syncthreads(); // also: every wave's bitmap updates are complete
        int any = 0;
        for (int w = 0; w < kClusterWaves; ++w)
            any |= s_again[w];
        if (!any) break;
        __syncthreads(); // s_again / candidate space / regions are rewritten by the next iteration
    }

    // ---- 5. cluster union: prefix popcount of the bitmap, union entries, list expansion ------------------------
    uint32_t ucnt = 0;
    if (local && !abandoned)
    {
        // every thread takes a run of B consecutive candidate bits (not whole words: ~100 words for 256 threads
        // left most threads idle and gave the others 32-bit serial chains)
        const uint32_t nbits = s_cOff[numCand];
        const uint32_t B     = (nbits + kCluster - 1) / kCluster;
        const uint32_t b0 = min(nbits, threadIdx.x * B), b1 = min(nbits, b0 + B);
        const uint32_t wb = b0 >> 5, we = b1 > b0 ? ((b1 - 1) >> 5) + 1 : wb; // words touched: [wb, we)
        auto           mine = [&](uint32_t w) -> uint32_t { // word w's bits within [b0, b1)
            uint32_t       v    = s_bits[w];
            const uint32_t base = w * 32;
            if (b0 > base) v &= ~0u << (b0 - base);
            if (b1 < base + 32) v &= (1u << (b1 - base)) - 1u;
            return v;
        };
        uint32_t sum = 0;
        for (uint32_t w = wb; w < we; ++w)
            sum += __popc(mine(w));
        // workgroup exclusive scan of the per-thread sums
        uint32_t incl = sum;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1)
        {
            uint32_t t = __shfl_up(incl, o, kWave);
            if (lane >= o) incl += t;
        }
        if (lane == kWave - 1) s_wsum[wave] = incl;
        __syncthreads();
        uint32_t off = 0;
        for (int w = 0; w < wave; ++w)
            off += s_wsum[w];
        for (int w = 0; w < kClusterWaves; ++w)
            ucnt += s_wsum[w];
        // per-word prefix (bitRank): set by the thread whose run holds the word's first bit
        uint32_t run = off + incl - sum;
        for (uint32_t w = wb; w < we; ++w)
        {
            if (w * 32 >= b0) s_pre[w] = run;
            run += __popc(mine(w));
        }
        // union entries: candidate index -> global index, through the leaf it belongs to
        uint32_t* uni = a.uni + (size_t)c * a.ucap + a.uoff; // a skin build's union: the slot's upper part
        run           = off + incl - sum;
        // first candidate leaf of this thread's run by binary search (s_cOff ascending), then walk forward
        int cc = 0;
        {
            int lo = 0, hi = numCand; // last cc with s_cOff[cc] <= b0
            while (lo < hi)
            {
                const int mid = (lo + hi + 1) >> 1;
                if (s_cOff[mid] <= b0) lo = mid;
                else hi = mid - 1;
            }
            cc = lo;
        }
        for (uint32_t w = wb; w < we; ++w)
        {
            uint32_t bits = mine(w);
            while (bits)
            {
                const uint32_t idx = w * 32 + __builtin_ctz(bits);
                bits &= bits - 1u;
                while (s_cOff[cc + 1] <= idx)
                    ++cc;
                if (run < a.ucap - a.uoff) uni[run] = s_p0[cc] + (idx - s_cOff[cc]);
                else if (!(a.skin1 > 0.0f)) atomicOr(&a.stats[0], 1u | 8u); // union beyond its capacity (bit 8);
                // a skin build records the true size (ucount) instead: the filter sends such a cluster to the exact search
                ++run;
            }
        }
        __syncthreads(); // s_pre complete
        // the last batch's chunk tables -> union positions
        for (int q = 0; q < nq; ++q)
        {
            // slots nobody hit hold stale indices: bounded into the candidate space, never referenced
            const uint32_t ci = wl.tab[q][lane] & (kCandSpace - 1);
            wl.tab[q][lane]   = (uint16_t)bitRank(s_bits, s_pre, ci);
        }
        // entries written early as candidate indices -> union positions (ascending either way); batches of 8 list
        // words, the 8 loads issued together (one L2 round trip per batch)
        if (__ballot(nEarly > 0))
        {
            // complete words only: with nEarly odd the last early entry is still the pending half (translated below)
            __builtin_amdgcn_s_waitcnt(0); // the early expansion's stores precede these loads
            const uint32_t nwl = nEarly >> 1;
            constexpr int  kRB = 8;
            for (uint32_t k0 = 0; k0 < nwl; k0 += kRB)
            {
                uint32_t v[kRB];
#pragma unroll
                for (int u = 0; u < kRB; ++u)
                    v[u] = (k0 + u < nwl) ? ll[(size_t)(k0 + u) * kWave] : 0u;
#pragma unroll
                for (int u = 0; u < kRB; ++u)
                {
                    const uint32_t k = k0 + u;
                    if (k < nwl)
                    {
                        const uint32_t lo = bitRank(s_bits, s_pre, v[u] & 0xffffu);
                        const uint32_t hp = bitRank(s_bits, s_pre, v[u] >> 16);
                        ll[(size_t)k * kWave] = lo | (hp << 16);
                    }
                }
            }
            if (nEarly & 1u) pend = bitRank(s_bits, s_pre, pend);
        }
        if (threadIdx.x == 0) a.ucount[c] = ucnt;
        __syncthreads(); // the candidate space and the union bitmap are dead: the masks take their bytes
        // the last batch: union positions straight into the lists (the early entries' last pending half included)
        expandFinal();
        if (stored & 1u) ll[(size_t)(stored >> 1) * kWave] = pend;
    }

    if (valid && !abandoned)
    {
        a.nc[i] = count + 1;
        if (a.iterateH) a.h[i] = hi;
        if (a.rxOut) a.rxOut[i] = RecX{xi, yi, zi, hi, a.m[i]};
    }
    // statistics (NcStats-like): per wave, then per cluster into clStats (reduced after the launch)
    const unsigned           failed = (valid && a.iterateH && iteration >= 10) ? 1u : 0u;
    const unsigned           nfail  = waveSum(failed);
    const unsigned           maxCnt = waveMax(valid ? count : 0u);
    const unsigned long long nstore = waveSum((unsigned long long)(valid ? stored : 0u));
    const unsigned long long tested = waveSum(valid ? candTested : 0ull);
    if (lane == 0)
    {
        if (nfail && !abandoned) atomicAdd(&a.stats[1], nfail); // failures only: rare
        s_cst[wave] = make_uint4(maxCnt, (uint32_t)nstore, (uint32_t)tested, 0u);
    }
    if (threadIdx.x == 0) s_next = grabCluster(a.work, numClusters, ticket);
    __syncthreads();
    if (threadIdx.x == 0 && !abandoned)
    {
        uint4 t = s_cst[0];
        for (int w = 1; w < kClusterWaves; ++w)
        {
            const uint4 u = s_cst[w];
            t.x = max(t.x, u.x), t.y += u.y, t.z += u.z;
        }
        t.w          = local ? ucnt : 0u;
        a.clStats[c] = t;
    }
    __syncthreads(); // LDS is reused by the next cluster (s_next was written before this barrier)
    ci = __builtin_amdgcn_readfirstlane(s_next);
    }
}


//! lane-interleaved lists (either format) -> row-major global lists out[(i-first)*ngmax + k]
__global__ void exportKernel(NsArgs a, uint32_t* out)
{
    uint32_t i = a.first + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.last) return;
    uint32_t ni = i - a.first, g = ni / kGroupSize, lane = ni % kGroupSize, c = ni / kCluster;
    uint32_t cnt = a.nc[i] - 1;
    cnt          = cnt < a.ngmax ? cnt : a.ngmax;
    const uint32_t W = nlocWords(a.ngmax);
    for (uint32_t k = 0; k < a.ngmax; ++k)
    {
        uint32_t j = 0;
        if (k < cnt)
        {
            if (a.localLists)
            {
                const bool lB = listsB(a.lb, c);
                uint32_t   w  = (lB ? a.lb.nloc : a.nloc)[((size_t)g * W + k / 2) * kWave + lane];
                j = a.uni[(size_t)c * a.ucap + (lB ? a.lb.uoff : 0u) + ((k & 1) ? (w >> 16) : (w & 0xffffu))];
            }
            else { j = a.nidx[((size_t)g * a.ngmax + k) * kWave + lane]; }
        }
        out[(size_t)ni * a.ngmax + k] = j;
    }
}

__global__ void importKernel(uint32_t* nidx, uint32_t first, uint32_t last, uint32_t ngmax, const uint32_t* in)
{
    uint32_t i = first + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= last) return;
    uint32_t ni = i - first, g = ni / kGroupSize, lane = ni % kGroupSize;
    for (uint32_t k = 0; k < ngmax; ++k)
        nidx[((size_t)g * ngmax + k) * kWave + lane] = in[(size_t)ni * ngmax + k];
}

//! workgroups of this build resident on the whole chip (occupancy x CUs): the persistent grid of one search
unsigned searchGrid()
{
    static unsigned grid = 0;
    if (!grid)
    {
        int dev = 0, cus = 256, perCu = 1;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCu, findNeighborsKernel, kCluster, 0);
        grid = (unsigned)std::max(1, cus) * (unsigned)std::max(1, perCu);
        if (getenv("SX_NS_DEBUG_GRID")) fprintf(stderr, "search grid %u (%d per CU)\n", grid, perCu);
    }
    return grid;
}

//! hit-mask scratch of this build's persistent grid
size_t searchScratchWords() { return (size_t)searchGrid() * kClusterWaves * kBatch * kWave; }

//! this build's search over [first, last): a persistent grid taking clusters from the work counters a.work[0..8)
//! (zeroed by the caller on the stream)
hipError_t findNeighborsOnce(const NsArgs& a, hipStream_t s)
{
    if (a.numGroups == 0) return hipSuccess;
    const unsigned clusters = (a.numGroups + kClusterWaves - 1) / kClusterWaves;
    unsigned       grid     = std::min(searchGrid(), clusters); // a redo list holds <= clusters
    if (a.maxGrid) grid = std::min(grid, a.maxGrid);
    findNeighborsKernel<<<grid, kCluster, 0, s>>>(a);
    return hipGetLastError();
}

#ifndef SX_NS_SMALL
namespace small
{
hipError_t findNeighborsOnce(const NsArgs& a, hipStream_t s);
size_t     searchScratchWords();
} // namespace small

size_t searchScratchBytes() { return std::max(searchScratchWords(), small::searchScratchWords()) * sizeof(uint64_t); }

static hipError_t reduceClusterStats(const NsArgs& a, hipStream_t s)
{
    return reduceClusterStats(a.clStats, (a.numGroups + kClusterWaves - 1) / kClusterWaves, a.stats, s);
}

hipError_t findNeighbors(const NsArgs& a, hipStream_t s)
{
    if (a.numGroups == 0) return hipSuccess;
    hipError_t e;
    // work counters: [0, 8) the first launch, [8, 16) the fallback launch
    if ((e = hipMemsetAsync(a.work, 0, 16 * sizeof(uint32_t), s))) return e;
    const int mode = a.policy ? a.policy->mode : 1;
    const uint32_t ncl = (a.numGroups + kClusterWaves - 1) / kClusterWaves;
    if (!a.hSave || mode == 1 || (mode == 0 && a.policy->useLarge()))
    {
        NsArgs    l    = a;
        uint32_t* over = a.hSave ? reinterpret_cast<uint32_t*>(a.hSave) : nullptr;
        l.redoList     = a.subset; // only the listed clusters, or all
        l.redo         = over;     // clusters over its capacities: again with smaller search regions (below)
        if (over && (e = hipMemsetAsync(over, 0, sizeof(uint32_t), s))) return e;
        if ((e = findNeighborsOnce(l, s))) return e;
        if (over)
        {
            NsArgs t    = a;
            t.redoList  = over;
            t.coherence = 10.0f;
            t.work      = a.work + 8;
            if ((e = findNeighborsOnce(t, s))) return e;
        }
        return reduceClusterStats(a, s);
    }
    // compact build first: a cluster over its capacities is not written and goes to a redo list (in the hSave
    // scratch: clusters + 1 words fit in its last - first floats), which the large build then takes -- only those
    // clusters, no host synchronisation, h untouched for them; a cluster over the large build's capacities goes to
    // a second list (after the first in the same scratch) that the large build takes again with smaller search
    // regions (coherence 10: a group spanning a strong density gradient, e.g. a collapsing core and its envelope)
    uint32_t*      redo  = reinterpret_cast<uint32_t*>(a.hSave);
    uint32_t*      redo2 = redo + ncl + 1;
    if ((e = hipMemsetAsync(redo, 0, sizeof(uint32_t), s))) return e;
    if ((e = hipMemsetAsync(redo2, 0, sizeof(uint32_t), s))) return e;
    NsArgs c        = a;
    c.forceOverflow = mode == 3;
    c.redo          = redo;
    c.redoList      = a.subset;
    if ((e = small::findNeighborsOnce(c, s))) return e;
    NsArgs b   = a;
    b.redoList = redo;
    b.redo     = redo2;
    b.work     = a.work + 8;
    if ((e = findNeighborsOnce(b, s))) return e;
    NsArgs t     = a;
    t.redoList   = redo2;
    t.coherence  = 10.0f;
    t.work       = a.work; // the compact build's counters: reset below, after it finished (stream order)
    if ((e = hipMemsetAsync(a.work, 0, 8 * sizeof(uint32_t), s))) return e;
    if ((e = findNeighborsOnce(t, s))) return e;
    return reduceClusterStats(a, s);
}
#endif

hipError_t exportNeighbors(const NsArgs& a, uint32_t* out, hipStream_t s)
{
    uint32_t n = a.last - a.first;
    if (n) exportKernel<<<(n + 255) / 256, 256, 0, s>>>(a, out);
    return hipGetLastError();
}

hipError_t importNeighbors(uint32_t* nidx, uint32_t first, uint32_t last, uint32_t ngmax, const uint32_t* in,
                           hipStream_t s)
{
    uint32_t n = last - first;
    if (n) importKernel<<<(n + 255) / 256, 256, 0, s>>>(nidx, first, last, ngmax, in);
    return hipGetLastError();
}

#ifdef SX_NS_SMALL
} // namespace small
#endif
} // namespace sx
