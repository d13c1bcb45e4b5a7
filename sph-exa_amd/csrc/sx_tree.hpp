/*! @file sx_tree.hpp
 * @brief device arena, tree container and host launchers of the cstone part (sx_tree.hip) and the neighbor
 *        search (sx_neighbors.hip).
 */
#pragma once

#include <algorithm>
#include <map>
#include <string>
#include <vector>

#include "sx_device.hpp"

namespace sx
{

//! grow-only named device (and pinned host) buffers owned by a context; no allocation inside a steady-state step
class Arena
{
public:
    ~Arena() { release(); }

    template<class T>
    T* get(const std::string& tag, size_t count)
    {
        return static_cast<T*>(getBytes(tag, std::max<size_t>(1, count) * sizeof(T), false));
    }
    template<class T>
    T* pinned(const std::string& tag, size_t count)
    {
        return static_cast<T*>(getBytes(tag, std::max<size_t>(1, count) * sizeof(T), true));
    }
    size_t bytesAllocated() const
    {
        size_t s = 0;
        for (auto& kv : bufs_)
            if (!kv.second.host) s += kv.second.bytes;
        return s;
    }
    void release()
    {
        for (auto& kv : bufs_)
        {
            if (kv.second.host) (void)hipHostFree(kv.second.ptr);
            else (void)hipFree(kv.second.ptr);
        }
        bufs_.clear();
    }
    bool failed() const { return failed_; }

private:
    struct Buf
    {
        void*  ptr{nullptr};
        size_t bytes{0};
        bool   host{false};
    };
    void* getBytes(const std::string& tag, size_t bytes, bool host)
    {
        auto it = bufs_.find(tag);
        if (it != bufs_.end() && it->second.bytes >= bytes) return it->second.ptr;
        if (it != bufs_.end())
        {
            (void)hipDeviceSynchronize();
            if (it->second.host) (void)hipHostFree(it->second.ptr);
            else (void)hipFree(it->second.ptr);
            bufs_.erase(it);
        }
        size_t alloc = bytes + bytes / 8 + 256; // 12.5 % growth headroom (allocGrowthRate-style)
        void*  p     = nullptr;
        hipError_t e = host ? hipHostMalloc(&p, alloc) : hipMalloc(&p, alloc);
        if (e != hipSuccess)
        {
            failed_ = true;
            return nullptr;
        }
        bufs_[tag] = Buf{p, alloc, host};
        return p;
    }
    std::map<std::string, Buf> bufs_;
    bool                       failed_{false};
};

//! the converged tree of one sync, in the reference OctreeData + OctreeNsView format
struct DevTree
{
    int       numLeaves{0}, numNodes{0}, numInternal{0};
    uint64_t* leaves{nullptr};   // numLeaves + 1
    uint32_t* counts{nullptr};   // numLeaves + 1 (trailing 0 for the layout scan)
    uint32_t* layout{nullptr};   // numLeaves + 1
    uint64_t* prefixes{nullptr}; // numNodes
    int32_t*  childOffsets{nullptr};
    int32_t*  parents{nullptr};
    int32_t*  levelRange{nullptr};
    int32_t*  internalToLeaf{nullptr};
    int32_t*  leafToInternal{nullptr};
    double*   centers{nullptr};
    double*   sizes{nullptr};
    std::vector<int32_t> levelRangeHost; // host copy of levelRange (per-level upsweep launches)

    int  parentsSize() const { return std::max(1, (numNodes - 1) / 8); }
    void reserve(Arena& a)
    {
        leaves         = a.get<uint64_t>("dt.leaves", numLeaves + 1);
        counts         = a.get<uint32_t>("dt.counts", numLeaves + 1);
        layout         = a.get<uint32_t>("dt.layout", numLeaves + 1);
        prefixes       = a.get<uint64_t>("dt.prefixes", numNodes);
        childOffsets   = a.get<int32_t>("dt.childOffsets", numNodes + 1);
        parents        = a.get<int32_t>("dt.parents", parentsSize());
        levelRange     = a.get<int32_t>("dt.levelRange", kMaxLevel + 2);
        internalToLeaf = a.get<int32_t>("dt.internalToLeaf", numNodes);
        leafToInternal = a.get<int32_t>("dt.leafToInternal", numNodes);
        centers        = a.get<double>("dt.centers", 3 * (size_t)numNodes);
        sizes          = a.get<double>("dt.sizes", 3 * (size_t)numNodes);
    }
};

//! the neighbor lists of one search over [first, last): global u32 lists or cluster unions + u16 positions
struct NbLists
{
    int       local{0};
    uint32_t  first{0}, last{0}, ngmax{0}, ucap{0};
    uint32_t* nidx{nullptr};
    uint32_t* nloc{nullptr};
    uint32_t* uni{nullptr};
    uint32_t* ucount{nullptr};

    size_t groups() const { return (size_t(last - first) + kGroupSize - 1) / kGroupSize; }
    size_t clusters() const { return (size_t(last - first) + kCluster - 1) / kCluster; }
    //! cluster-local u16 positions need unions below 2^16 entries
    static bool localPossible(uint32_t ngmax) { return unionCap(ngmax) <= 65536u; }
    bool reserve(Arena& a, uint32_t f, uint32_t l, uint32_t ng, bool wantLocal)
    {
        first = f, last = l, ngmax = ng;
        local = (wantLocal && localPossible(ng)) ? 1 : 0;
        size_t gr = std::max<size_t>(1, groups()), cl = std::max<size_t>(1, clusters());
        if (local)
        {
            ucap   = unionCap(ng);
            nloc   = a.get<uint32_t>("nb.nloc", gr * nlocWords(ng) * kWave);
            uni    = a.get<uint32_t>("nb.uni", cl * ucap);
            ucount = a.get<uint32_t>("nb.ucount", cl);
            return nloc && uni && ucount;
        }
        nidx = a.get<uint32_t>("nb.nidx", gr * ng * kWave);
        return nidx != nullptr;
    }
};

constexpr int kStatsWords = 28; //!< [0] error flags, [1] failures, [2] max count, [3] scratch, u64 at [4] stored
                                //!< neighbors, [6] candidates tested, [8] union entries, [10] clusters the
                                //!< compact build handed to the large one, [11] the compact build ran first,
                                //!< [12] the largest cluster union (local lists), [13] clusters whose skin
                                //!< the next step's drift would exhaust (sx_skin.hip), [14] 1 + a cluster
                                //!< over the large build's capacities, [15] its candidate leaves (capped),
                                //!< [16] its search regions, [17] clusters the large build handed to its
                                //!< smaller-region pass, [18..27] spare

//! which search build runs: the compact one (four workgroups per CU) with a device-side fallback to the large one,
//! or the large one directly.  Host state of one caller (context or sim), fed with the stats of each finished
//! search through observe() -- never with stale or foreign data (statsHost is zeroed when allocated).
struct NsPolicy
{
    int      mode{0};        //!< 0 auto, 1 large build only, 2 compact first (fallback on overflow), 3 = 2 with a
                             //!< forced overflow of every cluster (test hook: the device-side fallback path)
    int      largeRuns{0};   //!< searches left that go straight to the large build (after many compact overflows)
    uint64_t prevStored{0};  //!< stored neighbors of the previous search
    uint32_t prevTargets{0}; //!< its target count
    uint32_t lastBuild{0};   //!< 0 compact, 1 large, 2 compact with some clusters redone by the large build

    void observe(const uint32_t* statsHost, uint32_t targets)
    {
        lastBuild = statsHost[10] ? 2u : (statsHost[11] ? 0u : 1u);
        // redoing a few clusters costs little; when more than an eighth of them overflow, go large directly
        const uint64_t clusters = (targets + kCluster - 1) / kCluster;
        if (8ull * statsHost[10] > clusters) largeRuns = 64;
        prevStored  = *reinterpret_cast<const uint64_t*>(statsHost + 4);
        prevTargets = targets;
    }
    //! the large build directly only after a search in which many clusters overflowed the compact one (with the
    //! deferred list expansion the compact build stays faster at every neighbor count measured: Noh -n 300 at 100-120
    //! stored neighbors per target, compact + redo 9.3-10.5 ms against 12.0-14.8 ms for the large build)
    bool useLarge()
    {
        if (largeRuns > 0)
        {
            --largeRuns;
            return true;
        }
        return false;
    }
};

//! neighbor-search arguments (sx_neighbors.hip)
struct NsArgs
{
    uint32_t        first, last, numGroups, ngmax, ng0;
    int             iterateH;
    const double *  x, *y, *z;
    float*          h;
    uint32_t*       nc;
    uint32_t*       nidx; // global lists [group][k][lane] (localLists == 0)
    // cluster lists (localLists == 1): per 256-particle cluster c, the union of its targets' neighbors
    // uni[c*ucap + u] (global indices, stream order), ucount[c] = U, and per target the u16 positions into that
    // union, two per word: nloc[(group*nlocWords + k/2)*64 + lane]
    int             localLists;
    ListsB          lb; // exportNeighbors only: the second set of cluster lists (sx_device.hpp)
    uint32_t*       nloc;
    uint32_t*       uni;
    uint32_t*       ucount;
    uint32_t        ucap;
    // tree (OctreeNsView)
    const int32_t*  childOffsets;
    const int32_t*  internalToLeaf;
    const uint32_t* layout;
    const double*   centers;
    const double*   sizes;
    DevBox          box;
    double          margin; // node-box inflation covering key quantisation round-off
    double          extFactor; // OctreeNsView::searchExtFactor (findneighbors.hpp:112): tree-node reach radius
                               // scaled by it (> 1 on ve-bdt substeps: particles drifted out of their cells); 0 = 1
    const float*    powTab; // glibc powf(1 + 1023*ng0/nc, 0.1f) by nc (updateH)
    int             prefilter; // 1: packed f32 distance test in the cluster frame, exact double test only for the
                               // ambiguous chunks; 0: the exact double test for every candidate
    uint32_t*       stats;     // kStatsWords words, see above
    const uint8_t*  active;    // nullable: targets with active[i] == 0 are skipped (no h iteration, h and nc kept)
    uint4*          clStats;   // per cluster {max count, stored, tested, union}: reduced into stats by one small
                               // kernel after the search (per-wave atomics on the stats words serialised: 10 ms of a
                               // 64M-particle search)
    // optional (both non-null): the compact build runs first (policy permitting); a cluster that exceeds one of its
    // capacities is left unwritten and listed in hSave (scratch of last - first floats, used as a u32 list), and the
    // large build then redoes exactly the listed clusters -- no host synchronisation
    float*          hSave;
    NsPolicy*       policy;
    uint32_t*       redo;           // set by findNeighbors, compact build: [0] count, [1..] clusters it gave up
    const uint32_t* redoList;       // set by findNeighbors, large build: process only these clusters
    int             forceOverflow; // compact build only: report a capacity overflow for every cluster (mode 3)
    // set by findNeighbors: a search region (group box) is coherent while the box grown by the group's largest search
    // radius is no wider than `coherence` of its smallest h (0: 20); the last fallback takes 10 (smaller boxes)
    float           coherence;
    // persistent-grid state (findNeighbors sets up both): 16 work counters (8 XCD ranges per launch) and the
    // per-workgroup hit-mask scratch, searchScratchBytes() bytes
    uint32_t*       work;
    uint64_t*       hitMasks;
    // > 0: at most this many workgroups in the large build's persistent grid (two searches sharing the GPU, sx_sim.cpp
    // skinSearch); 0: the whole resident grid
    uint32_t        maxGrid;
    // optional: the targets' final neighbor records {x, y, z, h, m} (the pair kernels' RecX), written by the search
    // for every target it completes, so no separate packing pass is needed for [first, last)
    RecX*           rxOut;
    const float*    m;
    // skin build (sx_skin.hpp): > 0 scales every search radius by skin1 = 1 + s (the caller passes iterateH = 0, the
    // skin lists as nloc with their capacity as ngmax, the skin counts as nc, no rxOut); a union beyond ucap is then
    // recorded in ucount instead of failing the search
    float           skin1;
    uint32_t        uoff; // the union is written at uni[c*ucap + uoff ...] (capacity ucap - uoff); 0 but for skin builds
    // nullable: search only the clusters subset[1 .. subset[0]] (findNeighbors; device-resident list)
    const uint32_t* subset;

    void setLists(const NbLists& L)
    {
        localLists = L.local;
        nidx       = L.nidx;
        nloc       = L.nloc;
        uni        = L.uni;
        ucount     = L.ucount;
        ucap       = L.ucap;
    }
};

hipError_t launchSfcKeys(const double* x, const double* y, const double* z, uint64_t* keys, size_t n,
                         const DevBox& b, hipStream_t s);
hipError_t sortKeys(Arena& arena, uint64_t* keys, uint32_t* order, size_t n, hipStream_t s);
//! stable radix sort of keys on bits [beginBit, 63) into the arena's "sort.kout" (returned) with the permutation
hipError_t countDescents(const uint64_t* keys, size_t n, uint32_t* out, hipStream_t s);
uint64_t*  sortKeysBits(Arena& arena, const uint64_t* keys, uint32_t* order, size_t n, int beginBit, hipStream_t s,
                        hipError_t& e);
//! countDescents, and top[i] = keys[i] >> shift in the same pass
hipError_t countDescentsTop(const uint64_t* keys, size_t n, int shift, uint32_t* top, uint32_t* out, hipStream_t s);
//! stable radix sort of the 32-bit keys top on bits [0, bits): order = the permutation (values 0..n-1)
hipError_t sortTopBits(Arena& arena, const uint32_t* top, uint32_t* order, size_t n, int bits, hipStream_t s);
//! out[0] += descents of keys[order[i]] over i, out[1] += positions with order[i] != i
hipError_t checkSorted(const uint64_t* keys, const uint32_t* order, size_t n, uint32_t* out, hipStream_t s);
hipError_t gather(const uint32_t* order, size_t n, const void* src, void* dst, int elemBytes, hipStream_t s);
//! up to kMaxGatherFields fields of 4 or 8 bytes reordered by one kernel (the index is read once per particle)
constexpr int kMaxGatherFields = 16;
struct GatherSet
{
    int         count;
    const void* src[kMaxGatherFields];
    void*       dst[kMaxGatherFields];
    int         bytes[kMaxGatherFields];
};
hipError_t gatherMany(const uint32_t* order, size_t n, const GatherSet& set, hipStream_t s);
//! number of positions i < n with order[i] != i, added to *count
hipError_t movedCount(const uint32_t* order, size_t n, uint32_t* count, hipStream_t s);
/*! in-place reorder of the fields set.src[f] (== set.dst[f]) where order moves them: field[i] = old field[order[i]]
 *  for every i with order[i] != i, through tmp (n x the set's bytes per particle, columns 256-byte aligned): every
 *  moved value is read before any is written (two kernels); the fixed points of order are not touched */
hipError_t permuteMoved(const uint32_t* order, size_t n, const GatherSet& set, char* tmp, hipStream_t s);
hipError_t buildTree(Arena& arena, const uint64_t* keys, size_t n, uint32_t bucket, const DevBox& box, DevTree& t,
                     hipStream_t s);
hipError_t nodeCenters(const uint64_t* prefixes, int numNodes, const DevBox& b, double* centers, double* sizes,
                       hipStream_t s);
hipError_t leafLayout(Arena& arena, const uint32_t* counts, int numLeaves, uint32_t* layout, hipStream_t s);
hipError_t maxFloat(const float* v, uint32_t first, uint32_t last, unsigned* out, hipStream_t s);
void       packX(size_t n, const double* x, const double* y, const double* z, const float* h, const float* m, RecX* out,
                 hipStream_t s);
void       packV(size_t n, const float* vx, const float* vy, const float* vz, const float* c, RecV* out, hipStream_t s);
void       packT(size_t n, const float* xm, const float* kx, const float* prho, const float* alpha, RecT* out,
                 hipStream_t s);
//! xm, kx (nullable): RecC::vol = xm / kx (the AV switches' neighbor volume)
void       packC(size_t n, const float* c11, const float* c12, const float* c13, const float* c22, const float* c23,
                 const float* c33, const float* divv, RecC* out, hipStream_t s, const float* xm = nullptr,
                 const float* kx = nullptr);
void       packS(size_t n, const float* rho, const float* p, RecS* out, hipStream_t s);
void       tablePairs(const float* t, float2* out, hipStream_t s);

//! computeGroupSplits<64> with tolFactor: group boundaries groups[0..numGroups] (device, capacity cap)
hipError_t spatialGroups(Arena& arena, uint32_t first, uint32_t last, const double* x, const double* y,
                         const double* z, const uint64_t* leaves, int numLeaves, const uint32_t* layout,
                         const DevBox& b, float tolFactor, uint32_t* groups, uint32_t cap, uint32_t* numGroups,
                         hipStream_t s);
hipError_t findNeighbors(const NsArgs& a, hipStream_t s);
//! bytes of NsArgs::hitMasks the search needs (both builds' persistent grids)
size_t     searchScratchBytes();
//! workgroups of the large build resident on the whole chip (its persistent grid)
unsigned   searchGrid();
//! a's list fields (nidx or nloc/uni/ucap), first, last, ngmax and nc select the lists to export
hipError_t exportNeighbors(const NsArgs& a, uint32_t* out, hipStream_t s);
hipError_t importNeighbors(uint32_t* nidx, uint32_t first, uint32_t last, uint32_t ngmax, const uint32_t* in,
                           hipStream_t s);

} // namespace sx
