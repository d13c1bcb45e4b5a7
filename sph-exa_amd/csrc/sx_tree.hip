/*! @file sx_tree.hip
 * @brief cstone SFC + tree on gfx950: Hilbert keys, key sort, converged cornerstone leaves, linked octree in the
 *        reference's OctreeData format, geometric node centers, leaf layout, record packing, gathers.
 *
 * Compiled with -ffp-contract=off: the key quantisation floor(x*m) - xmin*m and the node centers must round
 * exactly like the reference (sfc/sfc.hpp:157-194, sfc/box.hpp:333-348).
 *
 * Tree construction is level-synchronous and top-down: the converged cornerstone tree (csarray.hpp:456-467) is
 * the unique tree whose split nodes are exactly those holding more than bucketSize particles above level 21, so
 * one pass per level expands every split node into its 8 children (counts by binary search in the sorted keys).
 * The per-level child lists ARE the reference's level-sorted node order (octree.hpp:185-213: prefixes sorted by
 * placeholder-bit key = level-major, key-minor), so prefixes/childOffsets/parents/levelRange come out directly;
 * internalToLeaf / leafToInternal of internal nodes reproduce the reference's binary-radix "unsorted" index
 * (createUnsortedLayoutCpu, octree.hpp:79-107) so that every array is bit-identical to buildOctreeCpu.
 */
#include <hipcub/hipcub.hpp>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "sx_tree.hpp"
#include "sx_sfc.hpp"

namespace sx
{

// ---- key helpers (sfc/common.hpp) ------------------------------------------------------------------------

__host__ __device__ __forceinline__ int clz64(uint64_t v) { return v ? __builtin_clzll(v) : 64; }
__host__ __device__ __forceinline__ uint64_t nodeRange(unsigned level)
{
    return uint64_t(1) << (3u * (kMaxLevel - level));
}
__host__ __device__ __forceinline__ uint64_t encodePlaceholderBit(uint64_t code, int prefixLength)
{
    return (uint64_t(1) << prefixLength) | (code >> (3 * kMaxLevel - prefixLength));
}
__device__ __forceinline__ unsigned decodePrefixLength(uint64_t code) { return 63 - clz64(code); }
__device__ __forceinline__ uint64_t decodePlaceholderBit(uint64_t code)
{
    int pl = (int)decodePrefixLength(code);
    return (code ^ (uint64_t(1) << pl)) << (3 * kMaxLevel - pl);
}
__device__ __forceinline__ unsigned octalDigit(uint64_t code, unsigned pos)
{
    return (unsigned)(code >> (3u * (kMaxLevel - pos))) & 7u;
}
__device__ __forceinline__ int digitWeight(int digit)
{
    int m = -(int)(digit >= 4);
    return ((7 - digit) & m) - (digit & ~m);
}

__device__ __forceinline__ size_t lowerBound(const uint64_t* a, size_t n, uint64_t v)
{
    size_t lo = 0, hi = n;
    while (lo < hi)
    {
        size_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

//! decodeHilbert<uint64_t> (sfc/hilbert.hpp:145-190)
__device__ __forceinline__ void decodeHilbert(uint64_t key, unsigned& ox, unsigned& oy, unsigned& oz)
{
    unsigned px = 0, py = 0, pz = 0;
    for (unsigned level = 0; level < kMaxLevel; ++level)
    {
        unsigned       octant = (key >> (3 * level)) & 7u;
        const unsigned xi = octant >> 2u, yi = (octant >> 1u) & 1u, zi = octant & 1u;
        if (yi ^ zi)
        {
            unsigned pt = px;
            px          = pz;
            pz          = py;
            py          = pt;
        }
        else if ((!xi & !yi & !zi) || (xi & yi & zi))
        {
            unsigned pt = px;
            px          = pz;
            pz          = pt;
        }
        unsigned mask = (1u << level) - 1;
        px ^= mask & (-(xi & (yi | zi)));
        py ^= mask & (-((xi & ((!yi) | (!zi))) | ((!xi) & yi & zi)));
        pz ^= mask & (-((xi & (!yi) & (!zi)) | (yi & zi)));
        px |= (xi << level);
        py |= ((xi ^ yi) << level);
        pz |= ((yi ^ zi) << level);
    }
    ox = px;
    oy = py;
    oz = pz;
}

// ---- kernels -----------------------------------------------------------------------------------------------

//! computeSfcKeys / sfc3D<HilbertKey<uint64_t>> (sfc/sfc.hpp:157-194, 284-291)
__global__ void sfcKeysKernel(const double* x, const double* y, const double* z, uint64_t* keys, size_t n, DevBox b)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    keys[i] = sfcKey(x[i], y[i], z[i], b);
}

__global__ void iotaKernel(uint32_t* a, size_t n)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < n) a[i] = (uint32_t)i;
}

template<class T>
__global__ void gatherKernel(const uint32_t* __restrict__ order, size_t n, const T* __restrict__ src, T* __restrict__ dst)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[order[i]];
}

/*! One level of the top-down split.  Input: the split (internal) nodes of level L in key order.  Each thread
 *  handles one child (8 per node): count = #keys in [start, start + range(L+1)).  Output per child: its key,
 *  count and split flag (count > bucket && L+1 < 21). */
__global__ void expandLevelKernel(const uint64_t* __restrict__ active, int numActive, unsigned level,
                                  const uint64_t* __restrict__ keys, size_t n, uint32_t bucket, uint64_t* childKey,
                                  uint32_t* childCount, uint32_t* splitFlag)
{
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= numActive * 8) return;
    uint64_t start  = active[t >> 3] + uint64_t(t & 7) * nodeRange(level + 1);
    uint64_t end    = start + nodeRange(level + 1);
    size_t   lo     = lowerBound(keys, n, start);
    size_t   hi     = (end == nodeRange(0)) ? n : lowerBound(keys, n, end);
    uint32_t c      = (uint32_t)(hi - lo);
    childKey[t]     = start;
    childCount[t]   = c;
    splitFlag[t]    = (c > bucket && level + 1 < (unsigned)kMaxLevel) ? 1u : 0u;
}

//! scatter the children of one level into the global node arrays (level-major order) and compact split nodes
__global__ void placeLevelKernel(const uint64_t* childKey, const uint32_t* childCount, const uint32_t* splitFlag,
                                 const uint32_t* splitScan, int numChildren, unsigned level, int nodeOffset,
                                 uint64_t* nodePrefix, uint32_t* nodeCount, uint8_t* nodeIsSplit, uint64_t* nextActive)
{
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= numChildren) return;
    nodePrefix[nodeOffset + t]  = encodePlaceholderBit(childKey[t], 3 * (int)(level + 1));
    nodeCount[nodeOffset + t]   = childCount[t];
    nodeIsSplit[nodeOffset + t] = (uint8_t)splitFlag[t];
    if (splitFlag[t]) nextActive[splitScan[t]] = childKey[t];
}

__global__ void splitFromLeafKernel(const uint32_t* leafFlag, uint32_t* split, int numNodes)
{
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < numNodes) split[t] = 1u - leafFlag[t];
    if (t == numNodes) split[t] = 0;
}

//! mark leaves (non-split nodes) for the leaf compaction
__global__ void leafFlagKernel(const uint8_t* nodeIsSplit, int numNodes, uint32_t* flag)
{
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < numNodes) flag[t] = nodeIsSplit[t] ? 0u : 1u;
}

__global__ void leafKeysKernel(const uint64_t* nodePrefix, const uint32_t* nodeCount, const uint32_t* leafFlag,
                               const uint32_t* leafScan, int numNodes, uint64_t* leafKey, uint32_t* leafCnt,
                               int32_t* leafNode)
{
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= numNodes || !leafFlag[t]) return;
    uint32_t k = leafScan[t];
    leafKey[k] = decodePlaceholderBit(nodePrefix[t]);
    leafCnt[k] = nodeCount[t];
    leafNode[k] = t;
}

/*! Linked-octree arrays from level-major nodes.  For node t (prefixes are already level-major sorted):
 *   - childOffsets[t] = first child index, for split nodes (nodes of the next level are the children of the split
 *     nodes of this level in key order, so the k-th split node's children start at levelStart(L+1) + 8k)
 *   - internalToLeaf/leafToInternal as createUnsortedLayoutCpu + buildOctreeCpu produce them. */
__global__ void linkKernel(const uint64_t* prefixes, const uint8_t* isSplit, const uint32_t* splitRank,
                           const int32_t* levelRange, int numNodes, int numInternal, const uint64_t* leaves,
                           int numLeaves, int32_t* childOffsets, int32_t* parents, int32_t* internalToLeaf,
                           int32_t* leafToInternal)
{
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= numNodes) return;
    uint64_t prefix = prefixes[t];
    unsigned pl     = decodePrefixLength(prefix);
    unsigned level  = pl / 3;
    uint64_t key    = decodePlaceholderBit(prefix);
    if (isSplit[t])
    {
        // rank of t among split nodes of its level
        int first = levelRange[level + 1] + 8 * (int)(splitRank[t] - splitRank[levelRange[level]]);
        childOffsets[t]          = first;
        parents[(first - 1) / 8] = t;
        // unsorted binary-radix index: leaf pair straddling the boundary between children 3 and 4
        uint64_t mid  = key + 4 * nodeRange(level + 1);
        int      tid  = (int)lowerBound(leaves, (size_t)numLeaves, mid) - 1;
        int      wsum = 0;
        for (unsigned l = 1; l <= level + 1; ++l)
            wsum += digitWeight((int)octalDigit(leaves[tid], l));
        int octIndex             = (tid + wsum) / 7;
        internalToLeaf[t]        = octIndex - numInternal;
        leafToInternal[octIndex] = t;
    }
    else
    {
        childOffsets[t] = 0;
        int leafIdx     = (int)lowerBound(leaves, (size_t)numLeaves, key);
        internalToLeaf[t]                      = leafIdx;
        leafToInternal[leafIdx + numInternal] = t;
    }
}

//! nodeFpCenters (focus/source_center.hpp:146-157), hilbertIBox + centerAndSize (box.hpp:333-348)
__global__ void nodeCentersKernel(const uint64_t* prefixes, int numNodes, DevBox b, double* centers, double* sizes)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= numNodes) return;
    constexpr int    maxCoord = 1 << kMaxLevel;
    constexpr double uL       = 1.0 / maxCoord;
    double           hx = 0.5 * uL * b.l[0], hy = 0.5 * uL * b.l[1], hz = 0.5 * uL * b.l[2];
    uint64_t         prefix     = prefixes[i];
    uint64_t         startKey   = decodePlaceholderBit(prefix);
    unsigned         level      = decodePrefixLength(prefix) / 3;
    unsigned         cubeLength = (unsigned)maxCoord >> level;
    unsigned         mask       = ~(cubeLength - 1);
    unsigned         ix, iy, iz;
    decodeHilbert(startKey, ix, iy, iz);
    ix &= mask;
    iy &= mask;
    iz &= mask;
    int xmin = (int)ix, xmax = (int)(ix + cubeLength), ymin = (int)iy, ymax = (int)(iy + cubeLength);
    int zmin = (int)iz, zmax = (int)(iz + cubeLength);
    centers[3 * i + 0] = b.lim[0] + (xmax + xmin) * hx;
    centers[3 * i + 1] = b.lim[2] + (ymax + ymin) * hy;
    centers[3 * i + 2] = b.lim[4] + (zmax + zmin) * hz;
    sizes[3 * i + 0]   = (xmax - xmin) * hx;
    sizes[3 * i + 1]   = (ymax - ymin) * hy;
    sizes[3 * i + 2]   = (zmax - zmin) * hz;
}

// ---- record packing ----------------------------------------------------------------------------------------

__global__ void packXKernel(size_t n, const double* x, const double* y, const double* z, const float* h,
                            const float* m, RecX* out)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    RecX r{x[i], y[i], z[i], h[i], m[i]};
    out[i] = r;
}

__global__ void packVKernel(size_t n, const float* vx, const float* vy, const float* vz, const float* c, RecV* out)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = RecV{vx ? vx[i] : 0.f, vy ? vy[i] : 0.f, vz ? vz[i] : 0.f, c ? c[i] : 0.f};
}

__global__ void packTKernel(size_t n, const float* xm, const float* kx, const float* prho, const float* alpha,
                            RecT* out)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = RecT{xm ? xm[i] : 0.f, kx ? kx[i] : 0.f, prho ? prho[i] : 0.f, alpha ? alpha[i] : 0.f};
}

__global__ void packCKernel(size_t n, const float* c11, const float* c12, const float* c13, const float* c22,
                            const float* c23, const float* c33, const float* divv, const float* xm, const float* kx,
                            RecC* out)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = RecC{c11 ? c11[i] : 0.f, c12 ? c12[i] : 0.f, c13 ? c13[i] : 0.f, c22 ? c22[i] : 0.f,
                  c23 ? c23[i] : 0.f, c33 ? c33[i] : 0.f, divv ? divv[i] : 0.f, (xm && kx) ? xm[i] / kx[i] : 0.f};
}

__global__ void tablePairKernel(const float* t, float2* out)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= kTableSize) return;
    float a = t[i];
    float b = (i + 1 < kTableSize) ? t[i + 1] - a : 0.0f;
    out[i]  = make_float2(a, b);
}

//! max over [first,last) of divv (MinMaxGpu in rhoTimestep), one atomic per block on the ordered-int image
__global__ void maxFloatKernel(const float* v, uint32_t first, uint32_t last, unsigned* out)
{
    float    m = -INFINITY;
    for (uint32_t i = first + blockIdx.x * blockDim.x + threadIdx.x; i < last; i += gridDim.x * blockDim.x)
        m = v[i] > m ? v[i] : m;
    m = waveMax(m);
    __shared__ float s[4];
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        float r = s[0];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
            r = s[w] > r ? s[w] : r;
        unsigned u = __float_as_uint(r);
        u          = (u & 0x80000000u) ? ~u : (u | 0x80000000u); // order-preserving map
        atomicMax(out, u);
    }
}

// ---- host-side launchers -----------------------------------------------------------------------------------

static inline unsigned grid(size_t n, int b = 256) { return (unsigned)((n + b - 1) / b); }

hipError_t launchSfcKeys(const double* x, const double* y, const double* z, uint64_t* keys, size_t n,
                         const DevBox& b, hipStream_t s)
{
    if (n) sfcKeysKernel<<<grid(n), 256, 0, s>>>(x, y, z, keys, n, b);
    return hipGetLastError();
}

//! number of descents keys[i] > keys[i+1] (added to *out)
__global__ __launch_bounds__(256) void descentsKernel(const uint64_t* __restrict__ keys, size_t n, uint32_t* out)
{
    uint32_t cnt = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i + 1 < n; i += (size_t)gridDim.x * blockDim.x)
        cnt += keys[i] > keys[i + 1] ? 1u : 0u;
    cnt = waveSum(cnt);
    __shared__ uint32_t s_c[4];
    if ((threadIdx.x & 63) == 0) s_c[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        const uint32_t t = s_c[0] + s_c[1] + s_c[2] + s_c[3];
        if (t) atomicAdd(out, t);
    }
}

hipError_t countDescents(const uint64_t* keys, size_t n, uint32_t* out, hipStream_t s)
{
    if (n < 2) return hipSuccess;
    descentsKernel<<<(unsigned)std::min<size_t>(2048, (n + 255) / 256), 256, 0, s>>>(keys, n, out);
    return hipGetLastError();
}

//! descents keys[i] > keys[i+1] (added to *out) and top[i] = keys[i] >> shift (the key bits the local sort orders)
__global__ __launch_bounds__(256) void descentsTopKernel(const uint64_t* __restrict__ keys, size_t n, int shift,
                                                         uint32_t* __restrict__ top, uint32_t* out)
{
    uint32_t cnt = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    {
        const uint64_t k = keys[i];
        top[i]           = (uint32_t)(k >> shift);
        if (i + 1 < n) cnt += k > keys[i + 1] ? 1u : 0u;
    }
    cnt = waveSum(cnt);
    __shared__ uint32_t s_c[4];
    if ((threadIdx.x & 63) == 0) s_c[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        const uint32_t t = s_c[0] + s_c[1] + s_c[2] + s_c[3];
        if (t) atomicAdd(out, t);
    }
}

hipError_t countDescentsTop(const uint64_t* keys, size_t n, int shift, uint32_t* top, uint32_t* out, hipStream_t s)
{
    if (!n) return hipSuccess;
    descentsTopKernel<<<(unsigned)std::min<size_t>(2048, (n + 255) / 256), 256, 0, s>>>(keys, n, shift, top, out);
    return hipGetLastError();
}

//! onesweep with 10-bit digits: 30 bits in 3 passes instead of 4 (64M nearly sorted keys: 1.81 ms against 2.06 for
//! the library's 8-bit default and 2.39 for 64-bit keys, scripts/sort_bench.hip)
using TopSortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 12>, rocprim::kernel_config<1024, 12>, 10,
                                        rocprim::block_radix_rank_algorithm::match>>;

hipError_t sortTopBits(Arena& arena, const uint32_t* top, uint32_t* order, size_t n, int bits, hipStream_t s)
{
    if (!n) return hipSuccess;
    uint32_t*                            tOut = arena.get<uint32_t>("sort.topout", n);
    rocprim::counting_iterator<uint32_t> ids(0u);
    size_t                               tmpBytes = 0;
    hipError_t e = rocprim::radix_sort_pairs<TopSortConfig>(nullptr, tmpBytes, top, tOut, ids, order, n, 0u,
                                                            (unsigned)bits, s);
    if (e) return e;
    void* tmp = arena.get<char>("sort.tmp", tmpBytes);
    return rocprim::radix_sort_pairs<TopSortConfig>(tmp, tmpBytes, top, tOut, ids, order, n, 0u, (unsigned)bits, s);
}

//! after a sort of the top bits: out[0] += descents of keys[order[.]] (0: the order is the full keys' stable sort),
//! out[1] += positions with order[i] != i
__global__ __launch_bounds__(256) void sortedCheckKernel(const uint64_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ order, size_t n, uint32_t* out)
{
    uint32_t desc = 0, moved = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    {
        const uint32_t o = order[i];
        moved += o != (uint32_t)i ? 1u : 0u;
        if (i + 1 < n) desc += keys[o] > keys[order[i + 1]] ? 1u : 0u;
    }
    desc  = waveSum(desc);
    moved = waveSum(moved);
    __shared__ uint32_t s_c[8];
    if ((threadIdx.x & 63) == 0) s_c[threadIdx.x >> 6] = desc, s_c[4 + (threadIdx.x >> 6)] = moved;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        const uint32_t d = s_c[0] + s_c[1] + s_c[2] + s_c[3], m = s_c[4] + s_c[5] + s_c[6] + s_c[7];
        if (d) atomicAdd(out, d);
        if (m) atomicAdd(out + 1, m);
    }
}

hipError_t checkSorted(const uint64_t* keys, const uint32_t* order, size_t n, uint32_t* out, hipStream_t s)
{
    if (!n) return hipSuccess;
    sortedCheckKernel<<<(unsigned)std::min<size_t>(2048, (n + 255) / 256), 256, 0, s>>>(keys, order, n, out);
    return hipGetLastError();
}

uint64_t* sortKeysBits(Arena& arena, const uint64_t* keys, uint32_t* order, size_t n, int beginBit, hipStream_t s,
                       hipError_t& e)
{
    uint64_t* kOut = arena.get<uint64_t>("sort.kout", n);
    uint32_t* vIn  = arena.get<uint32_t>("sort.vin", n);
    iotaKernel<<<grid(n), 256, 0, s>>>(vIn, n);
    size_t tmpBytes = 0;
    e = hipcub::DeviceRadixSort::SortPairs(nullptr, tmpBytes, keys, kOut, vIn, order, (int)n, beginBit, 63, s);
    if (e) return nullptr;
    void* tmp = arena.get<char>("sort.tmp", tmpBytes);
    e         = hipcub::DeviceRadixSort::SortPairs(tmp, tmpBytes, keys, kOut, vIn, order, (int)n, beginBit, 63, s);
    return kOut;
}

hipError_t sortKeys(Arena& arena, uint64_t* keys, uint32_t* order, size_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    uint64_t* kOut = arena.get<uint64_t>("sort.kout", n);
    uint32_t* vIn  = arena.get<uint32_t>("sort.vin", n);
    iotaKernel<<<grid(n), 256, 0, s>>>(vIn, n);
    size_t tmpBytes = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, tmpBytes, keys, kOut, vIn, order, (int)n, 0, 63, s);
    void* tmp = arena.get<char>("sort.tmp", tmpBytes);
    hipcub::DeviceRadixSort::SortPairs(tmp, tmpBytes, keys, kOut, vIn, order, (int)n, 0, 63, s);
    return hipMemcpyAsync(keys, kOut, n * sizeof(uint64_t), hipMemcpyDeviceToDevice, s);
}

hipError_t gather(const uint32_t* order, size_t n, const void* src, void* dst, int elemBytes, hipStream_t s)
{
    if (!n) return hipSuccess;
    switch (elemBytes)
    {
        case 1: gatherKernel<<<grid(n), 256, 0, s>>>(order, n, (const uint8_t*)src, (uint8_t*)dst); break;
        case 2: gatherKernel<<<grid(n), 256, 0, s>>>(order, n, (const uint16_t*)src, (uint16_t*)dst); break;
        case 4: gatherKernel<<<grid(n), 256, 0, s>>>(order, n, (const uint32_t*)src, (uint32_t*)dst); break;
        case 8: gatherKernel<<<grid(n), 256, 0, s>>>(order, n, (const uint64_t*)src, (uint64_t*)dst); break;
        case 16: gatherKernel<<<grid(n), 256, 0, s>>>(order, n, (const uint4*)src, (uint4*)dst); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

__global__ void gatherManyKernel(const uint32_t* __restrict__ order, size_t n, GatherSet set)
{
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t o = order[i];
    for (int f = 0; f < set.count; ++f) // uniform: every lane walks the same field list
    {
        if (set.bytes[f] == 8) static_cast<uint64_t*>(set.dst[f])[i] = static_cast<const uint64_t*>(set.src[f])[o];
        else if (set.bytes[f] == 4) static_cast<uint32_t*>(set.dst[f])[i] = static_cast<const uint32_t*>(set.src[f])[o];
        else static_cast<uint8_t*>(set.dst[f])[i] = static_cast<const uint8_t*>(set.src[f])[o];
    }
}

hipError_t gatherMany(const uint32_t* order, size_t n, const GatherSet& set, hipStream_t s)
{
    if (!n || !set.count) return hipSuccess;
    for (int f = 0; f < set.count; ++f)
        if (set.bytes[f] != 1 && set.bytes[f] != 4 && set.bytes[f] != 8) return hipErrorInvalidValue;
    gatherManyKernel<<<grid(n), 256, 0, s>>>(order, n, set);
    return hipGetLastError();
}

//! number of positions i < n with order[i] != i (added to *count): a capped grid, one atomic per block
__global__ __launch_bounds__(256) void movedCountKernel(const uint32_t* __restrict__ order, size_t n, uint32_t* count)
{
    uint32_t c = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        c += order[i] != (uint32_t)i ? 1u : 0u;
    c = waveSum(c);
    __shared__ uint32_t s_c[4];
    if ((threadIdx.x & 63) == 0) s_c[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        const uint32_t t = s_c[0] + s_c[1] + s_c[2] + s_c[3];
        if (t) atomicAdd(count, t);
    }
}

hipError_t movedCount(const uint32_t* order, size_t n, uint32_t* count, hipStream_t s)
{
    if (!n) return hipSuccess;
    movedCountKernel<<<(unsigned)std::min<size_t>(2048, (n + 255) / 256), 256, 0, s>>>(order, n, count);
    return hipGetLastError();
}

//! GATHER: tmp_f[i] = field_f[order[i]]; else field_f[i] = tmp_f[i]; both only where order[i] != i
template<bool GATHER>
__global__ __launch_bounds__(256) void movedCopyKernel(const uint32_t* __restrict__ order, size_t n, GatherSet set,
                                                       GatherSet tmp)
{
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t o = order[i];
    if (o == (uint32_t)i) return;
    for (int f = 0; f < set.count; ++f) // uniform
    {
        void* t = tmp.dst[f];
        if (set.bytes[f] == 8)
        {
            if (GATHER) static_cast<uint64_t*>(t)[i] = static_cast<const uint64_t*>(set.src[f])[o];
            else static_cast<uint64_t*>(set.dst[f])[i] = static_cast<const uint64_t*>(t)[i];
        }
        else if (set.bytes[f] == 4)
        {
            if (GATHER) static_cast<uint32_t*>(t)[i] = static_cast<const uint32_t*>(set.src[f])[o];
            else static_cast<uint32_t*>(set.dst[f])[i] = static_cast<const uint32_t*>(t)[i];
        }
        else
        {
            if (GATHER) static_cast<uint8_t*>(t)[i] = static_cast<const uint8_t*>(set.src[f])[o];
            else static_cast<uint8_t*>(set.dst[f])[i] = static_cast<const uint8_t*>(t)[i];
        }
    }
}

hipError_t permuteMoved(const uint32_t* order, size_t n, const GatherSet& set, char* tmp, hipStream_t s)
{
    if (!n || !set.count) return hipSuccess;
    GatherSet cols = set;
    size_t    off  = 0;
    for (int f = 0; f < set.count; ++f)
    {
        if (set.bytes[f] != 1 && set.bytes[f] != 4 && set.bytes[f] != 8) return hipErrorInvalidValue;
        if (set.src[f] != set.dst[f]) return hipErrorInvalidValue; // in place only
        cols.dst[f] = tmp + off;
        off += (n * set.bytes[f] + 255) & ~size_t(255);
    }
    movedCopyKernel<true><<<grid(n), 256, 0, s>>>(order, n, set, cols);
    movedCopyKernel<false><<<grid(n), 256, 0, s>>>(order, n, set, cols);
    return hipGetLastError();
}

template<class T>
static hipError_t exclusiveScan(Arena& arena, const char* tag, const T* in, T* out, int n, hipStream_t s)
{
    size_t bytes = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, n, s);
    void* tmp = arena.get<char>(tag, bytes);
    return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, out, n, s);
}

/*! Build the converged tree (leaves + linked octree + centers + layout) for sorted keys.  Host-synchronous per
 *  level (one 4-byte read-back per level; ~10 levels). */
hipError_t buildTree(Arena& arena, const uint64_t* keys, size_t n, uint32_t bucket, const DevBox& box, DevTree& t,
                     hipStream_t s)
{
    // level 0: the root. It is split iff n > bucket.
    std::vector<int> levelStart{0};
    int              numNodes = 1;
    bool             rootSplit = n > bucket;

    size_t    cap       = std::max<size_t>(64, 2 * (n / std::max<uint32_t>(1, bucket)) * 8 + 64);
    uint64_t* nodePrefix = arena.get<uint64_t>("tree.nodePrefix", cap);
    uint32_t* nodeCount  = arena.get<uint32_t>("tree.nodeCount", cap);
    uint8_t*  nodeSplit  = arena.get<uint8_t>("tree.nodeSplit", cap);
    uint64_t* active     = arena.get<uint64_t>("tree.active", cap / 8 + 8);
    uint64_t* nextActive = arena.get<uint64_t>("tree.nextActive", cap / 8 + 8);
    uint64_t* childKey   = arena.get<uint64_t>("tree.childKey", cap);
    uint32_t* childCount = arena.get<uint32_t>("tree.childCount", cap);
    uint32_t* splitFlag  = arena.get<uint32_t>("tree.splitFlag", cap + 1);
    uint32_t* splitScan  = arena.get<uint32_t>("tree.splitScan", cap + 1);
    uint32_t* hostWord   = arena.pinned<uint32_t>("tree.hostWord", 2);

    uint64_t rootPrefix = encodePlaceholderBit(0, 0);
    uint32_t rootCount  = (uint32_t)n;
    uint8_t  rootFlag   = rootSplit ? 1 : 0;
    hipMemcpyAsync(nodePrefix, &rootPrefix, 8, hipMemcpyHostToDevice, s);
    hipMemcpyAsync(nodeCount, &rootCount, 4, hipMemcpyHostToDevice, s);
    hipMemcpyAsync(nodeSplit, &rootFlag, 1, hipMemcpyHostToDevice, s);
    uint64_t zero = 0;
    hipMemcpyAsync(active, &zero, 8, hipMemcpyHostToDevice, s);

    int numActive = rootSplit ? 1 : 0;
    unsigned level = 0;
    while (numActive > 0)
    {
        int numChildren = numActive * 8;
        if ((size_t)(numNodes + numChildren) > cap) return hipErrorOutOfMemory;
        expandLevelKernel<<<grid(numChildren), 256, 0, s>>>(active, numActive, level, keys, n, bucket, childKey,
                                                             childCount, splitFlag);
        exclusiveScan(arena, "tree.scanTmp", splitFlag, splitScan, numChildren + 1, s);
        // splitFlag[numChildren] is garbage for the scan's last element: total = scan[last] + flag[last]
        hipMemcpyAsync(hostWord, splitScan + numChildren - 1, 4, hipMemcpyDeviceToHost, s);
        hipMemcpyAsync(hostWord + 1, splitFlag + numChildren - 1, 4, hipMemcpyDeviceToHost, s);
        placeLevelKernel<<<grid(numChildren), 256, 0, s>>>(childKey, childCount, splitFlag, splitScan, numChildren,
                                                            level, numNodes, nodePrefix, nodeCount, nodeSplit,
                                                            nextActive);
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) return e;
        levelStart.push_back(numNodes);
        numNodes += numChildren;
        numActive = (int)(hostWord[0] + hostWord[1]);
        std::swap(active, nextActive);
        ++level;
    }
    int numInternal = 0;
    {
        // internal nodes = split nodes; numLeaves = numNodes - numInternal = 7 * numInternal + 1
        int total = numNodes;
        numInternal = (total - 1) / 8;
    }
    int numLeaves = numNodes - numInternal;

    t.numLeaves   = numLeaves;
    t.numNodes    = numNodes;
    t.numInternal = numInternal;
    t.reserve(arena);

    // levelRange (getLevelRangeCpu): first node of each level, then numNodes
    std::vector<int32_t>& lr = t.levelRangeHost;
    lr.assign(kMaxLevel + 2, numNodes);
    for (size_t l = 0; l < levelStart.size() && l <= (size_t)kMaxLevel; ++l)
        lr[l] = levelStart[l];
    lr[kMaxLevel + 1] = numNodes;
    hipMemcpyAsync(t.levelRange, lr.data(), lr.size() * 4, hipMemcpyHostToDevice, s);
    hipMemcpyAsync(t.prefixes, nodePrefix, numNodes * 8, hipMemcpyDeviceToDevice, s);

    // leaves in key order: level-major node order is not key order across levels -> sort leaf keys
    uint32_t* leafFlag = arena.get<uint32_t>("tree.leafFlag", numNodes + 1);
    uint32_t* leafScan = arena.get<uint32_t>("tree.leafScan", numNodes + 1);
    leafFlagKernel<<<grid(numNodes), 256, 0, s>>>(nodeSplit, numNodes, leafFlag);
    exclusiveScan(arena, "tree.scanTmp", leafFlag, leafScan, numNodes, s);
    uint64_t* lkUns  = arena.get<uint64_t>("tree.lkUns", numLeaves);
    uint32_t* lcUns  = arena.get<uint32_t>("tree.lcUns", numLeaves);
    int32_t*  lnUns  = arena.get<int32_t>("tree.lnUns", numLeaves);
    leafKeysKernel<<<grid(numNodes), 256, 0, s>>>(nodePrefix, nodeCount, leafFlag, leafScan, numNodes, lkUns, lcUns,
                                                   lnUns);
    {
        uint32_t* ord  = arena.get<uint32_t>("tree.leafOrd", numLeaves);
        uint32_t* vin  = arena.get<uint32_t>("tree.leafVin", numLeaves);
        iotaKernel<<<grid(numLeaves), 256, 0, s>>>(vin, numLeaves);
        // every leaf sits at a level <= the deepest one expanded: its key is a multiple of that level's node range,
        // so the bits below it are zero and only the bits above are sorted (Sedov 64M: 24 of 63 bits, 3 passes)
        const int begin = level > 0 ? 3 * (kMaxLevel - (int)level) : 0;
        size_t    bytes = 0;
        hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, lkUns, t.leaves, vin, ord, numLeaves, begin, 63, s);
        void* tmp = arena.get<char>("tree.leafSortTmp", bytes);
        hipcub::DeviceRadixSort::SortPairs(tmp, bytes, lkUns, t.leaves, vin, ord, numLeaves, begin, 63, s);
        gatherKernel<<<grid(numLeaves), 256, 0, s>>>(ord, (size_t)numLeaves, lcUns, t.counts);
        uint64_t endKey = nodeRange(0);
        hipMemcpyAsync(t.leaves + numLeaves, &endKey, 8, hipMemcpyHostToDevice, s);
    }
    // split-node rank for childOffsets: exclusive scan of isSplit over all nodes
    uint32_t* splitU32  = arena.get<uint32_t>("tree.splitU32", numNodes + 1);
    uint32_t* splitRank = arena.get<uint32_t>("tree.splitRank", numNodes + 1);
    {
        // split = 1 - leaf, trailing zero
        splitFromLeafKernel<<<grid(numNodes + 1), 256, 0, s>>>(leafFlag, splitU32, numNodes);
        exclusiveScan(arena, "tree.scanTmp", splitU32, splitRank, numNodes + 1, s);
    }
    hipMemsetAsync(t.parents, 0, sizeof(int32_t) * t.parentsSize(), s);
    linkKernel<<<grid(numNodes), 256, 0, s>>>(t.prefixes, nodeSplit, splitRank, t.levelRange, numNodes, numInternal,
                                              t.leaves, numLeaves, t.childOffsets, t.parents, t.internalToLeaf,
                                              t.leafToInternal);
    hipMemsetAsync(t.childOffsets + numNodes, 0, 4, s);
    hipMemsetAsync(t.counts + numLeaves, 0, 4, s);
    nodeCentersKernel<<<grid(numNodes), 256, 0, s>>>(t.prefixes, numNodes, box, t.centers, t.sizes);
    exclusiveScan(arena, "tree.scanTmp", t.counts, t.layout, numLeaves + 1, s);
    return hipGetLastError();
}

hipError_t nodeCenters(const uint64_t* prefixes, int numNodes, const DevBox& b, double* centers, double* sizes,
                       hipStream_t s)
{
    if (numNodes) nodeCentersKernel<<<grid(numNodes), 256, 0, s>>>(prefixes, numNodes, b, centers, sizes);
    return hipGetLastError();
}

hipError_t leafLayout(Arena& arena, const uint32_t* counts, int numLeaves, uint32_t* layout, hipStream_t s)
{
    // layout has numLeaves+1 entries: scan over counts with a trailing zero
    uint32_t* tmp = arena.get<uint32_t>("layout.in", numLeaves + 1);
    hipMemcpyAsync(tmp, counts, numLeaves * 4, hipMemcpyDeviceToDevice, s);
    hipMemsetAsync(tmp + numLeaves, 0, 4, s);
    return exclusiveScan(arena, "layout.tmp", tmp, layout, numLeaves + 1, s);
}

void packX(size_t n, const double* x, const double* y, const double* z, const float* h, const float* m, RecX* out,
           hipStream_t s)
{
    if (n) packXKernel<<<grid(n), 256, 0, s>>>(n, x, y, z, h, m, out);
}
void packV(size_t n, const float* vx, const float* vy, const float* vz, const float* c, RecV* out, hipStream_t s)
{
    if (n) packVKernel<<<grid(n), 256, 0, s>>>(n, vx, vy, vz, c, out);
}
void packT(size_t n, const float* xm, const float* kx, const float* prho, const float* alpha, RecT* out,
           hipStream_t s)
{
    if (n) packTKernel<<<grid(n), 256, 0, s>>>(n, xm, kx, prho, alpha, out);
}
void packS(size_t n, const float* rho, const float* p, RecS* out, hipStream_t s)
{
    static_assert(sizeof(RecS) == sizeof(RecT) && alignof(RecS) == alignof(RecT), "RecS shares the RecT packer");
    if (n) packTKernel<<<grid(n), 256, 0, s>>>(n, rho, p, nullptr, nullptr, reinterpret_cast<RecT*>(out));
}
void packC(size_t n, const float* c11, const float* c12, const float* c13, const float* c22, const float* c23,
           const float* c33, const float* divv, RecC* out, hipStream_t s, const float* xm, const float* kx)
{
    if (n) packCKernel<<<grid(n), 256, 0, s>>>(n, c11, c12, c13, c22, c23, c33, divv, xm, kx, out);
}
void tablePairs(const float* t, float2* out, hipStream_t s) { tablePairKernel<<<grid(kTableSize), 256, 0, s>>>(t, out); }

// ---- target groups: computeGroupSplits<64> (traversal/groups.cuh:55-310, caller sph/groups.cu:30-47) -----------
// One wavefront per fixed group of 64 SFC-consecutive targets: the reference's warp on AMD (GpuConfig::warpSize 64),
// so one 64-bit split mask per group.  A split follows lane l when the distance to particle l+1, in box-scaled
// coordinates (x * 1/lx, no origin shift), exceeds tolFactor * cbrt(smallest leaf volume of the group).

__global__ void groupSplitsKernel(uint32_t first, uint32_t last, const double* __restrict__ x,
                                  const double* __restrict__ y, const double* __restrict__ z,
                                  const uint64_t* __restrict__ leaves, int numLeaves,
                                  const uint32_t* __restrict__ layout, DevBox b, float tolFactor, uint32_t numFixed,
                                  uint64_t* __restrict__ masks, uint32_t* __restrict__ numSub)
{
    const uint32_t g    = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int      lane = threadIdx.x & 63;
    if (g >= numFixed) return;
    const uint32_t body = min(first + g * 64u + (uint32_t)lane, last - 1);
    // leafIdx = upper_bound(layout, layout + numLeaves, body) - layout - 1
    int lo = 0, hi = numLeaves;
    while (lo < hi)
    {
        const int mid = (lo + hi) >> 1;
        if (layout[mid] <= body) lo = mid + 1;
        else hi = mid;
    }
    const int      leaf  = lo - 1;
    const uint64_t range = leaves[leaf + 1] - leaves[leaf];
    const unsigned level = (unsigned)(clz64(range - 1) - 1) / 3u; // treeLevel (64-bit keys: one unused bit)
    // centerAndSize in the unit box (float): half-size 2^-(level+1), vol = 8 s^3, all powers of two
    const float half = 0.5f * (1.0f / (float)(1u << kMaxLevel));
    const float sz   = (float)(1u << (kMaxLevel - level)) * half;
    float       vol  = 8.0f * sz * sz * sz;
    vol              = fminf(vol, 1.0f);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1)
        vol = fminf(vol, __shfl_xor(vol, o, 64));
    const double distCrit   = (double)(cbrtf(vol) * tolFactor);
    const double distCritSq = distCrit * distCrit;
    const double X = x[body] * b.il[0], Y = y[body] * b.il[1], Z = z[body] * b.il[2];
    // shflDown by one; lane 63 keeps its own value (HIP: out-of-range source lane)
    const double Xn = __shfl_down(X, 1, 64), Yn = __shfl_down(Y, 1, 64), Zn = __shfl_down(Z, 1, 64);
    const double dx = Xn - X, dy = Yn - Y, dz = Zn - Z;
    const double d2 = dx * dx + (dy * dy + dz * dz);
    const uint64_t m = __ballot(d2 > distCritSq);
    if (lane == 0)
    {
        masks[g]  = m;
        numSub[g] = 1u + (uint32_t)__popcll(m);
    }
}

//! makeSplits (groups.cuh:116-150) + the boundary scan: group boundaries of fixed group g from its split mask
__global__ void groupBoundsKernel(uint32_t first, uint32_t numFixed, const uint64_t* __restrict__ masks,
                                  const uint32_t* __restrict__ off, uint32_t* __restrict__ groups)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= numFixed) return;
    uint64_t m   = masks[g];
    uint32_t pos = first + 64u * g, k = off[g];
    groups[k++]  = pos;
    while (m)
    {
        const int length = __builtin_ctzll(m) + 1;
        pos += (uint32_t)length;
        groups[k++] = pos;
        m           = length < 64 ? m >> length : 0ull;
    }
}

hipError_t spatialGroups(Arena& arena, uint32_t first, uint32_t last, const double* x, const double* y,
                         const double* z, const uint64_t* leaves, int numLeaves, const uint32_t* layout,
                         const DevBox& b, float tolFactor, uint32_t* groups, uint32_t cap, uint32_t* numGroups,
                         hipStream_t s)
{
    *numGroups = 0;
    if (last <= first) return hipSuccess;
    const uint32_t numFixed = (last - first + 63) / 64;
    uint64_t*      masks    = arena.get<uint64_t>("grp.masks", numFixed);
    uint32_t*      nsub     = arena.get<uint32_t>("grp.nsub", numFixed + 1);
    uint32_t*      off      = arena.get<uint32_t>("grp.off", numFixed + 1);
    uint32_t*      hostN    = arena.pinned<uint32_t>("grp.n", 1);
    if (!masks || !nsub || !off || !hostN) return hipErrorOutOfMemory;
    hipError_t e;
    if ((e = hipMemsetAsync(nsub + numFixed, 0, 4, s))) return e;
    groupSplitsKernel<<<(numFixed + 3) / 4, 256, 0, s>>>(first, last, x, y, z, leaves, numLeaves, layout, b,
                                                          tolFactor, numFixed, masks, nsub);
    if ((e = exclusiveScan(arena, "grp.scan", nsub, off, (int)numFixed + 1, s))) return e;
    if ((e = hipMemcpyAsync(hostN, off + numFixed, 4, hipMemcpyDeviceToHost, s))) return e;
    if ((e = hipStreamSynchronize(s))) return e;
    const uint32_t ng = *hostN;
    if (ng + 1 > cap) return hipErrorInvalidValue;
    groupBoundsKernel<<<(numFixed + 255) / 256, 256, 0, s>>>(first, numFixed, masks, off, groups);
    if ((e = hipMemcpyAsync(groups + ng, &last, 4, hipMemcpyHostToDevice, s))) return e;
    if ((e = hipStreamSynchronize(s))) return e; // `last` lives on this stack frame
    *numGroups = ng;
    return hipGetLastError();
}

hipError_t maxFloat(const float* v, uint32_t first, uint32_t last, unsigned* out, hipStream_t s)
{
    hipMemsetAsync(out, 0, 4, s);
    uint32_t n = last - first;
    unsigned g = std::min<unsigned>(1024, grid(n));
    if (n) maxFloatKernel<<<g, 256, 0, s>>>(v, first, last, out);
    return hipGetLastError();
}

} // namespace sx
