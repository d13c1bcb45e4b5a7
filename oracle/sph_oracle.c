/* sph_oracle.c -- CPU restatement of the SPH-EXA VE hot path, in plain C11 + OpenMP.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker: tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it (via oracle/pyoracle.py); the product library (sph-exa_amd/) never links or
 * calls anything here.  Parity status: PINNED -- tests/test_oracle_vs_ref.py checks every function below
 * bit-for-bit against the reference's own CPU path compiled from /root/reference (oracle/_ref), and
 * tests/test_oracle_golden.py against the committed fixtures under tests/golden/ (generated from _ref by
 * oracle/gen_golden.py) and the reference's known-answer test data (sph/test/ve.cpp:112-233).
 *
 * Every function restates one reference function; citations are /root/reference paths.  Expressions
 * keep the reference's operand order *and* its implicit float/double promotions (e.g. `K` is double,
 * so `rho0 * K * h3Inv` is evaluated in double), so that with identical neighbor order the results are
 * bitwise identical to the reference compiled with the same flags (no FMA contraction).
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "sx_host_types.h"

#define KTABLE 20000
#define MAXLEVEL 21 /* maxTreeLevel<uint64_t> (sfc/sfc.hpp:119-127) */
#define UNUSED_BITS 1

typedef uint64_t key_t_;

/* ------------------------------------------------------------------------------------------------
 * kernel tables (sph_kernel_tables.hpp, kernels.hpp:35-59)
 * ------------------------------------------------------------------------------------------------ */

static double wharmonic_std(double v) /* kernels.hpp:35-42 */
{
    if (v == 0.0) return 1.0;
    const double Pv = M_PI_2 * v;
    return sin(Pv) / Pv;
}

static double wharmonic_derivative_std(double v) /* kernels.hpp:48-57 */
{
    if (v == 0.0) return 0.0;
    const double piHalf = M_PI_2;
    const double Pv     = piHalf * v;
    const double sincv  = sin(Pv) / (Pv);
    return sincv * piHalf * ((cos(Pv) / sin(Pv)) - 1.0 / Pv);
}

static double sinc6(double x) { return pow(wharmonic_std(x), 6.0); } /* getSphKernel sinc_n, :143-147 */

static double sinc6_derivative(double x) /* powSincDerivative, :104-108 */
{
    return 6.0 * pow(wharmonic_std(x), 6.0 - 1) * wharmonic_derivative_std(x);
}

static int cmp_double(const void* a, const void* b)
{
    double x = *(const double*)a, y = *(const double*)b;
    return (x > y) - (x < y);
}

static double kernel_vol(double x) { return 4.0 * M_PI * x * x * sinc6(x); }

/* util::simpson (sph_kernel_tables.hpp:27-56), samples sorted before accumulation */
static double simpson(double a, double b, uint64_t n)
{
    uint64_t numOdd  = n / 2;
    uint64_t numEven = (numOdd >= 1) ? numOdd - 1 : 0;
    double   h       = (b - a) / (double)n;
    double*  odd     = (double*)malloc(sizeof(double) * (numOdd ? numOdd : 1));
    double*  even    = (double*)malloc(sizeof(double) * (numEven ? numEven : 1));
    for (uint64_t i = 0; i < numOdd; ++i)
        odd[i] = kernel_vol(a + (double)(2 * (i + 1) - 1) * h);
    for (uint64_t i = 0; i < numEven; ++i)
        even[i] = kernel_vol(a + (double)(2 * (i + 1)) * h);
    qsort(odd, numOdd, sizeof(double), cmp_double);
    qsort(even, numEven, sizeof(double), cmp_double);
    double so = 0.0, se = 0.0;
    for (uint64_t i = 0; i < numOdd; ++i)
        so += odd[i];
    for (uint64_t i = 0; i < numEven; ++i)
        se += even[i];
    free(odd);
    free(even);
    return h / 3.0 * (kernel_vol(a) + kernel_vol(b) + 4.0 * so + 2.0 * se);
}

/* kernel_3D_k (:78-85) and tabulateFunction<float, 20000> (:88-101) */
void ox_kernel_tables(float* wh, float* whd, double* K)
{
    *K                 = 1.0 / simpson(0, 2.0, 2000);
    const float dx     = (float)((2.0 - 0.0) / (KTABLE - 1));
    for (size_t i = 0; i < KTABLE; ++i)
    {
        float nv = (float)(0.0 + (float)i * dx);
        wh[i]    = (float)sinc6((double)nv);
        whd[i]   = (float)sinc6_derivative((double)nv);
    }
}

/* lt::lookup<float> (table_lookup.hpp:14-26) */
static inline float lookup(const float* table, float v)
{
    const int   numIntervals = KTABLE - 1;
    const float support      = 2.0f;
    const float dx           = support / numIntervals;
    const float invDx        = 1.0f / dx;
    int         idx          = (int)(v * invDx);
    float derivative = (idx >= numIntervals) ? 0.0f : (table[idx + 1] - table[idx]) * invDx;
    return (idx >= numIntervals) ? 0.0f : table[idx] + derivative * (v - (float)idx * dx);
}

float ox_lookup(const float* table, float v) { return lookup(table, v); }

/* updateH<float> (kernels.hpp:26-32) */
float ox_update_h(unsigned ng0, unsigned nc, float h)
{
    const float c0 = 1023.0f;
    const float ex = (float)(1.0 / 10.0);
    return h * 0.5f * powf(1.0f + c0 * ng0 / (float)nc, ex);
}

/* ------------------------------------------------------------------------------------------------
 * box helpers (cstone/sfc/box.hpp:193-267)
 * ------------------------------------------------------------------------------------------------ */

static inline double box_l(const ox_box* b, int d) { return b->lim[2 * d + 1] - b->lim[2 * d]; }
static inline double box_il(const ox_box* b, int d) { return 1.0 / (b->lim[2 * d + 1] - b->lim[2 * d]); }
static inline int    box_pbc(const ox_box* b, int d) { return b->bnd[d] == 1; }

/* legacy applyPBC<double,float> (:233-255): xx -= lx is evaluated in double, then rounded */
static inline void applyPBC(const ox_box* b, float r, float* xx, float* yy, float* zz)
{
    if (box_pbc(b, 0) && *xx > r) *xx = (float)((double)*xx - box_l(b, 0));
    else if (box_pbc(b, 0) && *xx < -r) *xx = (float)((double)*xx + box_l(b, 0));
    if (box_pbc(b, 1) && *yy > r) *yy = (float)((double)*yy - box_l(b, 1));
    else if (box_pbc(b, 1) && *yy < -r) *yy = (float)((double)*yy + box_l(b, 1));
    if (box_pbc(b, 2) && *zz > r) *zz = (float)((double)*zz - box_l(b, 2));
    else if (box_pbc(b, 2) && *zz < -r) *zz = (float)((double)*zz + box_l(b, 2));
}

/* distancePBC<double,float> (:257-267) */
static inline float distancePBC(const ox_box* b, float hi, double x1, double y1, double z1, double x2, double y2,
                                double z2)
{
    float xx = (float)(x1 - x2);
    float yy = (float)(y1 - y2);
    float zz = (float)(z1 - z2);
    applyPBC(b, 2.0f * hi, &xx, &yy, &zz);
    return sqrtf(xx * xx + yy * yy + zz * zz);
}

/* ------------------------------------------------------------------------------------------------
 * Hilbert SFC (sfc/hilbert.hpp:60-105, 145-190; sfc/sfc.hpp:157-194)
 * ------------------------------------------------------------------------------------------------ */

static key_t_ iHilbert(unsigned px, unsigned py, unsigned pz)
{
    static const unsigned mortonToHilbert[8] = {0, 1, 3, 2, 7, 6, 4, 5};
    key_t_ key = 0;
    for (int level = MAXLEVEL - 1; level >= 0; --level)
    {
        unsigned xi     = (px >> level) & 1u;
        unsigned yi     = (py >> level) & 1u;
        unsigned zi     = (pz >> level) & 1u;
        unsigned octant = (xi << 2) | (yi << 1) | zi;
        key             = (key << 3) + mortonToHilbert[octant];
        px ^= -(xi & ((!yi) | zi));
        py ^= -((xi & (yi | zi)) | (yi & (!zi)));
        pz ^= -((xi & (!yi) & (!zi)) | (yi & (!zi)));
        if (zi)
        {
            unsigned pt = px;
            px          = py;
            py          = pz;
            pz          = pt;
        }
        else if (!yi)
        {
            unsigned pt = px;
            px          = pz;
            pz          = pt;
        }
    }
    return key;
}

static void decodeHilbert(key_t_ key, unsigned* ox, unsigned* oy, unsigned* oz)
{
    unsigned px = 0, py = 0, pz = 0;
    for (unsigned level = 0; level < MAXLEVEL; ++level)
    {
        unsigned       octant = (key >> (3 * level)) & 7u;
        const unsigned xi     = octant >> 2u;
        const unsigned yi     = (octant >> 1u) & 1u;
        const unsigned zi     = octant & 1u;
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
    *ox = px;
    *oy = py;
    *oz = pz;
}

/* sfc3D<HilbertKey<uint64_t>, double> (sfc.hpp:157-194) */
static key_t_ sfc3D(double x, double y, double z, const ox_box* b)
{
    const unsigned cubeLength = 1u << MAXLEVEL;
    const int      mcoord     = (1 << MAXLEVEL) - 1;
    double mx = cubeLength * box_il(b, 0), my = cubeLength * box_il(b, 1), mz = cubeLength * box_il(b, 2);
    int    ix = (int)(floor(x * mx) - b->lim[0] * mx);
    int    iy = (int)(floor(y * my) - b->lim[2] * my);
    int    iz = (int)(floor(z * mz) - b->lim[4] * mz);
    ix        = ix < mcoord ? ix : mcoord;
    iy        = iy < mcoord ? iy : mcoord;
    iz        = iz < mcoord ? iz : mcoord;
    return iHilbert((unsigned)ix, (unsigned)iy, (unsigned)iz);
}

void ox_sfc_keys(const double* x, const double* y, const double* z, size_t n, const ox_box* b, uint64_t* keys)
{
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n; ++i)
        keys[i] = sfc3D(x[i], y[i], z[i], b);
}

/* ------------------------------------------------------------------------------------------------
 * cornerstone octree (tree/csarray.hpp:290-467, tree/octree.hpp:95-213, sfc/common.hpp)
 * ------------------------------------------------------------------------------------------------ */

static inline int      clz64(key_t_ v) { return v ? __builtin_clzll(v) : 64; }
static inline key_t_   nodeRange(unsigned level) { return (key_t_)1 << (3u * (MAXLEVEL - level)); }
static inline unsigned treeLevel(key_t_ range) { return (unsigned)(clz64(range - 1) - UNUSED_BITS) / 3; }
static inline int      commonPrefix(key_t_ a, key_t_ b) { return clz64(a ^ b) - UNUSED_BITS; }
static inline key_t_   encodePlaceholderBit(key_t_ code, int prefixLength)
{
    int nShifts = 3 * MAXLEVEL - prefixLength;
    return ((key_t_)1 << prefixLength) | (code >> nShifts);
}
static inline unsigned decodePrefixLength(key_t_ code) { return 8 * sizeof(key_t_) - 1 - clz64(code); }
static inline key_t_   decodePlaceholderBit(key_t_ code)
{
    int prefixLength = (int)decodePrefixLength(code);
    return (code ^ ((key_t_)1 << prefixLength)) << (3 * MAXLEVEL - prefixLength);
}
static inline unsigned octalDigit(key_t_ code, unsigned position)
{
    return (unsigned)(code >> (3u * (MAXLEVEL - position))) & 7u;
}
static inline int digitWeight(int digit)
{
    int fourGeqMask = -(int)(digit >= 4);
    return ((7 - digit) & fourGeqMask) - (digit & ~fourGeqMask);
}

static size_t lower_bound_u64(const key_t_* a, size_t n, key_t_ v)
{
    size_t lo = 0, hi = n;
    while (lo < hi)
    {
        size_t mid = (lo + hi) / 2;
        if (a[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

typedef struct
{
    key_t_*   leaves;
    unsigned* counts;
    size_t    n, cap;
} leafbuf;

static void push_leaf(leafbuf* lb, key_t_ k, unsigned c)
{
    if (lb->n == lb->cap)
    {
        lb->cap    = lb->cap ? 2 * lb->cap : 1024;
        lb->leaves = (key_t_*)realloc(lb->leaves, lb->cap * sizeof(key_t_));
        lb->counts = (unsigned*)realloc(lb->counts, lb->cap * sizeof(unsigned));
    }
    lb->leaves[lb->n] = k;
    lb->counts[lb->n] = c;
    lb->n++;
}

/* The converged cornerstone tree of computeOctree (csarray.hpp:456-467) is the unique tree in which a
 * node is split iff its particle count exceeds the bucket size and it is above the maximum level
 * (calculateNodeOp, :233-255): restated here as a depth-first split in key order. */
static void split_node(const key_t_* keys, size_t n, key_t_ start, unsigned level, unsigned bucket, leafbuf* lb)
{
    key_t_ end   = start + nodeRange(level);
    size_t lo    = lower_bound_u64(keys, n, start);
    size_t hi    = lower_bound_u64(keys, n, end);
    size_t count = hi - lo;
    if (count > bucket && level < MAXLEVEL)
    {
        for (int s = 0; s < 8; ++s)
            split_node(keys + lo, count, start + (key_t_)s * nodeRange(level + 1), level + 1, bucket, lb);
    }
    else { push_leaf(lb, start, (unsigned)count); }
}

int ox_compute_octree(const uint64_t* keys, size_t n, unsigned bucket, uint64_t* leaves, unsigned* counts, int cap)
{
    leafbuf lb = {0, 0, 0, 0};
    split_node(keys, n, 0, 0, bucket, &lb);
    int nLeaf = (int)lb.n;
    if (cap >= nLeaf)
    {
        memcpy(leaves, lb.leaves, nLeaf * sizeof(key_t_));
        leaves[nLeaf] = nodeRange(0);
        memcpy(counts, lb.counts, nLeaf * sizeof(unsigned));
    }
    free(lb.leaves);
    free(lb.counts);
    return nLeaf;
}

static int binaryKeyWeight(key_t_ key, unsigned level) /* octree.hpp:58-68 */
{
    int ret = 0;
    for (unsigned l = 1; l <= level + 1; ++l)
        ret += digitWeight((int)octalDigit(key, l));
    return ret;
}

typedef struct
{
    key_t_ prefix;
    int    idx;
} prefix_pair;

static int cmp_prefix(const void* a, const void* b)
{
    key_t_ x = ((const prefix_pair*)a)->prefix, y = ((const prefix_pair*)b)->prefix;
    return (x > y) - (x < y);
}

/* buildOctreeCpu (octree.hpp:185-213) with createUnsortedLayoutCpu (:79-107), linkTreeCpu (:124-158),
 * getLevelRangeCpu (:161-172) */
void ox_build_octree(const uint64_t* leaves, int numLeaves, uint64_t* prefixes, int* childOffsets, int* parents,
                     int* levelRange, int* internalToLeaf, int* leafToInternal)
{
    int          nInt = (numLeaves - 1) / 7;
    int          nTot = numLeaves + nInt;
    prefix_pair* pp   = (prefix_pair*)malloc(sizeof(prefix_pair) * nTot);
    for (int tid = 0; tid < numLeaves; ++tid)
    {
        key_t_   key         = leaves[tid];
        unsigned level       = treeLevel(leaves[tid + 1] - key);
        pp[tid + nInt].prefix = encodePlaceholderBit(key, 3 * (int)level);
        pp[tid + nInt].idx    = tid + nInt;
        int prefixLength     = commonPrefix(key, leaves[tid + 1]);
        if (prefixLength % 3 == 0 && tid < numLeaves - 1)
        {
            int octIndex         = (tid + binaryKeyWeight(key, (unsigned)prefixLength / 3)) / 7;
            pp[octIndex].prefix  = encodePlaceholderBit(key, prefixLength);
            pp[octIndex].idx     = octIndex;
        }
    }
    qsort(pp, nTot, sizeof(prefix_pair), cmp_prefix); /* prefixes are unique: stable not needed */
    for (int i = 0; i < nTot; ++i)
    {
        prefixes[i]       = pp[i].prefix;
        internalToLeaf[i] = pp[i].idx;
    }
    free(pp);
    for (int i = 0; i < nTot; ++i)
        leafToInternal[internalToLeaf[i]] = i;
    for (int i = 0; i < nTot; ++i)
        internalToLeaf[i] -= nInt;
    for (unsigned level = 0; level <= MAXLEVEL; ++level)
        levelRange[level] = (int)lower_bound_u64(prefixes, nTot, encodePlaceholderBit(0, 3 * (int)level));
    levelRange[MAXLEVEL + 1] = nTot;
    for (int i = 0; i < nTot; ++i)
        childOffsets[i] = 0;
    for (int i = 0; i < nInt; ++i)
    {
        int      idxA         = leafToInternal[i];
        key_t_   prefix       = prefixes[idxA];
        key_t_   nodeKey      = decodePlaceholderBit(prefix);
        unsigned prefixLength = decodePrefixLength(prefix);
        unsigned level        = prefixLength / 3;
        key_t_   childPrefix  = encodePlaceholderBit(nodeKey, (int)prefixLength + 3);
        int      s0 = levelRange[level + 1], s1 = levelRange[level + 2];
        int      childIdx = s0 + (int)lower_bound_u64(prefixes + s0, (size_t)(s1 - s0), childPrefix);
        if (childIdx != s1 && childPrefix == prefixes[childIdx])
        {
            childOffsets[idxA]          = childIdx;
            parents[(childIdx - 1) / 8] = idxA;
        }
    }
}

/* nodeFpCenters (focus/source_center.hpp:146-157) with hilbertIBox (hilbert.hpp:274-290) and
 * centerAndSize (sfc/box.hpp:333-348) */
/* ------------------------------------------------------------------------------------------------
 * Target groups: computeGroupSplits<64> (cstone/traversal/groups.cuh:195-310; caller sph/groups.cu:30-47 with
 * tolFactor 2).  Restated for the 64-wide wavefront of the AMD build (GpuConfig::warpSize = 64, so one fixed group
 * of 64 particles = one warp and one 64-bit split mask, nwt = 1).
 * ------------------------------------------------------------------------------------------------ */

/* findSplits (groups.cuh:55-93) for one fixed group: bit l set when |X[l+1] - X[l]|^2 > distCritSq, X in
 * box-scaled coordinates (x * ilx, no origin shift), lane 63 and clamped lanes compare with themselves */
static uint64_t find_splits(const double* X, const double* Y, const double* Z, double distCritSq)
{
    uint64_t m = 0;
    for (int l = 0; l < 64; ++l)
    {
        int    n  = l < 63 ? l + 1 : l;
        double dx = X[n] - X[l], dy = Y[n] - Y[l], dz = Z[n] - Z[l];
        double d2 = dx * dx + (dy * dy + dz * dz); /* norm2 = right fold dot (util/array.hpp:253) */
        if (d2 > distCritSq) m |= 1ull << l;
    }
    return m;
}

/* makeSplits (groups.cuh:116-150): lengths of the runs of the split mask, the last one extended to 64 */
int ox_make_splits(uint64_t mask, uint32_t* lengths)
{
    int k = 0, remaining = 64;
    while (mask)
    {
        int length = __builtin_ctzll(mask) + 1;
        remaining -= length;
        lengths[k++] = (uint32_t)length;
        mask = length < 64 ? mask >> length : 0;
    }
    lengths[k++] = (uint32_t)remaining;
    return k;
}

/* groupSplitsKernel (groups.cuh:180-250) per fixed group g; returns the split mask */
uint64_t ox_group_split_mask(uint32_t first, uint32_t last, uint32_t g, const double* x, const double* y,
                             const double* z, const uint64_t* leaves, int numLeaves, const uint32_t* layout,
                             const ox_box* b, float tolFactor)
{
    double X[64], Y[64], Z[64];
    float  nodeVolume = 1.0f;
    for (int l = 0; l < 64; ++l)
    {
        uint32_t body = first + g * 64 + l;
        if (body > last - 1) body = last - 1;
        /* leafIdx = upper_bound(layout, layout + numLeaves, body) - layout - 1 */
        int lo = 0, hi = numLeaves;
        while (lo < hi)
        {
            int mid = (lo + hi) / 2;
            if (layout[mid] <= body) lo = mid + 1;
            else hi = mid;
        }
        int leaf = lo - 1;
        /* centerAndSize<KeyType>(sfcIBox(leaf range), unit box) in float: half-size of a cube of
         * (range)^(1/3) integer units, 2^-21 per unit; vol = 8 * sx * sy * sz (all powers of two) */
        uint64_t range = leaves[leaf + 1] - leaves[leaf];
        unsigned level = treeLevel(range);
        float    uL    = 1.0f / (float)(1u << MAXLEVEL);
        float    half  = 0.5f * uL * 1.0f;
        float    side  = (float)(1u << (MAXLEVEL - level));
        float    sz    = side * half;
        float    vol   = 8.0f * sz * sz * sz;
        nodeVolume     = vol < nodeVolume ? vol : nodeVolume;
        X[l] = x[body] * box_il(b, 0);
        Y[l] = y[body] * box_il(b, 1);
        Z[l] = z[body] * box_il(b, 2);
    }
    double distCrit = (double)(cbrtf(nodeVolume) * tolFactor);
    return find_splits(X, Y, Z, distCrit * distCrit);
}

/* computeGroupSplits<64> (groups.cuh:255-310): group boundaries groups[0..numGroups] (groups[numGroups] = last);
 * returns numGroups; groups == NULL: size query */
int ox_group_splits(uint32_t first, uint32_t last, const double* x, const double* y, const double* z,
                    const uint64_t* leaves, int numLeaves, const uint32_t* layout, const ox_box* b, float tolFactor,
                    uint32_t* groups)
{
    if (last <= first) return 0;
    uint32_t numFixed = (last - first + 63) / 64;
    uint32_t pos = first;
    int      ng  = 0;
    for (uint32_t g = 0; g < numFixed; ++g)
    {
        uint64_t m = ox_group_split_mask(first, last, g, x, y, z, leaves, numLeaves, layout, b, tolFactor);
        uint32_t len[65];
        int      k = ox_make_splits(m, len);
        for (int q = 0; q < k; ++q)
        {
            if (groups) groups[ng] = pos;
            pos += len[q];
            ng++;
        }
    }
    if (groups) groups[ng] = last;
    return ng;
}

void ox_node_centers(const uint64_t* prefixes, int numNodes, const ox_box* b, double* centers, double* sizes)
{
    const int    maxCoord = 1 << MAXLEVEL;
    const double uL       = 1.0 / maxCoord;
    double       hx = 0.5 * uL * box_l(b, 0), hy = 0.5 * uL * box_l(b, 1), hz = 0.5 * uL * box_l(b, 2);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < numNodes; ++i)
    {
        key_t_   prefix     = prefixes[i];
        key_t_   startKey   = decodePlaceholderBit(prefix);
        unsigned level      = decodePrefixLength(prefix) / 3;
        unsigned cubeLength = (unsigned)maxCoord >> level;
        unsigned mask       = ~(cubeLength - 1);
        unsigned ix, iy, iz;
        decodeHilbert(startKey, &ix, &iy, &iz);
        ix &= mask;
        iy &= mask;
        iz &= mask;
        int xmin = (int)ix, xmax = (int)(ix + cubeLength), ymin = (int)iy, ymax = (int)(iy + cubeLength);
        int zmin = (int)iz, zmax = (int)(iz + cubeLength);
        centers[3 * i + 0] = b->lim[0] + (xmax + xmin) * hx;
        centers[3 * i + 1] = b->lim[2] + (ymax + ymin) * hy;
        centers[3 * i + 2] = b->lim[4] + (zmax + zmin) * hz;
        sizes[3 * i + 0]   = (xmax - xmin) * hx;
        sizes[3 * i + 1]   = (ymax - ymin) * hy;
        sizes[3 * i + 2]   = (zmax - zmin) * hz;
    }
}

/* ------------------------------------------------------------------------------------------------
 * neighbor search (cstone/findneighbors.hpp:95-188, traversal/traversal.hpp:69-110,
 * traversal/boxoverlap.hpp:186-216, sph/find_neighbors.hpp:10-44)
 * ------------------------------------------------------------------------------------------------ */

typedef struct
{
    int             numLeafNodes;
    const key_t_*   prefixes;
    const int*      childOffsets;
    const int*      internalToLeaf;
    const uint32_t* layout;
    const double*   centers;
    const double*   sizes;
    float           searchExtFactor;
} ns_view;

static inline double rint_pbc(double dx, const ox_box* b, int d)
{
    return dx - box_pbc(b, d) * box_l(b, d) * rint(dx * box_il(b, d));
}

/* norm2(minDistance(...)) with and without PBC (boxoverlap.hpp:197-216); dot = right fold */
static inline double minDist2(const double* p, const double* c, const double* s, const ox_box* b, int pbc)
{
    double d[3];
    for (int k = 0; k < 3; ++k)
    {
        double dx = c[k] - p[k];
        if (pbc) dx = rint_pbc(dx, b, k);
        dx = fabs(dx);
        dx -= s[k];
        dx += fabs(dx);
        dx *= 0.5;
        d[k] = dx;
    }
    return d[0] * d[0] + (d[1] * d[1] + d[2] * d[2]);
}

static unsigned findNeighbors1(uint32_t i, const double* x, const double* y, const double* z, const float* h,
                               const ns_view* t, const ox_box* b, unsigned ngmax, uint32_t* neighbors)
{
    double xi = x[i], yi = y[i], zi = z[i];
    float  hi = h[i];

    float  radiusSq     = 4.0f * hi * hi;
    float  cellRadiusSq = radiusSq * t->searchExtFactor * t->searchExtFactor;
    double particle[3]  = {xi, yi, zi};
    unsigned numNeighbors = 0;

    int anyPbc = box_pbc(b, 0) || box_pbc(b, 1) || box_pbc(b, 2);
    /* insideBox(particle, {2h,2h,2h}, box) */
    double tw     = 2.0 * (double)hi;
    int    inside = (xi - tw >= b->lim[0]) && (yi - tw >= b->lim[2]) && (zi - tw >= b->lim[4]) &&
                 (xi + tw <= b->lim[1]) && (yi + tw <= b->lim[3]) && (zi + tw <= b->lim[5]);
    int usePbc = anyPbc && !inside;

#define OVERLAPS(idx) (minDist2(particle, t->centers + 3 * (idx), t->sizes + 3 * (idx), b, usePbc) < cellRadiusSq)
#define SEARCH_BOX(idx)                                                                                                \
    do {                                                                                                               \
        int      leafIdx = t->internalToLeaf[idx];                                                                     \
        uint32_t first = t->layout[leafIdx], last = t->layout[leafIdx + 1];                                            \
        for (uint32_t j = first; j < last; ++j)                                                                        \
        {                                                                                                              \
            if (j == i) continue;                                                                                      \
            double dx = x[j] - particle[0], dy = y[j] - particle[1], dz = z[j] - particle[2];                          \
            if (usePbc)                                                                                                \
            {                                                                                                          \
                dx = rint_pbc(dx, b, 0);                                                                               \
                dy = rint_pbc(dy, b, 1);                                                                               \
                dz = rint_pbc(dz, b, 2);                                                                               \
            }                                                                                                          \
            if (dx * dx + dy * dy + dz * dz < radiusSq)                                                                \
            {                                                                                                          \
                if (numNeighbors < ngmax) neighbors[numNeighbors] = j;                                                 \
                numNeighbors++;                                                                                        \
            }                                                                                                          \
        }                                                                                                              \
    } while (0)

    /* singleTraversal (traversal.hpp:69-110) */
    if (!OVERLAPS(0)) return numNeighbors;
    if (t->childOffsets[0] == 0)
    {
        SEARCH_BOX(0);
        return numNeighbors;
    }
    int stack[128];
    stack[0]     = 0;
    int stackPos = 1;
    int node     = 0;
    do
    {
        for (int octant = 0; octant < 8; ++octant)
        {
            int child = t->childOffsets[node] + octant;
            if (OVERLAPS(child))
            {
                if (t->childOffsets[child] == 0) { SEARCH_BOX(child); }
                else { stack[stackPos++] = child; }
            }
        }
        node = stack[--stackPos];
    } while (node != 0);
#undef OVERLAPS
#undef SEARCH_BOX
    return numNeighbors;
}

/* Tree for an already sorted key array (same construction as the reference harness). */
typedef struct
{
    key_t_*   leaves;
    unsigned* counts;
    key_t_*   prefixes;
    int *     childOffsets, *parents, *levelRange, *internalToLeaf, *leafToInternal;
    double *  centers, *sizes;
    uint32_t* layout;
    int       nLeaf, nTot;
} ox_tree;

static void tree_build(ox_tree* t, const uint64_t* keys, size_t n, unsigned bucket, const ox_box* b)
{
    int nLeaf        = ox_compute_octree(keys, n, bucket, NULL, NULL, 0);
    t->nLeaf         = nLeaf;
    t->leaves        = (key_t_*)malloc(sizeof(key_t_) * (nLeaf + 1));
    t->counts        = (unsigned*)malloc(sizeof(unsigned) * nLeaf);
    ox_compute_octree(keys, n, bucket, t->leaves, t->counts, nLeaf);
    int nInt          = (nLeaf - 1) / 7;
    int nTot          = nLeaf + nInt;
    t->nTot           = nTot;
    t->prefixes       = (key_t_*)malloc(sizeof(key_t_) * nTot);
    t->childOffsets   = (int*)calloc(nTot + 1, sizeof(int));
    t->parents        = (int*)calloc((nTot - 1) / 8 > 1 ? (nTot - 1) / 8 : 1, sizeof(int));
    t->levelRange     = (int*)calloc(MAXLEVEL + 2, sizeof(int));
    t->internalToLeaf = (int*)calloc(nTot, sizeof(int));
    t->leafToInternal = (int*)calloc(nTot, sizeof(int));
    ox_build_octree(t->leaves, nLeaf, t->prefixes, t->childOffsets, t->parents, t->levelRange, t->internalToLeaf,
                    t->leafToInternal);
    t->centers = (double*)malloc(sizeof(double) * 3 * nTot);
    t->sizes   = (double*)malloc(sizeof(double) * 3 * nTot);
    ox_node_centers(t->prefixes, nTot, b, t->centers, t->sizes);
    t->layout    = (uint32_t*)malloc(sizeof(uint32_t) * (nLeaf + 1));
    uint32_t acc = 0;
    for (int i = 0; i < nLeaf; ++i)
    {
        t->layout[i] = acc;
        acc += t->counts[i];
    }
    t->layout[nLeaf] = acc;
}

static void tree_free(ox_tree* t)
{
    free(t->leaves);
    free(t->counts);
    free(t->prefixes);
    free(t->childOffsets);
    free(t->parents);
    free(t->levelRange);
    free(t->internalToLeaf);
    free(t->leafToInternal);
    free(t->centers);
    free(t->sizes);
    free(t->layout);
}

static ns_view tree_view(const ox_tree* t)
{
    ns_view v = {t->nLeaf, t->prefixes, t->childOffsets, t->internalToLeaf, t->layout, t->centers, t->sizes, 1.0f};
    return v;
}

/* findNeighborsSph (sph/find_neighbors.hpp:10-44): nc includes self; returns the number of failures */
static size_t findNeighborsSph(const double* x, const double* y, const double* z, float* h, uint32_t firstId,
                               uint32_t lastId, const ox_box* b, const ns_view* t, unsigned ng0, unsigned ngmax,
                               uint32_t* neighbors, uint32_t* nc)
{
    uint32_t numWork  = lastId - firstId;
    unsigned ngmin    = ng0 / 4;
    size_t   numFails = 0;
#pragma omp parallel for reduction(+ : numFails)
    for (uint32_t i = 0; i < numWork; ++i)
    {
        uint32_t id    = i + firstId;
        unsigned ncSph = 1 + findNeighbors1(id, x, y, z, h, t, b, ngmax, neighbors + (size_t)i * ngmax);
        int      iteration = 0;
        while ((ngmin > ncSph || (ncSph - 1) > ngmax) && iteration++ < 10)
        {
            h[id] = ox_update_h(ng0, ncSph, h[id]);
            ncSph = 1 + findNeighbors1(id, x, y, z, h, t, b, ngmax, neighbors + (size_t)i * ngmax);
        }
        numFails += (iteration >= 10);
        nc[i] = ncSph;
    }
    return numFails;
}

void ox_find_neighbors(const double* x, const double* y, const double* z, float* h, const uint64_t* keys, size_t n,
                       unsigned first, unsigned last, const ox_box* b, unsigned bucket, unsigned ng0, unsigned ngmax,
                       int iterate_h, uint32_t* neighbors, uint32_t* nc)
{
    ox_tree t;
    tree_build(&t, keys, n, bucket, b);
    ns_view v = tree_view(&t);
    if (iterate_h) { findNeighborsSph(x, y, z, h, first, last, b, &v, ng0, ngmax, neighbors, nc); }
    else
    {
        uint32_t numWork = last - first;
#pragma omp parallel for
        for (uint32_t i = 0; i < numWork; ++i)
            nc[i] = findNeighbors1(i + first, x, y, z, h, &v, b, ngmax, neighbors + (size_t)i * ngmax);
    }
    tree_free(&t);
}

/* ------------------------------------------------------------------------------------------------
 * VE kernels (sph/hydro_ve/<kernel>_kern.hpp), driven like the compute*Impl loops
 * ------------------------------------------------------------------------------------------------ */

static float g_wh[KTABLE], g_whd[KTABLE];
static double g_K;
static int    g_tables = 0;

static void ensure_tables(void)
{
    if (!g_tables)
    {
#pragma omp critical(ox_tables)
        {
            if (!g_tables)
            {
                ox_kernel_tables(g_wh, g_whd, &g_K);
                g_tables = 1;
            }
        }
    }
}

static inline unsigned nc_capped(const uint32_t* nc, size_t i, unsigned ngmax)
{
    unsigned v = nc[i] - 1;
    return v < ngmax ? v : ngmax;
}

/* Neighbor-list consumers check every index they are about to read against the state size first: a list exported
 * from the GPU path under test is INPUT to this checker, so a bad index must fail the test (ox_list_errors() > 0,
 * raised by pyoracle), not crash the process.  A kernel given a bad list computes nothing. */
static unsigned long long g_listErrors = 0;

unsigned long long ox_list_errors(void) { return g_listErrors; }
void               ox_clear_list_errors(void) { g_listErrors = 0; }

static int lists_ok(const ox_state* s, const uint32_t* neighbors, unsigned first, unsigned last, unsigned ngmax)
{
    unsigned long long bad = 0;
#pragma omp parallel for reduction(+ : bad)
    for (size_t i = first; i < last; ++i)
    {
        const unsigned  cnt = nc_capped(s->nc, i, ngmax);
        const uint32_t* row = neighbors + (size_t)ngmax * (i - first);
        for (unsigned k = 0; k < cnt; ++k)
            bad += row[k] >= s->n ? 1 : 0;
    }
    if (s->n && last > s->n) bad += 1;
    g_listErrors += bad;
    return bad == 0;
}

/* Error scales of the neighbor sums (tests only): when registered by ox_set_scales, the J-loops also accumulate,
 * per particle, the magnitude of the terms their float sums are made of -- the scale of the rounding error of a
 * float sum in any order (SURVEY.md 8(c) tier 1).  a: L1 over the three components; dv: divv, curlv and dV;
 * gradh and alpha: the sums propagated through the closing formula. */
static double *g_sc_du, *g_sc_a, *g_sc_dv, *g_sc_gradh, *g_sc_alpha;

void ox_set_scales(double* du, double* a, double* dv, double* gradh, double* alpha)
{
    g_sc_du = du, g_sc_a = a, g_sc_dv = dv, g_sc_gradh = gradh, g_sc_alpha = alpha;
}

/* xmassJLoop (xmass_kern.hpp:50-79) */
static float xmassJLoop(uint32_t i, double K, const ox_box* b, const uint32_t* nb, unsigned cnt, const ox_state* s)
{
    double xi = s->x[i], yi = s->y[i], zi = s->z[i];
    float  hi = s->h[i], mi = s->m[i];
    float  hInv  = (float)(1.0 / hi);
    float  h3Inv = hInv * hInv * hInv;
    float  rho0i = mi;
    for (unsigned pj = 0; pj < cnt; ++pj)
    {
        uint32_t j    = nb[pj];
        float    dist = distancePBC(b, hi, xi, yi, zi, s->x[j], s->y[j], s->z[j]);
        float    vloc = dist * hInv;
        float    w    = lookup(g_wh, vloc);
        rho0i += w * s->m[j];
    }
    /* veDefinition deduces T = double from (rho0i * K * h3Inv) */
    return (float)((double)mi / ((double)rho0i * K * (double)h3Inv));
}

void ox_xmass(ox_state* s, const ox_params* p, const ox_box* b, const uint32_t* neighbors, unsigned first,
              unsigned last)
{
    if (!lists_ok(s, neighbors, first, last, p->ngmax)) return;
    ensure_tables();
#pragma omp parallel for
    for (size_t i = first; i < last; i++)
    {
        size_t ni = i - first;
        s->xm[i]  = xmassJLoop((uint32_t)i, p->K, b, neighbors + p->ngmax * ni, nc_capped(s->nc, i, p->ngmax), s);
    }
}

/* veDefGradhJLoop (ve_def_gradh_kern.hpp:43-90) */
static void veDefGradhJLoop(uint32_t i, double K, const ox_box* b, const uint32_t* nb, unsigned cnt,
                            const ox_state* s, float* kxo, float* gradho)
{
    double xi = s->x[i], yi = s->y[i], zi = s->z[i];
    float  hi = s->h[i], mi = s->m[i], xmassi = s->xm[i];
    float  hInv     = 1.0f / hi;
    float  h3Inv    = hInv * hInv * hInv;
    float  kxi      = xmassi;
    float  whomegai = -3.0f * xmassi;
    float  wrho0i   = -3.0f * mi;
    double sOm = 3.0 * fabs((double)xmassi), sRh = 3.0 * fabs((double)mi);
    for (unsigned pj = 0; pj < cnt; ++pj)
    {
        uint32_t j      = nb[pj];
        float    dist   = distancePBC(b, hi, xi, yi, zi, s->x[j], s->y[j], s->z[j]);
        float    vloc   = dist * hInv;
        float    w      = lookup(g_wh, vloc);
        float    dw     = lookup(g_whd, vloc);
        float    dterh  = -(3.0f * w + vloc * dw);
        float    xmassj = s->xm[j];
        kxi += w * xmassj;
        whomegai += dterh * xmassj;
        wrho0i += dterh * s->m[j];
        if (g_sc_gradh)
        {
            sOm += fabs((double)dterh * xmassj);
            sRh += fabs((double)dterh * s->m[j]);
        }
    }
    kxi      = (float)((double)kxi * (K * (double)h3Inv));
    whomegai = (float)((double)whomegai * (K * (double)h3Inv * (double)hInv));
    wrho0i   = (float)((double)wrho0i * (K * (double)h3Inv * (double)hInv));
    whomegai = (float)((double)(whomegai * mi / xmassi) +
                       ((double)kxi - K * (double)xmassi * (double)h3Inv) * (double)wrho0i);
    float rhoi   = kxi * mi / xmassi;
    float dhdrho = -hi / (rhoi * 3.0f);
    *kxo         = kxi;
    *gradho      = 1.0f - dhdrho * whomegai;
    if (g_sc_gradh)
    {
        const double k4 = K * (double)h3Inv * (double)hInv;
        g_sc_gradh[i]   = 1.0 + fabs((double)dhdrho) * k4 *
                                  (fabs((double)mi / xmassi) * sOm +
                                   (fabs((double)kxi) + K * fabs((double)xmassi) * (double)h3Inv) * sRh);
    }
}

void ox_ve_def_gradh(ox_state* s, const ox_params* p, const ox_box* b, const uint32_t* neighbors, unsigned first,
                     unsigned last)
{
    if (!lists_ok(s, neighbors, first, last, p->ngmax)) return;
    ensure_tables();
#pragma omp parallel for
    for (size_t i = first; i < last; i++)
    {
        size_t ni = i - first;
        veDefGradhJLoop((uint32_t)i, p->K, b, neighbors + p->ngmax * ni, nc_capped(s->nc, i, p->ngmax), s, &s->kx[i],
                        &s->gradh[i]);
    }
}

/* computeEOS_Impl (hydro_ve/eos.hpp:52-77) with idealGasEOS/idealGasCv (sph/eos.hpp:13-40) */
static float ideal_gas_cv_f(float mui, double gamma)
{
    const float R = 8.317e7f;
    return (float)((double)(R / mui) / (gamma - 1.0f));
}

void ox_eos(ox_state* s, const ox_params* p, unsigned first, unsigned last)
{
#pragma omp parallel for schedule(static)
    for (size_t i = first; i < last; ++i)
    {
        float  rho = s->kx[i] * s->m[i] / s->xm[i];
        double tmp = (double)ideal_gas_cv_f(p->muiConst, p->gamma) * s->temp[i] * (p->gamma - 1.0);
        double pi  = (double)rho * tmp;
        double ci  = sqrt(tmp);
        s->prho[i] = (float)(pi / (double)(s->kx[i] * s->m[i] * s->m[i] * s->gradh[i]));
        s->c[i]    = (float)ci;
    }
}

/* IADJLoop (iad_kern.hpp:43-109) */
/* volume weight of neighbor j: xm_j / kx_j (VE, iad_kern.hpp:74) or m_j / rho_j (std IADJLoopSTD,
 * hydro_std/iad_kern.hpp:40), both evaluated as (num / den) * w */
static void IADJLoopVol(uint32_t i, double K, const ox_box* b, const uint32_t* nb, unsigned cnt, ox_state* s,
                        const float* num, const float* den)
{
    float  tau11 = 0, tau12 = 0, tau13 = 0, tau22 = 0, tau23 = 0, tau33 = 0;
    double xi = s->x[i], yi = s->y[i], zi = s->z[i];
    float  hi    = s->h[i];
    float  hiInv = 1.0f / hi;
    for (unsigned pj = 0; pj < cnt; ++pj)
    {
        uint32_t j  = nb[pj];
        float    rx = (float)(xi - s->x[j]);
        float    ry = (float)(yi - s->y[j]);
        float    rz = (float)(zi - s->z[j]);
        applyPBC(b, 2.0f * hi, &rx, &ry, &rz);
        float dist   = sqrtf(rx * rx + ry * ry + rz * rz);
        float vloc   = dist * hiInv;
        float w      = lookup(g_wh, vloc);
        float volj_w = num[j] / den[j] * w;
        tau11 += rx * rx * volj_w;
        tau12 += rx * ry * volj_w;
        tau13 += rx * rz * volj_w;
        tau22 += ry * ry * volj_w;
        tau23 += ry * rz * volj_w;
        tau33 += rz * rz * volj_w;
    }
#define GETEXP(v) ((v) == 0.0f ? 0 : ilogbf(v))
    int tauExpSum = GETEXP(tau11) + GETEXP(tau12) + GETEXP(tau13) + GETEXP(tau22) + GETEXP(tau23) + GETEXP(tau33);
#undef GETEXP
    float normalization = ldexpf(1.0f, -tauExpSum / 6);
    tau11 *= normalization;
    tau12 *= normalization;
    tau13 *= normalization;
    tau22 *= normalization;
    tau23 *= normalization;
    tau33 *= normalization;
    float det = tau11 * tau22 * tau33 + 2.0f * tau12 * tau23 * tau13 - tau11 * tau23 * tau23 -
                tau22 * tau13 * tau13 - tau33 * tau12 * tau12;
    float factor = (float)((double)(normalization * (hi * hi * hi)) / ((double)det * K));
    s->c11[i]    = (tau22 * tau33 - tau23 * tau23) * factor;
    s->c12[i]    = (tau13 * tau23 - tau33 * tau12) * factor;
    s->c13[i]    = (tau12 * tau23 - tau22 * tau13) * factor;
    s->c22[i]    = (tau11 * tau33 - tau13 * tau13) * factor;
    s->c23[i]    = (tau13 * tau12 - tau11 * tau23) * factor;
    s->c33[i]    = (tau11 * tau22 - tau12 * tau12) * factor;
}

/* divV_curlVJLoop (divv_curlv_kern.hpp:43-123), curlv stored; doGradV (dV11.size() == x.size(),
 * iad_divv_curlv.hpp) writes the velocity-gradient fields of the avClean propagator (:113-121) */
static void divVcurlVJLoop(uint32_t i, double K, const ox_box* b, const uint32_t* nb, unsigned cnt, ox_state* s,
                           int doGradV)
{
    double xi = s->x[i], yi = s->y[i], zi = s->z[i];
    float  vxi = s->vx[i], vyi = s->vy[i], vzi = s->vz[i];
    float  hi = s->h[i], kxi = s->kx[i];
    float  hiInv  = 1.0f / hi;
    float  hiInv3 = hiInv * hiInv * hiInv;
    float  dVx[3] = {0, 0, 0}, dVy[3] = {0, 0, 0}, dVz[3] = {0, 0, 0};
    float  c11i = s->c11[i], c12i = s->c12[i], c13i = s->c13[i], c22i = s->c22[i], c23i = s->c23[i],
          c33i = s->c33[i];
    double sdv = 0.0;
    for (unsigned pj = 0; pj < cnt; ++pj)
    {
        uint32_t j  = nb[pj];
        float    rx = (float)(xi - s->x[j]);
        float    ry = (float)(yi - s->y[j]);
        float    rz = (float)(zi - s->z[j]);
        applyPBC(b, 2.0f * hi, &rx, &ry, &rz);
        float r2    = rx * rx + ry * ry + rz * rz;
        float dist  = sqrtf(r2);
        float vx_ji = s->vx[j] - vxi;
        float vy_ji = s->vy[j] - vyi;
        float vz_ji = s->vz[j] - vzi;
        float v1    = dist * hiInv;
        float Wi    = lookup(g_wh, v1);
        float tA[3];
        tA[0]        = -(c11i * rx + c12i * ry + c13i * rz) * Wi;
        tA[1]        = -(c12i * rx + c22i * ry + c23i * rz) * Wi;
        tA[2]        = -(c13i * rx + c23i * ry + c33i * rz) * Wi;
        float xmassj = s->xm[j];
        float fx = vx_ji * xmassj, fy = vy_ji * xmassj, fz = vz_ji * xmassj;
        for (int k = 0; k < 3; ++k)
        {
            dVx[k] = dVx[k] + tA[k] * fx;
            dVy[k] = dVy[k] + tA[k] * fy;
            dVz[k] = dVz[k] + tA[k] * fz;
        }
        if (g_sc_dv)
            sdv += (fabs((double)tA[0]) + fabs((double)tA[1]) + fabs((double)tA[2])) *
                   (fabs((double)fx) + fabs((double)fy) + fabs((double)fz));
    }
    float norm_kxi = (float)(K * (double)hiInv3 / (double)kxi);
    if (g_sc_dv) g_sc_dv[i] = fabs((double)norm_kxi) * sdv;
    s->divv[i]     = norm_kxi * (dVx[0] + dVy[1] + dVz[2]);
    if (s->curlv)
    {
        float cv0 = dVz[1] - dVy[2], cv1 = dVx[2] - dVz[0], cv2 = dVy[0] - dVx[1];
        s->curlv[i] = norm_kxi * sqrtf(cv0 * cv0 + (cv1 * cv1 + cv2 * cv2));
    }
    if (doGradV)
    {
        s->dV11[i] = norm_kxi * dVx[0];
        s->dV12[i] = norm_kxi * (dVx[1] + dVy[0]);
        s->dV13[i] = norm_kxi * (dVx[2] + dVz[0]);
        s->dV22[i] = norm_kxi * dVy[1];
        s->dV23[i] = norm_kxi * (dVy[2] + dVz[1]);
        s->dV33[i] = norm_kxi * dVz[2];
    }
}

void ox_iad_divv_curlv(ox_state* s, const ox_params* p, const ox_box* b, const uint32_t* neighbors, unsigned first,
                       unsigned last)
{
    if (!lists_ok(s, neighbors, first, last, p->ngmax)) return;
    ensure_tables();
#pragma omp parallel for
    for (size_t i = first; i < last; ++i)
    {
        size_t   ni  = i - first;
        unsigned cnt = nc_capped(s->nc, i, p->ngmax);
        IADJLoopVol((uint32_t)i, p->K, b, neighbors + p->ngmax * ni, cnt, s, s->xm, s->kx);
        divVcurlVJLoop((uint32_t)i, p->K, b, neighbors + p->ngmax * ni, cnt, s, p->avClean);
    }
}

/* AVswitchesJLoop (av_switches_kern.hpp:43-137) */
static float AVswitchesJLoop(uint32_t i, double K, const ox_box* b, const uint32_t* nb, unsigned cnt,
                             const ox_state* s, double dt, float alphamin, float alphamax, float decay_constant,
                             float alpha_i)
{
    double xi = s->x[i], yi = s->y[i], zi = s->z[i];
    float  vxi = s->vx[i], vyi = s->vy[i], vzi = s->vz[i];
    float  hi = s->h[i], ci = s->c[i];
    float  c11i = s->c11[i], c12i = s->c12[i], c13i = s->c13[i], c22i = s->c22[i], c23i = s->c23[i],
          c33i = s->c33[i];
    float vijsignal_i = 1.e-40f * ci;
    float hiInv       = 1.0f / hi;
    float hiInv3      = hiInv * hiInv * hiInv;
    float divv_i      = s->divv[i];
    float gx = 0, gy = 0, gz = 0;
    double sg = 0.0;
    for (unsigned pj = 0; pj < cnt; ++pj)
    {
        uint32_t j  = nb[pj];
        float    rx = (float)(xi - s->x[j]);
        float    ry = (float)(yi - s->y[j]);
        float    rz = (float)(zi - s->z[j]);
        applyPBC(b, 2.0f * hi, &rx, &ry, &rz);
        float r2           = rx * rx + ry * ry + rz * rz;
        float dist         = sqrtf(r2);
        float vx_ij        = vxi - s->vx[j];
        float vy_ij        = vyi - s->vy[j];
        float vz_ij        = vzi - s->vz[j];
        float rv           = rx * vx_ij + ry * vy_ij + rz * vz_ij;
        float vijsignal_ij = 0.0f;
        if (rv < 0.0f) { vijsignal_ij = ci + s->c[j] - 3.0f * rv / dist; }
        if (vijsignal_i < vijsignal_ij) vijsignal_i = vijsignal_ij; /* stl::max */
        float v1     = dist * hiInv;
        float Wi     = (float)(K * (double)hiInv3 * (double)lookup(g_wh, v1));
        float termA1 = -(c11i * rx + c12i * ry + c13i * rz) * Wi;
        float termA2 = -(c12i * rx + c22i * ry + c23i * rz) * Wi;
        float termA3 = -(c13i * rx + c23i * ry + c33i * rz) * Wi;
        float volj   = s->xm[j] / s->kx[j];
        float factor = volj * (divv_i - s->divv[j]);
        gx += factor * termA1;
        gy += factor * termA2;
        gz += factor * termA3;
        if (g_sc_alpha)
            sg += fabs((double)factor) * (fabs((double)termA1) + fabs((double)termA2) + fabs((double)termA3));
    }
    float graddivv = sqrtf(gx * gx + gy * gy + gz * gz);
    /* d alphaloc / d graddivv <= alphamax h^2 / (h^2 graddivv + h |divv| + 0.05 c) */
    if (g_sc_alpha)
        g_sc_alpha[i] = (double)alphamax * (double)hi * hi * sg /
                        ((double)hi * hi * graddivv + (double)hi * fabs((double)divv_i) + 0.05 * ci);
    float alphaloc = 0.0f;
    if (divv_i < 0.0f)
    {
        float a_const = hi * hi * graddivv;
        alphaloc      = alphamax * a_const / (a_const + hi * fabsf(divv_i) + 0.05f * ci);
    }
    if (alphaloc >= alpha_i) { alpha_i = alphaloc; }
    else
    {
        float decay    = hi / (decay_constant * vijsignal_i);
        float alphadot = 0.0f;
        if (alphaloc >= alphamin) { alphadot = (alphaloc - alpha_i) / decay; }
        else { alphadot = (alphamin - alpha_i) / decay; }
        alpha_i = (float)((double)alpha_i + (double)alphadot * dt);
    }
    return alpha_i;
}

void ox_av_switches(ox_state* s, const ox_params* p, const ox_box* b, const uint32_t* neighbors, unsigned first,
                    unsigned last)
{
    if (!lists_ok(s, neighbors, first, last, p->ngmax)) return;
    ensure_tables();
#pragma omp parallel for
    for (size_t i = first; i < last; ++i)
    {
        size_t ni   = i - first;
        s->alpha[i] = AVswitchesJLoop((uint32_t)i, p->K, b, neighbors + p->ngmax * ni, nc_capped(s->nc, i, p->ngmax),
                                      s, s->minDt, p->alphamin, p->alphamax, p->decay_constant, s->alpha[i]);
    }
}

/* momentumAndEnergyJLoop<avClean=false> (momentum_energy_kern.hpp:65-222), tdpdTrho == nullptr.
 * The Atwood ramp calls unqualified `pow(float, float)` inside namespace sph (momentum_energy_kern.hpp:192-193);
 * with libstdc++ that resolves to ::pow(double, double) from <math.h>, so each product is formed in double and
 * rounded once to float -- verified bit-for-bit against oracle/_ref on the Noh IC, where powf() differs. */
/* avRvCorrection<float, float> (momentum_energy_kern.hpp:43-63): symv is the upper-triangle product
 * (kernels.hpp:88-95) and dot the right fold a0*b0 + (a1*b1 + a2*b2) (util/array.hpp:253-256) */
static inline float dot3(float a0, float a1, float a2, float b0, float b1, float b2)
{
    return a0 * b0 + (a1 * b1 + a2 * b2);
}
static float avRvCorrection(float rx, float ry, float rz, float eta_ab, float eta_crit, const float* gi,
                            const float* gj)
{
    float dmy1 = dot3(rx, ry, rz, gi[0] * rx + gi[1] * ry + gi[2] * rz, gi[3] * ry + gi[4] * rz, gi[5] * rz);
    float dmy2 = dot3(rx, ry, rz, gj[0] * rx + gj[1] * ry + gj[2] * rz, gj[3] * ry + gj[4] * rz, gj[5] * rz);
    float dmy3 = 1.0f;
    if (eta_ab < eta_crit)
    {
        float etaDiff = 5.0f * (eta_ab - eta_crit);
        dmy3          = expf(-etaDiff * etaDiff);
    }
    float A_ab   = (dmy2 != 0.0f) ? dmy1 / dmy2 : 0.0f;
    float A_abp1 = 1.0f + A_ab;
    float q      = 4.0f * A_ab / (A_abp1 * A_abp1);
    q            = q < 1.0f ? q : 1.0f;  /* stl::min(T(1), x) */
    q            = 0.0f < q ? q : 0.0f;  /* stl::max(T(0), x) */
    float phi_ab = 0.5f * dmy3 * q;
    return -phi_ab * (dmy1 + dmy2);
}

/* error scale of the avClean correction (tests only, with the scales on): per unit of the checker's rtol, the change
 * of avRvCorrection when the velocity gradients gi, gj carry a relative error of that size.  The correction is
 * ill-conditioned where its quadratic forms dmy1, dmy2 cancel (A_ab = dmy1 / dmy2): the sensitivity of q is
 * propagated, capped at q's full range [0, 1] (5e4 = 1 / 2e-5, the step checker's rtol) */
static double avRvCorrectionScale(float rx, float ry, float rz, float eta_ab, float eta_crit, const float* gi,
                                  const float* gj)
{
    const double x = fabs((double)rx), y = fabs((double)ry), z = fabs((double)rz);
    const double d1 = dot3(rx, ry, rz, gi[0] * rx + gi[1] * ry + gi[2] * rz, gi[3] * ry + gi[4] * rz, gi[5] * rz);
    const double d2 = dot3(rx, ry, rz, gj[0] * rx + gj[1] * ry + gj[2] * rz, gj[3] * ry + gj[4] * rz, gj[5] * rz);
    const double S1 = x * (fabs(gi[0]) * x + fabs(gi[1]) * y + fabs(gi[2]) * z) + y * (fabs(gi[3]) * y + fabs(gi[4]) * z) +
                      z * fabs(gi[5]) * z;
    const double S2 = x * (fabs(gj[0]) * x + fabs(gj[1]) * y + fabs(gj[2]) * z) + y * (fabs(gj[3]) * y + fabs(gj[4]) * z) +
                      z * fabs(gj[5]) * z;
    double dmy3 = 1.0;
    if (eta_ab < eta_crit)
    {
        const double e = 5.0 * ((double)eta_ab - eta_crit);
        dmy3           = exp(-e * e);
    }
    const double kCap = 5e4;
    double       uq   = kCap, q = 1.0;
    if (d2 != 0.0 && d1 != 0.0)
    {
        const double A  = d1 / d2;
        const double uA = fabs(A) * (S1 / fabs(d1) + S2 / fabs(d2));
        q               = 4.0 * A / ((1.0 + A) * (1.0 + A));
        q               = q < 0.0 ? 0.0 : (q > 1.0 ? 1.0 : q);
        const double dq = fabs(4.0 * (1.0 - A) / ((1.0 + A) * (1.0 + A) * (1.0 + A)));
        uq              = fmin(kCap, dq * uA);
    }
    return 0.5 * dmy3 * (uq * fabs(d1 + d2) + q * (S1 + S2));
}

static void momentumJLoop(uint32_t i, double K, const ox_box* b, const uint32_t* nb, unsigned cnt, ox_state* s,
                          float Atmin, float Atmax, float ramp, int avClean, float* maxvsignal)
{
    double xi = s->x[i], yi = s->y[i], zi = s->z[i];
    float  vxi = s->vx[i], vyi = s->vy[i], vzi = s->vz[i];
    float  hi = s->h[i], mi = s->m[i], ci = s->c[i], kxi = s->kx[i];
    float  alpha_i = s->alpha[i];
    float  xmassi  = s->xm[i];
    float  rhoi    = kxi * mi / xmassi;
    float  prhoi   = s->prho[i];
    float  hiInv   = 1.0f / hi;
    float  hiInv3  = hiInv * hiInv * hiInv;
    float  maxvsignali = 0.0f;
    float  mx = 0, my = 0, mz = 0, energy = 0, a_visc_energy = 0;
    float  c11i = s->c11[i], c12i = s->c12[i], c13i = s->c13[i], c22i = s->c22[i], c23i = s->c23[i],
          c33i = s->c33[i];
    float gradV_i[6] = {0, 0, 0, 0, 0, 0};
    if (avClean)
    {
        gradV_i[0] = s->dV11[i], gradV_i[1] = s->dV12[i], gradV_i[2] = s->dV13[i];
        gradV_i[3] = s->dV22[i], gradV_i[4] = s->dV23[i], gradV_i[5] = s->dV33[i];
    }
    /* T(32) * M_PI / T(3) / T(neighborsCount + 1) is formed in double, cbrt in double, stored as float */
    float eta_crit = (float)cbrt((double)32.0f * M_PI / (double)3.0f / (double)(float)(cnt + 1));
    double sE = 0.0, sV = 0.0, sA = 0.0;
    for (unsigned pj = 0; pj < cnt; ++pj)
    {
        uint32_t j   = nb[pj];
        float    rx  = (float)(xi - s->x[j]);
        float    ry  = (float)(yi - s->y[j]);
        float    rz  = (float)(zi - s->z[j]);
        float    vxj = s->vx[j], vyj = s->vy[j], vzj = s->vz[j];
        applyPBC(b, 2.0f * hi, &rx, &ry, &rz);
        float r2     = rx * rx + ry * ry + rz * rz;
        float dist   = sqrtf(r2);
        float vx_ij  = vxi - vxj;
        float vy_ij  = vyi - vyj;
        float vz_ij  = vzi - vzj;
        float hj     = s->h[j];
        float hjInv  = 1.0f / hj;
        float v1     = dist * hiInv;
        float v2     = dist * hjInv;
        float hjInv3 = hjInv * hjInv * hjInv;
        float Wi     = hiInv3 * lookup(g_wh, v1);
        float Wj     = hjInv3 * lookup(g_wh, v2);
        float tA1i   = -(c11i * rx + c12i * ry + c13i * rz) * Wi;
        float tA2i   = -(c12i * rx + c22i * ry + c23i * rz) * Wi;
        float tA3i   = -(c13i * rx + c23i * ry + c33i * rz) * Wi;
        float c11j = s->c11[j], c12j = s->c12[j], c13j = s->c13[j], c22j = s->c22[j], c23j = s->c23[j],
              c33j = s->c33[j];
        float tA1j   = -(c11j * rx + c12j * ry + c13j * rz) * Wj;
        float tA2j   = -(c12j * rx + c22j * ry + c23j * rz) * Wj;
        float tA3j   = -(c13j * rx + c23j * ry + c33j * rz) * Wj;
        float mj     = s->m[j];
        float cj     = s->c[j];
        float kxj    = s->kx[j];
        float xmassj = s->xm[j];
        float rhoj   = kxj * mj / xmassj;
        float rv     = rx * vx_ij + ry * vy_ij + rz * vz_ij;
        double urv   = 0.0; /* avClean: error scale of rv (avRvCorrectionScale), with the scales on */
        if (avClean)
        {
            float gradV_j[6] = {s->dV11[j], s->dV12[j], s->dV13[j], s->dV22[j], s->dV23[j], s->dV33[j]};
            rv += avRvCorrection(rx, ry, rz, v2 < v1 ? v2 : v1, eta_crit, gradV_i, gradV_j); /* stl::min */
            if (g_sc_du)
                urv = avRvCorrectionScale(rx, ry, rz, v2 < v1 ? v2 : v1, eta_crit, gradV_i, gradV_j) +
                      0.01 * (fabs((double)rx * vx_ij) + fabs((double)ry * vy_ij) + fabs((double)rz * vz_ij));
        }
        float wij    = rv / dist;
        /* artificial_viscosity<float> (kernels.hpp:70-84): (alpha_i + alpha_j) / 4.0 is a double */
        float viscosity_ij = 0.0f;
        if (wij < 0.0f)
        {
            float vij_signal =
                (float)((double)(alpha_i + s->alpha[j]) / 4.0 * (double)(ci + cj) - (double)(2.0f * wij));
            viscosity_ij = -vij_signal * wij;
        }
        float vijsignal = 0.5f * (ci + cj) - 2.0f * wij;
        maxvsignali     = (vijsignal > maxvsignali) ? vijsignal : maxvsignali;
        float a_mom, b_mom;
        float Atwood = fabsf(rhoi - rhoj) / (rhoi + rhoj);
        if (Atwood < Atmin)
        {
            a_mom = xmassi * xmassi;
            b_mom = xmassj * xmassj;
        }
        else if (Atwood > Atmax)
        {
            a_mom = xmassi * xmassj;
            b_mom = a_mom;
        }
        else
        {
            float sigma_ij = ramp * (Atwood - Atmin);
            a_mom          = (float)(pow(xmassi, 2.0f - sigma_ij) * pow(xmassj, sigma_ij));
            b_mom          = (float)(pow(xmassj, 2.0f - sigma_ij) * pow(xmassi, sigma_ij));
        }
        float a_visc   = mj / rhoi * viscosity_ij;
        float b_visc   = mj / rhoj * viscosity_ij;
        float a_visc_x = 0.5f * (a_visc * tA1i + b_visc * tA1j);
        float a_visc_y = 0.5f * (a_visc * tA2i + b_visc * tA2j);
        float a_visc_z = 0.5f * (a_visc * tA3i + b_visc * tA3j);
        a_visc_energy += a_visc_x * vx_ij + a_visc_y * vy_ij + a_visc_z * vz_ij;
        energy += mj * a_mom * (vx_ij * tA1i + vy_ij * tA2i + vz_ij * tA3i);
        float momentum_i = mj * prhoi * a_mom;
        float momentum_j = mj * s->prho[j] * b_mom;
        mx += momentum_i * tA1i + momentum_j * tA1j + a_visc_x;
        my += momentum_i * tA2i + momentum_j * tA2j + a_visc_y;
        mz += momentum_i * tA3i + momentum_j * tA3j + a_visc_z;
        if (g_sc_du)
        {
            sE += fabs((double)mj * a_mom) *
                  (fabs((double)vx_ij * tA1i) + fabs((double)vy_ij * tA2i) + fabs((double)vz_ij * tA3i));
            sV += fabs((double)a_visc_x * vx_ij) + fabs((double)a_visc_y * vy_ij) + fabs((double)a_visc_z * vz_ij);
            sA += fabs((double)momentum_i) * (fabs((double)tA1i) + fabs((double)tA2i) + fabs((double)tA3i)) +
                  fabs((double)momentum_j) * (fabs((double)tA1j) + fabs((double)tA2j) + fabs((double)tA3j)) +
                  fabs((double)a_visc_x) + fabs((double)a_visc_y) + fabs((double)a_visc_z);
            if (urv > 0.0 && wij < 0.0)
            {
                /* the viscosity's change with rv: d(-s w)/dw, s = (alpha_i + alpha_j)/4 (c_i + c_j) - 2 w */
                const double dvis = fabs((double)(alpha_i + s->alpha[j]) / 4.0 * (ci + cj) - 4.0 * wij) * urv / dist;
                const double wi = (double)mj / rhoi, wj = (double)mj / rhoj;
                sV += dvis * 0.5 *
                      (wi * (fabs((double)tA1i * vx_ij) + fabs((double)tA2i * vy_ij) + fabs((double)tA3i * vz_ij)) +
                       wj * (fabs((double)tA1j * vx_ij) + fabs((double)tA2j * vy_ij) + fabs((double)tA3j * vz_ij)));
                sA += dvis * 0.5 *
                      (wi * (fabs((double)tA1i) + fabs((double)tA2i) + fabs((double)tA3i)) +
                       wj * (fabs((double)tA1j) + fabs((double)tA2j) + fabs((double)tA3j)));
            }
        }
    }
    if (g_sc_du)
    {
        g_sc_du[i] = K * (fabs((double)prhoi) * sE + 0.5 * sV);
        if (g_sc_a) g_sc_a[i] = K * sA;
    }
    if (a_visc_energy < 0.0f) a_visc_energy = 0.0f; /* stl::max(T(0), x) */
    float eCoeff = prhoi;
    s->du[i]     = K * (double)(eCoeff * energy + 0.5f * a_visc_energy);
    s->ax[i]     = (float)(-K * (double)mx);
    s->ay[i]     = (float)(-K * (double)my);
    s->az[i]     = (float)(-K * (double)mz);
    *maxvsignal  = maxvsignali;
}

/* tsKCourant<float> (kernels.hpp:12-18); Kcour is a float parameter */
static inline float tsKCourant(float maxvsignal, float h, float c, float Kcour)
{
    float v = maxvsignal > 0.0f ? maxvsignal : c;
    return Kcour * h / v;
}

double ox_momentum_energy(ox_state* s, const ox_params* p, const ox_box* b, const uint32_t* neighbors,
                          unsigned first, unsigned last)
{
    if (!lists_ok(s, neighbors, first, last, p->ngmax)) return 0.0;
    ensure_tables();
    float minDt = INFINITY;
#pragma omp parallel for schedule(static) reduction(min : minDt)
    for (size_t i = first; i < last; ++i)
    {
        size_t ni         = i - first;
        float  maxvsignal = 0;
        momentumJLoop((uint32_t)i, p->K, b, neighbors + p->ngmax * ni, nc_capped(s->nc, i, p->ngmax), s, p->Atmin,
                      p->Atmax, p->ramp, p->avClean, &maxvsignal);
        float dt_i = tsKCourant(maxvsignal, s->h[i], s->c[i], (float)p->Kcour);
        minDt      = minDt < dt_i ? minDt : dt_i;
    }
    s->minDtCourant = minDt;
    return minDt;
}

/* ------------------------------------------------------------------------------------------------
 * std propagator kernels (HydroProp, std_hydro.hpp:124-184)
 * ------------------------------------------------------------------------------------------------ */

/* computeDensityImpl (hydro_std/density.hpp:41-52): xmassJLoop written to rho, then rho = m / rho */
void ox_density(ox_state* s, const ox_params* p, const ox_box* b, const uint32_t* neighbors, unsigned first,
                unsigned last)
{
    if (!lists_ok(s, neighbors, first, last, p->ngmax)) return;
    ensure_tables();
#pragma omp parallel for
    for (size_t i = first; i < last; i++)
    {
        size_t ni  = i - first;
        float  xmi = xmassJLoop((uint32_t)i, p->K, b, neighbors + p->ngmax * ni, nc_capped(s->nc, i, p->ngmax), s);
        s->rho[i]  = s->m[i] / xmi;
    }
}

/* computeEOS_HydroStdImpl (hydro_std/eos.hpp:43-56): idealGasEOS(temp, rho, mui, gamma) in double */
void ox_eos_std(ox_state* s, const ox_params* p, unsigned first, unsigned last)
{
#pragma omp parallel for schedule(static)
    for (size_t i = first; i < last; ++i)
    {
        double tmp = (double)ideal_gas_cv_f(p->muiConst, p->gamma) * s->temp[i] * (p->gamma - 1.0);
        s->p[i]    = (float)((double)s->rho[i] * tmp);
        s->c[i]    = (float)sqrt(tmp);
    }
}

/* computeIADImpl (hydro_std/iad.hpp:41-70) with IADJLoopSTD (hydro_std/iad_kern.hpp:12-77) */
void ox_iad_std(ox_state* s, const ox_params* p, const ox_box* b, const uint32_t* neighbors, unsigned first,
                unsigned last)
{
    if (!lists_ok(s, neighbors, first, last, p->ngmax)) return;
    ensure_tables();
#pragma omp parallel for
    for (size_t i = first; i < last; ++i)
    {
        size_t ni = i - first;
        IADJLoopVol((uint32_t)i, p->K, b, neighbors + p->ngmax * ni, nc_capped(s->nc, i, p->ngmax), s, s->m, s->rho);
    }
}

/* momentumAndEnergyJLoop of the std propagator (hydro_std/momentum_energy_kern.hpp:12-134): gradh = 1, constant
 * alpha = 1 with the halved AV, r_ij and v_ij as i - j and the sign applied at the end (du only) */
static void momentumStdJLoop(uint32_t i, double K, const ox_box* b, const uint32_t* nb, unsigned cnt, ox_state* s,
                             float* maxvsignal)
{
    const float gradh_i = 1.0f, gradh_j = 1.0f;
    double      xi = s->x[i], yi = s->y[i], zi = s->z[i];
    float       vxi = s->vx[i], vyi = s->vy[i], vzi = s->vz[i];
    float       hi = s->h[i], roi = s->rho[i], pri = s->p[i], ci = s->c[i];
    float       mi_roi = s->m[i] / s->rho[i];
    float       hiInv  = 1.0f / hi;
    float       hiInv3 = hiInv * hiInv * hiInv;
    float       maxvsignali = 0.0f;
    float       momentum_x = 0, momentum_y = 0, momentum_z = 0, energy = 0;
    double      sA = 0.0, sE = 0.0;
    float c11i = s->c11[i], c12i = s->c12[i], c13i = s->c13[i], c22i = s->c22[i], c23i = s->c23[i], c33i = s->c33[i];
    for (unsigned pj = 0; pj < cnt; ++pj)
    {
        uint32_t j  = nb[pj];
        float    rx = (float)(xi - s->x[j]);
        float    ry = (float)(yi - s->y[j]);
        float    rz = (float)(zi - s->z[j]);
        applyPBC(b, 2.0f * hi, &rx, &ry, &rz);
        float r2     = rx * rx + ry * ry + rz * rz;
        float dist   = sqrtf(r2);
        float vx_ij  = vxi - s->vx[j];
        float vy_ij  = vyi - s->vy[j];
        float vz_ij  = vzi - s->vz[j];
        float hj     = s->h[j];
        float hjInv  = 1.0f / hj;
        float v1     = dist * hiInv;
        float v2     = dist * hjInv;
        float rv     = rx * vx_ij + ry * vy_ij + rz * vz_ij;
        float hjInv3 = hjInv * hjInv * hjInv;
        float Wi     = hiInv3 * lookup(g_wh, v1);
        float Wj     = hjInv3 * lookup(g_wh, v2);
        float tA1i   = c11i * rx + c12i * ry + c13i * rz;
        float tA2i   = c12i * rx + c22i * ry + c23i * rz;
        float tA3i   = c13i * rx + c23i * ry + c33i * rz;
        float c11j = s->c11[j], c12j = s->c12[j], c13j = s->c13[j], c22j = s->c22[j], c23j = s->c23[j],
              c33j = s->c33[j];
        float tA1j = c11j * rx + c12j * ry + c13j * rz;
        float tA2j = c12j * rx + c22j * ry + c23j * rz;
        float tA3j = c13j * rx + c23j * ry + c33j * rz;
        float roj  = s->rho[j];
        float cj   = s->c[j];
        float wij  = rv / dist;
        /* 0.5 * artificial_viscosity(1, 1, ci, cj, wij) (kernels.hpp:70-84): (1 + 1) / 4.0 is a double */
        float visc = 0.0f;
        if (wij < 0.0f)
        {
            float vij_signal = (float)((double)(1.0f + 1.0f) / 4.0 * (double)(ci + cj) - (double)(2.0f * wij));
            visc             = -vij_signal * wij;
        }
        float viscosity_ij = 0.5f * visc;
        float vijsignal    = ci + cj - 3.0f * wij;
        maxvsignali        = (vijsignal > maxvsignali) ? vijsignal : maxvsignali;
        float mj        = s->m[j];
        float mj_roj_Wj = mj / roj * Wj;
        float mj_pro_i  = mj * pri / (gradh_i * roi * roi);
        float am        = Wi * (mj_pro_i + viscosity_ij * mi_roi);
        float bm        = mj_roj_Wj * (s->p[j] / (roj * gradh_j) + viscosity_ij);
        momentum_x += am * tA1i + bm * tA1j;
        momentum_y += am * tA2i + bm * tA2j;
        momentum_z += am * tA3i + bm * tA3j;
        float ae = Wi * (2.0f * mj_pro_i + viscosity_ij * mi_roi);
        float be = viscosity_ij * mj_roj_Wj;
        energy += vx_ij * (ae * tA1i + be * tA1j) + vy_ij * (ae * tA2i + be * tA2j) + vz_ij * (ae * tA3i + be * tA3j);
        if (g_sc_du)
        {
            const double ta = fabs((double)tA1i) + fabs((double)tA2i) + fabs((double)tA3i),
                         tb = fabs((double)tA1j) + fabs((double)tA2j) + fabs((double)tA3j),
                         vv = fabs((double)vx_ij) + fabs((double)vy_ij) + fabs((double)vz_ij);
            sA += fabs((double)am) * ta + fabs((double)bm) * tb;
            sE += vv * (fabs((double)ae) * ta + fabs((double)be) * tb);
        }
    }
    if (g_sc_du)
    {
        g_sc_du[i] = K * 0.5 * sE;
        if (g_sc_a) g_sc_a[i] = K * sA;
    }
    s->du[i]    = -K * 0.5 * (double)energy;
    s->ax[i]    = (float)(K * (double)momentum_x);
    s->ay[i]    = (float)(K * (double)momentum_y);
    s->az[i]    = (float)(K * (double)momentum_z);
    *maxvsignal = maxvsignali;
}

/* computeMomentumEnergyStdImpl (hydro_std/momentum_energy.hpp:40-84) */
double ox_momentum_energy_std(ox_state* s, const ox_params* p, const ox_box* b, const uint32_t* neighbors,
                              unsigned first, unsigned last)
{
    if (!lists_ok(s, neighbors, first, last, p->ngmax)) return 0.0;
    ensure_tables();
    float minDt = INFINITY;
#pragma omp parallel for schedule(static) reduction(min : minDt)
    for (size_t i = first; i < last; ++i)
    {
        size_t ni         = i - first;
        float  maxvsignal = 0;
        momentumStdJLoop((uint32_t)i, p->K, b, neighbors + p->ngmax * ni, nc_capped(s->nc, i, p->ngmax), s,
                         &maxvsignal);
        float dt_i = tsKCourant(maxvsignal, s->h[i], s->c[i], (float)p->Kcour);
        minDt      = minDt < dt_i ? minDt : dt_i;
    }
    s->minDtCourant = minDt;
    return minDt;
}

/* ------------------------------------------------------------------------------------------------
 * integration (sph/positions.hpp:54-139 with the F2 fix, update_h.hpp:12-22, ts_global.hpp:72-112)
 * ------------------------------------------------------------------------------------------------ */

void ox_positions(ox_state* s, const ox_params* p, const ox_box* b, unsigned first, unsigned last)
{
    double dt = s->minDt, dt_m1 = s->minDt_m1;
    float  constCv = ideal_gas_cv_f(p->muiConst, p->gamma);
#pragma omp parallel for schedule(static)
    for (size_t i = first; i < last; i++)
    {
        /* positionUpdate<double> (:77-88); fixed-boundary branch (:99-108) applies to bnd == 2 only */
        int skip = 0;
        if ((b->bnd[0] == 2 || b->bnd[1] == 2 || b->bnd[2] == 2) && s->vx[i] == 0.0f && s->vy[i] == 0.0f &&
            s->vz[i] == 0.0f)
        {
            double X[3] = {s->x[i], s->y[i], s->z[i]};
            for (int d = 0; d < 3; ++d)
            {
                double top = b->lim[2 * d + 1], bot = b->lim[2 * d];
                if (b->bnd[d] == 2 &&
                    (fabs(top - X[d]) < 2.0f * s->h[i] || fabs(bot - X[d]) < 2.0f * s->h[i]))
                    skip = 1;
            }
        }
        if (!skip)
        {
            double A[3]  = {s->ax[i], s->ay[i], s->az[i]};
            double X[3]  = {s->x[i], s->y[i], s->z[i]};
            double dX[3] = {s->x_m1[i], s->y_m1[i], s->z_m1[i]};
            double Xn[3], Vn1[3], dXn1[3];
            double inv = 1.0 / dt_m1, hdm1 = 0.5 * dt_m1, adt = fabs(dt);
            for (int k = 0; k < 3; ++k)
            {
                double Vnmhalf = dX[k] * inv;
                double Vn      = Vnmhalf + A[k] * hdm1;
                Vn1[k]         = Vn + A[k] * dt;
                dXn1[k]        = (Vn + (A[k] * 0.5) * adt) * dt;
                Xn[k]          = X[k] + dXn1[k];
            }
            /* putInBox (box.hpp:209-230) */
            for (int d = 0; d < 3; ++d)
            {
                int pbc = box_pbc(b, d);
                if (pbc && Xn[d] > b->lim[2 * d + 1]) Xn[d] -= box_l(b, d);
                else if (pbc && Xn[d] < b->lim[2 * d]) Xn[d] += box_l(b, d);
            }
            s->x[i]    = Xn[0];
            s->y[i]    = Xn[1];
            s->z[i]    = Xn[2];
            s->x_m1[i] = (float)dXn1[0];
            s->y_m1[i] = (float)dXn1[1];
            s->z_m1[i] = (float)dXn1[2];
            s->vx[i]   = (float)Vn1[0];
            s->vy[i]   = (float)Vn1[1];
            s->vz[i]   = (float)Vn1[2];
        }
        /* updateTempHost with energyUpdate<double,double> (:54-61, :121-139), F2 fixed */
        double u_old = (double)constCv * s->temp[i];
        double du = s->du[i], du_m1 = (double)s->du_m1[i];
        double u_new = u_old + du * dt + 0.5 * (du - du_m1) / dt_m1 * fabs(dt) * dt;
        if (u_new < 0.) { u_new = u_old * exp(u_new * dt / u_old); }
        s->temp[i]  = u_new / (double)constCv;
        s->du_m1[i] = (float)s->du[i];
    }
}

/* ------------------------------------------------------------------------------------------------
 * Block time-steps (HydroVeBdtProp seam): positions_gpu.cu:45-179, ts_groups.cu:17-108, restated per group
 * [gs[g], ge[g]).  dt, dt_m1 per rung and cv as the GPU seam passes them (float), evaluated in double like
 * positionUpdate / energyUpdate (positions.hpp:54-88).
 * ------------------------------------------------------------------------------------------------ */
static double energy_update(double u_old, double dt, double dt_m1, double du, double du_m1)
{
    double u_new = u_old + du * dt + 0.5 * (du - du_m1) / dt_m1 * fabs(dt) * dt;
    if (u_new < 0.) { u_new = u_old * exp(u_new * dt / u_old); }
    return u_new;
}

static void position_update(double dt, double dt_m1, const double* X, const double* A, const double* dX,
                            const ox_box* b, double* Xn, double* V, double* dXn)
{
    double inv = 1.0 / dt_m1, hdm1 = 0.5 * dt_m1, adt = fabs(dt);
    for (int k = 0; k < 3; ++k)
    {
        double Vnmhalf = dX[k] * inv;
        double Vn      = Vnmhalf + A[k] * hdm1;
        V[k]           = Vn + A[k] * dt;
        dXn[k]         = (Vn + (A[k] * 0.5) * adt) * dt;
        Xn[k]          = X[k] + dXn[k];
    }
    if (b)
        for (int d = 0; d < 3; ++d)
        {
            int pbc = box_pbc(b, d);
            if (pbc && Xn[d] > b->lim[2 * d + 1]) Xn[d] -= box_l(b, d);
            else if (pbc && Xn[d] < b->lim[2 * d]) Xn[d] += box_l(b, d);
        }
}

/* computePositionsKernel (positions_gpu.cu:110-160), temp form, cv = (float)constCv (Thydro cv) */
void ox_positions_rungs(ox_state* s, const uint32_t* gs, const uint32_t* ge, unsigned ng, float dt, const float* dt_m1,
                        const uint8_t* rung, double constCv, const ox_box* b)
{
    float cv = (float)constCv;
    for (unsigned g = 0; g < ng; ++g)
        for (uint32_t i = gs[g]; i < ge[g]; ++i)
        {
            int fbc = b->bnd[0] == 2 || b->bnd[1] == 2 || b->bnd[2] == 2, skip = 0;
            if (fbc && s->vx[i] == 0.0f && s->vy[i] == 0.0f && s->vz[i] == 0.0f)
            {
                double X[3] = {s->x[i], s->y[i], s->z[i]};
                for (int d = 0; d < 3; ++d)
                {
                    double top = b->lim[2 * d + 1], bot = b->lim[2 * d];
                    if (b->bnd[d] == 2 && (fabs(top - X[d]) < 2.0f * s->h[i] || fabs(bot - X[d]) < 2.0f * s->h[i]))
                        skip = 1;
                }
            }
            if (skip) continue;
            double dm1  = rung ? dt_m1[rung[i]] : dt_m1[0];
            double A[3] = {s->ax[i], s->ay[i], s->az[i]}, X[3] = {s->x[i], s->y[i], s->z[i]},
                   dX[3] = {s->x_m1[i], s->y_m1[i], s->z_m1[i]};
            double Xn[3], V[3], dXn[3];
            position_update(dt, dm1, X, A, dX, b, Xn, V, dXn);
            s->x[i] = Xn[0], s->y[i] = Xn[1], s->z[i] = Xn[2];
            s->x_m1[i] = (float)dXn[0], s->y_m1[i] = (float)dXn[1], s->z_m1[i] = (float)dXn[2];
            s->vx[i] = (float)V[0], s->vy[i] = (float)V[1], s->vz[i] = (float)V[2];
            s->temp[i]  = energy_update(s->temp[i] * cv, dt, dm1, s->du[i], (double)s->du_m1[i]) / cv;
            s->du_m1[i] = (float)s->du[i];
        }
}

/* driftKernel (positions_gpu.cu:45-86): open box, x_m1 and du_m1 kept */
void ox_drift_positions(ox_state* s, const uint32_t* gs, const uint32_t* ge, unsigned ng, float dt, float dt_back,
                        const float* dt_m1, const uint8_t* rung, double constCv)
{
    float cv = (float)constCv;
    for (unsigned g = 0; g < ng; ++g)
        for (uint32_t i = gs[g]; i < ge[g]; ++i)
        {
            double dm1  = rung ? dt_m1[rung[i]] : dt_m1[0];
            double A[3] = {s->ax[i], s->ay[i], s->az[i]}, Xb[3] = {s->x[i], s->y[i], s->z[i]},
                   dX[3] = {s->x_m1[i], s->y_m1[i], s->z_m1[i]};
            double X0[3], V[3], dXn[3], X1[3];
            position_update(-(double)dt_back, dm1, Xb, A, dX, NULL, X0, V, dXn);
            position_update(dt, dm1, X0, A, dX, NULL, X1, V, dXn);
            s->x[i] = X1[0], s->y[i] = X1[1], s->z[i] = X1[2];
            s->vx[i] = (float)V[0], s->vy[i] = (float)V[1], s->vz[i] = (float)V[2];
            double u_recov = energy_update(s->temp[i] * cv, -(double)dt_back, dm1, s->du[i], (double)s->du_m1[i]);
            s->temp[i]     = energy_update(u_recov, dt, dm1, s->du[i], (double)s->du_m1[i]) / cv;
        }
}

/* groupDivvKernel / groupAccKernel (ts_groups.cu:17-68) */
void ox_group_divv_dt(float Krho, const uint32_t* gs, const uint32_t* ge, unsigned ng, const float* divv,
                      float* groupDt)
{
    for (unsigned g = 0; g < ng; ++g)
    {
        float m = -INFINITY;
        for (uint32_t i = gs[g]; i < ge[g]; ++i)
            m = m > divv[i] ? m : divv[i];
        float v    = Krho / fabsf(m);
        groupDt[g] = groupDt[g] < v ? groupDt[g] : v;
    }
}

void ox_group_acc_dt(float etaAcc, const uint32_t* gs, const uint32_t* ge, unsigned ng, const float* ax,
                     const float* ay, const float* az, float* groupDt)
{
    for (unsigned g = 0; g < ng; ++g)
    {
        float m = 0.0f;
        for (uint32_t i = gs[g]; i < ge[g]; ++i)
        {
            float a2 = ax[i] * ax[i] + (ay[i] * ay[i] + az[i] * az[i]);
            m        = m > a2 ? m : a2;
        }
        float v    = etaAcc / sqrtf(sqrtf(m));
        groupDt[g] = groupDt[g] < v ? groupDt[g] : v;
    }
}

void ox_update_h_range(ox_state* s, unsigned ng0, unsigned first, unsigned last)
{
#pragma omp parallel for schedule(static)
    for (size_t i = first; i < last; i++)
        s->h[i] = ox_update_h(ng0, s->nc[i], s->h[i]);
}


/* ------------------------------------------------------------------------------------------------
 * self-gravity (ryoanji CPU path, single rank, open box): expansion centers and MAC radii of the focus tree
 * (octree_focus_mpi.hpp:325-392 updateCenters, :432-459 setMacRadius), Cartesian quadrupoles
 * (upsweep_cpu.hpp:53-86, cartesian_qpole.hpp:88-257), Barnes-Hut traversal (traversal_cpu.hpp:80-230)
 * ------------------------------------------------------------------------------------------------ */

/* cstone::massCenter<double> + normalizeMass (source_center.hpp:45-81) */
static void grav_mass_center(const double* x, const double* y, const double* z, const float* m, uint32_t first,
                             uint32_t last, double* c)
{
    c[0] = c[1] = c[2] = c[3] = 0.0;
    for (uint32_t i = first; i < last; ++i)
    {
        double w = (double)m[i];
        c[0] += w * x[i];
        c[1] += w * y[i];
        c[2] += w * z[i];
        c[3] += w;
    }
    double invM = (c[3] != 0.0) ? 1.0 / c[3] : 0.0;
    c[0] *= invM;
    c[1] *= invM;
    c[2] *= invM;
}

/* P2M<double, float, float> (cartesian_qpole.hpp:88-126): float accumulators, each update formed in double */
static void grav_p2m(const double* x, const double* y, const double* z, const float* m, uint32_t begin, uint32_t end,
                     const double* center, float* gv)
{
    for (int k = 0; k < 8; ++k)
        gv[k] = 0.0f;
    if (begin == end) return;
    for (uint32_t i = begin; i < end; ++i)
    {
        double m_i = (double)m[i];
        double rx = x[i] - center[0], ry = y[i] - center[1], rz = z[i] - center[2];
        gv[0] = (float)((double)gv[0] + m_i);
        gv[1] = (float)((double)gv[1] + rx * rx * m_i);
        gv[2] = (float)((double)gv[2] + rx * ry * m_i);
        gv[3] = (float)((double)gv[3] + rx * rz * m_i);
        gv[4] = (float)((double)gv[4] + ry * ry * m_i);
        gv[5] = (float)((double)gv[5] + ry * rz * m_i);
        gv[6] = (float)((double)gv[6] + rz * rz * m_i);
    }
    float traceQ = gv[1] + gv[4] + gv[6];
    gv[7]        = traceQ;
    gv[1]        = 3 * gv[1] - traceQ;
    gv[4]        = 3 * gv[4] - traceQ;
    gv[6]        = 3 * gv[6] - traceQ;
    gv[2] *= 3;
    gv[3] *= 3;
    gv[5] *= 3;
}

/* addQuadrupole<float, double> (cartesian_qpole.hpp:210-232), parallel axis theorem */
static void grav_add_quadrupole(float* comp, double rx, double ry, double rz, const float* add)
{
    double rx_2 = rx * rx, ry_2 = ry * ry, rz_2 = rz * rz;
    double r_2  = (rx_2 + ry_2 + rz_2) * (1.0 / 3.0);
    double ml   = (double)(add[0] * 3);
    comp[7]     = (float)((double)(comp[7] + add[7]) + ml * r_2);
    comp[0] += add[0];
    comp[1] = (float)((double)comp[1] + ((double)add[1] + ml * (rx_2 - r_2)));
    comp[2] = (float)((double)comp[2] + ((double)add[2] + ml * rx * ry));
    comp[3] = (float)((double)comp[3] + ((double)add[3] + ml * rx * rz));
    comp[4] = (float)((double)comp[4] + ((double)add[4] + ml * (ry_2 - r_2)));
    comp[5] = (float)((double)comp[5] + ((double)add[5] + ml * ry * rz));
    comp[6] = (float)((double)comp[6] + ((double)add[6] + ml * (rz_2 - r_2)));
}

/* expansion centers (mass centers, upsweep with CombineSourceCenter) and setMac (computeVecMacR2,
 * traversal/macs.hpp:82-97), then leaf P2M + upsweepMultipoles (M2M); centers4[4*node] = {x,y,z,mac^2} */
static void grav_upsweep(const ox_state* s, const ox_tree* t, float invTheta, double* centers4, float* mp)
{
    int nInt = t->nTot - t->nLeaf;
#pragma omp parallel for schedule(static)
    for (int L = 0; L < t->nLeaf; ++L)
    {
        int node = t->leafToInternal[nInt + L];
        grav_mass_center(s->x, s->y, s->z, s->m, t->layout[L], t->layout[L + 1], centers4 + 4 * (size_t)node);
    }
    for (int level = MAXLEVEL; level >= 0; --level)
    {
#pragma omp parallel for schedule(static)
        for (int i = t->levelRange[level]; i < t->levelRange[level + 1]; ++i)
        {
            int c = t->childOffsets[i];
            if (!c) continue;
            double acc[4] = {0, 0, 0, 0};
            for (int k = c; k < c + 8; ++k)
            {
                double w = centers4[4 * (size_t)k + 3];
                acc[0] += w * centers4[4 * (size_t)k + 0];
                acc[1] += w * centers4[4 * (size_t)k + 1];
                acc[2] += w * centers4[4 * (size_t)k + 2];
                acc[3] += w;
            }
            double invM = (acc[3] != 0.0) ? 1.0 / acc[3] : 0.0;
            centers4[4 * (size_t)i + 0] = acc[0] * invM;
            centers4[4 * (size_t)i + 1] = acc[1] * invM;
            centers4[4 * (size_t)i + 2] = acc[2] * invM;
            centers4[4 * (size_t)i + 3] = acc[3];
        }
    }
#pragma omp parallel for schedule(static)
    for (int i = 0; i < t->nTot; ++i)
    {
        double* c  = centers4 + 4 * (size_t)i;
        double  dx = c[0] - t->centers[3 * (size_t)i], dy = c[1] - t->centers[3 * (size_t)i + 1],
               dz = c[2] - t->centers[3 * (size_t)i + 2];
        double sx = t->sizes[3 * (size_t)i], sy = t->sizes[3 * (size_t)i + 1], sz = t->sizes[3 * (size_t)i + 2];
        double smax = sx > sy ? sx : sy;
        smax        = smax > sz ? smax : sz;
        double sd   = sqrt(dx * dx + (dy * dy + dz * dz)); /* norm2 = right fold */
        double l    = 2.0 * smax;
        double mac  = l * (double)invTheta + sd;
        c[3]        = (c[3] != 0.0) ? mac * mac : 0.0;
    }
#pragma omp parallel for schedule(static)
    for (int L = 0; L < t->nLeaf; ++L)
    {
        int node = t->leafToInternal[nInt + L];
        grav_p2m(s->x, s->y, s->z, s->m, t->layout[L], t->layout[L + 1], centers4 + 4 * (size_t)node,
                 mp + 8 * (size_t)node);
    }
    for (int level = MAXLEVEL; level >= 0; --level)
    {
#pragma omp parallel for schedule(static)
        for (int i = t->levelRange[level]; i < t->levelRange[level + 1]; ++i)
        {
            int c = t->childOffsets[i];
            if (!c) continue;
            float* out = mp + 8 * (size_t)i;
            for (int k = 0; k < 8; ++k)
                out[k] = 0.0f;
            for (int k = c; k < c + 8; ++k)
            {
                const double* Xo = centers4 + 4 * (size_t)i;
                const double* Xi = centers4 + 4 * (size_t)k;
                grav_add_quadrupole(out, Xo[0] - Xi[0], Xo[1] - Xi[1], Xo[2] - Xi[2], mp + 8 * (size_t)k);
            }
        }
    }
}

/* M2P<double, double, float> (cartesian_qpole.hpp:175-201); inverseSquareRoot on the host = 1/sqrt */
static inline void grav_m2p(double* acc, double tx, double ty, double tz, const double* com, const float* M)
{
    double r0 = tx - com[0], r1 = ty - com[1], r2 = tz - com[2];
    double rr       = r0 * r0 + (r1 * r1 + r2 * r2);
    double r_minus1 = 1.0 / sqrt(rr);
    double r_minus2 = r_minus1 * r_minus1;
    double r_minus5 = r_minus2 * r_minus2 * r_minus1;
    double Qrx      = r0 * (double)M[1] + r1 * (double)M[2] + r2 * (double)M[3];
    double Qry      = r0 * (double)M[2] + r1 * (double)M[4] + r2 * (double)M[5];
    double Qrz      = r0 * (double)M[3] + r1 * (double)M[5] + r2 * (double)M[6];
    double rQr      = r0 * Qrx + r1 * Qry + r2 * Qrz;
    double rQrAndMonopole = (-2.5 * rQr * r_minus5 - (double)M[0] * r_minus1) * r_minus2;
    acc[0] += -((double)M[0] * r_minus1 + 0.5 * r_minus5 * rQr);
    acc[1] += r_minus5 * Qrx + rQrAndMonopole * r0;
    acc[2] += r_minus5 * Qry + rQrAndMonopole * r1;
    acc[3] += r_minus5 * Qrz + rQrAndMonopole * r2;
    /* magnitude of the terms (error scale, ox_set_scales) */
    acc[4] += fabs(r_minus5) * (fabs(Qrx) + fabs(Qry) + fabs(Qrz)) +
              fabs(rQrAndMonopole) * (fabs(r0) + fabs(r1) + fabs(r2));
}

/* P2P<double, double, float, float> (kernel.hpp:514-535), softened by h_i + h_j */
static inline void grav_p2p(double* acc, double xi, double yi, double zi, double xj, double yj, double zj, float mj,
                            float hi, float hj)
{
    double dx = xj - xi, dy = yj - yi, dz = zj - zi;
    double R2     = dx * dx + (dy * dy + dz * dz);
    float  h_ij   = hi + hj;
    float  h_ij2  = h_ij * h_ij;
    double R2eff  = (R2 < (double)h_ij2) ? (double)h_ij2 : R2;
    double invR   = 1.0 / sqrt(R2eff);
    double invR2  = invR * invR;
    double invR3m = (double)mj * invR * invR2;
    acc[0] -= invR3m * R2;
    acc[1] += dx * invR3m;
    acc[2] += dy * invR3m;
    acc[3] += dz * invR3m;
    acc[4] += fabs(invR3m) * (fabs(dx) + fabs(dy) + fabs(dz));
}

#define GRAV_GROUP 16

/* computeGravity (traversal_cpu.hpp:166-230) over targets [first, last) in groups of 16 consecutive particles,
 * computeGravityGroup (:80-151) with singleTraversal (traversal.hpp:69-110).  The reference sizes the target box of
 * a partial last group over all 16 array slots (uninitialised past the valid ones); the valid targets are used
 * here.  Adds G*acc to ax, ay, az; returns 0.5 * sum G m_i phi_i. */
static double grav_traverse(ox_state* s, const ox_tree* t, const double* centers4, const float* mp, float G,
                            uint32_t first, uint32_t last)
{
    double egrav = 0.0;
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : egrav)
    for (uint32_t i0 = first; i0 < last; i0 += GRAV_GROUP)
    {
        uint32_t nt = last - i0 < GRAV_GROUP ? last - i0 : GRAV_GROUP;
        double   acc[GRAV_GROUP][5];
        double   lo[3], hi[3];
        for (uint32_t k = 0; k < nt; ++k)
        {
            acc[k][0] = acc[k][1] = acc[k][2] = acc[k][3] = acc[k][4] = 0.0;
            double p[3] = {s->x[i0 + k], s->y[i0 + k], s->z[i0 + k]};
            for (int d = 0; d < 3; ++d)
            {
                if (k == 0 || p[d] < lo[d]) lo[d] = p[d];
                if (k == 0 || p[d] > hi[d]) hi[d] = p[d];
            }
        }
        double tc[3], ts[3];
        for (int d = 0; d < 3; ++d)
        {
            tc[d] = (hi[d] + lo[d]) * 0.5;
            ts[d] = (hi[d] - lo[d]) * 0.5;
        }
#define GRAV_DESCEND(node, out)                                                                                        \
    do {                                                                                                               \
        const double* com_ = centers4 + 4 * (size_t)(node);                                                            \
        double        d0 = fabs(tc[0] - com_[0]) - ts[0], d1 = fabs(tc[1] - com_[1]) - ts[1],                          \
               d2 = fabs(tc[2] - com_[2]) - ts[2];                                                                     \
        d0 += fabs(d0);                                                                                                \
        d1 += fabs(d1);                                                                                                \
        d2 += fabs(d2);                                                                                                \
        d0 *= 0.5;                                                                                                     \
        d1 *= 0.5;                                                                                                     \
        d2 *= 0.5;                                                                                                     \
        double R2_ = d0 * d0 + (d1 * d1 + d2 * d2);                                                                    \
        (out)      = R2_ < fabs(com_[3]);                                                                              \
        if (!(out))                                                                                                    \
            for (uint32_t k = 0; k < nt; ++k)                                                                          \
                grav_m2p(acc[k], s->x[i0 + k], s->y[i0 + k], s->z[i0 + k], com_, mp + 8 * (size_t)(node));            \
    } while (0)
#define GRAV_LEAF(node)                                                                                                \
    do {                                                                                                               \
        int      lidx_ = t->internalToLeaf[node];                                                                      \
        uint32_t s0_ = t->layout[lidx_], s1_ = t->layout[lidx_ + 1];                                                   \
        for (uint32_t k = 0; k < nt; ++k)                                                                              \
            for (uint32_t j = s0_; j < s1_; ++j)                                                                       \
                grav_p2p(acc[k], s->x[i0 + k], s->y[i0 + k], s->z[i0 + k], s->x[j], s->y[j], s->z[j], s->m[j],         \
                         s->h[i0 + k], s->h[j]);                                                                       \
    } while (0)
        int descend;
        GRAV_DESCEND(0, descend);
        if (descend)
        {
            if (t->childOffsets[0] == 0) { GRAV_LEAF(0); }
            else
            {
                int stack[128];
                stack[0]     = 0;
                int stackPos = 1, node = 0;
                do
                {
                    for (int octant = 0; octant < 8; ++octant)
                    {
                        int child = t->childOffsets[node] + octant;
                        int d;
                        GRAV_DESCEND(child, d);
                        if (d)
                        {
                            if (t->childOffsets[child] == 0) { GRAV_LEAF(child); }
                            else { stack[stackPos++] = child; }
                        }
                    }
                    node = stack[--stackPos];
                } while (node != 0);
            }
        }
#undef GRAV_DESCEND
#undef GRAV_LEAF
        for (uint32_t k = 0; k < nt; ++k)
        {
            double u = (double)(G * s->m[i0 + k]) * acc[k][0];
            egrav += u;
            s->ax[i0 + k] = (float)((double)s->ax[i0 + k] + (double)G * acc[k][1]);
            s->ay[i0 + k] = (float)((double)s->ay[i0 + k] + (double)G * acc[k][2]);
            s->az[i0 + k] = (float)((double)s->az[i0 + k] + (double)G * acc[k][3]);
            if (g_sc_a) g_sc_a[i0 + k] += fabs((double)G) * acc[k][4];
        }
    }
    return 0.5 * egrav;
}

/* upsweep + traversal on the tree of the (key-sorted) state: adds gravity to ax, ay, az of [first, last), returns
 * egrav; centers4/multipoles (numNodes x 4 doubles / x 8 floats) are written when non-null */
double ox_gravity(ox_state* s, const ox_params* p, const ox_box* b, unsigned bucket, unsigned first, unsigned last,
                  double* centersOut, float* multipolesOut, int cap)
{
    ox_tree t;
    tree_build(&t, s->keys, s->n, bucket, b);
    if (cap < 0)
    {
        int nTot = t.nTot; /* size query */
        tree_free(&t);
        return (double)nTot;
    }
    double* c4 = (double*)calloc(4 * (size_t)t.nTot, sizeof(double));
    float*  mp = (float*)calloc(8 * (size_t)t.nTot, sizeof(float));
    grav_upsweep(s, &t, 1.0f / p->theta, c4, mp);
    double egrav = grav_traverse(s, &t, c4, mp, (float)p->g, first, last);
    if (centersOut && cap >= t.nTot) memcpy(centersOut, c4, sizeof(double) * 4 * (size_t)t.nTot);
    if (multipolesOut && cap >= t.nTot) memcpy(multipolesOut, mp, sizeof(float) * 8 * (size_t)t.nTot);
    free(c4);
    free(mp);
    tree_free(&t);
    return egrav;
}

/* accelerationTimestep (ts_global.hpp:47-67) over [first, last) */
double ox_acc_timestep(const ox_state* s, const ox_params* p, unsigned first, unsigned last)
{
    double maxAccSq = 0.0;
    for (size_t i = first; i < last; ++i)
    {
        double ax = s->ax[i], ay = s->ay[i], az = s->az[i];
        double a2 = ax * ax + (ay * ay + az * az);
        maxAccSq  = a2 > maxAccSq ? a2 : maxAccSq;
    }
    return p->etaAcc * sqrt(p->eps / sqrt(maxAccSq));
}

/* rhoTimestep (ts_global.hpp:72-94): Krho / |max divv| over n values (float max, double quotient) */
double ox_rho_timestep(const float* divv, size_t n, double Krho)
{
    float maxDivv = -INFINITY;
#pragma omp parallel for reduction(max : maxDivv)
    for (size_t i = 0; i < n; ++i)
        maxDivv = divv[i] > maxDivv ? divv[i] : maxDivv;
    return Krho / fabs((double)maxDivv);
}

/* computeTimestep (ts_global.hpp:97-112), one rank: min of the acceleration (g != 0), Courant, rho and growth
 * limits; io[0..6] = minDt, minDt_m1, ttot, minDtCourant, minDtRho, g, maxDtIncrease, the first three updated */
void ox_compute_timestep(double* io, const float* ax, const float* ay, const float* az, size_t n, double etaAcc,
                         double eps)
{
    double minDtAcc = INFINITY;
    if (io[5] != 0.0)
    {
        double maxAccSq = 0.0;
        for (size_t i = 0; i < n; ++i)
        {
            double x = ax[i], y = ay[i], z = az[i];
            double a2 = x * x + (y * y + z * z);
            maxAccSq  = a2 > maxAccSq ? a2 : maxAccSq;
        }
        minDtAcc = etaAcc * sqrt(eps / sqrt(maxAccSq));
    }
    double minDtLoc = INFINITY;
    double cand[4]  = {minDtAcc, io[3], io[4], io[6] * io[0]};
    for (int k = 0; k < 4; ++k)
        minDtLoc = cand[k] < minDtLoc ? cand[k] : minDtLoc;
    io[2] += minDtLoc;
    io[1] = io[0];
    io[0] = minDtLoc;
}

typedef struct
{
    uint64_t key;
    uint64_t idx;
} kv_pair;

static int cmp_kv(const void* a, const void* b)
{
    uint64_t x = ((const kv_pair*)a)->key, y = ((const kv_pair*)b)->key;
    if (x != y) return (x > y) - (x < y);
    uint64_t i = ((const kv_pair*)a)->idx, j = ((const kv_pair*)b)->idx;
    return (i > j) - (i < j);
}

#define PERMUTE(field, type)                                                                                           \
    do {                                                                                                               \
        type* tmp_ = (type*)scratch;                                                                                   \
        _Pragma("omp parallel for schedule(static)") for (size_t i = 0; i < n; ++i) tmp_[i] = s->field[ord[i].idx];   \
        memcpy(s->field, tmp_, n * sizeof(type));                                                                      \
    } while (0)

/* One VE step, single rank: sync (keys, sort, reorder, tree) + computeForces + integrate
 * (ve_hydro.hpp:132-218). Returns the number of h-nc convergence failures. */
int ox_step(ox_state* s, const ox_params* p, const ox_box* b, unsigned bucket)
{
    ensure_tables();
    size_t n = s->n;
    ox_sfc_keys(s->x, s->y, s->z, n, b, s->keys);
    kv_pair* ord = (kv_pair*)malloc(sizeof(kv_pair) * n);
    for (size_t i = 0; i < n; ++i)
    {
        ord[i].key = s->keys[i];
        ord[i].idx = i;
    }
    qsort(ord, n, sizeof(kv_pair), cmp_kv);
    void* scratch = malloc(n * sizeof(double));
    for (size_t i = 0; i < n; ++i)
        s->keys[i] = ord[i].key;
    PERMUTE(x, double);
    PERMUTE(y, double);
    PERMUTE(z, double);
    PERMUTE(h, float);
    PERMUTE(m, float);
    PERMUTE(temp, double);
    PERMUTE(vx, float);
    PERMUTE(vy, float);
    PERMUTE(vz, float);
    PERMUTE(x_m1, float);
    PERMUTE(y_m1, float);
    PERMUTE(z_m1, float);
    PERMUTE(du_m1, float);
    PERMUTE(alpha, float);
    PERMUTE(id, uint64_t);
    free(scratch);
    free(ord);

    ox_tree t;
    tree_build(&t, s->keys, n, bucket, b);
    ns_view   v   = tree_view(&t);
    uint32_t* nbr = (uint32_t*)malloc(sizeof(uint32_t) * n * p->ngmax);

    size_t fails = findNeighborsSph(s->x, s->y, s->z, s->h, 0, (uint32_t)n, b, &v, p->ng0, p->ngmax, nbr, s->nc);
    if (p->prop == 1)
    {
        /* HydroProp::computeForces (std_hydro.hpp:124-166); minDtRho is never set (stays INFINITY) */
        ox_density(s, p, b, nbr, 0, (unsigned)n);
        ox_eos_std(s, p, 0, (unsigned)n);
        ox_iad_std(s, p, b, nbr, 0, (unsigned)n);
        ox_momentum_energy_std(s, p, b, nbr, 0, (unsigned)n);
        s->minDtRho = INFINITY;
    }
    else
    {
        ox_xmass(s, p, b, nbr, 0, (unsigned)n);
        ox_ve_def_gradh(s, p, b, nbr, 0, (unsigned)n);
        ox_eos(s, p, 0, (unsigned)n);
        ox_iad_divv_curlv(s, p, b, nbr, 0, (unsigned)n);
        s->minDtRho = ox_rho_timestep(s->divv, n, p->Krho);
        ox_av_switches(s, p, b, nbr, 0, (unsigned)n);
        ox_momentum_energy(s, p, b, nbr, 0, (unsigned)n);
    }
    if (p->g != 0.0)
    {
        /* mHolder_.upsweep + traverse (ve_hydro.hpp:193-202) on the same tree; accelerationTimestep below */
        double* c4 = (double*)calloc(4 * (size_t)t.nTot, sizeof(double));
        float*  mp = (float*)calloc(8 * (size_t)t.nTot, sizeof(float));
        grav_upsweep(s, &t, 1.0f / p->theta, c4, mp);
        s->egrav = grav_traverse(s, &t, c4, mp, (float)p->g, 0, (unsigned)n);
        free(c4);
        free(mp);
    }
    double io[7] = {s->minDt, s->minDt_m1, s->ttot, s->minDtCourant, s->minDtRho, p->g, p->maxDtIncrease};
    ox_compute_timestep(io, s->ax, s->ay, s->az, n, p->etaAcc, p->eps);
    s->minDt = io[0], s->minDt_m1 = io[1], s->ttot = io[2];
    ox_positions(s, p, b, 0, (unsigned)n);
    ox_update_h_range(s, p->ng0, 0, (unsigned)n);

    free(nbr);
    tree_free(&t);
    return (int)fails;
}
