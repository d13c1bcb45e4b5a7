/*! @file sx_device.hpp
 * @brief gfx950 device helpers shared by the hot-path kernels: box / periodic folding, kernel-table lookup,
 *        packed neighbor records, wave64 reductions.
 *
 * Arithmetic follows the reference expressions and promotions exactly (see oracle/sph_oracle.c for the CPU
 * restatement): e.g. the legacy applyPBC<double,float> subtracts the box length in double and rounds to float
 * (cstone/sfc/box.hpp:233-255).  Files compiled with -ffp-contract=off (the "exact" variant) reproduce the CPU
 * reference bit-for-bit given the same neighbor order; the default variant lets the compiler form FMAs.
 */
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sx
{

constexpr int kWave       = 64;    // CDNA4 wavefront
constexpr int kTableSize  = 20000; // sph::lt::kTableSize (table_lookup.hpp:12)
constexpr int kMaxLevel   = 21;    // maxTreeLevel<uint64_t>
constexpr int kGroupSize  = 64;    // particles per neighbor-list block = one wavefront
constexpr int kClusterWaves = 4;   // groups per cluster = waves per cluster workgroup
constexpr int kCluster      = kGroupSize * kClusterWaves; // particles sharing one neighbor union

//! words of u16 cluster-local neighbor positions per target (two per word)
__host__ __device__ constexpr uint32_t nlocWords(uint32_t ngmax) { return (ngmax + 1) / 2; }
//! union capacity per cluster: every union entry is a stored neighbor of at least one of its targets
__host__ __device__ constexpr uint32_t unionCap(uint32_t ngmax) { return kCluster * ngmax; }

//! the skin filter's second set of exact lists (sx_skin.hpp, round 6): per cluster c, bit kListsBSel of sel[c]
//! selects this set's nloc / uni[c*ucap + uoff] / ucount[c] instead of the primary ones (the filter keeps the last two
//! different hit sets of every cluster: a lattice's h moves between two shells).  sel == nullptr: the primary set
struct ListsB
{
    const uint8_t*  sel;
    const uint32_t* nloc;
    const uint32_t* ucount;
    uint32_t        uoff;
};
constexpr uint8_t kListsBSel = 4; //!< sel bit: the second set is current (bits 0 / 1: set A / B valid, the filter's)
__host__ __device__ inline bool listsB(const ListsB& b, uint32_t c) { return b.sel && (b.sel[c] & kListsBSel); }

//! box data as the kernels need it (cstone::Box<double>, sfc/box.hpp:111-191)
struct DevBox
{
    double lim[6];
    double l[3];  // lengths_  = max - min
    double il[3]; // inverseLengths_ = 1 / (max - min)
    int    pbc[3];
    int    fbc[3];
    int    anyPbc;
};

//! packed per-particle records gathered by neighbor index (16-byte aligned, one or two dwordx4 each)
struct __attribute__((aligned(16))) RecX
{
    double x, y, z;
    float  h, m;
};
struct __attribute__((aligned(16))) RecV
{
    float vx, vy, vz, c;
};
struct __attribute__((aligned(16))) RecT
{
    float xm, kx, prho, alpha;
};
//! std propagator (HydroProp): density and pressure of a neighbor (no xm/kx/prho/alpha there)
struct __attribute__((aligned(16))) RecS
{
    float rho, p, pad0, pad1;
};
//! IAD's outputs as a neighbor record; vol = xm / kx (the AV switches' neighbor volume, written where xm and kx are
//! known: by IAD for its targets, by the packing pass for the halos)
struct __attribute__((aligned(16))) RecC
{
    float c11, c12, c13, c22, c23, c33, divv, vol;
};

//! lt::lookup<float> (table_lookup.hpp:14-26) on a pair table {t[i], t[i+1]-t[i]}: one 8-byte gather.
//! The stored difference is the same float subtraction the reference performs, so results are identical.
__device__ __forceinline__ float lookup(const float2* __restrict__ tab, float v)
{
    constexpr int   numIntervals = kTableSize - 1;
    constexpr float dx           = 2.0f / numIntervals;
    constexpr float invDx        = 1.0f / dx;
    int             idx          = (int)(v * invDx);
    if (idx >= numIntervals) return 0.0f;
    float2 e          = tab[idx];
    float  derivative = e.y * invDx;
    return e.x + derivative * (v - (float)idx * dx);
}

//! legacy applyPBC<double,float> (box.hpp:233-255)
__device__ __forceinline__ void applyPBC(const DevBox& b, float r, float& xx, float& yy, float& zz)
{
    if (b.pbc[0] && xx > r) xx = (float)((double)xx - b.l[0]);
    else if (b.pbc[0] && xx < -r) xx = (float)((double)xx + b.l[0]);
    if (b.pbc[1] && yy > r) yy = (float)((double)yy - b.l[1]);
    else if (b.pbc[1] && yy < -r) yy = (float)((double)yy + b.l[1]);
    if (b.pbc[2] && zz > r) zz = (float)((double)zz - b.l[2]);
    else if (b.pbc[2] && zz < -r) zz = (float)((double)zz + b.l[2]);
}

constexpr uint32_t kPowTable = 1u << 16; //!< nc values covered by the host-computed powf table

/*! updateH<float> (kernels.hpp:26-32): h * 0.5 * std::pow(1 + 1023*ng0/nc, 0.1f).
 *  The reference calls glibc powf, which is not correctly rounded (0.5+ ULP on e.g. nc = 166 is reached only
 *  via 1 + 102300/nc; 112 of nc <= 2e5 differ from a correctly rounded pow).  nc is an integer and ng0 fixed per
 *  run, so the factor is tabulated on the host with glibc powf itself (powTab[nc], nc < 2^16) and the device
 *  result is bit-identical; beyond the table a double pow is used (never reached: nc <= N and the h iteration
 *  keeps nc near ng0). */
//! the beyond-the-table factor, out of line: inlined, the double pow's polynomial constants stay live across the
//! caller's loops (the neighbor search kept 16 of them in scratch)
__device__ __noinline__ float updateHFactorFar(unsigned ng0, unsigned nc)
{
    const float c0   = 1023.0f;
    const float ex   = (float)(1.0 / 10.0);
    float       base = 1.0f + c0 * ng0 / (float)nc;
    return (float)pow((double)base, (double)ex);
}

__device__ __forceinline__ float updateH(unsigned ng0, unsigned nc, float h, const float* __restrict__ powTab)
{
    const float f = nc < kPowTable ? powTab[nc] : updateHFactorFar(ng0, nc);
    return h * 0.5f * f;
}

//! tsKCourant<float> (kernels.hpp:12-18)
__device__ __forceinline__ float tsKCourant(float maxvsignal, float h, float c, float Kcour)
{
    float v = maxvsignal > 0.0f ? maxvsignal : c;
    return Kcour * h / v;
}

//! idealGasCv<float,double> (sph/eos.hpp:13-18)
__host__ __device__ __forceinline__ float idealGasCv(float mui, double gamma)
{
    const float R = 8.317e7f;
    return (float)((double)(R / mui) / (gamma - 1.0f));
}

/*! XCD-aware block remap (HIP guide 5.5 T1): workgroups are dealt round-robin to the 8 XCDs (block b -> XCD b%8),
 *  so consecutive SFC blocks would land on different L2s and every XCD would stream the whole active window.
 *  This bijection gives XCD x a contiguous range of logical blocks, processed in order, so the neighbor records a
 *  block gathers are mostly already in that XCD's 4 MB L2. Placement only affects speed, never results. */
__device__ __forceinline__ uint32_t xcdBlock(uint32_t b, uint32_t nb)
{
    const uint32_t q = nb >> 3, r = nb & 7, x = b & 7, k = b >> 3;
    return (x < r) ? x * (q + 1) + k : r * (q + 1) + (x - r) * q + k;
}

// ---- wave64 reductions (cross-lane through DPP/ds_swizzle via __shfl_xor) ----------------------------------

template<class T>
__device__ __forceinline__ T waveMin(T v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
    {
        T w = __shfl_xor(v, o, kWave);
        v   = w < v ? w : v;
    }
    return v;
}

template<class T>
__device__ __forceinline__ T waveMax(T v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
    {
        T w = __shfl_xor(v, o, kWave);
        v   = w > v ? w : v;
    }
    return v;
}

template<class T>
__device__ __forceinline__ T waveSum(T v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o, kWave);
    return v;
}

//! OR over the wave (all lanes active), wave-uniform result: DPP quad/row steps + row broadcasts, no LDS traffic
//! (quad_perm [1,0,3,2] and [2,3,0,1], row_half_mirror, row_mirror, row_bcast15 into rows 1,3, row_bcast31 into
//! rows 2,3: lane 63 ends up with the OR of all 64 lanes)
__device__ __forceinline__ uint32_t waveOrU32(uint32_t v)
{
    int x = (int)v;
    x |= __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);
    x |= __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);
    x |= __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false);
    x |= __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, false);
    x |= __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);
    x |= __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);
    return (uint32_t)__builtin_amdgcn_readlane(x, 63);
}

__device__ __forceinline__ uint64_t waveOr64(uint64_t v)
{
    return ((uint64_t)waveOrU32((uint32_t)(v >> 32)) << 32) | waveOrU32((uint32_t)v);
}

__device__ __forceinline__ double readlaneD(double v, int k)
{
    int2 p = *reinterpret_cast<int2*>(&v);
    p.x    = __builtin_amdgcn_readlane(p.x, k);
    p.y    = __builtin_amdgcn_readlane(p.y, k);
    return *reinterpret_cast<double*>(&p);
}

//! a wave-uniform double moved to scalar registers
__device__ __forceinline__ double readfirstlaneD(double v)
{
    const uint64_t u = __double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

//! uniform grid over the box (skin lists, sx_skin.hpp: per-step displacement maxima by cell of the end-of-step position)
struct DispGrid
{
    double lo[3];
    double inv[3]; // cells per unit length
    int    n;      // cells per axis
    int    pbc[3];
};

//! cell index of coordinate v on axis d: clamped on open axes, unwrapped (callers wrap) on periodic ones
__host__ __device__ inline int gridCell(double v, const DispGrid& g, int d)
{
    const double f = (v - g.lo[d]) * g.inv[d];
    int          k = (int)floor(f);
    if (g.pbc[d]) return k;
    return k < 0 ? 0 : (k >= g.n ? g.n - 1 : k);
}

__host__ __device__ inline int wrapCell(int k, int n)
{
    k %= n;
    return k < 0 ? k + n : k;
}

//! order-preserving image of a float as an unsigned integer (atomic min / max of signed floats)
__host__ __device__ inline uint32_t orderedBits(float f)
{
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ inline float orderedFloat(uint32_t o)
{
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
//! per cell the ranges of the three displacement components as ordered bits, six planes of n^3 words: min x, min y,
//! min z (initialised to 0xffffffff), max x, max y, max z (initialised to 0); an empty cell keeps min > max
constexpr int kGridWords = 6;

/*! the cell of (x, y, z) takes the displacement (dx, dy, dz) into its component ranges, for every lane with `on`;
 *  called by every lane of the wave.  SFC-ordered particles: a wave's particles share one or a few cells, so the wave
 *  takes its cells one at a time -- the ranges of the cell's lanes reduced across the wave, six atomics by one lane */
__device__ inline void gridRangeAtomic(uint32_t* cells, const DispGrid& g, double x, double y, double z, float dx,
                                       float dy, float dz, bool on)
{
    uint32_t cell = 0;
    if (on)
    {
        const double p[3] = {x, y, z};
        int          k[3];
        for (int e = 0; e < 3; ++e)
            k[e] = g.pbc[e] ? wrapCell(gridCell(p[e], g, e), g.n) : gridCell(p[e], g, e);
        cell = ((uint32_t)k[2] * g.n + (uint32_t)k[1]) * g.n + (uint32_t)k[0];
    }
    const float  d[3] = {dx, dy, dz};
    const size_t nc   = (size_t)g.n * g.n * g.n;
    const int    lane = (int)(threadIdx.x & 63);
    uint64_t     left = __ballot(on);
    while (left)
    {
        const int      l0   = __builtin_ctzll(left);
        const uint32_t c0   = __builtin_amdgcn_readlane(cell, l0);
        const bool     same = on && cell == c0;
        left &= ~__ballot(same);
#pragma unroll
        for (int e = 0; e < 3; ++e)
        {
            float lo = same ? d[e] : INFINITY, hi = same ? d[e] : -INFINITY;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1)
            {
                lo = fminf(lo, __shfl_xor(lo, o, kWave));
                hi = fmaxf(hi, __shfl_xor(hi, o, kWave));
            }
            if (lane == l0)
            {
                atomicMin(&cells[e * nc + c0], orderedBits(lo));
                atomicMax(&cells[(3 + e) * nc + c0], orderedBits(hi));
            }
        }
    }
}

//! float atomic min for non-negative values via the ordered int representation
__device__ __forceinline__ void atomicMinPos(float* addr, float v)
{
    atomicMin(reinterpret_cast<int*>(addr), __float_as_int(v));
}

} // namespace sx
