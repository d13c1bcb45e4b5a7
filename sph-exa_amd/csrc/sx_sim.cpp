/*! @file sx_sim.cpp
 * @brief Device-resident VE time step (sx_sim_*): HydroVeProp::computeForces + integrate
 *        (main/src/propagator/ve_hydro.hpp:132-218), on one GPU or SFC-decomposed over several.
 *
 * Step = sync -> neighbor search with h-nc iteration -> XMass -> [halo xm] -> VeDefGradh -> EOS
 *        -> [halo v,prho,c,kx] -> IAD+divv/curlv -> [halo c_ij,divv] -> AV switches -> [halo alpha]
 *        -> momentum/energy -> global time-step min -> positions/energy -> h update.
 *
 * sync, one GPU: Hilbert keys, radix sort, reorder of every conserved field, converged tree.
 * sync, P GPUs (replaces cstone::Domain::sync, domain.hpp:196-244, with an MI355X-first design):
 *   1. sort local particles by key;
 *   2. global key histogram (2^18 bins, allreduce) -> equal-count SFC splitters, identical on every rank
 *      (the reference's global cornerstone tree + MPI_Allreduce of counts, update_mpi_gpu.cuh:75);
 *   3. particle exchange to the SFC owner (alltoallv of 80-byte AoS records; skipped when nothing moves);
 *   4. halo discovery: each rank publishes request boxes = AABB of every 2048-particle SFC chunk grown by
 *      2*hmax(chunk)*margin; every rank marks (wave-cooperative tree traversal of its own tree) the particles
 *      inside each peer's boxes -> send lists; halos land in place, [halos of lower ranks | local | higher];
 *   5. the combined array is key-sorted by construction -> one tree over locals + halos, built from the halos' keys
 *      (sent first, 8 B each) while their coordinates, h and m are exchanged on the communication stream.
 *   After the h iteration the request margin is checked; if some particle outgrew it, discovery is redone.
 * Halo exchanges carry exactly the reference's fields (ve_hydro.hpp:150-186): x,y,z,h,m at setup, then xm,
 * then vx,vy,vz,prho,c,kx, then c11..c33,divv, then alpha.
 */
#include <hip/hip_runtime.h>

#include <cstdio>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/sphexa_hip.h"
#include "sx_comm.hpp"
#include "sx_gravity.hpp"
#include "sx_hydro.hpp"
#include "sx_observables.hpp"
#include "sx_sim.hpp"
#include "sx_skin.hpp"
#include "sx_traverse.hpp"
#include "sx_tree.hpp"

using namespace sx;
using namespace sx::sim;

extern "C" void*          sx_ctx_stream_internal(sx_ctx* c);
extern "C" int            sx_ctx_exact_internal(sx_ctx* c);
extern "C" const float2*  sx_ctx_table_internal(sx_ctx* c, int which);
extern "C" const float*   sx_ctx_powtab_internal(sx_ctx* c, uint32_t ng0);
extern "C" sx::Transport* sx_comm_transport_internal(sx_comm* c);

namespace
{

constexpr int      kHistBits   = 18;    // global key histogram resolution (level 6)
constexpr uint32_t kChunk      = 2048;  // particles per halo request box

DevBox toDevBox(const sx_box* b)
{
    DevBox d{};
    for (int k = 0; k < 6; ++k)
        d.lim[k] = b->lim[k];
    for (int k = 0; k < 3; ++k)
    {
        d.l[k]   = b->lim[2 * k + 1] - b->lim[2 * k];
        d.il[k]  = 1.0 / (b->lim[2 * k + 1] - b->lim[2 * k]);
        d.pbc[k] = b->bnd[k] == 1;
        d.fbc[k] = b->bnd[k] == 2;
        d.anyPbc |= d.pbc[k];
    }
    return d;
}

//! max |a|^2 over [first, last) for accelerationTimestep (ts_global.hpp:47-67)
__global__ void maxAccSqKernel(const float* ax, const float* ay, const float* az, size_t first, size_t last,
                               unsigned long long* out)
{
    double v = 0.0;
    for (size_t i = first + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < last; i += (size_t)gridDim.x * blockDim.x)
    {
        double x = ax[i], y = ay[i], z = az[i], q = x * x + (y * y + z * z);
        v        = q > v ? q : v;
    }
    // wave max -> block max -> one atomic per block (a per-wave atomic on one address serialises: 0.74 ms at 4M)
    __shared__ double s[4];
    v = waveMax(v);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        double m = s[0];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
            m = s[w] > m ? s[w] : m;
        atomicMax(out, (unsigned long long)__double_as_longlong(m));
    }
}

//! particle record of the SFC exchange (conserved fields of the VE propagator, ve_hydro.hpp:74)
struct __attribute__((aligned(16))) PRec
{
    double   x, y, z, temp;
    float    h, m, vx, vy, vz, xm1, ym1, zm1, dum1, alpha;
    uint64_t id;
};
static_assert(sizeof(PRec) == 80, "PRec layout");

//! halo request box: AABB grown by the search radius
struct __attribute__((aligned(16))) ReqBox
{
    double c[3], s[3];
    double hmax;
    int32_t owner, pad;
};

// ---- time step --------------------------------------------------------------------------------------------

//! rhoTimestep (ts_global.hpp:72-94) and the rank-local part of computeTimestep (:97-112)
//! useRho = 0: the std propagator, which never sets minDtRho (std_hydro.hpp:170-178: stays INFINITY)
__global__ void dtCandidateKernel(Scalars* s, double Krho, double maxDtIncrease, double g, double eps, double etaAcc,
                                  int useRho)
{
    unsigned u = s->maxDivvU;
    u          = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
    float maxDivv   = __uint_as_float(u);
    s->minDtRho     = useRho ? Krho / (double)fabsf(maxDivv) : INFINITY;
    s->minDtCourant = (double)s->courant;
    double minDtAcc = INFINITY;
    if (g != 0.0) minDtAcc = etaAcc * sqrt(eps / sqrt(__longlong_as_double((long long)s->maxAccSqBits)));
    double m       = INFINITY;
    double cand[4] = {minDtAcc, s->minDtCourant, s->minDtRho, maxDtIncrease * s->minDt};
    for (int k = 0; k < 4; ++k)
        m = cand[k] < m ? cand[k] : m;
    s->dtCand = m;
}

//! after the (MPI_Allreduce-equivalent) global min: ttot, minDt_m1, minDt
__global__ void dtApplyKernel(Scalars* s)
{
    double m = s->dtCand;
    s->ttot += m;
    s->minDt_m1 = s->minDt;
    s->minDt    = m;
}

__global__ void resetScalarsKernel(Scalars* s)
{
    s->courant      = 1e10f;
    s->maxDivvU     = 0;
    s->egrav        = 0.0;
    s->maxAccSqBits = 0;
    s->gravErr      = 0;
}

// ---- initial conditions -----------------------------------------------------------------------------------

//! Sedov lattice (grid.hpp:102-132, sedov_init.hpp:48-96); particles [lfirst, lfirst + n) of the z-major lattice
__global__ void sedovInitKernel(uint32_t side, size_t lfirst, size_t n, double* x, double* y, double* z, float* h,
                                float* m, double* temp, float* vx, float* vy, float* vz, float* xm1, float* ym1,
                                float* zm1, float* dum1, float* alpha, uint64_t* id, float hInit, float mPart,
                                double ener0, double width2, double u0, float cv)
{
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= n) return;
    size_t       li = lfirst + t;
    const double r = 0.5, step = (2. * r) / side, r_ini = -r + 0.5 * step;
    size_t       i = li / ((size_t)side * side), j = (li / side) % side, k = li % side;
    double       lz = r_ini + (i * step), ly = r_ini + (j * step), lx = r_ini + (k * step);
    x[t] = lx;
    y[t] = ly;
    z[t] = lz;
    h[t] = hInit;
    m[t] = mPart;
    double r2 = lx * lx + ly * ly + lz * lz;
    double ui = ener0 * exp(-(r2 / width2)) + u0;
    temp[t]   = ui / (double)cv;
    vx[t] = vy[t] = vz[t] = 0.f;
    xm1[t] = ym1[t] = zm1[t] = 0.f;
    dum1[t]  = 0.f;
    alpha[t] = 0.05f;
    id[t]    = li;
}

// ---- domain decomposition kernels -------------------------------------------------------------------------

__global__ void histKernel(const uint64_t* keys, size_t n, uint32_t* bins)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(&bins[keys[i] >> (63 - kHistBits)], 1u);
}

//! out[q] = first local key >= split[q] (out[0] = 0, out[P] = n: the whole range is assigned)
__global__ void lowerBoundsKernel(const uint64_t* keys, size_t n, const uint64_t* split, int P, uint64_t* out)
{
    int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q > P) return;
    uint64_t v  = split[q];
    size_t   lo = 0, hi = n;
    while (lo < hi)
    {
        size_t mid = (lo + hi) >> 1;
        if (keys[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    out[q] = q == 0 ? 0 : (q == P ? n : lo);
}

//! per peer count = difference of consecutive segment boundaries (u64 or u32), into the count-exchange buffer
__global__ void diffCountsKernel(const uint64_t* b64, const uint32_t* b32, int P, uint64_t* out)
{
    int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P) return;
    out[q] = b64 ? b64[q + 1] - b64[q] : (uint64_t)(b32[q + 1] - b32[q]);
}

__global__ void packPRecKernel(Fields f, size_t n, PRec* out)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    // ve-bdt: the rung rides in the top byte of the id slot (particle ids < 2^56)
    const uint64_t id = f.rung ? (f.id[i] | (uint64_t)f.rung[i] << 56) : f.id[i];
    out[i] = PRec{f.x[i],   f.y[i],   f.z[i],   f.temp[i], f.h[i],    f.m[i],     f.vx[i], f.vy[i],
                  f.vz[i],  f.xm1[i], f.ym1[i], f.zm1[i],  f.dum1[i], f.alpha[i], id};
}

__global__ void unpackPRecKernel(const PRec* in, size_t n, Fields f)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    PRec r    = in[i];
    f.x[i]    = r.x;
    f.y[i]    = r.y;
    f.z[i]    = r.z;
    f.temp[i] = r.temp;
    f.h[i]    = r.h;
    f.m[i]    = r.m;
    f.vx[i]   = r.vx;
    f.vy[i]   = r.vy;
    f.vz[i]   = r.vz;
    f.xm1[i]  = r.xm1;
    f.ym1[i]  = r.ym1;
    f.zm1[i]  = r.zm1;
    f.dum1[i] = r.dum1;
    f.alpha[i] = r.alpha;
    f.id[i]   = f.rung ? r.id & ((1ull << 56) - 1) : r.id;
    if (f.rung) f.rung[i] = (uint8_t)(r.id >> 56);
}

//! request box of every kChunk SFC-consecutive local particles: AABB grown by 2*hmax*margin + quantisation margin
__global__ void chunkBoxKernel(const double* x, const double* y, const double* z, const float* h, size_t n,
                               double margin, double qmargin, int owner, ReqBox* out)
{
    const size_t c0   = (size_t)blockIdx.x * kChunk;
    const size_t c1   = min(n, c0 + kChunk);
    double       lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    float        hm   = 0;
    for (size_t i = c0 + threadIdx.x; i < c1; i += blockDim.x)
    {
        lo[0] = fmin(lo[0], x[i]), hi[0] = fmax(hi[0], x[i]);
        lo[1] = fmin(lo[1], y[i]), hi[1] = fmax(hi[1], y[i]);
        lo[2] = fmin(lo[2], z[i]), hi[2] = fmax(hi[2], z[i]);
        hm    = fmaxf(hm, h[i]);
    }
    __shared__ double s[6][4];
    __shared__ float  sh[4];
    for (int k = 0; k < 3; ++k)
    {
        lo[k] = waveMin(lo[k]);
        hi[k] = waveMax(hi[k]);
    }
    hm = waveMax(hm);
    int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
    {
        for (int k = 0; k < 3; ++k)
            s[k][w] = lo[k], s[3 + k][w] = hi[k];
        sh[w] = hm;
    }
    __syncthreads();
    if (threadIdx.x == 0)
    {
        int nw = blockDim.x >> 6;
        for (int v = 1; v < nw; ++v)
            for (int k = 0; k < 3; ++k)
                s[k][0] = fmin(s[k][0], s[k][v]), s[3 + k][0] = fmax(s[3 + k][0], s[3 + k][v]), sh[0] = fmaxf(sh[0], sh[v]);
        ReqBox b;
        double R = 2.0 * (double)sh[0] * margin + qmargin;
        for (int k = 0; k < 3; ++k)
        {
            b.c[k] = 0.5 * (s[k][0] + s[3 + k][0]);
            b.s[k] = 0.5 * (s[3 + k][0] - s[k][0]) + R;
        }
        b.hmax  = sh[0];
        b.owner = owner;
        b.pad   = 0;
        out[blockIdx.x] = b;
    }
}

//! 1 if some particle of the chunk grew beyond the chunk's request radius during the h iteration
__global__ void chunkCheckKernel(const float* h, size_t n, const ReqBox* boxes, double margin, unsigned* flag)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ReqBox& b = boxes[i / kChunk];
    if ((double)h[i] > b.hmax * margin) atomicOr(flag, 1u);
}

/*! 1 if some local's search sphere (2h around its current position) leaves its chunk's request box (minimum image):
 *  the peers sent every particle inside that box, so a sphere inside it sees all of them.  Unlike chunkCheckKernel
 *  this also covers the drift of the locals inside a ve-bdt hierarchy. */
__global__ void chunkCoverKernel(const double* x, const double* y, const double* z, const float* h, size_t n,
                                 const ReqBox* boxes, DevBox box, double qmargin, unsigned* flag)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ReqBox& b = boxes[i / kChunk];
    const double  r = 2.0 * (double)h[i] * (1.0 + 1e-6) + qmargin;
    const bool    out = fabs(foldPbc(x[i] - b.c[0], box, 0)) + r > b.s[0] || fabs(foldPbc(y[i] - b.c[1], box, 1)) + r > b.s[1] ||
                     fabs(foldPbc(z[i] - b.c[2], box, 2)) + r > b.s[2];
    if (out) atomicOr(flag, 1u);
}

/*! several ranks, a reuse step: the clusters list[1 .. list[0]] were searched again this step (a skin rebuilt from the
 *  current positions, or the exact search), over the locals and the halos of the last build only.  That search saw
 *  every particle within a target's radius only if the target's sphere lies inside its chunk's request box of that
 *  build: radius 2 r_i scale, r = hb (rebuilt skins: the h of their build, scale 1 + s) or h (exact search, scale 1).
 *  One workgroup per listed cluster; flag |= 1 when some sphere leaves its box (then every rank redoes the step from
 *  a full sync) */
__global__ void coverListKernel(const uint32_t* list, uint32_t maxList, uint32_t first, uint32_t last, const double* x,
                                const double* y, const double* z, const float* r, float scale, const ReqBox* boxes,
                                DevBox box, double qmargin, unsigned* flag)
{
    const uint32_t k = blockIdx.x;
    if (k >= min(list[0], maxList)) return;
    const uint32_t i = first + list[1 + k] * kCluster + threadIdx.x;
    if (i >= last) return;
    const ReqBox& b = boxes[(i - first) / kChunk];
    const double  R = 2.0 * (double)r[i] * (double)scale * (1.0 + 1e-6) + qmargin;
    const bool    out = fabs(foldPbc(x[i] - b.c[0], box, 0)) + R > b.s[0] ||
                     fabs(foldPbc(y[i] - b.c[1], box, 1)) + R > b.s[1] || fabs(foldPbc(z[i] - b.c[2], box, 2)) + R > b.s[2];
    if (out) atomicOr(flag, 1u);
}

/*! one wave per peer request box: traverse the local tree, mark local particles inside the box (minimum image)
 *  for the box owner.  mark: one bit per rank (<= 64 ranks). */
__global__ __launch_bounds__(256) void markHalosKernel(const ReqBox* boxes, int numBoxes, const int32_t* childOffsets,
                                                       const int32_t* internalToLeaf, const uint32_t* layout,
                                                       const double* centers, const double* sizes, const double* x,
                                                       const double* y, const double* z, DevBox box, double qmargin,
                                                       unsigned long long* mark, uint32_t* err)
{
    __shared__ int s_queue[4][kQCap];
    constexpr int  kCCap = 2048; // candidate leaves per wave of the halo discovery
    __shared__ int s_cand[4][kCCap];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int bi   = blockIdx.x * 4 + wave;
    if (bi >= numBoxes) return;
    const ReqBox b = boxes[bi];
    bool         overflow;
    const int    numCand = waveCollectLeaves<kCCap>(
        childOffsets,
        [&](int node) {
            return boxDist2(centers + 3 * (size_t)node, sizes + 3 * (size_t)node, b.c[0], b.c[1], b.c[2],
                            b.s[0] + qmargin, b.s[1] + qmargin, b.s[2] + qmargin, box) <= 0.0;
        },
        s_queue[wave], s_cand[wave], lane, overflow);
    if (overflow && lane == 0) atomicOr(err, 1u);
    const unsigned long long bit = 1ull << b.owner;
    for (int c = 0; c < numCand; ++c)
    {
        const int      node = __builtin_amdgcn_readfirstlane(s_cand[wave][c]);
        const int      leaf = internalToLeaf[node];
        const uint32_t p0 = layout[leaf], p1 = layout[leaf + 1];
        for (uint32_t p = p0 + lane; p < p1; p += 64)
        {
            double d0 = fabs(foldPbc(x[p] - b.c[0], box, 0));
            double d1 = fabs(foldPbc(y[p] - b.c[1], box, 1));
            double d2 = fabs(foldPbc(z[p] - b.c[2], box, 2));
            if (d0 <= b.s[0] && d1 <= b.s[1] && d2 <= b.s[2]) atomicOr(&mark[p], bit);
        }
    }
}

//! send flags of every peer at once: segment q of (n + 1) entries holds bit q of each particle's mark (0 for q == r
//! and for the segment's closing entry), so one exclusive scan numbers the send lists of all peers in peer order
//! send flags of peers [q0, q0 + Pb): one segment of n + 1 flags per peer (the extra 0 makes the scan's last entry
//! the batch total)
__global__ void maskFlagsKernel(const unsigned long long* mark, size_t n, int q0, int Pb, int r, uint32_t* flag)
{
    const size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (k >= (size_t)Pb * (n + 1)) return;
    const size_t j = k / (n + 1), i = k - j * (n + 1);
    const int    q = q0 + (int)j;
    flag[k]        = (i < n && q != r) ? (uint32_t)((mark[i] >> q) & 1ull) : 0u;
}

__global__ void scatterIdxKernel(const uint32_t* flag, const uint32_t* scan, size_t n, int Pb, uint64_t base,
                                 uint32_t* out)
{
    const size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (k < (size_t)Pb * (n + 1) && flag[k]) out[base + scan[k]] = (uint32_t)(k % (n + 1));
}

//! start of every peer's send list in the scan (P entries) and the total (entry P)
__global__ void segStartsKernel(const uint32_t* scan, size_t n, int P, uint32_t* out)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q <= P) out[q] = scan[q < P ? (size_t)q * (n + 1) : (size_t)P * (n + 1) - 1];
}

static inline unsigned grid(size_t n, int b = 256) { return (unsigned)((n + b - 1) / b); }

// ---- multi-rank gravity helpers (distributedGravity) ----------------------------------------------------------

constexpr int kCellShift = 63 - kHistBits; // level-6 cell of a key: the global histogram bins, one owner each

//! source record of a gravity halo: coordinates, mass, smoothing length and the SFC key of the owner's last sync
//! (inside a ve-bdt hierarchy the particles drift while the key order of the sync stays the tree's order)
struct __attribute__((aligned(8))) GPart
{
    double   x, y, z;
    float    m, h;
    uint64_t key;
};

__global__ void farKeysKernel(uint64_t* keys, size_t n)
{
    size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (c < n) keys[c] = (uint64_t)c << kCellShift;
}

__global__ void cellFlagKernel(const uint64_t* keys, size_t n, uint32_t* flag)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i > n) return;
    flag[i] = (i < n && (i == 0 || (keys[i] >> kCellShift) != (keys[i - 1] >> kCellShift))) ? 1u : 0u;
}

__global__ void cellCountCheckKernel(const uint32_t* total, uint32_t expected, unsigned* err)
{
    if (*total != expected) *err = 1u;
}

//! the buffers hold nCells (+1) entries, sized from the sync's histogram; a scan that disagrees (cellCountCheckKernel
//! reports it) writes nothing out of range
__global__ void cellScatterKernel(const uint64_t* keys, const uint32_t* flag, const uint32_t* scan, size_t n,
                                  uint32_t nCells, uint32_t* cellBeg, uint32_t* cellIds)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < n && flag[i] && scan[i] < nCells)
    {
        cellBeg[scan[i]] = (uint32_t)i;
        cellIds[scan[i]] = (uint32_t)(keys[i] >> kCellShift);
    }
    if (i == n && scan[n] <= nCells) cellBeg[scan[n]] = (uint32_t)n;
}

__global__ void nearToFarKernel(const uint32_t* nearFlag, size_t n, uint32_t* farFlag, uint32_t* reqFlag)
{
    size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (k > n) return;
    const uint32_t v = k < n ? nearFlag[k] : 0u;
    if (k < n) farFlag[k] = 1u - v;
    reqFlag[k] = v;
}

__global__ void reqScatterKernel(const GCell* cells, const uint32_t* reqFlag, const uint32_t* scan, size_t n,
                                 uint32_t* reqIds)
{
    size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (k < n && reqFlag[k]) reqIds[scan[k]] = cells[k].cell;
}

//! v[q] = scan[off[q]] for the P+1 segment boundaries
__global__ void segmentAtKernel(const uint32_t* scan, const uint64_t* off, int P, uint32_t* out)
{
    int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q <= P) out[q] = scan[off[q]];
}

//! owner side: requested cell -> particle range of the local cell (binary search over the sorted local cell ids)
__global__ void reqLookupKernel(const uint32_t* req, size_t nReq, const uint32_t* cellIds, const uint32_t* cellBeg,
                                int nCells, uint32_t* size, uint32_t* beg)
{
    size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (k > nReq) return;
    if (k == nReq)
    {
        size[k] = 0;
        return;
    }
    const uint32_t id = req[k];
    int            lo = 0, hi = nCells;
    while (lo < hi)
    {
        int mid = (lo + hi) >> 1;
        if (cellIds[mid] < id) lo = mid + 1;
        else hi = mid;
    }
    const bool found = lo < nCells && cellIds[lo] == id;
    beg[k]           = found ? cellBeg[lo] : 0u;
    size[k]          = found ? cellBeg[lo + 1] - cellBeg[lo] : 0u;
}

//! one wave per request: the cell's particles into the send buffer at its scanned offset
__global__ void gatherCellsKernel(const uint32_t* beg, const uint32_t* size, const uint32_t* off, size_t nReq,
                                  const double* x, const double* y, const double* z, const float* m, const float* h,
                                  const uint64_t* keys, GPart* out)
{
    const size_t k    = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    const int    lane = threadIdx.x & 63;
    if (k >= nReq) return;
    const uint32_t b = beg[k], c = size[k], o = off[k];
    for (uint32_t t = lane; t < c; t += 64)
    {
        const uint32_t i = b + t;
        out[o + t]       = GPart{x[i], y[i], z[i], m[i], h[i], keys[i]};
    }
}

__global__ void unpackGPartKernel(const GPart* in, size_t n, double* x, double* y, double* z, float* m, float* h,
                                  uint64_t* keys)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const GPart p = in[i];
    x[i] = p.x, y[i] = p.y, z[i] = p.z, m[i] = p.m, h[i] = p.h, keys[i] = p.key;
}

} // namespace

namespace sx::sim
{

void allocFields(sx_sim* s, size_t cap)
{
    auto& a  = s->mem;
    s->x     = a.get<double>("x", cap);
    s->y     = a.get<double>("y", cap);
    s->z     = a.get<double>("z", cap);
    s->temp  = a.get<double>("temp", cap);
    s->h     = a.get<float>("h", cap);
    s->m     = a.get<float>("m", cap);
    s->vx    = a.get<float>("vx", cap);
    s->vy    = a.get<float>("vy", cap);
    s->vz    = a.get<float>("vz", cap);
    s->xm1   = a.get<float>("x_m1", cap);
    s->ym1   = a.get<float>("y_m1", cap);
    s->zm1   = a.get<float>("z_m1", cap);
    s->dum1  = a.get<float>("du_m1", cap);
    s->alpha = a.get<float>("alpha", cap);
    s->id    = a.get<uint64_t>("id", cap);
    s->keys  = a.get<uint64_t>("keys", cap);
    s->order = a.get<uint32_t>("order", cap);
    s->nc    = a.get<uint32_t>("nc", cap);
    s->xm    = a.get<float>("xm", cap);
    s->kx    = a.get<float>("kx", cap);
    s->gradh = a.get<float>("gradh", cap);
    s->prho  = a.get<float>("prho", cap);
    s->c     = a.get<float>("c", cap);
    s->divv  = a.get<float>("divv", cap);
    s->curlv = a.get<float>("curlv", cap);
    s->c11   = a.get<float>("c11", cap);
    s->c12   = a.get<float>("c12", cap);
    s->c13   = a.get<float>("c13", cap);
    s->c22   = a.get<float>("c22", cap);
    s->c23   = a.get<float>("c23", cap);
    s->c33   = a.get<float>("c33", cap);
    s->ax    = a.get<float>("ax", cap);
    s->ay    = a.get<float>("ay", cap);
    s->az    = a.get<float>("az", cap);
    s->du    = a.get<double>("du", cap);
    if (s->p.avClean)
    {
        // GradVFields, allocated only with avClean (ve_hydro.hpp:80-85)
        s->dV[0] = a.get<float>("dV11", cap);
        s->dV[1] = a.get<float>("dV12", cap);
        s->dV[2] = a.get<float>("dV13", cap);
        s->dV[3] = a.get<float>("dV22", cap);
        s->dV[4] = a.get<float>("dV23", cap);
        s->dV[5] = a.get<float>("dV33", cap);
    }
    if (s->p.propagator == 1)
    {
        s->rho  = a.get<float>("rho", cap);
        s->pres = a.get<float>("p", cap);
    }
    s->rx    = a.get<RecX>("rx", cap);
    s->rv    = a.get<RecV>("rv", cap);
    s->rt    = a.get<RecT>("rt", cap);
    s->rs    = reinterpret_cast<RecS*>(s->rt);
    s->rc    = a.get<RecC>("rc", cap);
    auto spare = [&](auto*& field, const char* tag) {
        using T = std::remove_reference_t<decltype(*field)>;
        s->spares.push_back(
            {reinterpret_cast<void**>(&field), a.get<T>(std::string(tag) + ".alt", cap), (int)sizeof(T)});
    };
    spare(s->x, "x");
    spare(s->y, "y");
    spare(s->z, "z");
    spare(s->h, "h");
    spare(s->m, "m");
    spare(s->temp, "temp");
    spare(s->vx, "vx");
    spare(s->vy, "vy");
    spare(s->vz, "vz");
    spare(s->xm1, "x_m1");
    spare(s->ym1, "y_m1");
    spare(s->zm1, "z_m1");
    spare(s->dum1, "du_m1");
    spare(s->alpha, "alpha");
    spare(s->id, "id");
    if (s->p.propagator == 2)
    {
        s->rung = a.get<uint8_t>("rung", cap);
        spare(s->rung, "rung");
    }
    s->nb.reserve(a, 0, (uint32_t)cap, s->p.ngmax, true);
    s->stats      = a.get<uint32_t>("stats", kStatsWords);
    s->statsHost  = a.pinned<uint32_t>("statsHost", kStatsWords);
    s->clsHost    = a.pinned<uint32_t>("ovl.countHost", 2);
    if (s->statsHost) std::fill(s->statsHost, s->statsHost + kStatsWords, 0u);
    s->sc         = a.get<Scalars>("scalars", 1);
    s->scHost     = a.pinned<Scalars>("scalarsHost", 1);
}

PairArgs simPairArgs(sx_sim* s)
{
    PairArgs a{};
    a.lb             = s->skin.lb; // the step's second set of lists (skin filter), or none
    a.first          = (uint32_t)s->first;
    a.last           = (uint32_t)s->last;
    a.numGroups      = (uint32_t)((s->last - s->first + kGroupSize - 1) / kGroupSize);
    a.ngmax          = s->p.ngmax;
    a.localLists     = s->nb.local;
    a.nidx           = s->nb.nidx;
    a.nloc           = s->nb.nloc;
    a.uni            = s->nb.uni;
    a.ucount         = s->nb.ucount;
    a.ucap           = s->nb.ucap;
    a.nc             = s->nc;
    a.rx             = s->rx;
    a.rv             = s->rv;
    a.rt             = s->rt;
    a.rc             = s->rc;
    a.wh             = sx_ctx_table_internal(s->ctx, 0);
    a.whd            = sx_ctx_table_internal(s->ctx, 1);
    a.box            = s->dbox;
    a.K              = s->p.K;
    a.xm             = s->xm;
    a.kx             = s->kx;
    a.gradh          = s->gradh;
    a.c11            = s->c11;
    a.c12            = s->c12;
    a.c13            = s->c13;
    a.c22            = s->c22;
    a.c23            = s->c23;
    a.c33            = s->c33;
    a.divv           = s->divv;
    a.curlv          = s->curlv;
    a.alpha          = s->alpha;
    a.ax             = s->ax;
    a.ay             = s->ay;
    a.az             = s->az;
    a.du             = s->du;
    a.minDt          = &s->sc->courant;
    a.blockDt        = s->mem.get<float>("pair.blockdt", std::max<size_t>(1, (s->last - s->first + kCluster - 1) / kCluster));
    a.alphamin       = s->p.alphamin;
    a.alphamax       = s->p.alphamax;
    a.decay_constant = s->p.decay_constant;
    a.dtPtr          = &s->sc->minDt;
    a.Atmin          = s->p.Atmin;
    a.Atmax          = s->p.Atmax;
    a.ramp           = s->p.ramp;
    a.Kcour          = (float)s->p.Kcour;
    a.dV11 = s->dV[0], a.dV12 = s->dV[1], a.dV13 = s->dV[2], a.dV22 = s->dV[3], a.dV23 = s->dV[4], a.dV33 = s->dV[5];
    a.rs   = s->rs;
    a.avClean = s->p.avClean ? 1 : 0;
    return a;
}

double quantMargin(const DevBox& b)
{
    return 4.0 * std::max(b.l[0], std::max(b.l[1], b.l[2])) / double(1u << kMaxLevel);
}

#define SIM_HIP(call)                                                                                                  \
    do {                                                                                                               \
        if ((call) != hipSuccess) return SX_ERR_HIP;                                                                   \
    } while (0)
#define SIM_COMM(call)                                                                                                 \
    do {                                                                                                               \
        if (!(call)) return SX_ERR_HIP;                                                                                \
    } while (0)

//! sort the local particles [0,nl) of the primary arrays by key (keys[0..nl) computed) via the spare buffers
/*! SFC order of the locals, identical to the reference's stable sort of the full keys (Domain::sync):
 *  - keys already ascending (no descent): the stable sort is the identity, nothing moves;
 *  - else a stable radix sort of the top sortBits key bits, accepted when the result is ascending in the full keys
 *    (then keys equal in the sorted bits kept their input order AND that order is ascending in the lower bits, which
 *    is what the full stable sort gives); otherwise the full sort, and more bits from the next step on.
 *  Lattice-like states separate every particle within the top 10 levels (30 bits), so 4 of the 8 radix passes.
 *  Up to 32 bits the sort moves 32-bit keys (the top bits, extracted by the descent count) and an implicit identity
 *  permutation: 8 instead of 12 bytes per element and pass; the full keys are then reordered with the other fields
 *  (only the moved positions), instead of being copied back from the sort's output. */
int sortLocals(sx_sim* s, size_t nl, hipStream_t st)
{
    uint32_t* cnt  = s->work.get<uint32_t>("sort.desc", 2);
    uint32_t* cntH = s->work.pinned<uint32_t>("sort.desch", 2);
    auto      read = [&]() -> int {
        SIM_HIP(hipMemcpyAsync(cntH, cnt, 8, hipMemcpyDeviceToHost, st));
        SIM_HIP(hipStreamSynchronize(st));
        return SX_OK;
    };
    const int bits = std::clamp(s->sortBits, 1, 63);
    uint32_t* top  = bits <= 32 ? s->work.get<uint32_t>("sort.top", nl) : nullptr;
    SIM_HIP(hipMemsetAsync(cnt, 0, 8, st));
    if (top) SIM_HIP(countDescentsTop(s->keys, nl, 63 - bits, top, cnt, st));
    else SIM_HIP(countDescents(s->keys, nl, cnt, st));
    if (int e = read()) return e;
    s->sortStats[0]++;
    if (cntH[0] == 0) return SX_OK;
    hipError_t he          = hipSuccess;
    bool       permuteKeys = false; // the order is final and the keys are reordered with the fields
    uint32_t   moved       = 0;
    if (top)
    {
        SIM_HIP(sortTopBits(s->work, top, s->order, nl, bits, st));
        SIM_HIP(hipMemsetAsync(cnt, 0, 8, st));
        SIM_HIP(checkSorted(s->keys, s->order, nl, cnt, st));
        if (int e = read()) return e;
        permuteKeys = cntH[0] == 0;
        moved       = cntH[1];
    }
    if (!permuteKeys)
    {
        uint64_t* kOut = nullptr;
        if (!top && bits < 63)
        {
            kOut = sortKeysBits(s->work, s->keys, s->order, nl, 63 - bits, st, he);
            SIM_HIP(he);
            SIM_HIP(hipMemsetAsync(cnt, 0, 8, st));
            SIM_HIP(countDescents(kOut, nl, cnt, st));
            if (int e = read()) return e;
            if (cntH[0]) kOut = nullptr;
        }
        if (!kOut)
        {
            kOut = sortKeysBits(s->work, s->keys, s->order, nl, 0, st, he);
            SIM_HIP(he);
            if (bits < 63)
            {
                s->sortBits = std::min(63, bits + 9);
                s->sortStats[2]++;
            }
        }
        SIM_HIP(hipMemcpyAsync(s->keys, kOut, nl * sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
        SIM_HIP(hipMemsetAsync(cnt, 0, 8, st));
        SIM_HIP(movedCount(s->order, nl, cnt, st));
        if (int e = read()) return e;
        moved = cntH[0];
    }
    s->sortStats[1]++;
    // a nearly stationary state moves few positions per step (Sedov 64M: ~10 %): then only those are rewritten, in
    // place (read into a scratch copy, then written back), instead of gathering every field into its spare buffer
    if (moved <= nl / 4)
    {
        size_t colBytes = permuteKeys ? ((size_t)nl * sizeof(uint64_t) + 255) & ~size_t(255) : 0;
        for (auto& sp : s->spares)
            colBytes += ((size_t)nl * sp.elemBytes + 255) & ~size_t(255);
        char*     tmp = s->work.get<char>("sort.movedtmp", colBytes);
        GatherSet set{};
        auto      add = [&](void* field, int bytes) -> int {
            if (set.count == kMaxGatherFields)
            {
                SIM_HIP(permuteMoved(s->order, nl, set, tmp, st));
                set.count = 0;
            }
            set.src[set.count] = field, set.dst[set.count] = field, set.bytes[set.count] = bytes;
            ++set.count;
            return SX_OK;
        };
        if (permuteKeys)
            if (int e = add(s->keys, sizeof(uint64_t))) return e;
        for (auto& sp : s->spares)
            if (int e = add(*sp.field, sp.elemBytes)) return e;
        SIM_HIP(permuteMoved(s->order, nl, set, tmp, st));
        s->sortStats[3]++;
        return SX_OK;
    }
    GatherSet set{};
    auto      add = [&](const void* src, void* dst, int bytes) -> int {
        if (set.count == kMaxGatherFields)
        {
            SIM_HIP(gatherMany(s->order, nl, set, st));
            set.count = 0;
        }
        set.src[set.count] = src, set.dst[set.count] = dst, set.bytes[set.count] = bytes;
        ++set.count;
        return SX_OK;
    };
    uint64_t* kOut = permuteKeys ? s->work.get<uint64_t>("sort.kout", nl) : nullptr;
    if (kOut)
        if (int e = add(s->keys, kOut, sizeof(uint64_t))) return e;
    for (auto& sp : s->spares)
    {
        if (int e = add(*sp.field, sp.alt, sp.elemBytes)) return e;
        std::swap(*sp.field, sp.alt);
    }
    SIM_HIP(gatherMany(s->order, nl, set, st));
    if (kOut) SIM_HIP(hipMemcpyAsync(s->keys, kOut, nl * sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
    return SX_OK;
}

//! interior / boundary clusters: a cluster is interior when no entry of its neighbor union is a halo (outside
//! [first, last)).  One wave per cluster; the lists are compacted with one atomic per cluster (order is free: every
//! cluster is computed independently)
__global__ void classifyClustersKernel(const uint32_t* uni, const uint32_t* ucount, uint32_t ucap, ListsB lb,
                                       uint32_t first, uint32_t last, uint32_t numClusters, uint32_t* lists,
                                       uint32_t* counts)
{
    const uint32_t c    = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    if (c >= numClusters) return;
    // an overflowed union (ucount > ucap, stats bit 8, reported as an error after the step) is only partly stored:
    // read what is there and treat the cluster as boundary
    const bool      lB = listsB(lb, c);
    const uint32_t  uc = lB ? lb.ucount[c] : ucount[c];
    const uint32_t  U  = min(uc, ucap);
    const uint32_t* u  = uni + (size_t)c * ucap + (lB ? lb.uoff : 0u);
    bool            halo = uc > ucap;
    for (uint32_t k = lane; k < U; k += 64)
    {
        const uint32_t j = u[k];
        halo |= j < first || j >= last;
    }
    const bool any = __ballot(halo) != 0ull;
    if (lane == 0)
    {
        const uint32_t pos = atomicAdd(&counts[any ? 1 : 0], 1u);
        lists[(any ? numClusters : 0u) + pos] = c;
    }
}

//! RecX of the halos [0, first) and [last, n): the search wrote the locals' records (NsArgs::rxOut)
void packXHalos(sx_sim* s, hipStream_t st)
{
    if (s->first) packX(s->first, s->x, s->y, s->z, s->h, s->m, s->rx, st);
    if (s->n > s->last)
        packX(s->n - s->last, s->x + s->last, s->y + s->last, s->z + s->last, s->h + s->last, s->m + s->last,
              s->rx + s->last, st);
}

//! exchange one set of fields for the halos of this step (send lists built by discoverHalos)
int haloExchange(sx_sim* s, std::initializer_list<std::pair<void*, int>> fields, hipStream_t st)
{
    if (!s->comm || s->comm->size() == 1) return SX_OK;
    const int P = s->comm->size();
    for (auto [ptr, es] : fields)
    {
        char* f   = static_cast<char*>(ptr);
        char* buf = s->work.get<char>("halo.send", std::max<uint64_t>(1, s->numSend) * 8);
        if (s->numSend) SIM_HIP(gather(s->sendIdx, s->numSend, f + s->first * es, buf, es, st));
        std::vector<uint64_t> sb(P), so(P), rb(P), ro(P);
        for (int q = 0; q < P; ++q)
        {
            sb[q] = s->haloSend[q] * es;
            so[q] = s->haloSendOff[q] * es;
            rb[q] = s->haloRecv[q] * es;
            ro[q] = s->haloRecvOff[q] * es;
        }
        SIM_COMM(s->comm->alltoallv(buf, sb.data(), so.data(), f, rb.data(), ro.data(), st));
    }
    return SX_OK;
}

//! whether this step's exchanges overlap with interior clusters (several ranks, cluster lists, not disabled)
bool overlapping(const sx_sim* s, const HydroLaunch& H)
{
    return s->comm && s->comm->size() > 1 && s->overlap && s->nb.local && s->commStream && H.clusterLists;
}

/*! halo exchange of `fields` followed by the pair kernel `launch`, which needs the exchanged halo values.  Without
 *  overlap: exchange, pack(0, n), launch over all clusters.  With overlap: the exchange runs on commStream after the
 *  producer's kernels (event); meanwhile the compute stream packs the locals' records and runs the interior
 *  clusters; then it waits for the exchange, packs the halos' records and runs the boundary clusters.  Every cluster
 *  is computed exactly as in the serial order, so results are bitwise identical. */
template<class Pack, class Launch>
int exchangeThen(sx_sim* s, const HydroLaunch& H, std::initializer_list<std::pair<void*, int>> fields, Pack&& pack,
                 Launch&& launch, PairArgs pa, hipStream_t st)
{
    if (!overlapping(s, H))
    {
        if (int e = haloExchange(s, fields, st)) return e;
        pack(size_t(0), s->n);
        launch(pa);
        return SX_OK;
    }
    SIM_HIP(hipEventRecord(s->evProd, st));
    SIM_HIP(hipStreamWaitEvent(s->commStream, s->evProd, 0));
    if (int e = haloExchange(s, fields, s->commStream)) return e;
    SIM_HIP(hipEventRecord(s->evComm, s->commStream));
    pack(s->first, s->last);
    const uint32_t nc = (uint32_t)((s->last - s->first + kCluster - 1) / kCluster);
    pa.clusterList    = s->clsList;
    pa.listCount      = s->nInterior;
    launch(pa);
    SIM_HIP(hipStreamWaitEvent(st, s->evComm, 0));
    pack(size_t(0), s->first);
    pack(s->last, s->n);
    pa.clusterList = s->clsList + nc;
    pa.listCount   = s->nBoundary;
    launch(pa);
    return SX_OK;
}

/*! distributed sync: SFC assignment, particle exchange, halo discovery + setup exchange, combined tree.
 *  On entry the local particles are [first,last); on exit [first,last) again with halos around them. */
int anyRank(sx_sim* s, bool bad, hipStream_t st, bool& out);

//! a count exchange that doubles as a collective abort: a rank that cannot go on (capacity, scratch) sends
//! kAbortCount to every peer, so all ranks leave the sync at the same exchange (SX_ERR_NOMEM) instead of the others
//! waiting in the next collective; no extra host round trip
constexpr uint64_t kAbortCount = ~0ull;
int countsOrAbort(sx_sim* s, std::vector<uint64_t>& send, std::vector<uint64_t>& recv, bool fail, hipStream_t st)
{
    if (fail) send.assign(send.size(), kAbortCount);
    SIM_COMM(s->comm->exchangeCounts(send, recv, st, s->cntBuf));
    bool abort = fail;
    for (uint64_t c : recv)
        abort |= c == kAbortCount;
    return abort ? SX_ERR_NOMEM : SX_OK;
}

//! the same exchange for counts the device computed (cntBuf[0, P), e.g. diffCountsKernel): sent as they are (or the
//! abort marker), and the sent and received counts read back in one synchronisation; sendOff = prefix sums of send
int deviceCountsOrAbort(sx_sim* s, bool fail, hipStream_t st, std::vector<uint64_t>& send,
                        std::vector<uint64_t>& sendOff, std::vector<uint64_t>& recv)
{
    const int P = s->comm->size();
    uint64_t* h = s->work.pinned<uint64_t>("dom.cnth", 2 * (size_t)P);
    if (!h || !s->cntBuf) return SX_ERR_NOMEM;
    if (fail)
    {
        for (int q = 0; q < P; ++q)
            h[q] = kAbortCount;
        SIM_HIP(hipMemcpyAsync(s->cntBuf, h, 8 * (size_t)P, hipMemcpyHostToDevice, st));
    }
    std::vector<uint64_t> bytes(P, 8), off(P);
    for (int q = 0; q < P; ++q)
        off[q] = 8 * (uint64_t)q;
    SIM_COMM(s->comm->alltoallv(s->cntBuf, bytes.data(), off.data(), s->cntBuf + P, bytes.data(), off.data(), st));
    SIM_HIP(hipMemcpyAsync(h, s->cntBuf, 16 * (size_t)P, hipMemcpyDeviceToHost, st));
    SIM_HIP(hipStreamSynchronize(st));
    send.assign(h, h + P);
    recv.assign(h + P, h + 2 * P);
    sendOff.assign(P + 1, 0);
    bool abort = fail;
    for (int q = 0; q < P; ++q)
    {
        abort |= recv[q] == kAbortCount;
        sendOff[q + 1] = sendOff[q] + (fail ? 0 : send[q]);
    }
    return abort ? SX_ERR_NOMEM : SX_OK;
}

int distributedSync(sx_sim* s, hipStream_t st, double margin)
{
    sx::Transport* T  = s->comm;
    const int      P  = T->size(), r = T->rank();
    size_t         nl = s->last - s->first;
    const double   qm = quantMargin(s->dbox);

    // --- 1. local keys + sort (compacts locals to [0, nl))
    SIM_HIP(launchSfcKeys(s->x + s->first, s->y + s->first, s->z + s->first, s->keys, nl, s->dbox, st));
    if (s->first != 0)
    {
        for (auto& sp : s->spares)
        {
            SIM_HIP(hipMemcpyAsync(sp.alt, static_cast<char*>(*sp.field) + s->first * sp.elemBytes, nl * sp.elemBytes,
                                   hipMemcpyDeviceToDevice, st));
            std::swap(*sp.field, sp.alt);
        }
    }
    if (int e = sortLocals(s, nl, st)) return e;

    // --- 2. global histogram -> splitters (the small per-rank buffers of the sync were allocated by sx_sim_set_comm,
    //        so nothing here fails on one rank alone between two collectives)
    const size_t nb   = size_t(1) << kHistBits;
    uint32_t*    bins = s->work.get<uint32_t>("dom.bins", nb);
    if (!bins) return SX_ERR_NOMEM; // allocated by set_comm: cannot fail here
    SIM_HIP(hipMemsetAsync(bins, 0, nb * 4, st));
    if (nl) histKernel<<<grid(nl), 256, 0, st>>>(s->keys, nl, bins);
    SIM_COMM(T->allreduceSumU32(bins, nb, st));
    std::vector<uint32_t> hb(nb);
    SIM_HIP(hipMemcpyAsync(hb.data(), bins, nb * 4, hipMemcpyDeviceToHost, st));
    SIM_HIP(hipStreamSynchronize(st));
    std::vector<uint64_t> split(P + 1, 0);
    if (int e = sx_domain_splitters(hb.data(), kHistBits, P, split.data())) return e;
    // every rank's particle count after the exchange: the histogram bins of its range (splitters are bin
    // boundaries), so the request-box counts of step 4 need no exchange
    std::vector<uint64_t> nlOf(P, 0);
    s->cellsOf.assign(P, 0);
    for (int q = 0; q < P; ++q)
        for (uint64_t b = split[q] >> (63 - kHistBits); b < (split[q + 1] >> (63 - kHistBits)) && b < nb; ++b)
        {
            nlOf[q] += hb[b];
            s->cellsOf[q] += hb[b] != 0;
        }

    // --- 3. particle exchange
    uint64_t* dsplit = s->work.get<uint64_t>("dom.split", P + 1);
    uint64_t* dseg   = s->work.get<uint64_t>("dom.seg", P + 1);
    s->cntBuf = s->work.get<uint64_t>("dom.cnt", 2 * P);
    if (!dsplit || !dseg || !s->cntBuf) return SX_ERR_NOMEM; // allocated by set_comm: cannot fail here
    // the send counts stay on the device: segments of the sorted keys -> counts -> the count exchange, read back
    // together with the receive counts (one synchronisation)
    SIM_HIP(hipMemcpyAsync(dsplit, split.data(), 8 * (P + 1), hipMemcpyHostToDevice, st));
    lowerBoundsKernel<<<grid(P + 1, 64), 64, 0, st>>>(s->keys, nl, dsplit, P, dseg);
    diffCountsKernel<<<grid(P, 64), 64, 0, st>>>(dseg, nullptr, P, s->cntBuf);
    std::vector<uint64_t> sendCnt, seg, recvCnt;
    // the new local count is this rank's histogram bins (nlOf[r], the sum of the receive counts); the exchange
    // buffers are sized by it before the count exchange, so a failure is decided there on every rank
    PRec* sbuf = nullptr;
    PRec* rbuf = nullptr;
    bool  noRoom = nlOf[r] > s->cap;
    if (!noRoom)
    {
        sbuf   = s->work.get<PRec>("dom.psend", nl);
        rbuf   = s->work.get<PRec>("dom.precv", nlOf[r]);
        noRoom = !sbuf || !rbuf;
    }
    if (int e = deviceCountsOrAbort(s, noRoom, st, sendCnt, seg, recvCnt)) return e;
    bool moved = false;
    for (int q = 0; q < P; ++q)
        moved |= (q != r) && (sendCnt[q] || recvCnt[q]);
    // a local count that disagrees with the histogram cannot happen (the splitters are bin boundaries of the histogram
    // of these same keys); should it, this rank still takes part in every collective up to the halo count exchange,
    // sized by the histogram as its peers expect, and aborts all ranks there together (countsOrAbort)
    bool broken = false;
    if (moved)
    {
        uint64_t nNew = 0;
        for (int q = 0; q < P; ++q)
            nNew += recvCnt[q];
        broken = nNew != nlOf[r];
        if (broken) rbuf = s->work.get<PRec>("dom.precv", nNew); // the peers send nNew records
        if (nl) packPRecKernel<<<grid(nl), 256, 0, st>>>(s->fields(), nl, sbuf);
        std::vector<uint64_t> sb(P), so(P), rb(P), ro(P);
        uint64_t              acc = 0;
        for (int q = 0; q < P; ++q)
        {
            sb[q] = sendCnt[q] * sizeof(PRec);
            so[q] = seg[q] * sizeof(PRec);
            rb[q] = recvCnt[q] * sizeof(PRec);
            ro[q] = acc * sizeof(PRec);
            acc += recvCnt[q];
        }
        if (!rbuf) // only on the broken path: receive nothing (the peers abort with this rank below)
            for (int q = 0; q < P; ++q)
                rb[q] = 0;
        SIM_COMM(T->alltoallv(sbuf, sb.data(), so.data(), rbuf, rb.data(), ro.data(), st));
        if (!broken)
        {
            nl = nNew;
            if (nl) unpackPRecKernel<<<grid(nl), 256, 0, st>>>(rbuf, nl, s->fields());
            SIM_HIP(launchSfcKeys(s->x, s->y, s->z, s->keys, nl, s->dbox, st));
            if (int e = sortLocals(s, nl, st)) return e;
        }
    }

    // --- 4. halo discovery: request boxes, exchange, mark, send lists
    // the exchange delivers exactly this rank's bins (the peers size their box receives from nlOf): the splitters
    // are bin boundaries of the histogram of these same keys, so this holds on every rank by construction; a rank
    // where it does not (`broken`) sends boxes of the size its peers expect and aborts them at the count exchange below
    broken |= nl != nlOf[r];
    if (broken) nl = std::min<size_t>(nl, nlOf[r]);
    const size_t nChunks = (nlOf[r] + kChunk - 1) / kChunk;
    ReqBox*      myBoxes = s->work.get<ReqBox>("dom.mybox", nChunks);
    if (!myBoxes) return SX_ERR_NOMEM;
    if (broken) SIM_HIP(hipMemsetAsync(myBoxes, 0, nChunks * sizeof(ReqBox), st));
    else if (nChunks)
        chunkBoxKernel<<<(unsigned)nChunks, 256, 0, st>>>(s->x, s->y, s->z, s->h, nl, margin, qm, r, myBoxes);
    std::vector<uint64_t> boxCnt(P, nChunks), boxRecv(P);
    boxCnt[r] = 0;
    for (int q = 0; q < P; ++q)
        boxRecv[q] = q == r ? 0 : (nlOf[q] + kChunk - 1) / kChunk;
    uint64_t nRemote = 0;
    for (int q = 0; q < P; ++q)
        nRemote += boxRecv[q];
    ReqBox* remote = s->work.get<ReqBox>("dom.rbox", nRemote);
    {
        std::vector<uint64_t> sb(P), so(P, 0), rb(P), ro(P);
        uint64_t              acc = 0;
        for (int q = 0; q < P; ++q)
        {
            sb[q] = boxCnt[q] * sizeof(ReqBox);
            rb[q] = boxRecv[q] * sizeof(ReqBox);
            ro[q] = acc * sizeof(ReqBox);
            acc += boxRecv[q];
        }
        SIM_COMM(T->alltoallv(myBoxes, sb.data(), so.data(), remote, rb.data(), ro.data(), st));
    }
    SIM_HIP(buildTree(s->work, s->keys, nl, s->bucket, s->dbox, s->localTree, st));
    auto* mark = s->work.get<unsigned long long>("dom.mark", nl);
    auto* err  = s->work.get<uint32_t>("dom.err", 1);
    SIM_HIP(hipMemsetAsync(mark, 0, nl * 8, st));
    SIM_HIP(hipMemsetAsync(err, 0, 4, st));
    if (nRemote && nl)
        markHalosKernel<<<grid(nRemote, 4), 256, 0, st>>>(
            remote, (int)nRemote, s->localTree.childOffsets, s->localTree.internalToLeaf, s->localTree.layout,
            s->localTree.centers, s->localTree.sizes, s->x, s->y, s->z, s->dbox, qm, mark, err);
    // send lists of the peers from one flag array and one scan per batch of peers (peer order), one host read of the
    // batch's offsets; a batch holds as many peers as keep its flags within kFlagCap entries (and the scan's int
    // count), so the scratch does not grow with the rank count
    constexpr size_t kFlagCap = size_t(1) << 27;
    const int        Pb       = (int)std::max<size_t>(1, std::min<size_t>(P, kFlagCap / (nl + 1)));
    const size_t     nf       = (size_t)Pb * (nl + 1);
    // scratch failures are not returned here (the peers would wait in the count exchange below): they skip the
    // send-list work and abort every rank at that exchange (countsOrAbort)
    bool      fail = broken || nf > (size_t)INT32_MAX; // one peer's segment alone beyond the scan's range
    uint32_t* flag = fail ? nullptr : s->work.get<uint32_t>("dom.flag", nf);
    uint32_t* scan = fail ? nullptr : s->work.get<uint32_t>("dom.scan", nf);
    uint32_t* segs = s->work.get<uint32_t>("dom.segs", Pb + 1);
    uint32_t* hseg = s->work.pinned<uint32_t>("dom.hseg", Pb + 1);
    fail |= !flag || !scan || !segs || !hseg;
    s->haloSend.assign(P, 0);
    s->haloSendOff.assign(P, 0);
    size_t tmpB = 0;
    void*  tmp  = nullptr;
    if (!fail)
    {
        hipcub::DeviceScan::ExclusiveSum(nullptr, tmpB, flag, scan, (int)nf, st);
        tmp  = s->work.get<char>("dom.scantmp", tmpB);
        fail = !tmp;
    }
    // flags + scan of one batch; with scatter, the batch's send indices go to sendIdx[base, ...)
    auto batch = [&](int q0, int nb, bool scatter, uint64_t base) -> int
    {
        const size_t nfb = (size_t)nb * (nl + 1);
        maskFlagsKernel<<<grid(nfb), 256, 0, st>>>(mark, nl, q0, nb, r, flag);
        SIM_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmpB, flag, scan, (int)nfb, st));
        if (scatter) scatterIdxKernel<<<grid(nfb), 256, 0, st>>>(flag, scan, nl, nb, base, s->sendIdx);
        segStartsKernel<<<grid(nb + 1, 64), 64, 0, st>>>(scan, nl, nb, segs);
        SIM_HIP(hipMemcpyAsync(hseg, segs, 4 * (nb + 1), hipMemcpyDeviceToHost, st));
        SIM_HIP(hipStreamSynchronize(st));
        for (int j = 0; j < nb; ++j)
        {
            s->haloSendOff[q0 + j] = base + hseg[j];
            s->haloSend[q0 + j]    = (j < nb - 1 ? hseg[j + 1] : hseg[nb]) - hseg[j];
        }
        return SX_OK;
    };
    // the send list is sized by what the peers request (a local may go to several peers): with one batch the scan
    // is read before the scatter; with several, a counting pass first (the arena's growth does not keep contents)
    uint64_t total   = 0;
    bool     idxFail = false; // the send list could not be sized (one batch: decided after the count exchange)
    if (!fail && Pb >= P)
    {
        // one batch (the common case): the send counts stay on the device -- segment starts of the scan -> counts ->
        // the count exchange, read back with the halo receive counts in one synchronisation; the send list is sized
        // and scattered after it (flags and scan are kept)
        const size_t nfb = (size_t)P * (nl + 1);
        maskFlagsKernel<<<grid(nfb), 256, 0, st>>>(mark, nl, 0, P, r, flag);
        SIM_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmpB, flag, scan, (int)nfb, st));
        segStartsKernel<<<grid(P + 1, 64), 64, 0, st>>>(scan, nl, P, segs);
        diffCountsKernel<<<grid(P, 64), 64, 0, st>>>(nullptr, segs, P, s->cntBuf);
        std::vector<uint64_t> off;
        if (int e = deviceCountsOrAbort(s, false, st, s->haloSend, off, s->haloRecv)) return e;
        for (int q = 0; q < P; ++q)
            s->haloSendOff[q] = off[q];
        total      = off[P];
        s->sendIdx = s->work.get<uint32_t>("dom.sendIdx", std::max<uint64_t>(1, total));
        idxFail    = !s->sendIdx;
        if (!idxFail) scatterIdxKernel<<<grid(nfb), 256, 0, st>>>(flag, scan, nl, P, 0, s->sendIdx);
    }
    else
    {
        // several batches (the flags of all peers beyond kFlagCap): a counting pass, then the scatter pass, the
        // counts exchanged on the host's copy
        for (int q0 = 0; q0 < P && !fail; q0 += Pb)
        {
            const int nb = std::min(Pb, P - q0);
            if (int e = batch(q0, nb, false, total)) return e;
            total += hseg[nb];
        }
        s->sendIdx = fail ? nullptr : s->work.get<uint32_t>("dom.sendIdx", std::max<uint64_t>(1, total));
        fail |= !s->sendIdx;
        if (!fail)
        {
            uint64_t base = 0;
            for (int q0 = 0; q0 < P; q0 += Pb)
            {
                const int nb = std::min(Pb, P - q0);
                if (int e = batch(q0, nb, true, base)) return e;
                base += hseg[nb];
            }
        }
        if (int e = countsOrAbort(s, s->haloSend, s->haloRecv, fail, st)) return e;
    }
    s->numSend     = total;
    s->haloRecv[r] = 0;
    uint64_t nLow = 0, nHigh = 0;
    for (int q = 0; q < P; ++q)
        (q < r ? nLow : nHigh) += s->haloRecv[q];
    {
        // the halo capacity (known once the receive counts are) and the send list, decided on every rank together
        bool full = false;
        if (int e = anyRank(s, nLow + nl + nHigh > s->cap || idxFail, st, full)) return e;
        if (full) return SX_ERR_NOMEM;
    }
    s->haloRecvOff.assign(P, 0);
    {
        uint64_t lay[3];
        if (int e = sx_domain_halo_layout(s->haloRecv.data(), P, r, nl, s->haloRecvOff.data(), lay)) return e;
    }
    s->numHalos = nLow + nHigh;

    // --- 5. move locals to [nLow, nLow + nl), exchange x,y,z,h,m, keys + tree over everything
    if (nLow)
    {
        for (auto& sp : s->spares)
        {
            SIM_HIP(hipMemcpyAsync(static_cast<char*>(sp.alt) + nLow * sp.elemBytes, *sp.field, nl * sp.elemBytes,
                                   hipMemcpyDeviceToDevice, st));
            std::swap(*sp.field, sp.alt);
        }
    }
    s->first = nLow;
    s->last  = nLow + nl;
    s->n     = nLow + nl + nHigh;
    // the halos' keys come from their owners (8 B each; the owners computed them from the same coordinates), so the
    // combined tree is built while x,y,z,h,m (28 B per halo) are still in flight on the communication stream
    SIM_HIP(launchSfcKeys(s->x + s->first, s->y + s->first, s->z + s->first, s->keys + s->first, nl, s->dbox, st));
    if (int e = haloExchange(s, {{s->keys, 8}}, st)) return e;
    const bool ovl = s->overlap && s->commStream;
    hipStream_t cs = ovl ? s->commStream : st;
    if (ovl)
    {
        SIM_HIP(hipEventRecord(s->evProd, st));
        SIM_HIP(hipStreamWaitEvent(cs, s->evProd, 0));
    }
    if (int e = haloExchange(s, {{s->x, 8}, {s->y, 8}, {s->z, 8}, {s->h, 4}, {s->m, 4}}, cs)) return e;
    if (ovl) SIM_HIP(hipEventRecord(s->evComm, cs));
    SIM_HIP(buildTree(s->work, s->keys, s->n, s->bucket, s->dbox, s->tree, st));
    if (ovl) SIM_HIP(hipStreamWaitEvent(st, s->evComm, 0));
    s->syncErr = err; // read after the search, with its statistics (syncErrEnqueue / syncErrFailed)
    return SX_OK;
}

//! the last sync's halo-marking flag -> host, ordered on st before the caller's next synchronisation
int syncErrEnqueue(sx_sim* s, hipStream_t st)
{
    uint32_t* h = s->work.pinned<uint32_t>("dom.errh", 1);
    if (!h) return SX_ERR_NOMEM;
    *h = 0;
    if (s->syncErr) SIM_HIP(hipMemcpyAsync(h, s->syncErr, 4, hipMemcpyDeviceToHost, st));
    return SX_OK;
}

//! after that synchronisation: the halo marking of the last sync overflowed its traversal stack
bool syncErrFailed(sx_sim* s)
{
    const uint32_t* h = s->work.pinned<uint32_t>("dom.errh", 1);
    return h && *h != 0;
}

/*! the Ewald correction of periodic self-gravity (gravity_wrapper.hpp:135-157) for the locals [first, last), from the
 *  global root expansion (c4: mass center, m8: quadrupole) with the reference's EwaldSettings defaults (ewald.h:17-21)
 *  and the walk's one image shell; the box is a cube (checked by sx_sim_create) */
int ewaldStep(sx_sim* s, const double c4[4], const float m8[8], const uint8_t* active, hipStream_t st)
{
    EwaldArgs           ea{};
    std::vector<double> hs;
    const double        L = s->box.lim[1] - s->box.lim[0];
    if (ewaldInit(ea.p, hs, c4, m8, L, 1, 2.6, 2.8, 2.0, 3.0e-3)) return SX_ERR_ARG;
    double* hd = s->work.get<double>("ewald.hsum", std::max<size_t>(hs.size(), 5));
    if (!hd) return SX_ERR_NOMEM;
    SIM_HIP(hipMemcpyAsync(hd, hs.data(), hs.size() * sizeof(double), hipMemcpyHostToDevice, st));
    ea.first = (uint32_t)s->first, ea.last = (uint32_t)s->last;
    ea.x = s->x, ea.y = s->y, ea.z = s->z, ea.m = s->m;
    ea.ax = s->ax, ea.ay = s->ay, ea.az = s->az;
    ea.active = active;
    ea.G = (float)s->p.g, ea.hsum = hd, ea.usum = &s->sc->egrav, ea.uscale = 0.5 * (double)ea.G;
    SIM_HIP(ewaldCorrection(ea, st));
    // the host table must outlive the copy
    SIM_HIP(hipStreamSynchronize(st));
    return SX_OK;
}

/*! Self-gravity with several ranks (replaces syncGrav + MultipoleHolder::upsweep/traverse of the reference,
 *  domain.hpp:246-372, multipole_holder.cuh:40-66, and the global multipole exchange of
 *  ryoanji/interface/global_multipole.hpp).  Sources are split by level-6 SFC cells, each owned by one rank (the
 *  splitters are histogram-bin boundaries):
 *   1. every rank forms mass center, MAC radius and quadrupole of its own cells; all cells are all-gathered;
 *   2. a remote cell that satisfies the vector MAC against every request box of this rank (each box contains 2048
 *      SFC-consecutive locals) is "far": its multipole is a leaf of the uniform level-6 far tree, whose upsweep and
 *      Barnes-Hut traversal give the far field (all other leaves massless);
 *   3. the particles of the remaining ("near") remote cells are fetched from their owners as gravity halos, merged
 *      with the locals in key order ([lower ranks | locals | higher ranks]) and traversed with the single-rank
 *      upsweep + traversal on their own tree.
 *  Each source is counted once (locals and near cells in the near tree, far cells in the far tree); every far-cell
 *  multipole is accepted by the same MAC the reference applies, so the result matches the single-rank
 *  Barnes-Hut field within its opening-angle error. */
int distributedGravity(sx_sim* s, hipStream_t st, const uint8_t* active, bool drift)
{
    sx::Transport* T  = s->comm;
    const int      P  = T->size(), r = T->rank();
    const size_t   nl = s->last - s->first;
    const float    invTheta = 1.0f / s->p.theta;
    const size_t   nCellsAll = size_t(1) << kHistBits;
    // periodic self-gravity: both walks over the one image shell of the single-rank path (gravity_wrapper.hpp:135-157)
    const bool     pbc = periodicGravity(s);
    const double   boxL[3] = {s->box.lim[1] - s->box.lim[0], s->box.lim[3] - s->box.lim[2], s->box.lim[5] - s->box.lim[4]};

    // --- far tree: uniform level-6 octree (one synthetic key per cell, bucket 1), built once
    if (s->farTree.numLeaves != (int)nCellsAll)
    {
        uint64_t* fk = s->gravWork.get<uint64_t>("far.keys", nCellsAll);
        farKeysKernel<<<grid(nCellsAll), 256, 0, st>>>(fk, nCellsAll);
        SIM_HIP(buildTree(s->farMem, fk, nCellsAll, 1, s->dbox, s->farTree, st));
        if (s->farTree.numLeaves != (int)nCellsAll) return SX_ERR_HIP;
        GravArgs fa{};
        fa.numLeaves      = s->farTree.numLeaves;
        fa.numNodes       = s->farTree.numNodes;
        fa.childOffsets   = s->farTree.childOffsets;
        fa.internalToLeaf = s->farTree.internalToLeaf;
        fa.leafToNode     = s->farMem.get<int32_t>("far.leafToNode", nCellsAll);
        SIM_HIP(farTreeLeafMap(fa, st));
        uint32_t* lay = s->farMem.get<uint32_t>("far.emptyLayout", nCellsAll + 1);
        SIM_HIP(hipMemsetAsync(lay, 0, 4 * (nCellsAll + 1), st));
    }
    int32_t*  farL2N = s->farMem.get<int32_t>("far.leafToNode", nCellsAll);
    uint32_t* farLay = s->farMem.get<uint32_t>("far.emptyLayout", nCellsAll + 1);
    Arena&    W      = s->gravWork;

    // --- 1. local cells: ranges of the key-sorted locals, moments
    const uint64_t* lkeys = s->keys + s->first;
    uint32_t*       flag  = W.get<uint32_t>("g.flag", nl + 1);
    uint32_t*       scan  = W.get<uint32_t>("g.scan", nl + 1);
    cellFlagKernel<<<grid(nl + 1), 256, 0, st>>>(lkeys, nl, flag);
    size_t tmpB = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, tmpB, flag, scan, (int)nl + 1, st);
    SIM_HIP(hipcub::DeviceScan::ExclusiveSum(W.get<char>("g.scantmp", tmpB), tmpB, flag, scan, (int)nl + 1, st));
    // the cell count is known from the sync's histogram (cellsOf); the device checks the scan agrees
    if (s->cellsOf.size() != (size_t)P) return SX_ERR_ARG;
    const int nCells = (int)s->cellsOf[r];
    cellCountCheckKernel<<<1, 1, 0, st>>>(scan + nl, (uint32_t)nCells, &s->sc->gravErr);
    uint32_t* cellBeg = W.get<uint32_t>("g.cellBeg", nCells + 1);
    uint32_t* cellIds = W.get<uint32_t>("g.cellIds", nCells);
    cellScatterKernel<<<grid(nl + 1), 256, 0, st>>>(lkeys, flag, scan, nl, (uint32_t)nCells, cellBeg, cellIds);
    GCell* mine = W.get<GCell>("g.mine", nCells);
    SIM_HIP(cellMoments(s->x + s->first, s->y + s->first, s->z + s->first, s->m + s->first, cellBeg, cellIds, nCells,
                        farL2N, s->farTree.centers, s->farTree.sizes, invTheta, mine, st, drift));

    // --- 2. all-gather the cells (rank order = key order)
    std::vector<uint64_t> cnt(P, (uint64_t)nCells), rcnt(s->cellsOf);
    cnt[r]  = 0;
    rcnt[r] = 0;
    std::vector<uint64_t> aOff(P + 1, 0);
    for (int q = 0; q < P; ++q)
        aOff[q + 1] = aOff[q] + rcnt[q];
    const size_t nAll = aOff[P];
    GCell*       all  = W.get<GCell>("g.all", nAll);
    {
        std::vector<uint64_t> sb(P), so(P, 0), rb(P), ro(P);
        for (int q = 0; q < P; ++q)
        {
            sb[q] = cnt[q] * sizeof(GCell);
            rb[q] = rcnt[q] * sizeof(GCell);
            ro[q] = aOff[q] * sizeof(GCell);
        }
        SIM_COMM(T->alltoallv(mine, sb.data(), so.data(), all, rb.data(), ro.data(), st));
    }

    // --- 3. near / far classification against this rank's request boxes (distributedSync step 4)
    const size_t  nChunks = (nl + kChunk - 1) / kChunk;
    const ReqBox* boxes   = s->work.get<ReqBox>("dom.mybox", nChunks);
    if (drift)
    {
        // the locals have moved since the sync's request boxes: boxes of their current positions (the same chunks)
        ReqBox* cur = W.get<ReqBox>("g.curbox", nChunks);
        if (!cur) return SX_ERR_NOMEM;
        if (nChunks)
            chunkBoxKernel<<<(unsigned)nChunks, 256, 0, st>>>(s->x + s->first, s->y + s->first, s->z + s->first,
                                                             s->h + s->first, nl, kHaloMargin, quantMargin(s->dbox), r,
                                                             cur);
        boxes = cur;
    }
    uint32_t*     nearF   = W.get<uint32_t>("g.near", nAll + 1);
    uint32_t*     farF    = W.get<uint32_t>("g.far", nAll + 1);
    uint32_t*     reqF    = W.get<uint32_t>("g.reqFlag", nAll + 1);
    uint32_t*     reqS    = W.get<uint32_t>("g.reqScan", nAll + 1);
    SIM_HIP(cellNearFlags(all, (int)nAll, reinterpret_cast<const double*>(boxes), (int)nChunks, nearF, st,
                          pbc ? boxL : nullptr));
    nearToFarKernel<<<grid(nAll + 1), 256, 0, st>>>(nearF, nAll, farF, reqF);
    tmpB = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, tmpB, reqF, reqS, (int)nAll + 1, st);
    SIM_HIP(hipcub::DeviceScan::ExclusiveSum(W.get<char>("g.scantmp2", tmpB), tmpB, reqF, reqS, (int)nAll + 1, st));
    uint32_t* reqIds = W.get<uint32_t>("g.reqIds", nAll);
    reqScatterKernel<<<grid(nAll), 256, 0, st>>>(all, reqF, reqS, nAll, reqIds);
    uint64_t* dOff = W.get<uint64_t>("g.aOff", P + 1);
    uint32_t* dAt  = W.get<uint32_t>("g.at", P + 1);
    SIM_HIP(hipMemcpyAsync(dOff, aOff.data(), 8 * (P + 1), hipMemcpyHostToDevice, st));
    segmentAtKernel<<<grid(P + 1, 64), 64, 0, st>>>(reqS, dOff, P, dAt);
    // --- 4. requests to the owners (counts from the device, exchanged and read back in one synchronisation), owners
    //        send the cells' particles
    diffCountsKernel<<<grid(P, 64), 64, 0, st>>>(nullptr, dAt, P, s->cntBuf);
    std::vector<uint64_t> reqCnt, reqOff, reqRecv;
    if (int e = deviceCountsOrAbort(s, false, st, reqCnt, reqOff, reqRecv)) return e;
    const uint64_t hwReq = reqOff[P]; // near (requested) remote cells
    std::vector<uint64_t> rrOff(P + 1, 0);
    for (int q = 0; q < P; ++q)
        rrOff[q + 1] = rrOff[q] + reqRecv[q];
    const size_t nReq = rrOff[P];
    uint32_t*    req  = W.get<uint32_t>("g.req", nReq);
    {
        std::vector<uint64_t> sb(P), so(P), rb(P), ro(P);
        for (int q = 0; q < P; ++q)
            sb[q] = reqCnt[q] * 4, so[q] = reqOff[q] * 4, rb[q] = reqRecv[q] * 4, ro[q] = rrOff[q] * 4;
        SIM_COMM(T->alltoallv(reqIds, sb.data(), so.data(), req, rb.data(), ro.data(), st));
    }
    uint32_t* rsize = W.get<uint32_t>("g.rsize", nReq + 1);
    uint32_t* rbeg  = W.get<uint32_t>("g.rbeg", nReq + 1);
    uint32_t* roff  = W.get<uint32_t>("g.roff", nReq + 1);
    reqLookupKernel<<<grid(nReq + 1), 256, 0, st>>>(req, nReq, cellIds, cellBeg, nCells, rsize, rbeg);
    tmpB = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, tmpB, rsize, roff, (int)nReq + 1, st);
    SIM_HIP(hipcub::DeviceScan::ExclusiveSum(W.get<char>("g.scantmp3", tmpB), tmpB, rsize, roff, (int)nReq + 1, st));
    SIM_HIP(hipMemcpyAsync(dOff, rrOff.data(), 8 * (P + 1), hipMemcpyHostToDevice, st));
    segmentAtKernel<<<grid(P + 1, 64), 64, 0, st>>>(roff, dOff, P, dAt);
    diffCountsKernel<<<grid(P, 64), 64, 0, st>>>(nullptr, dAt, P, s->cntBuf);
    std::vector<uint64_t> pCnt, pOff, pRecv;
    if (int e = deviceCountsOrAbort(s, false, st, pCnt, pOff, pRecv)) return e;
    const size_t nSend = pOff[P];
    GPart*       psend = W.get<GPart>("g.psend", nSend);
    if (nReq)
        gatherCellsKernel<<<grid(nReq * 64), 256, 0, st>>>(rbeg, rsize, roff, nReq, s->x + s->first, s->y + s->first,
                                                           s->z + s->first, s->m + s->first, s->h + s->first,
                                                           s->keys + s->first, psend);
    uint64_t nLow = 0, nHigh = 0;
    for (int q = 0; q < P; ++q)
        (q < r ? nLow : nHigh) += (q == r ? 0 : pRecv[q]);
    const size_t nG    = nLow + nl + nHigh;
    GPart*       precv = W.get<GPart>("g.precv", nLow + nHigh);
    {
        std::vector<uint64_t> sb(P), so(P), rb(P), ro(P);
        uint64_t              acc = 0;
        for (int q = 0; q < P; ++q)
        {
            sb[q] = pCnt[q] * sizeof(GPart), so[q] = pOff[q] * sizeof(GPart);
            rb[q] = (q == r ? 0 : pRecv[q]) * sizeof(GPart), ro[q] = acc * sizeof(GPart);
            acc += (q == r ? 0 : pRecv[q]);
        }
        SIM_COMM(T->alltoallv(psend, sb.data(), so.data(), precv, rb.data(), ro.data(), st));
    }

    // --- 5. near sources: [lower-rank halos | locals | higher-rank halos], key sorted by construction
    double*   gx = W.get<double>("g.x", nG);
    double*   gy = W.get<double>("g.y", nG);
    double*   gz = W.get<double>("g.z", nG);
    float*    gm = W.get<float>("g.m", nG);
    float*    gh = W.get<float>("g.h", nG);
    uint64_t* gk = W.get<uint64_t>("g.keys", nG);
    if (nLow) unpackGPartKernel<<<grid(nLow), 256, 0, st>>>(precv, nLow, gx, gy, gz, gm, gh, gk);
    if (nHigh)
        unpackGPartKernel<<<grid(nHigh), 256, 0, st>>>(precv + nLow, nHigh, gx + nLow + nl, gy + nLow + nl,
                                                       gz + nLow + nl, gm + nLow + nl, gh + nLow + nl, gk + nLow + nl);
    SIM_HIP(hipMemcpyAsync(gx + nLow, s->x + s->first, 8 * nl, hipMemcpyDeviceToDevice, st));
    SIM_HIP(hipMemcpyAsync(gy + nLow, s->y + s->first, 8 * nl, hipMemcpyDeviceToDevice, st));
    SIM_HIP(hipMemcpyAsync(gz + nLow, s->z + s->first, 8 * nl, hipMemcpyDeviceToDevice, st));
    SIM_HIP(hipMemcpyAsync(gm + nLow, s->m + s->first, 4 * nl, hipMemcpyDeviceToDevice, st));
    SIM_HIP(hipMemcpyAsync(gh + nLow, s->h + s->first, 4 * nl, hipMemcpyDeviceToDevice, st));
    // the keys of the last sync, not of the current positions: the sources stay in the sync's key order (inside a
    // ve-bdt hierarchy particles drift out of their cells, as in the reference's fixed focus tree)
    SIM_HIP(hipMemcpyAsync(gk + nLow, s->keys + s->first, 8 * nl, hipMemcpyDeviceToDevice, st));
    SIM_HIP(buildTree(W, gk, nG, s->bucket, s->dbox, s->nearTree, st));

    GravArgs ga{};
    ga.first          = (uint32_t)nLow;
    ga.last           = (uint32_t)(nLow + nl);
    ga.numLeaves      = s->nearTree.numLeaves;
    ga.numNodes       = s->nearTree.numNodes;
    ga.childOffsets   = s->nearTree.childOffsets;
    ga.internalToLeaf = s->nearTree.internalToLeaf;
    ga.layout         = s->nearTree.layout;
    ga.geoCenters     = s->nearTree.centers;
    ga.geoSizes       = s->nearTree.sizes;
    ga.leafToNode     = W.get<int32_t>("g.leafToNode", (size_t)s->nearTree.numLeaves);
    if (drift)
    {
        // the near tree's cells come from the sync's keys: boxes holding each node's cell and its current particles
        double* c3 = W.get<double>("g.geoC", 3 * (size_t)s->nearTree.numNodes);
        double* s3 = W.get<double>("g.geoS", 3 * (size_t)s->nearTree.numNodes);
        if (!c3 || !s3) return SX_ERR_NOMEM;
        SIM_HIP(skinRefreshBoxes(s->nearTree, gx, gy, gz, s->dbox, c3, s3, st, true));
        ga.geoCenters = c3;
        ga.geoSizes   = s3;
    }
    ga.x = gx, ga.y = gy, ga.z = gz, ga.m = gm, ga.h = gh;
    ga.centers4   = W.get<double>("g.centers", 4 * (size_t)s->nearTree.numNodes);
    ga.multipoles = W.get<float>("g.multipoles", 8 * (size_t)s->nearTree.numNodes);
    ga.G          = (float)s->p.g;
    ga.invTheta   = invTheta;
    // target i of the near arrays is local particle s->first + (i - nLow)
    const ptrdiff_t shift = (ptrdiff_t)s->first - (ptrdiff_t)nLow;
    ga.ax    = s->ax + shift;
    ga.ay    = s->ay + shift;
    ga.az    = s->az + shift;
    ga.active = active ? active + shift : nullptr;
    ga.egrav = &s->sc->egrav;
    ga.err   = &s->sc->gravErr;
    ga.fast  = sx_ctx_exact_internal(s->ctx) ? 0 : 1;
    ga.interactions = s->gravCount && !pbc ? s->work.get<unsigned long long>("grav.inter", 2) : nullptr;
    if (pbc)
    {
        ga.numShells = 1;
        for (int d = 0; d < 3; ++d)
            ga.boxL[d] = boxL[d];
    }
    SIM_HIP(gravityUpsweep(ga, s->nearTree.levelRangeHost.data(), st));
    ga.waveE = s->work.get<double>("grav.waveE", (ga.last - ga.first + kWave - 1) / kWave + 1);
    SIM_HIP(gravityTraverse(ga, st));

    // --- 6. far field: far cells as leaves of the level-6 tree, traversed by the locals
    GravArgs fa{};
    fa.first          = (uint32_t)s->first;
    fa.last           = (uint32_t)s->last;
    fa.numLeaves      = s->farTree.numLeaves;
    fa.numNodes       = s->farTree.numNodes;
    fa.childOffsets   = s->farTree.childOffsets;
    fa.internalToLeaf = s->farTree.internalToLeaf;
    fa.layout         = farLay; // no particles: a far leaf is always accepted (MAC holds for every request box)
    fa.geoCenters     = s->farTree.centers;
    fa.geoSizes       = s->farTree.sizes;
    fa.leafToNode     = farL2N;
    fa.x = s->x, fa.y = s->y, fa.z = s->z, fa.m = s->m, fa.h = s->h;
    fa.centers4   = s->farMem.get<double>("far.centers", 4 * (size_t)s->farTree.numNodes);
    fa.multipoles = s->farMem.get<float>("far.multipoles", 8 * (size_t)s->farTree.numNodes);
    fa.G          = (float)s->p.g;
    fa.invTheta   = invTheta;
    fa.ax = s->ax, fa.ay = s->ay, fa.az = s->az;
    fa.active = active;
    fa.egrav = &s->sc->egrav;
    fa.err   = &s->sc->gravErr;
    fa.fast  = sx_ctx_exact_internal(s->ctx) ? 0 : 1;
    fa.interactions = ga.interactions;
    fa.numShells    = ga.numShells;
    for (int d = 0; d < 3; ++d)
        fa.boxL[d] = ga.boxL[d];
    if (drift)
    {
        double* c3 = s->farMem.get<double>("far.geoC", 3 * (size_t)s->farTree.numNodes);
        double* s3 = s->farMem.get<double>("far.geoS", 3 * (size_t)s->farTree.numNodes);
        if (!c3 || !s3) return SX_ERR_NOMEM;
        SIM_HIP(farRefreshBoxes(fa, all, farF, (int)nAll, s->farTree.levelRangeHost.data(), c3, s3, st));
        fa.geoCenters = c3;
        fa.geoSizes   = s3;
    }
    SIM_HIP(farUpsweep(fa, all, farF, (int)nAll, s->farTree.levelRangeHost.data(), st));
    fa.waveE = s->work.get<double>("grav.waveE", (fa.last - fa.first + kWave - 1) / kWave + 1);
    SIM_HIP(gravityTraverse(fa, st));
    if (pbc)
    {
        // the Ewald correction from the global root: the near tree (locals + near cells) and the far tree (far cells)
        // together hold every source once
        double cN[4], cF[4], c4[4];
        float  mN[8], mF[8], m8[8];
        SIM_HIP(hipMemcpyAsync(cN, ga.centers4, sizeof(cN), hipMemcpyDeviceToHost, st));
        SIM_HIP(hipMemcpyAsync(mN, ga.multipoles, sizeof(mN), hipMemcpyDeviceToHost, st));
        SIM_HIP(hipMemcpyAsync(cF, fa.centers4, sizeof(cF), hipMemcpyDeviceToHost, st));
        SIM_HIP(hipMemcpyAsync(mF, fa.multipoles, sizeof(mF), hipMemcpyDeviceToHost, st));
        SIM_HIP(hipStreamSynchronize(st));
        combineRoots(cN, mN, cF, mF, c4, m8);
        if (int e = ewaldStep(s, c4, m8, active, st)) return e;
    }
    s->gravHalos       = nLow + nHigh;
    s->gravRemoteCells = nAll;
    s->gravFarCells    = nAll - (reqOff.empty() ? 0 : hwReq);
    return SX_OK;
}

/*! a decision every rank must take together: true on all ranks if `bad` holds on any (one allreduce).  A rank that
 *  returned alone from the middle of distributedSync would leave its peers waiting in the next collective. */
int anyRank(sx_sim* s, bool bad, hipStream_t st, bool& out)
{
    auto*     flg  = s->work.get<uint32_t>("dom.agree", 1);
    uint32_t* hflg = s->work.pinned<uint32_t>("dom.agreeh", 1);
    if (!flg || !hflg) return SX_ERR_NOMEM;
    *hflg = bad ? 1u : 0u;
    SIM_HIP(hipMemcpyAsync(flg, hflg, 4, hipMemcpyHostToDevice, st));
    SIM_COMM(s->comm->allreduceSumU32(flg, 1, st));
    SIM_HIP(hipMemcpyAsync(hflg, flg, 4, hipMemcpyDeviceToHost, st));
    SIM_HIP(hipStreamSynchronize(st));
    out = *hflg != 0;
    return SX_OK;
}

int halosOutgrown(sx_sim* s, hipStream_t st, unsigned& hf)
{
    const size_t nl  = s->last - s->first;
    auto*        flg = s->work.get<unsigned>("dom.hflag", 1);
    SIM_HIP(hipMemsetAsync(flg, 0, 4, st));
    if (nl)
        chunkCoverKernel<<<grid(nl), 256, 0, st>>>(s->x + s->first, s->y + s->first, s->z + s->first, s->h + s->first,
                                                 nl, s->work.get<ReqBox>("dom.mybox", 1), s->dbox,
                                                 quantMargin(s->dbox), flg);
    // the retry decision must be global: a rank redoing the sync alone would deadlock the collectives
    SIM_COMM(s->comm->allreduceSumU32(flg, 1, st));
    unsigned* hflg = s->work.pinned<unsigned>("dom.hflagh", 1);
    SIM_HIP(hipMemcpyAsync(hflg, flg, 4, hipMemcpyDeviceToHost, st));
    if (int e = syncErrEnqueue(s, st)) return e;
    SIM_HIP(hipStreamSynchronize(st));
    if (syncErrFailed(s)) return SX_ERR_TRAVERSAL;
    hf = *hflg;
    return SX_OK;
}

void maxAccSq(sx_sim* s, hipStream_t st)
{
    const size_t nl = s->last - s->first;
    if (nl)
        maxAccSqKernel<<<std::min<unsigned>(grid(nl), 2048), 256, 0, st>>>(s->ax, s->ay, s->az, s->first, s->last,
                                                                          &s->sc->maxAccSqBits);
}

//! self-gravity with periodic images (the reference's test, gravity_wrapper.hpp:77,135: boundaryX; sx_sim_create
//! admits only boxes periodic along all three axes with self-gravity)
bool periodicGravity(const sx_sim* s) { return s->p.g != 0.0 && s->box.bnd[0] == 1; }

//! skin lists serve this sim: one rank, not ve-bdt, cluster lists.  With self-gravity a reuse step traverses the last
//! sync's tree, its multipoles formed from the current positions and its MAC geometry refreshed (cells + particles).
//! Not with periodic self-gravity: between syncs a particle that crossed a periodic face is wrapped to the far side of
//! the box while it stays in its old leaf, so the leaf's multipole (raw coordinates) would spread across the box
//! while its refreshed MAC box (minimum image) covers only the old cell -- every step syncs there
//! Several ranks: the halo set of a full build is requested with the skin radius, a reuse step refreshes the halos'
//! x, y, z, h, m over the build's send lists and reduces the displacement grid over all ranks, and every decision
//! about builds is taken on all ranks together (skinHaloRefresh, the decision exchange in sx_sim_step); self-gravity
//! on a reuse step splits near and far cells against boxes of the current positions and takes MAC boxes that hold
//! each cell (node) and its drifted particles (distributedGravity with drift)
bool skinUsable(const sx_sim* s)
{
    return s->skin.factor > 0.0f && s->p.propagator != 2 && NbLists::localPossible(s->p.ngmax) &&
           !periodicGravity(s);
}

//! widest skin the adaptation goes to: skin lists (1.16)^3 = 1.56x the neighbors; wider unions outgrow the filter's LDS
//! staging (kSkinCap) in dense regions (Noh at s = 0.25: 37% of the clusters)
constexpr float kMaxSkin = 0.16f;
//! reuse steps after which a skin has paid for its build several times over: a stale-forced build before them widens it
constexpr int kShortSkin = 10;

//! a skin that did not outlast two steps: the next build takes a twice wider one; at the widest, the next steps
//! search without skin (backoff, doubling up to 32 steps)
void skinTooThin(SkinState& K)
{
    K.forceBuild = true;
    if (K.cur < kMaxSkin) K.cur = std::min(2.0f * K.cur, kMaxSkin);
    else
    {
        K.backoff    = K.backoffLen;
        K.backoffLen = std::min(2 * K.backoffLen, 32);
    }
}

//! the displacement grid over the box: kSkinGridN cells per axis
SkinGrid skinGrid(const DevBox& b)
{
    SkinGrid g{};
    g.n = kSkinGridN;
    for (int d = 0; d < 3; ++d)
    {
        g.lo[d]  = b.lim[2 * d];
        g.inv[d] = (double)kSkinGridN / b.l[d];
        g.pbc[d] = b.pbc[d];
    }
    return g;
}

//! skin-list capacity per target: the neighbor capacity scaled by the skin volume, with room for density variation
uint32_t skinCapacity(uint32_t ngmax, float factor)
{
    const double f = std::pow(1.0 + factor, 3.0) * 1.15;
    const uint32_t c = (uint32_t)std::ceil(ngmax * f);
    return std::min<uint32_t>(256u, (c + 1u) & ~1u);
}

//! the skin arrays the position update feeds: per particle this step's displacement vector, and per cell of the grid
//! the component ranges (initialised here: the update scatters into them)
bool skinParticleBuffers(sx_sim* s, PosArgs& q, hipStream_t st)
{
    const size_t nc = (size_t)kSkinGridN * kSkinGridN * kSkinGridN;
    q.dispX = s->mem.get<float>("skin.dx", s->cap);
    q.dispY = s->mem.get<float>("skin.dy", s->cap);
    q.dispZ = s->mem.get<float>("skin.dz", s->cap);
    q.cells = s->mem.get<uint32_t>("skin.cells", kGridWords * nc);
    q.grid  = skinGrid(s->dbox);
    if (!q.dispX || !q.dispY || !q.dispZ || !q.cells) return false;
    return hipMemsetAsync(q.cells, 0xff, 3 * nc * sizeof(uint32_t), st) == hipSuccess &&
           hipMemsetAsync(q.cells + 3 * nc, 0, 3 * nc * sizeof(uint32_t), st) == hipSuccess;
}

constexpr int kSkinResync = 1000; //!< skinSearch: redo this step's search from a full sync (not an error code)

//! a step's skin search on this rank: clusters, stale ones (rebuilt at once or sent to the exact search directly),
//! those rebuilt, and those that took the exact search
struct SkinCounts
{
    uint32_t clusters{0}, stale{0}, rebuilt{0}, exact{0};
};

/*! The step's neighbor search through skin lists (sx_skin.hpp).  A full build (after a full sync) builds every
 *  cluster's skin and filters it; a reuse step only filters.  Stale clusters are rebuilt at once on node boxes refreshed
 *  from the current positions (reuse steps) and filtered; clusters stale again take the exact search (on a reuse step
 *  over the refreshed boxes: should it outgrow a capacity there, kSkinResync makes the caller restore h and redo the
 *  step's search from a full sync).  na: the step's search arguments (exact lists, h, nc, tree).  One host read of the
 *  stale count, two or three when some cluster is stale. */
int skinSearch(sx_sim* s, const NsArgs& na, bool reuse, hipStream_t st, float* xmOut, RecT* rtXm, SkinCounts& out)
{
    auto&          K   = s->skin;
    const uint32_t ncl = (na.numGroups + kClusterWaves - 1) / kClusterWaves;
    out                = SkinCounts{};
    out.clusters       = ncl;
    if (!reuse) K.built = K.cur; // (also with no local cluster: every rank's skin state stays the same)
    if (!ncl) return SX_OK;
    if (!reuse) K.ngmaxS = skinCapacity(s->p.ngmax, K.built);
    const size_t G    = kSkinGridN;
    float*       rel  = s->mem.get<float>("skin.rel", s->cap);
    float*       dx   = s->mem.get<float>("skin.dx", s->cap);
    float*       dy   = s->mem.get<float>("skin.dy", s->cap);
    float*       dz   = s->mem.get<float>("skin.dz", s->cap);
    uint32_t*   sloc = s->mem.get<uint32_t>("skin.sloc", na.numGroups * (size_t)nlocWords(K.ngmaxS) * kWave);
    uint32_t*   scnt = s->mem.get<uint32_t>("skin.scnt", s->cap);
    float*      hb   = s->mem.get<float>("skin.hb", s->cap);
    float*      acc  = s->mem.get<float>("skin.acc", ncl);
    uint32_t*   cells = s->mem.get<uint32_t>("skin.cells", kGridWords * G * G * G);
    uint32_t*   ucS   = s->mem.get<uint32_t>("skin.ucount", ncl);
    uint32_t*   l1    = s->mem.get<uint32_t>("skin.l1", ncl + 1);
    uint32_t*   l2    = s->mem.get<uint32_t>("skin.l2", ncl + 1);
    uint32_t*   l3    = s->mem.get<uint32_t>("skin.l3", ncl + 1);
    uint32_t*   hl    = s->mem.pinned<uint32_t>("skin.host", 4);
    uint8_t*    strk  = s->mem.get<uint8_t>("skin.streak", ncl);
    uint32_t*   hmask = s->mem.get<uint32_t>("skin.hitmask", na.numGroups * (size_t)kSkinMaskWords * kWave);
    uint8_t*    same  = s->mem.get<uint8_t>("skin.same", ncl);
    float2*     frz   = s->mem.get<float2>("skin.frz", ncl);
    // the second set of exact lists (SkinArgs::nlocB): its union in the slot's second quarter, below the skin union
    const bool  twoSets = na.ucap / 4 >= (uint32_t)kSkinCap && !getenv("SX_SKIN_ONESET");
    uint32_t*   nlocB = twoSets ? s->mem.get<uint32_t>("skin.nlocB", na.numGroups * (size_t)nlocWords(na.ngmax) * kWave)
                                : nullptr;
    uint32_t*   ucB   = twoSets ? s->mem.get<uint32_t>("skin.ucountB", ncl) : nullptr;
    uint32_t*   hmB   = twoSets ? s->mem.get<uint32_t>("skin.hitmaskB", na.numGroups * (size_t)kSkinMaskWords * kWave)
                                : nullptr;
    if (!rel || !dx || !dy || !dz || !sloc || !scnt || !hb || !acc || !cells || !ucS || !l1 || !l2 || !l3 || !hl || !strk ||
        !hmask || !same || !frz || (twoSets && (!nlocB || !ucB || !hmB)))
        return SX_ERR_NOMEM;

    const SkinGrid g = skinGrid(s->dbox);
    SkinArgs fa{};
    fa.first = na.first, fa.last = na.last, fa.numGroups = na.numGroups, fa.ngmax = na.ngmax, fa.ng0 = na.ng0;
    fa.ngmaxS = K.ngmaxS, fa.iterateH = na.iterateH, fa.skin1 = 1.0f + K.built;
    fa.x = na.x, fa.y = na.y, fa.z = na.z, fa.h = na.h, fa.m = na.m, fa.nc = na.nc, fa.rxOut = na.rxOut;
    // the skin union lives in the upper half of each cluster's union slot, the exact union (the pair kernels') at its
    // start
    const uint32_t uoff = na.ucap / 2;
    fa.nloc = na.nloc, fa.uni = na.uni, fa.ucount = na.ucount, fa.ucap = na.ucap, fa.uoff = uoff, fa.ucountS = ucS;
    fa.sloc = sloc, fa.scnt = scnt, fa.hb = hb, fa.rel = rel, fa.acc = acc, fa.cells = cells, fa.grid = g;
    fa.dispX = dx, fa.dispY = dy, fa.dispZ = dz;
    fa.xmOut = xmOut, fa.rtXm = rtXm, fa.K = s->p.K;
    K.xmFused   = xmOut != nullptr;
    K.exactList = l2;
    fa.box = na.box, fa.powTab = na.powTab, fa.stats = na.stats, fa.clStats = na.clStats;
    // exact lists kept where no target's hits changed: only over the lists, masks and flags the last skin search of
    // this simulation left (no other search or allocation since)
    fa.hitMask   = hmask;
    fa.same      = same;
    fa.nlocB = nlocB, fa.ucountB = ucB, fa.hitMaskB = hmB, fa.uoffB = na.ucap / 4;
    fa.frz       = getenv("SX_SKIN_NOFREEZE") ? nullptr : frz; // (A/B: every reuse step walks its skin lists)
    fa.keepLists = reuse && K.listsKept && K.keptNloc == na.nloc && K.keptUni == na.uni && K.keptMask == hmask &&
                   K.keptSame == same && K.keptFrz == frz && K.keptNlocB == nlocB;
    K.listsKept  = false; // until this search completes

    // the skin build: the search with radii 2 h (1 + s), no h iteration, skin lists and counts as its outputs
    NsArgs b   = na;
    b.skin1    = 1.0f + K.built;
    b.iterateH = 0;
    b.nloc     = sloc;
    b.ngmax    = K.ngmaxS;
    b.nc       = scnt;
    b.rxOut    = nullptr;
    b.uoff     = uoff;
    b.ucount   = ucS;

    SIM_HIP(hipMemsetAsync(l1, 0, 4, st));
    SIM_HIP(hipMemsetAsync(l2, 0, 4, st));
    if (!reuse)
    {
        SIM_HIP(hipMemsetAsync(strk, 0, ncl, st));
        SIM_HIP(findNeighbors(b, st));
        fa.fresh = 1;
    }
    else fa.fresh = 0; // the grid of this step's displacements came from the last position update
    fa.list  = nullptr;
    fa.stale = l1;
    // reuse steps: a cluster stale again on the step after its rebuild goes straight to the exact search (l2)
    fa.streak = reuse ? strk : nullptr;
    fa.direct = reuse ? l2 : nullptr;
    SIM_HIP(skinFilter(fa, ncl, st));
    SIM_HIP(hipMemcpyAsync(hl, l1, 4, hipMemcpyDeviceToHost, st));
    SIM_HIP(hipMemcpyAsync(hl + 1, l2, 4, hipMemcpyDeviceToHost, st));
    SIM_HIP(hipStreamSynchronize(st));
    const uint32_t n1 = hl[0], nd = hl[1];
    uint32_t       n2 = nd;
    out.rebuilt = n1, out.stale = n1 + nd, out.exact = nd;
    NsArgs         x  = na; // the exact search, for clusters whose h iteration outgrows even a fresh skin
    // subset searches of a reuse step run the large build directly: on the refreshed (overlapping) boxes many of the
    // few clusters overflow the compact one, whose launch then only adds a tail (Noh -n 300: 20.4 -> 20.1 ms/step)
    NsPolicy large;
    large.mode = 1;
    if (reuse) b.policy = x.policy = &large;
    if ((n1 || nd) && reuse)
    {
        // particles have left the cells of the last full sync's tree: the walk takes boxes of the current positions
        double* c3 = s->mem.get<double>("skin.centers", 3 * (size_t)s->tree.numNodes);
        double* s3 = s->mem.get<double>("skin.sizes", 3 * (size_t)s->tree.numNodes);
        if (!c3 || !s3) return SX_ERR_NOMEM;
        SIM_HIP(skinRefreshBoxes(s->tree, na.x, na.y, na.z, na.box, c3, s3, st));
        b.centers = x.centers = c3;
        b.sizes = x.sizes = s3;
    }
    // the directly stale clusters' exact search does not depend on the rebuild of the others (disjoint clusters: their
    // lists, unions, h, nc and records; only the statistics words are shared, reduced again below): with both, it runs
    // on the auxiliary stream with its own search scratch while the rebuild and its filter run here
    const bool early = n1 && nd && reuse && s->auxStream && s->evAuxIn && s->evAuxOut && !getenv("SX_SKIN_SERIAL_EXACT");
    if (early)
    {
        NsArgs xd   = x;
        xd.subset   = l2;
        xd.work     = s->mem.get<uint32_t>("skin.aux.work", 16);
        xd.hSave    = s->mem.get<float>("skin.aux.over", ncl + 1);
        xd.hitMasks = s->mem.get<uint64_t>("skin.aux.masks", searchScratchBytes() / sizeof(uint64_t));
        // one workgroup per cluster here, the rest of the resident grid for the rebuild: a persistent rebuild grid
        // holding every slot would leave this search waiting for it (SX_SKIN_AUX_SHARE=0: both take the whole grid)
        const char* sh = getenv("SX_SKIN_AUX_SHARE");
        if (!sh || atoi(sh) != 0)
        {
            const unsigned G = searchGrid();
            xd.maxGrid       = std::min(nd, G / 2);
            b.maxGrid        = G - xd.maxGrid;
        }
        if (!xd.work || !xd.hSave || !xd.hitMasks) return SX_ERR_NOMEM;
        SIM_HIP(hipEventRecord(s->evAuxIn, st));
        SIM_HIP(hipStreamWaitEvent(s->auxStream, s->evAuxIn, 0));
        SIM_HIP(findNeighbors(xd, s->auxStream));
        SIM_HIP(hipEventRecord(s->evAuxOut, s->auxStream));
    }
    uint32_t* lx = l2; // the exact search's list below: l2 (the direct clusters, then those stale after the rebuild)
    if (n1)
    {
        b.subset  = l1;
        SIM_HIP(findNeighbors(b, st));
        fa.fresh  = 1;
        fa.list   = l1;
        // appended after the direct ones, or (their search already running) a list of their own
        if (early) SIM_HIP(hipMemsetAsync(l3, 0, 4, st));
        fa.stale  = early ? l3 : l2;
        fa.streak = nullptr;
        fa.direct = nullptr;
        SIM_HIP(skinFilter(fa, ncl, st));
        SIM_HIP(hipMemcpyAsync(hl + 2, fa.stale, 4, hipMemcpyDeviceToHost, st));
        SIM_HIP(hipStreamSynchronize(st));
        n2 = hl[2];
    }
    uint32_t n3 = 0; // early: the clusters stale after the rebuild (l3), searched below
    if (early)
    {
        n3 = n2, n2 = nd + n3, lx = l3;
        K.earlyExact += nd;
        SIM_HIP(hipStreamWaitEvent(st, s->evAuxOut, 0));
    }
    out.exact = n2;
    {
        if (early ? n3 : n2)
        {
            x.subset = lx;
            SIM_HIP(findNeighbors(x, st));
        }
        if (early)
        {
            // one list of every exact-search cluster (XMass, skinMarkStale): l3's entries after the direct ones
            if (n3) SIM_HIP(hipMemcpyAsync(l2 + 1 + nd, l3 + 1, 4 * (size_t)n3, hipMemcpyDeviceToDevice, st));
            hl[3] = n2;
            SIM_HIP(hipMemcpyAsync(l2, hl + 3, 4, hipMemcpyHostToDevice, st)); // read by the synchronisation below
        }
        if (n2)
        {
            if (reuse)
            {
                // on a reuse step the walk takes the drifted tree's refreshed boxes, which overlap: should the exact
                // search outgrow its capacities there, the step's search is redone from a full sync
                SIM_HIP(hipMemcpyAsync(hl, na.stats, 4, hipMemcpyDeviceToHost, st));
                SIM_HIP(hipStreamSynchronize(st));
                if (hl[0] & 1u)
                {
                    SIM_HIP(hipMemsetAsync(na.stats, 0, 4, st));
                    return kSkinResync;
                }
            }
            SIM_HIP(skinMarkStale(l2, ncl, acc, st)); // their skins are rebuilt next step
        }
    }
    SIM_HIP(reduceClusterStats(na.clStats, ncl, na.stats, st));
    K.listsKept = true, K.keptNloc = na.nloc, K.keptUni = na.uni, K.keptMask = hmask, K.keptSame = same, K.keptFrz = frz;
    K.keptNlocB = nlocB;
    // the pair kernels read each cluster's current set
    K.lb = twoSets ? ListsB{same, nlocB, ucB, na.ucap / 4} : ListsB{};
    if (getenv("SX_SKIN_DEBUG"))
    {
        uint32_t f = 0;
        SIM_HIP(hipMemcpyAsync(&f, na.stats, 4, hipMemcpyDeviceToHost, st));
        SIM_HIP(hipStreamSynchronize(st));
        fprintf(stderr, "skin: reuse %d s %.3f clusters %u stale %u exact %u (direct %u) flags 0x%x mode %d\n",
                (int)reuse, K.built, ncl, n1 + nd, n2, nd, f, s->nsPolicy.mode);
    }
    return SX_OK;
}

/*! the skin's bookkeeping after a step's search: statistics of this rank, and the build decisions from the stale share
 *  of all ranks (staleAll of clustersAll: with several ranks the sums over every rank, so that every rank takes the
 *  same decisions and the next step is a full sync + build on all of them or on none) */
void skinDecide(SkinState& K, bool reuse, const SkinCounts& c, uint64_t staleAll, uint64_t clustersAll)
{
    K.lastStale = c.stale, K.lastExact = c.exact;
    K.staleClusters += c.stale, K.exactClusters += c.exact;
    if (reuse)
    {
        K.reuseSteps++;
        K.sinceBuild++;
    }
    else
    {
        K.builds++;
        K.valid      = true;
        K.forceBuild = false;
        K.sinceBuild = 0;
    }
    // many clusters rebuilt one by one: the next step syncs (SFC order restored) and builds them all at once.  A
    // stale-heavy step costs about a build; a skin with fewer than two clean reuse steps since its build saved
    // nothing, so the next steps search without it (backoff, doubling up to 32 steps with every such skin)
    const bool clean = (double)staleAll <= K.staleLimit * (double)clustersAll;
    if (!reuse) K.cleanSinceBuild = 0;
    else if (clean) K.cleanSinceBuild++;
    if (!clean)
    {
        K.forceBuild = true;
        if (!reuse || K.cleanSinceBuild < 2) skinTooThin(K);
        // a skin used up by the flow in fewer than kShortSkin steps (Noh's shock at s = 0.05: a full build every ~6
        // steps) is widened a little for the next build; one that lasts until maxReuse (Sedov) stays as it is
        else if (K.sinceBuild < kShortSkin) K.cur = std::min(1.25f * K.cur, kMaxSkin);
    }
    if (clean && K.cleanSinceBuild >= 2) K.backoffLen = 4;
}

//! a reuse step with several ranks: the halos of the last build get their owners' current x, y, z, h, m over the
//! build's send lists (the particles stay where they are: no exchange to the SFC owners until the next build), and
//! the displacement grid of the last position update becomes the grid of every rank's particles (u32 min / max of the
//! ordered-float component ranges): a particle that was no halo at the build can only reach a target's 2h sphere
//! through the region around its cluster, where its steps now count in the filter's drift bound (sx_skin.hpp)
int skinHaloRefresh(sx_sim* s, hipStream_t st)
{
    if (int e = haloExchange(s, {{s->x, 8}, {s->y, 8}, {s->z, 8}, {s->h, 4}, {s->m, 4}}, st)) return e;
    const size_t nc    = (size_t)kSkinGridN * kSkinGridN * kSkinGridN;
    uint32_t*    cells = s->mem.get<uint32_t>("skin.cells", kGridWords * nc);
    if (!cells) return SX_ERR_NOMEM;
    SIM_COMM(s->comm->allreduceMinU32(cells, 3 * nc, st));
    SIM_COMM(s->comm->allreduceMaxU32(cells + 3 * nc, 3 * nc, st));
    return SX_OK;
}

//! XMass of the step: all clusters, or after a filter that computed it only the exact-search clusters
void xmassRest(sx_sim* s, const HydroLaunch& H, PairArgs a, hipStream_t st)
{
    if (!s->skin.xmFused) return H.xmass(a, st);
    if (!s->skin.lastExact) return;
    a.clusterList = s->skin.exactList + 1;
    a.listCount   = s->skin.lastExact;
    H.xmass(a, st);
}

int localSync(sx_sim* s, hipStream_t st)
{
    const size_t n = s->n;
    // keys written by the last position update (PosArgs::keys) are those of the current coordinates
    if (!s->keysFresh) SIM_HIP(launchSfcKeys(s->x, s->y, s->z, s->keys, n, s->dbox, st));
    s->keysFresh = false;
    if (int e = sortLocals(s, n, st)) return e;
    SIM_HIP(buildTree(s->work, s->keys, n, s->bucket, s->dbox, s->tree, st));
    s->first = 0;
    s->last  = n;
    return SX_OK;
}

} // namespace sx::sim

extern "C"
{

    int sx_sim_create(sx_sim** out, sx_ctx* ctx, size_t capacity, const sx_params* p, const sx_box* box,
                      uint32_t bucketSize)
    {
        if (p->propagator < 0 || p->propagator > 2) return SX_ERR_ARG;
        // self-gravity in a periodic box: the image walk + Ewald correction of the VE / std step (single rank).  The
        // reference decides on boundaryX alone (gravity_wrapper.hpp:77,135) and walks images along all three axes;
        // here a mixed box (some axes periodic, some not) is refused rather than given images along open axes, the
        // Ewald sum needs a cubic box (ewald.hpp:149-214), and the ve-bdt driver's gravity has no image walk
        if (p->g != 0.0 && (box->bnd[0] == 1 || box->bnd[1] == 1 || box->bnd[2] == 1))
        {
            const bool allPbc = box->bnd[0] == 1 && box->bnd[1] == 1 && box->bnd[2] == 1;
            const double lx = box->lim[1] - box->lim[0], ly = box->lim[3] - box->lim[2], lz = box->lim[5] - box->lim[4];
            if (!allPbc || lx != ly || lx != lz || p->propagator == 2) return SX_ERR_ARG;
        }
        auto* s   = new sx_sim;
        s->ctx    = ctx;
        s->p      = *p;
        s->box    = *box;
        s->dbox   = toDevBox(box);
        s->bucket = bucketSize;
        s->cap    = capacity;
        allocFields(s, capacity);
        if (s->p.propagator == 2) allocBdt(s);
        if (s->mem.failed())
        {
            delete s;
            return SX_ERR_NOMEM;
        }
        const char* names[] = {"sync",         "FindNeighbors", "XMass",          "VeDefGradh", "EOS",
                               "IadDivvCurlv", "AVswitches",    "MomentumEnergy", "Gravity",    "UpdateQuantities"};
        s->stageNames.assign(std::begin(names), std::end(names));
        s->ev.resize(s->stageNames.size() + 1);
        for (auto& e : s->ev)
            (void)hipEventCreate(&e);
        s->stageMs.assign(s->stageNames.size(), 0.f);
        const char* knames[] = {"findNeighbors", "xmass",          "veDefGradh", "iadDivvCurlv",
                                "avSwitches",    "momentumEnergy", "gravity"};
        s->kernelNames.assign(std::begin(knames), std::end(knames));
        s->kev.resize(2 * s->kernelNames.size());
        for (auto& e : s->kev)
            (void)hipEventCreate(&e);
        s->kernelMs.assign(s->kernelNames.size(), 0.f);
        if (hipStreamCreateWithFlags(&s->commStream, hipStreamNonBlocking) != hipSuccess) s->commStream = nullptr;
        (void)hipEventCreateWithFlags(&s->evProd, hipEventDisableTiming);
        (void)hipEventCreateWithFlags(&s->evComm, hipEventDisableTiming);
        (void)hipEventCreateWithFlags(&s->evStats, hipEventDisableTiming);
        {
            // the highest priority: its few workgroups (one per directly stale cluster) are dispatched ahead of the
            // rebuild's persistent grid instead of sharing the CUs with it (SX_SKIN_AUX_PRIO=0: default priority)
            int least = 0, greatest = 0;
            (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
            const char* ap = getenv("SX_SKIN_AUX_PRIO");
            const int   pr = ap && atoi(ap) == 0 ? least : greatest;
            if (hipStreamCreateWithPriority(&s->auxStream, hipStreamNonBlocking, pr) != hipSuccess) s->auxStream = nullptr;
        }
        (void)hipEventCreateWithFlags(&s->evAuxIn, hipEventDisableTiming);
        (void)hipEventCreateWithFlags(&s->evAuxOut, hipEventDisableTiming);
        Scalars init{1e-6, 1e-6, 0.0, INFINITY, INFINITY, 0.0, 1e10f, 0, 0.0, 0ull, 0u};
        (void)hipMemcpy(s->sc, &init, sizeof(Scalars), hipMemcpyHostToDevice);
        *out = s;
        return SX_OK;
    }

    void sx_sim_destroy(sx_sim* s)
    {
        if (!s) return;
        (void)hipDeviceSynchronize();
        for (auto& e : s->ev)
            (void)hipEventDestroy(e);
        for (auto& e : s->kev)
            (void)hipEventDestroy(e);
        if (s->evProd) (void)hipEventDestroy(s->evProd);
        if (s->evComm) (void)hipEventDestroy(s->evComm);
        if (s->evStats) (void)hipEventDestroy(s->evStats);
        if (s->commStream) (void)hipStreamDestroy(s->commStream);
        if (s->evAuxIn) (void)hipEventDestroy(s->evAuxIn);
        if (s->evAuxOut) (void)hipEventDestroy(s->evAuxOut);
        if (s->auxStream) (void)hipStreamDestroy(s->auxStream);
        delete s;
    }

    int sx_sim_set_comm(sx_sim* s, sx_comm* c)
    {
        sx::Transport* T = sx_comm_transport_internal(c);
        if (T && T->size() > 1)
        {
            // the sync's small per-rank buffers, allocated here so that no rank fails alone between two collectives
            // of a step (its peers would wait in the next one)
            const size_t P  = (size_t)T->size();
            const bool   ok = s->work.get<uint32_t>("dom.bins", size_t(1) << kHistBits) &&
                            s->work.get<uint64_t>("dom.split", P + 1) && s->work.get<uint64_t>("dom.seg", P + 1) &&
                            s->work.get<uint64_t>("dom.cnt", 2 * P) && s->work.pinned<uint64_t>("dom.cnth", 2 * P) &&
                            s->work.get<uint32_t>("dom.agree", 1) && s->work.pinned<uint32_t>("dom.agreeh", 1) &&
                            s->work.get<unsigned>("dom.hflag", 1) && s->work.pinned<unsigned>("dom.hflagh", 1) &&
                            s->work.pinned<uint32_t>("dom.errh", 1);
            if (!ok) return SX_ERR_NOMEM;
        }
        s->keysFresh  = false;
        s->skin.valid = false;
        s->comm       = T;
        s->commHandle = c;
        return SX_OK;
    }

    int sx_sim_set_overlap(sx_sim* s, int on)
    {
        s->overlap = on != 0;
        return SX_OK;
    }

    int sx_sim_overlap_stats(sx_sim* s, uint32_t out[2])
    {
        out[0] = s->nInterior;
        out[1] = s->nBoundary;
        return SX_OK;
    }

    int sx_sim_set_skin(sx_sim* s, float factor, int maxReuse)
    {
        if (!s || !(factor >= 0.0f) || factor > 1.0f || maxReuse < 1) return SX_ERR_ARG;
        s->skin.factor   = factor;
        s->skin.cur      = factor;
        s->skin.built    = factor;
        s->skin.maxReuse = maxReuse;
        s->skin.valid    = false;
        return SX_OK;
    }

    int sx_sim_rebuild_lists(sx_sim* s)
    {
        if (!s) return SX_ERR_ARG;
        s->skin.forceBuild = true;
        return SX_OK;
    }

    int sx_sim_skin_stats(sx_sim* s, uint64_t out[14])
    {
        if (!s) return SX_ERR_ARG;
        const auto& K = s->skin;
        out[0] = K.builds, out[1] = K.reuseSteps, out[2] = K.staleClusters, out[3] = K.exactClusters;
        out[4] = K.lastStale, out[5] = K.lastExact, out[6] = K.ngmaxS, out[7] = K.plainSteps;
        out[8] = (uint64_t)std::lround(1e6 * K.built), out[9] = (uint64_t)std::lround(1e6 * K.cur);
        out[10] = K.resyncs, out[11] = K.keptClusters, out[12] = K.frozenClusters, out[13] = K.earlyExact;
        return SX_OK;
    }

    int sx_sim_export_neighbors(sx_sim* s, uint32_t* out)
    {
        if (!s || !out) return SX_ERR_ARG;
        if (s->nb.first != s->first || s->nb.last != s->last || s->nb.ngmax != s->p.ngmax) return SX_ERR_ARG;
        NsArgs a{};
        a.first = (uint32_t)s->first, a.last = (uint32_t)s->last, a.ngmax = s->p.ngmax, a.nc = s->nc;
        a.setLists(s->nb);
        a.lb = s->skin.lb; // the lists the last step's pair kernels read
        hipStream_t st = (hipStream_t)sx_ctx_stream_internal(s->ctx);
        SIM_HIP(exportNeighbors(a, out, st));
        SIM_HIP(hipStreamSynchronize(st));
        return SX_OK;
    }

    size_t sx_sim_size(sx_sim* s) { return s->last - s->first; }

    int sx_sim_layout(sx_sim* s, uint64_t out[4])
    {
        out[0] = s->first;
        out[1] = s->last;
        out[2] = s->n;
        out[3] = s->haloRetries + s->bdt.haloShort;
        return SX_OK;
    }

    int sx_sim_init_sedov_rank(sx_sim* s, uint32_t side, int rank, int size)
    {
        s->keysFresh  = false;
        s->skin.valid = false;
        size_t N  = (size_t)side * side * side;
        size_t f  = N * rank / size, l = N * (rank + 1) / size;
        size_t n  = l - f;
        if (n > s->cap) return SX_ERR_ARG;
        s->n          = n;
        s->first      = 0;
        s->last       = n;
        double r      = 0.5;
        double hInit  = std::cbrt(3.0 / (4 * M_PI) * s->p.ng0 * std::pow(2 * r, 3) / N) * 0.5;
        double width  = 0.1;
        double ener0  = 1.0 / std::pow(M_PI, 1.5) / 1. / std::pow(width, 3.0);
        float  cv     = idealGasCv(s->p.muiConst, s->p.gamma);
        auto   st     = (hipStream_t)sx_ctx_stream_internal(s->ctx);
        if (n)
            sedovInitKernel<<<grid(n), 256, 0, st>>>(side, f, n, s->x, s->y, s->z, s->h, s->m, s->temp, s->vx, s->vy,
                                                     s->vz, s->xm1, s->ym1, s->zm1, s->dum1, s->alpha, s->id,
                                                     (float)hInit, (float)(1.0 / N), ener0, width * width, 1e-8, cv);
        if (s->rung && n) SIM_HIP(hipMemsetAsync(s->rung, 0, n, st));
        s->bdt.started = false;
        Scalars init{1e-6, 1e-6, 0.0, INFINITY, INFINITY, 0.0, 1e10f, 0, 0.0, 0ull, 0u};
        SIM_HIP(hipMemcpyAsync(s->sc, &init, sizeof(Scalars), hipMemcpyHostToDevice, st));
        SIM_HIP(hipStreamSynchronize(st));
        return SX_OK;
    }

    int sx_sim_init_sedov(sx_sim* s, uint32_t side) { return sx_sim_init_sedov_rank(s, side, 0, 1); }

    int sx_sim_set_state(sx_sim* s, size_t n, const double* x, const double* y, const double* z, const float* h,
                         const float* m, const double* temp, const float* vx, const float* vy, const float* vz,
                         const float* x_m1, const float* y_m1, const float* z_m1, const float* du_m1,
                         const float* alpha, const uint64_t* id, double minDt, double minDt_m1)
    {
        s->keysFresh  = false;
        s->skin.valid = false;
        if (n > s->cap) return SX_ERR_ARG;
        if (s->p.propagator == 2)
        {   // ve-bdt carries the rung in the id's top byte through the particle exchange (PRec): ids must fit 56 bits
            for (size_t i = 0; i < n; ++i)
                if (id[i] >> 56) return SX_ERR_ARG;
        }
        s->n     = n;
        s->first = 0;
        s->last  = n;
        auto cp  = [n](void* d, const void* h, size_t es) { return hipMemcpy(d, h, n * es, hipMemcpyHostToDevice); };
        SIM_HIP(cp(s->x, x, 8));
        SIM_HIP(cp(s->y, y, 8));
        SIM_HIP(cp(s->z, z, 8));
        SIM_HIP(cp(s->h, h, 4));
        SIM_HIP(cp(s->m, m, 4));
        SIM_HIP(cp(s->temp, temp, 8));
        SIM_HIP(cp(s->vx, vx, 4));
        SIM_HIP(cp(s->vy, vy, 4));
        SIM_HIP(cp(s->vz, vz, 4));
        SIM_HIP(cp(s->xm1, x_m1, 4));
        SIM_HIP(cp(s->ym1, y_m1, 4));
        SIM_HIP(cp(s->zm1, z_m1, 4));
        SIM_HIP(cp(s->dum1, du_m1, 4));
        SIM_HIP(cp(s->alpha, alpha, 4));
        SIM_HIP(cp(s->id, id, 8));
        if (s->rung) SIM_HIP(hipMemset(s->rung, 0, n));
        s->bdt.started = false;
        Scalars init{minDt, minDt_m1, 0.0, INFINITY, INFINITY, 0.0, 1e10f, 0};
        SIM_HIP(hipMemcpy(s->sc, &init, sizeof(Scalars), hipMemcpyHostToDevice));
        return SX_OK;
    }

    int sx_sim_fields(sx_sim* s, sx_fields* f, uint64_t** id)
    {
        // pointers to the LOCAL particles [first, last) of the last step
        std::memset(f, 0, sizeof(*f));
        size_t o = s->first;
        f->n     = s->last - s->first;
        f->x     = s->x + o;
        f->y     = s->y + o;
        f->z     = s->z + o;
        f->x_m1  = s->xm1 + o;
        f->y_m1  = s->ym1 + o;
        f->z_m1  = s->zm1 + o;
        f->vx    = s->vx + o;
        f->vy    = s->vy + o;
        f->vz    = s->vz + o;
        f->prho  = s->prho + o;
        f->rho   = s->rho ? s->rho + o : nullptr;
        f->p     = s->pres ? s->pres + o : nullptr;
        f->h     = s->h + o;
        f->m     = s->m + o;
        f->c     = s->c + o;
        f->ax    = s->ax + o;
        f->ay    = s->ay + o;
        f->az    = s->az + o;
        f->du    = s->du + o;
        f->du_m1 = s->dum1 + o;
        f->c11   = s->c11 + o;
        f->c12   = s->c12 + o;
        f->c13   = s->c13 + o;
        f->c22   = s->c22 + o;
        f->c23   = s->c23 + o;
        f->c33   = s->c33 + o;
        f->temp  = s->temp + o;
        f->xm    = s->xm + o;
        f->kx    = s->kx + o;
        f->divv  = s->divv + o;
        f->curlv = s->curlv + o;
        f->alpha = s->alpha + o;
        f->gradh = s->gradh + o;
        f->keys  = s->keys + o;
        f->nc    = s->nc + o;
        f->rung  = s->rung ? s->rung + o : nullptr;
        if (s->dV[0])
        {
            f->dV11 = s->dV[0] + o, f->dV12 = s->dV[1] + o, f->dV13 = s->dV[2] + o;
            f->dV22 = s->dV[3] + o, f->dV23 = s->dV[4] + o, f->dV33 = s->dV[5] + o;
        }
        if (id) *id = s->id + o;
        return SX_OK;
    }

    int sx_sim_conserved(sx_sim* s, double out[13])
    {
        hipStream_t   st = (hipStream_t)sx_ctx_stream_internal(s->ctx);
        ConservedArgs a{s->first, s->last, s->x, s->y, s->z, s->vx, s->vy, s->vz, s->m, s->temp, nullptr, s->nc,
                        (double)idealGasCv(s->p.muiConst, s->p.gamma)};
        double* scratch = s->work.get<double>("obs.scratch", conservedScratch(s->last - s->first));
        double* q       = s->work.get<double>("obs.q", 10);
        SIM_HIP(conservedQuantities(a, scratch, q, st));
        // egrav of the last step joins the sum (computeConservedQuantities, conserved_quantities.hpp:145-153)
        SIM_HIP(hipMemcpyAsync(q + 9, &s->sc->egrav, 8, hipMemcpyDeviceToDevice, st));
        if (s->comm && s->comm->size() > 1) SIM_COMM(s->comm->allreduceSumF64(q, 10, st));
        double h[10];
        SIM_HIP(hipMemcpyAsync(h, q, sizeof(h), hipMemcpyDeviceToHost, st));
        SIM_HIP(hipStreamSynchronize(st));
        const double ecin = h[0], eint = h[1], egrav = h[9];
        out[0] = ecin, out[1] = eint, out[2] = egrav, out[3] = ecin + eint + egrav;
        out[4] = std::sqrt(h[2] * h[2] + h[3] * h[3] + h[4] * h[4]);
        out[5] = std::sqrt(h[5] * h[5] + h[6] * h[6] + h[7] * h[7]);
        out[6] = h[8];
        for (int k = 0; k < 6; ++k)
            out[7 + k] = h[2 + k];
        return SX_OK;
    }

    int sx_sim_set_gravity_counting(sx_sim* s, int enable)
    {
        if (!s || s->p.g == 0.0) return SX_ERR_ARG;
        // the ve-bdt substeps (sx_bdt.cpp) do not count: refusing beats zeros that read as valid counts
        if (enable && s->p.propagator == 2) return SX_ERR_ARG;
        s->gravCount = enable != 0;
        if (s->gravCount)
        {
            // counts of a step without counting read as zeros, not as stale values
            hipStream_t st = (hipStream_t)sx_ctx_stream_internal(s->ctx);
            SIM_HIP(hipMemsetAsync(s->work.get<unsigned long long>("grav.inter", 2), 0, 16, st));
        }
        return SX_OK;
    }

    int sx_sim_gravity_interactions(sx_sim* s, uint64_t out[2])
    {
        if (!s || s->p.g == 0.0) return SX_ERR_ARG;
        if (!s->gravCount)
        {
            out[0] = out[1] = 0;
            return SX_OK;
        }
        hipStream_t st = (hipStream_t)sx_ctx_stream_internal(s->ctx);
        SIM_HIP(hipMemcpyAsync(out, s->work.get<unsigned long long>("grav.inter", 2), 16, hipMemcpyDeviceToHost, st));
        SIM_HIP(hipStreamSynchronize(st));
        return SX_OK;
    }

    int sx_sim_gravity_stats(sx_sim* s, uint64_t out[3])
    {
        out[0] = s->gravHalos;
        out[1] = s->gravFarCells;
        out[2] = s->gravRemoteCells;
        return SX_OK;
    }

    int sx_sim_step(sx_sim* s)
    {
        if (s->p.propagator == 2) return stepBdt(s);
        hipStream_t        st  = (hipStream_t)sx_ctx_stream_internal(s->ctx);
        const HydroLaunch& H   = sx_ctx_exact_internal(s->ctx) ? hydro_exact() : hydro_fast();
        const bool         dist = s->comm && s->comm->size() > 1;
        int                ev  = 0;
        SIM_HIP(hipEventRecord(s->ev[ev++], st));

        // skin lists (sx_skin.hpp): a reuse step keeps the order and tree of the last full build and filters the
        // skin lists instead of syncing and searching
        bool skinOn = skinUsable(s);
        if (skinOn && s->skin.backoff > 0)
        {
            s->skin.backoff--;
            s->skin.plainSteps++;
            skinOn = false;
        }
        bool reuse = skinOn && s->skin.valid && !s->skin.forceBuild && s->skin.sinceBuild < s->skin.maxReuse;
        if (!skinOn) s->skin.valid = false;
        // h before a reuse step's filter (its h iteration), for a search redone from a full sync (kSkinResync)
        float* hReuse = reuse ? s->mem.get<float>("skin.h0", s->cap) : nullptr;
        if (reuse && !hReuse) return SX_ERR_NOMEM;
        if (reuse) SIM_HIP(hipMemcpyAsync(hReuse, s->h + s->first, (s->last - s->first) * 4, hipMemcpyDeviceToDevice, st));
        bool synced = false;
        // h before the h iteration, to redo the search if the halo margin proves too small
        float* h0     = dist ? s->work.get<float>("h0", s->cap) : nullptr;
        double margin = kHaloMargin;
        NsArgs na{};
        bool   restoreH0 = false; // a retry with a larger halo margin: the locals' h as before the last search
        SkinCounts skc{};
        for (int attempt = 0;; ++attempt)
        {
            // a skin build requests its halos within the skin radius: the build's lists see every particle within
            // 2 h (1 + s) of a target (several ranks)
            const double skinMargin = skinOn ? 1.0 + (double)s->skin.cur : 1.0;
            if (dist && reuse)
            {
                if (int e = skinHaloRefresh(s, st)) return e;
            }
            else if (dist)
            {
                // restore pre-iteration h of the locals, then rediscover halos with a larger margin
                if (restoreH0)
                    SIM_HIP(hipMemcpyAsync(s->h + s->first, h0, (s->last - s->first) * 4, hipMemcpyDeviceToDevice, st));
                if (int e = distributedSync(s, st, margin * skinMargin)) return e;
                SIM_HIP(hipMemcpyAsync(h0, s->h + s->first, (s->last - s->first) * 4, hipMemcpyDeviceToDevice, st));
            }
            else if (!reuse && !synced)
            {
                if (int e = localSync(s, st)) return e;
                synced = true;
            }
            if (attempt == 0) SIM_HIP(hipEventRecord(s->ev[ev++], st));

            // ---- neighbors + h iteration on the local targets --------------------------------------------
            na.first          = (uint32_t)s->first;
            na.last           = (uint32_t)s->last;
            na.numGroups      = (uint32_t)((s->last - s->first + kGroupSize - 1) / kGroupSize);
            na.ngmax          = s->p.ngmax;
            na.ng0            = s->p.ng0;
            na.iterateH       = 1;
            na.x              = s->x;
            na.y              = s->y;
            na.z              = s->z;
            na.h              = s->h;
            na.nc             = s->nc;
            if (!s->nb.reserve(s->mem, (uint32_t)s->first, (uint32_t)s->last, s->p.ngmax, true)) return SX_ERR_NOMEM;
            na.setLists(s->nb);
            na.childOffsets   = s->tree.childOffsets;
            na.internalToLeaf = s->tree.internalToLeaf;
            na.layout         = s->tree.layout;
            na.centers        = s->tree.centers;
            na.sizes          = s->tree.sizes;
            na.box            = s->dbox;
            na.margin         = quantMargin(s->dbox);
            na.stats          = s->stats;
            na.powTab         = sx_ctx_powtab_internal(s->ctx, s->p.ng0);
            na.prefilter      = 1;
            na.hSave          = s->mem.get<float>("ns.hsave", std::max<size_t>(2 * ((s->last - s->first) / kCluster + 2), s->last - s->first)); // the two redo lists
            na.policy         = &s->nsPolicy;
            na.clStats        = s->mem.get<uint4>("ns.clstats", (na.numGroups + kClusterWaves - 1) / kClusterWaves);
            na.work           = s->mem.get<uint32_t>("ns.work", 16);
            na.hitMasks       = s->mem.get<uint64_t>("ns.masks", searchScratchBytes() / sizeof(uint64_t));
            na.rxOut          = s->rx; // the locals' RecX: packed by the search itself (packXHalos below)
            na.m              = s->m;
            if (!na.hSave || !na.clStats || !na.work || !na.hitMasks) return SX_ERR_NOMEM;
            if (const char* reps = getenv("SX_SEARCH_REPS"); reps && attempt == 0)
            {
                // timing hook for search A/B runs (scripts/ab_search.sh): the search without the h iteration,
                // repeated on this step's state before the real search
                NsArgs x     = na;
                x.iterateH   = 0;
                NsPolicy pol;
                pol.mode = getenv("SX_SEARCH_LARGE") ? 1 : 2; // compact build first (as in the real search)
                x.policy = &pol;
                const int R  = std::max(1, atoi(reps));
                s->skin.listsKept = false; // this search rewrites the exact lists
                s->skin.lb        = ListsB{};
                SIM_HIP(hipEventRecord(s->kev[0], st));
                for (int r = 0; r < R; ++r)
                {
                    SIM_HIP(hipMemsetAsync(s->stats, 0, kStatsWords * 4, st));
                    SIM_HIP(findNeighbors(x, st));
                }
                SIM_HIP(hipEventRecord(s->kev[1], st));
                SIM_HIP(hipEventSynchronize(s->kev[1]));
                float ms = 0;
                (void)hipEventElapsedTime(&ms, s->kev[0], s->kev[1]);
                fprintf(stderr, "search-reps: %.3f ms per search (%d reps)\n", ms / R, R);
            }
            SIM_HIP(hipMemsetAsync(s->stats, 0, kStatsWords * 4, st));
            resetScalarsKernel<<<1, 1, 0, st>>>(s->sc);
            SIM_HIP(hipEventRecord(s->kev[0], st));
            bool resync = false; // this rank's reuse step must be redone from a full sync + build
            if (skinOn)
            {
                // the fast variant's XMass (or the std density's xmass pass) rides on the filter's final pass
                const bool fastXm = !sx_ctx_exact_internal(s->ctx);
                float*     xmOut  = fastXm ? (s->p.propagator == 1 ? s->rho : s->xm) : nullptr;
                // no RecT {xm} for the locals: VeDefGradh reads xm from the dense field and writes the records
                RecT*      rtXm   = nullptr;
                const int e = skinSearch(s, na, reuse, st, xmOut, rtXm, skc);
                resync      = e == kSkinResync;
                if (e && !resync) return e;
                if (!dist)
                {
                    if (resync)
                    {
                        // h as before the filter, then this step's search again after a full sync + build
                        SIM_HIP(hipMemcpyAsync(s->h + s->first, hReuse, (s->last - s->first) * 4,
                                               hipMemcpyDeviceToDevice, st));
                        s->skin.resyncs++;
                        if (s->skin.cleanSinceBuild < 2) skinTooThin(s->skin);
                        reuse = false;
                        continue;
                    }
                    skinDecide(s->skin, reuse, skc, skc.stale, skc.clusters);
                    s->skin.stepClusters = skc.clusters;
                }
            }
            else
            {
                s->skin.xmFused   = false;
                s->skin.listsKept = false;
                s->skin.lb        = ListsB{}; // the plain search writes the primary set
                SIM_HIP(findNeighbors(na, st));
            }
            SIM_HIP(hipEventRecord(s->kev[1], st));
            SIM_HIP(hipMemcpyAsync(s->statsHost, s->stats, kStatsWords * 4, hipMemcpyDeviceToHost, st));
            if (s->evStats) SIM_HIP(hipEventRecord(s->evStats, st));
            if (!dist) break;
            // halo sufficiency: every local particle's final h within its chunk's request margin (a build or a plain
            // search); on a reuse step, the spheres of the clusters searched again this step (coverListKernel).
            // One exchange of five words carries every decision the ranks take together: [0] halo margin too small,
            // [1] the reuse step must be redone from a full sync + build, [2] stale clusters, [3] clusters, [4] clusters
            // whose skin would not survive another such drift (the filter's stats[13])
            const size_t nl  = s->last - s->first;
            auto*        flg = s->work.get<unsigned>("dom.hflag", 5);
            uint32_t*    dec = s->work.pinned<uint32_t>("dom.dech", 8);
            if (!flg || !dec) return SX_ERR_NOMEM;
            dec[0] = 0, dec[1] = resync ? 1u : 0u, dec[2] = skc.stale, dec[3] = skc.clusters, dec[4] = 0;
            SIM_HIP(hipMemcpyAsync(flg, dec, 5 * 4, hipMemcpyHostToDevice, st));
            const ReqBox* myBoxes = s->work.get<ReqBox>("dom.mybox", 1);
            if (!reuse)
            {
                if (nl)
                    chunkCheckKernel<<<grid(nl), 256, 0, st>>>(s->h + s->first, nl, myBoxes, margin * skinMargin, flg);
            }
            else
            {
                const double qm = quantMargin(s->dbox);
                if (skc.rebuilt)
                    coverListKernel<<<skc.rebuilt, kCluster, 0, st>>>(
                        s->mem.get<uint32_t>("skin.l1", 1), skc.rebuilt, (uint32_t)s->first, (uint32_t)s->last, s->x,
                        s->y, s->z, s->mem.get<float>("skin.hb", 1), 1.0f + s->skin.built, myBoxes, s->dbox, qm,
                        flg + 1);
                if (skc.exact)
                    coverListKernel<<<skc.exact, kCluster, 0, st>>>(s->mem.get<uint32_t>("skin.l2", 1), skc.exact,
                                                                    (uint32_t)s->first, (uint32_t)s->last, s->x, s->y,
                                                                    s->z, s->h, 1.0f, myBoxes, s->dbox, qm, flg + 1);
            }
            if (skinOn) SIM_HIP(hipMemcpyAsync(flg + 4, s->stats + 13, 4, hipMemcpyDeviceToDevice, st));
            unsigned hf = 0;
            // the retry decision must be global: a rank redoing the sync alone would deadlock the collectives
            SIM_COMM(s->comm->allreduceSumU32(flg, 5, st));
            SIM_HIP(hipMemcpyAsync(dec, flg, 5 * 4, hipMemcpyDeviceToHost, st));
            if (overlapping(s, H))
            {
                const uint32_t ncl = (uint32_t)((nl + kCluster - 1) / kCluster);
                s->clsList         = s->work.get<uint32_t>("ovl.list", 2 * (size_t)std::max(1u, ncl));
                s->clsCount        = s->work.get<uint32_t>("ovl.count", 2);
                SIM_HIP(hipMemsetAsync(s->clsCount, 0, 8, st));
                if (ncl)
                    classifyClustersKernel<<<(ncl + 3) / 4, 256, 0, st>>>(s->nb.uni, s->nb.ucount, s->nb.ucap,
                                                                         s->skin.lb, (uint32_t)s->first,
                                                                         (uint32_t)s->last, ncl, s->clsList,
                                                                         s->clsCount);
                SIM_HIP(hipMemcpyAsync(s->clsHost, s->clsCount, 8, hipMemcpyDeviceToHost, st));
            }
            if (int e = syncErrEnqueue(s, st)) return e;
            SIM_HIP(hipStreamSynchronize(st));
            if (syncErrFailed(s)) return SX_ERR_TRAVERSAL;
            if (overlapping(s, H)) s->nInterior = s->clsHost[0], s->nBoundary = s->clsHost[1];
            hf                = dec[0];
            s->statsHost[3]   = hf;
            if (skinOn && dec[1])
            {
                // some rank's reuse step cannot stand (a sphere searched again outside the build's halo region, or
                // the exact search over capacity): every rank restores h and redoes the step from a full sync + build
                SIM_HIP(hipMemcpyAsync(s->h + s->first, hReuse, (s->last - s->first) * 4, hipMemcpyDeviceToDevice, st));
                s->skin.resyncs++;
                if (s->skin.cleanSinceBuild < 2) skinTooThin(s->skin);
                reuse     = false;
                restoreH0 = false;
                continue;
            }
            if (hf)
            {
                if (attempt >= 3) return SX_ERR_NOT_CONVERGED;
                margin *= 1.5;
                restoreH0 = true;
                s->haloRetries++;
                continue;
            }
            if (skinOn)
            {
                skinDecide(s->skin, reuse, skc, dec[2], dec[3]);
                s->skin.stepClusters = dec[3];
                s->skin.stepS13      = dec[4];
            }
            break;
        }
        SIM_HIP(hipEventRecord(s->ev[ev++], st));

        const size_t n  = s->n;
        PairArgs     pa = simPairArgs(s);
        if (s->p.propagator == 1)
        {
            // ---- HydroProp::computeForces (std_hydro.hpp:124-166): density, EOS, [v,rho,p,c] halos, IAD,
            //      [c_ij] halos, momentum + energy.  The stage/kernel event slots follow the VE order:
            //      density in "xmass", IAD in "iadDivvCurlv", momentumEnergySTD in "momentumEnergy".
            packXHalos(s, st);
            SIM_HIP(hipEventRecord(s->kev[2], st));
            PairArgs da = pa;
            da.xm       = s->rho; // computeDensity: xmass written to rho (xmass_gpu.cu:151-153)
            xmassRest(s, H, da, st);
            H.xmassToRho((uint32_t)s->first, (uint32_t)s->last, s->m, s->rho, st);
            SIM_HIP(hipEventRecord(s->kev[3], st));
            SIM_HIP(hipEventRecord(s->ev[ev++], st));
            SIM_HIP(hipEventRecord(s->kev[4], st));
            SIM_HIP(hipEventRecord(s->kev[5], st));
            EosArgs ea{(uint32_t)s->first, (uint32_t)s->last, s->p.muiConst, s->p.gamma, s->temp, s->m, nullptr, nullptr,
                       nullptr, nullptr, s->c, s->rho, s->pres};
            H.eosStd(ea, st);
            SIM_HIP(hipEventRecord(s->ev[ev++], st));
            SIM_HIP(hipEventRecord(s->ev[ev++], st));
            SIM_HIP(hipEventRecord(s->kev[6], st));
            if (int e = exchangeThen(
                    s, H, {{s->vx, 4}, {s->vy, 4}, {s->vz, 4}, {s->rho, 4}, {s->pres, 4}, {s->c, 4}},
                    [&](size_t a, size_t b)
                    {
                        packV(b - a, s->vx + a, s->vy + a, s->vz + a, s->c + a, s->rv + a, st);
                        packS(b - a, s->rho + a, s->pres + a, s->rs + a, st);
                    },
                    [&](const PairArgs& p) { H.iadStd(p, st); }, pa, st))
                return e;
            SIM_HIP(hipEventRecord(s->kev[7], st));
            SIM_HIP(hipEventRecord(s->ev[ev++], st));
            SIM_HIP(hipEventRecord(s->kev[8], st));
            SIM_HIP(hipEventRecord(s->kev[9], st));
            SIM_HIP(hipEventRecord(s->ev[ev++], st));
            SIM_HIP(hipEventRecord(s->kev[10], st));
            if (int e = exchangeThen(
                    s, H, {{s->c11, 4}, {s->c12, 4}, {s->c13, 4}, {s->c22, 4}, {s->c23, 4}, {s->c33, 4}},
                    [&](size_t a, size_t b)
                    {
                        packC(b - a, s->c11 + a, s->c12 + a, s->c13 + a, s->c22 + a, s->c23 + a, s->c33 + a, nullptr,
                              s->rc + a, st);
                    },
                    [&](const PairArgs& p) { H.momentumStd(p, st); }, pa, st))
                return e;
            SIM_HIP(hipEventRecord(s->kev[11], st));
            SIM_HIP(hipEventRecord(s->ev[ev++], st));
        }
        else
        {
            // ---- XMass
            packXHalos(s, st);
            // the cluster kernels write the locals' records as they produce them (PairArgs::rtOut / rcOut, EosArgs):
            // the packing passes below then cover only the halos (halo()); the exact kernels leave it to them
            // only the cluster kernels write records; they run when the lists are in the local (union) format, and
            // ngmax > 256 keeps the global format, whose gather kernels read packed records of every particle
            const bool fused = H.clusterLists && pa.localLists && !pa.active;
            auto       halo  = [&](size_t a, size_t b, auto&& fn) {
                if (!fused) return fn(a, b);
                if (a < s->first) fn(a, std::min(b, (size_t)s->first));
                if (b > s->last) fn(std::max(a, (size_t)s->last), b);
            };
            SIM_HIP(hipEventRecord(s->kev[2], st));
            {
                PairArgs xa = pa;
                xa.rtOut    = fused ? s->rt : nullptr;
                xmassRest(s, H, xa, st);
            }
            SIM_HIP(hipEventRecord(s->kev[3], st));
            // ---- [xm] halos, VeDefGradh (overlapped: interior clusters while the halos are in flight)
            SIM_HIP(hipEventRecord(s->ev[ev++], st));
            SIM_HIP(hipEventRecord(s->kev[4], st));
            // the cluster VeDefGradh also runs the EOS of its targets (PairArgs::eos): kx and gradh stay in registers
            PairArgs va = pa;
            if (fused)
                va.eos = EosFuse{s->temp,  (double)idealGasCv(s->p.muiConst, s->p.gamma), s->p.gamma, s->prho, s->c,
                                 s->vx,    s->vy, s->vz, s->alpha, s->rv, s->rt};
            if (int e = exchangeThen(
                    s, H, {{s->xm, 4}},
                    [&](size_t a, size_t b)
                    {
                        halo(a, b, [&](size_t u, size_t v)
                             { packT(v - u, s->xm + u, nullptr, nullptr, nullptr, s->rt + u, st); });
                    },
                    [&](const PairArgs& p) { H.veDefGradh(p, st); }, va, st))
                return e;
            SIM_HIP(hipEventRecord(s->kev[5], st));
            SIM_HIP(hipEventRecord(s->ev[ev++], st));
            // ---- EOS (unless fused above), then the v/prho/c/kx halo exchange
            if (!fused)
            {
                EosArgs ea{(uint32_t)s->first, (uint32_t)s->last, s->p.muiConst, s->p.gamma, s->temp, s->m, s->kx,
                           s->xm, s->gradh, s->prho, s->c, nullptr, nullptr};
                H.eos(ea, st);
            }
            SIM_HIP(hipEventRecord(s->ev[ev++], st));
            // ---- [v, prho, c, kx] halos, IAD + divv/curlv, rho time-step
            auto packVT = [&](size_t a, size_t b)
            {
                halo(a, b,
                     [&](size_t u, size_t v)
                     {
                         packV(v - u, s->vx + u, s->vy + u, s->vz + u, s->c + u, s->rv + u, st);
                         packT(v - u, s->xm + u, s->kx + u, s->prho + u, s->alpha + u, s->rt + u, st);
                     });
            };
            pa.rcOut = fused ? s->rc : nullptr; // IAD writes the locals' {c_ij, divv}
            SIM_HIP(hipEventRecord(s->kev[6], st));
            if (int e = exchangeThen(s, H, {{s->vx, 4}, {s->vy, 4}, {s->vz, 4}, {s->prho, 4}, {s->c, 4}, {s->kx, 4}},
                                     packVT, [&](const PairArgs& p) { H.iadDivvCurlv(p, st); }, pa, st))
                return e;
            SIM_HIP(hipEventRecord(s->kev[7], st));
            SIM_HIP(maxFloat(s->divv, (uint32_t)s->first, (uint32_t)s->last, &s->sc->maxDivvU, st));
            SIM_HIP(hipEventRecord(s->ev[ev++], st));
            // ---- [c_ij, divv] halos, AV switches
            SIM_HIP(hipEventRecord(s->kev[8], st));
            if (int e = exchangeThen(
                    s, H, {{s->c11, 4}, {s->c12, 4}, {s->c13, 4}, {s->c22, 4}, {s->c23, 4}, {s->c33, 4}, {s->divv, 4}},
                    [&](size_t a, size_t b)
                    {
                        halo(a, b,
                             [&](size_t u, size_t v)
                             {
                                 packC(v - u, s->c11 + u, s->c12 + u, s->c13 + u, s->c22 + u, s->c23 + u, s->c33 + u,
                                       s->divv + u, s->rc + u, st, s->xm + u, s->kx + u);
                             });
                    },
                    [&](const PairArgs& p)
                    {
                        PairArgs q = p;
                        q.rcOut    = nullptr;
                        q.rtOut    = fused ? s->rt : nullptr; // AV writes the locals' records with the new alpha
                        // the largest union of this step's search: the host waits here for the search to finish
                        // (long done on the device when the kernels queued before AV still run, so nothing idles)
                        if (s->evStats && hipEventSynchronize(s->evStats) == hipSuccess) q.unionMax = s->statsHost[12];
                        H.avSwitches(q, st);
                    },
                    pa, st))
                return e;
            pa.rcOut = nullptr;
            SIM_HIP(hipEventRecord(s->kev[9], st));
            SIM_HIP(hipEventRecord(s->ev[ev++], st));
            // ---- [alpha (+ dV)] halos, momentum + energy.  With avClean the reference exchanges dV11,dV12,dV22,
            //      dV23,dV33 + alpha (ve_hydro.hpp:182-185) and leaves the halo dV13 undefined; all six are exchanged
            //      here so the result does not depend on the decomposition
            auto packTa = [&](size_t a, size_t b)
            {
                halo(a, b, [&](size_t u, size_t v)
                     { packT(v - u, s->xm + u, s->kx + u, s->prho + u, s->alpha + u, s->rt + u, st); });
            };
            auto launchMe = [&](const PairArgs& p) { H.momentumEnergy(p, st); };
            SIM_HIP(hipEventRecord(s->kev[10], st));
            if (s->p.avClean)
            {
                if (int e = exchangeThen(s, H,
                                         {{s->dV[0], 4}, {s->dV[1], 4}, {s->dV[2], 4}, {s->dV[3], 4}, {s->dV[4], 4},
                                          {s->dV[5], 4}, {s->alpha, 4}},
                                         packTa, launchMe, pa, st))
                    return e;
            }
            else if (int e = exchangeThen(s, H, {{s->alpha, 4}}, packTa, launchMe, pa, st)) return e;
            SIM_HIP(hipEventRecord(s->kev[11], st));
            SIM_HIP(hipEventRecord(s->ev[ev++], st));
        }
        // ---- self-gravity (ve_hydro.hpp:193-202): upsweep + traversal on the step's tree, added to ax, ay, az
        SIM_HIP(hipEventRecord(s->kev[12], st));
        if (s->p.g != 0.0)
        {
            // P2P, M2P of this step (BhStats), counted only on request (sx_sim_set_gravity_counting)
            auto* inter = s->gravCount ? s->work.get<unsigned long long>("grav.inter", 2) : nullptr;
            if (inter) SIM_HIP(hipMemsetAsync(inter, 0, 2 * sizeof(unsigned long long), st));
            if (dist)
            {
                if (int e = distributedGravity(s, st, nullptr, reuse)) return e;
            }
            else
            {
            GravArgs ga{};
            ga.first          = (uint32_t)s->first;
            ga.last           = (uint32_t)s->last;
            ga.numLeaves      = s->tree.numLeaves;
            ga.numNodes       = s->tree.numNodes;
            ga.childOffsets   = s->tree.childOffsets;
            ga.internalToLeaf = s->tree.internalToLeaf;
            ga.layout         = s->tree.layout;
            ga.geoCenters     = s->tree.centers;
            ga.geoSizes       = s->tree.sizes;
            if (reuse)
            {
                // no sync this step: particles may have left their cells; the MAC takes boxes that hold both
                double* gc3 = s->work.get<double>("grav.geoC", 3 * (size_t)s->tree.numNodes);
                double* gs3 = s->work.get<double>("grav.geoS", 3 * (size_t)s->tree.numNodes);
                if (!gc3 || !gs3) return SX_ERR_NOMEM;
                SIM_HIP(skinRefreshBoxes(s->tree, s->x, s->y, s->z, s->dbox, gc3, gs3, st, true));
                ga.geoCenters = gc3;
                ga.geoSizes   = gs3;
            }
            ga.leafToNode     = s->work.get<int32_t>("grav.leafToNode", (size_t)s->tree.numLeaves);
            ga.x = s->x, ga.y = s->y, ga.z = s->z, ga.m = s->m, ga.h = s->h;
            ga.centers4   = s->work.get<double>("grav.centers", 4 * (size_t)s->tree.numNodes);
            ga.multipoles = s->work.get<float>("grav.multipoles", 8 * (size_t)s->tree.numNodes);
            ga.G          = (float)s->p.g;
            ga.invTheta   = 1.0f / s->p.theta;
            ga.ax = s->ax, ga.ay = s->ay, ga.az = s->az;
            ga.egrav = &s->sc->egrav;
            ga.err   = &s->sc->gravErr;
            ga.fast  = sx_ctx_exact_internal(s->ctx) ? 0 : 1;
            ga.interactions = inter;
            SIM_HIP(gravityUpsweep(ga, s->tree.levelRangeHost.data(), st));
            ga.waveE = s->work.get<double>("grav.waveE", (ga.last - ga.first + kWave - 1) / kWave + 1);
            const bool pbc = periodicGravity(s);
            if (pbc)
            {
                // periodic (gravity_wrapper.hpp:135-157): the walk over one image shell, then the Ewald correction
                // with the reference's EwaldSettings defaults (ewald.h:17-21)
                ga.numShells = 1;
                ga.boxL[0] = s->box.lim[1] - s->box.lim[0], ga.boxL[1] = s->box.lim[3] - s->box.lim[2];
                ga.boxL[2] = s->box.lim[5] - s->box.lim[4];
                ga.interactions = nullptr;
            }
            SIM_HIP(gravityTraverse(ga, st));
            if (pbc)
            {
                double c4[4];
                float  m8[8];
                SIM_HIP(hipMemcpyAsync(c4, ga.centers4, sizeof(c4), hipMemcpyDeviceToHost, st));
                SIM_HIP(hipMemcpyAsync(m8, ga.multipoles, sizeof(m8), hipMemcpyDeviceToHost, st));
                SIM_HIP(hipStreamSynchronize(st));
                if (int e = ewaldStep(s, c4, m8, nullptr, st)) return e;
            }
            }
            maxAccSq(s, st);
        }
        SIM_HIP(hipEventRecord(s->kev[13], st));
        SIM_HIP(hipEventRecord(s->ev[ev++], st));
        // ---- integrate: global time-step, positions, h
        dtCandidateKernel<<<1, 1, 0, st>>>(s->sc, s->p.Krho, s->p.maxDtIncrease, s->p.g, s->p.eps, s->p.etaAcc,
                                           s->p.propagator != 1);
        if (dist) SIM_COMM(s->comm->allreduceMinF64(&s->sc->dtCand, 1, st));
        dtApplyKernel<<<1, 1, 0, st>>>(s->sc);
        PosArgs qa{};
        qa.first   = (uint32_t)s->first;
        qa.last    = (uint32_t)s->last;
        qa.dtPtr   = &s->sc->minDt;
        qa.box     = s->dbox;
        qa.x       = s->x;
        qa.y       = s->y;
        qa.z       = s->z;
        qa.x_m1    = s->xm1;
        qa.y_m1    = s->ym1;
        qa.z_m1    = s->zm1;
        qa.vx      = s->vx;
        qa.vy      = s->vy;
        qa.vz      = s->vz;
        qa.ax      = s->ax;
        qa.ay      = s->ay;
        qa.az      = s->az;
        qa.temp    = s->temp;
        qa.du      = s->du;
        qa.du_m1   = s->dum1;
        qa.h       = s->h;
        qa.constCv = idealGasCv(s->p.muiConst, s->p.gamma);
        // one rank: the next localSync's keys come from this pass (the coordinates are in registers here)
        // (not when the next step will be served by the skin filter: it does not sync; should it resync after all,
        // localSync computes the keys itself, keysFresh being false)
        const SkinState& K = s->skin;
        const bool reuseNext = skinOn && K.valid && !K.forceBuild && K.sinceBuild < K.maxReuse && K.backoff == 0;
        qa.keys    = (!dist && s->p.propagator != 2 && !reuseNext) ? s->keys : nullptr;
        if (skinOn && !skinParticleBuffers(s, qa, st)) return SX_ERR_NOMEM;
        H.positions(qa, st);
        s->keysFresh = qa.keys != nullptr;
        H.updateH((uint32_t)s->first, (uint32_t)s->last, s->p.ng0, s->nc, s->h, na.powTab, st);
        SIM_HIP(hipEventRecord(s->ev[ev++], st));
        SIM_HIP(hipGetLastError());
        SIM_HIP(hipStreamSynchronize(st));

        for (size_t k = 0; k < s->stageMs.size(); ++k)
            (void)hipEventElapsedTime(&s->stageMs[k], s->ev[k], s->ev[k + 1]);
        for (size_t k = 0; k < s->kernelMs.size(); ++k)
            (void)hipEventElapsedTime(&s->kernelMs[k], s->kev[2 * k], s->kev[2 * k + 1]);
        s->lastStats.numFailed     = s->statsHost[1];
        s->lastStats.maxNeighbors  = s->statsHost[2];
        s->lastStats.sumNeighbors  = *reinterpret_cast<uint64_t*>(s->statsHost + 4);
        s->lastStats.sumCandidates = *reinterpret_cast<uint64_t*>(s->statsHost + 6);
        s->lastStats.sumUnion      = *reinterpret_cast<uint64_t*>(s->statsHost + 8);
        s->lastStats.maxUnion      = s->statsHost[12];
        if (skinOn && reuse) s->skin.keptClusters += s->statsHost[18], s->skin.frozenClusters += s->statsHost[19];
        s->nsPolicy.observe(s->statsHost, (uint32_t)(s->last - s->first));
        if (reuse && s->skin.cleanSinceBuild <= 1 && !s->skin.forceBuild)
        {
            // the first clean step after a build, but most clusters would not survive another such drift: the skin
            // cannot outlast two steps; stop using it now rather than after a stale-heavy step (several ranks: the
            // counts of all ranks, exchanged with the step's decisions)
            const double s13 = dist ? (double)s->skin.stepS13 : (double)s->statsHost[13];
            if (s13 > s->skin.staleLimit * (double)s->skin.stepClusters) skinTooThin(s->skin);
        }
        s->lastStats.build         = s->nsPolicy.lastBuild;
        if (s->statsHost[0] & 1u)
        {
            fprintf(stderr, "sx_sim_step: neighbor search capacity exceeded (flags 0x%x: 2 walk capacity -- 0x40 traversal "
                            "queue, 0x20 candidate leaves, 0x10 search regions --, 4 candidate space, 8 union); cluster %d: %u "
                            "candidate leaves, %u search regions\n",
                    s->statsHost[0], (int)s->statsHost[14] - 1, s->statsHost[15], s->statsHost[16]);
            return SX_ERR_TRAVERSAL;
        }
        if (s->p.g != 0.0)
        {
            SIM_HIP(hipMemcpy(s->scHost, s->sc, sizeof(Scalars), hipMemcpyDeviceToHost));
            if (s->scHost->gravErr)
            {
                fprintf(stderr, "sx_sim_step: GPU traversal stack exhausted in Barnes-Hut\n");
                return SX_ERR_TRAVERSAL;
            }
        }
        return SX_OK;
    }

    int sx_sim_set_time(sx_sim* s, double ttot)
    {
        if (!s) return SX_ERR_ARG;
        hipStream_t st = (hipStream_t)sx_ctx_stream_internal(s->ctx);
        SIM_HIP(hipMemcpyAsync(s->scHost, s->sc, sizeof(Scalars), hipMemcpyDeviceToHost, st));
        SIM_HIP(hipStreamSynchronize(st));
        s->scHost->ttot = ttot;
        SIM_HIP(hipMemcpyAsync(s->sc, s->scHost, sizeof(Scalars), hipMemcpyHostToDevice, st));
        SIM_HIP(hipStreamSynchronize(st));
        s->bdt.ttot = ttot; // ve-bdt keeps d.ttot on the host between substeps
        return SX_OK;
    }

    int sx_sim_scalars(sx_sim* s, double out[6])
    {
        hipStream_t st = (hipStream_t)sx_ctx_stream_internal(s->ctx);
        SIM_HIP(hipMemcpyAsync(s->scHost, s->sc, sizeof(Scalars), hipMemcpyDeviceToHost, st));
        SIM_HIP(hipStreamSynchronize(st));
        out[0] = s->scHost->minDt;
        out[1] = s->scHost->minDt_m1;
        out[2] = s->scHost->ttot;
        out[3] = s->scHost->minDtCourant;
        out[4] = s->scHost->minDtRho;
        out[5] = s->scHost->egrav;
        return SX_OK;
    }

    int sx_sim_kernel_times(sx_sim* s, float* ms, int cap, const char** names)
    {
        int k = 0;
        for (; k < cap && k < (int)s->kernelMs.size(); ++k)
        {
            ms[k] = s->kernelMs[k];
            if (names) names[k] = s->kernelNames[k].c_str();
        }
        return k;
    }

    int sx_sim_stage_times(sx_sim* s, float* ms, int cap, const char** names)
    {
        int k = 0;
        for (; k < cap && k < (int)s->stageMs.size(); ++k)
        {
            ms[k] = s->stageMs[k];
            if (names) names[k] = s->stageNames[k].c_str();
        }
        return k;
    }

    int sx_sim_last_stats(sx_sim* s, sx_nbstats* st)
    {
        *st = s->lastStats;
        return SX_OK;
    }

} // extern "C"
