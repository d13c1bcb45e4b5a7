/*! @file sx_hydro_cluster.hip
 * @brief Fast-variant VE pair kernels on cluster neighbor lists (gfx950): XMass, VeDefGradh, IAD + divv/curlv,
 *        AV switches, momentum + energy.
 *
 * One 256-thread workgroup per 256-particle SFC cluster (four wave64 groups, one lane per target).  The neighbor
 * search (sx_neighbors.hip) leaves, per cluster, the UNION of its targets' neighbors (uni[], typically 6-7 entries
 * per target instead of ~120 per target) and, per target, u16 positions into it, two per word, lane-interleaved.
 *
 *   1. stage: the workgroup gathers the union's packed records (coalesced runs: the union is in leaf order) and
 *      writes one compact LDS record per union entry: positions relative to the cluster origin (minimum image,
 *      folded in double, rounded to float) plus the per-kernel neighbor fields, derived quantities precomputed
 *      (vol = xm/kx, rho = kx*m/xm, 1/h, m/rho);
 *   2. each lane walks its position list (one coalesced 256-B word load per two neighbors, prefetched four words
 *      ahead) and reads its neighbors' records from LDS (ds_read_b128); the SPH kernel W(v) = sinc(pi v/2)^6 and
 *      dW/dv are evaluated in registers with a degree-6 polynomial in v^2 (|error| < 2e-7 over [0,2), the same
 *      order as the reference's 20000-point table interpolation), so the inner loop touches no global memory;
 *   3. unions larger than the LDS capacity CH are processed in CH-sized chunks, every lane advancing through its
 *      sorted position list chunk by chunk.
 *
 * The per-pair arithmetic follows the reference kernels (citations per kernel) in float with FMA contraction and
 * reciprocal multiplies; results agree with the CPU reference to float rounding (tests/test_gpu_parity.py states
 * the tolerance).  Bit-reproducible results come from the exact variant (sx_hydro.hip, -ffp-contract=off).
 */
#include "sx_hydro.hpp"
#include "sx_kernel_poly.hpp"
#include "sx_traverse.hpp"

namespace sx
{
namespace cluster
{

constexpr int kB = kCluster; // threads per workgroup

#ifndef SX_LEAN_DEPTH
#define SX_LEAN_DEPTH 2
#endif
#ifndef SX_ME_LEAN
#define SX_ME_LEAN true // momentum: one record in flight (see neighborLoop)
#endif

//! per-workgroup cluster bookkeeping
struct Clu
{
    uint32_t        c, gw, i, iSafe, U;
    bool            valid;
    unsigned        cnt;        // this target's stored neighbors
    uint32_t        wBeg, wEnd; // this wave's share of the target's list words (split-K over the wave's part)
    int             part;       // which share: 0 .. SPLIT-1
    int             tid;        // target slot within the cluster: 0 .. 255
    const uint32_t* un;         // union of this cluster
    const uint32_t* nl;         // this lane's position words, stride 64
    double          ox, oy, oz;
    bool            pbc; // positions need the applyPBC rule after folding (tiny periodic boxes)
};

//! LDS neighbor records as loaded by the pipelined loop
struct Rec5
{
    float4 a;
    float  s;
};
struct Rec8
{
    float4 a, b;
};
struct Rec9
{
    float4 a, b;
    float  s;
};
__device__ __forceinline__ float relc(double x, double o, const DevBox& b, int k) { return (float)foldPbc(x - o, b, k); }

//! sets up the cluster and decides (workgroup-uniformly) whether folded coordinates are minimum-image for every
//! neighbor pair: |x_i - o| + 2 h_i < L/2 on every periodic axis.  With SPLIT > 1 the workgroup has SPLIT waves per
//! group: wave w serves group w % 4 and takes the words [wBeg, wEnd) of share w / 4 of every lane's list.
template<int SPLIT>
__device__ __forceinline__ Clu setup(const PairArgs& a, float* s_red)
{
    Clu            cu;
    const int      wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int      sub  = wave & (kClusterWaves - 1);
    cu.part             = wave / kClusterWaves;
    cu.tid              = sub * kWave + lane;
    const uint32_t blk  = xcdBlock(blockIdx.x, gridDim.x);
    cu.c                = a.clusterList ? a.clusterList[blk] : blk;
    cu.gw               = cu.c * kClusterWaves + sub;
    const uint32_t c0   = a.first + cu.c * kCluster;
    cu.i                = c0 + cu.tid;
    cu.valid            = cu.gw < a.numGroups && cu.i < a.last && (!a.active || a.active[cu.i]);
    cu.iSafe            = cu.valid ? cu.i : c0;
    cu.cnt              = 0;
    if (cu.valid)
    {
        unsigned c1 = a.nc[cu.i] - 1;
        cu.cnt      = c1 < a.ngmax ? c1 : a.ngmax;
    }
    const uint32_t nw = (cu.cnt + 1) >> 1;
    cu.wBeg           = nw * cu.part / SPLIT;
    cu.wEnd           = nw * (cu.part + 1) / SPLIT;
    const bool lB     = listsB(a.lb, cu.c); // the cluster's current set of lists
    cu.U              = lB ? a.lb.ucount[cu.c] : a.ucount[cu.c];
    cu.un             = a.uni + (size_t)cu.c * a.ucap + (lB ? a.lb.uoff : 0u);
    cu.nl             = (lB ? a.lb.nloc : a.nloc) + (size_t)cu.gw * nlocWords(a.ngmax) * kWave + lane;
    const RecX o      = a.rx[c0];
    cu.ox = o.x, cu.oy = o.y, cu.oz = o.z;

    const RecX r    = a.rx[cu.iSafe];
    const float h2  = 2.0f * r.h;
    float       ext = 0.0f;
    if (a.box.pbc[0]) ext = fmaxf(ext, (fabsf(relc(r.x, cu.ox, a.box, 0)) + h2) * (float)a.box.il[0]);
    if (a.box.pbc[1]) ext = fmaxf(ext, (fabsf(relc(r.y, cu.oy, a.box, 1)) + h2) * (float)a.box.il[1]);
    if (a.box.pbc[2]) ext = fmaxf(ext, (fabsf(relc(r.z, cu.oz, a.box, 2)) + h2) * (float)a.box.il[2]);
    ext = waveMax(ext);
    if (lane == 0) s_red[wave] = ext;
    __syncthreads();
    float e = s_red[0];
    for (int w = 1; w < kClusterWaves * SPLIT; ++w)
        e = fmaxf(e, s_red[w]);
    cu.pbc = __builtin_amdgcn_readfirstlane(e >= 0.49f ? 1 : 0);
    return cu;
}

/*! Partial sums of the SPLIT shares of each target -> every share (same order everywhere, so all shares agree).
 *  v[f] is summed (or max-ed where bit f of maxMask is set); scratch holds NV * SPLIT * 256 floats. */
template<int SPLIT, int NV>
__device__ __forceinline__ void combineShares(const Clu& cu, float (&v)[NV], float* scratch, unsigned maxMask = 0,
                                              bool scratchAliasesRecords = false)
{
    if constexpr (SPLIT > 1)
    {
        constexpr int T = SPLIT * kCluster;
        if (scratchAliasesRecords) __syncthreads(); // every share is done reading the staged records
#pragma unroll
        for (int f = 0; f < NV; ++f)
            scratch[f * T + cu.part * kCluster + cu.tid] = v[f];
        __syncthreads();
#pragma unroll
        for (int f = 0; f < NV; ++f)
        {
            float acc = scratch[f * T + cu.tid];
            for (int q = 1; q < SPLIT; ++q)
            {
                const float x = scratch[f * T + q * kCluster + cu.tid];
                acc           = ((maxMask >> f) & 1u) ? fmaxf(acc, x) : acc + x;
            }
            v[f] = acc;
        }
    }
}

/*! Run compute(load(p)) over this lane's share of its neighbors, p = LDS slot.  stage(j, slot) writes the record
 *  of particle j.  `resident` carries "the whole union is already in LDS" from a previous pass over the same records.
 *  With the union resident the loop is software-pipelined: the LDS records of the next two neighbors (one list
 *  word) are read while the current two are computed, and list words are prefetched four ahead. */
template<int CH, int SPLIT, bool PF = true, bool LEAN = false, class Stage, class Load, class Compute>
__device__ __forceinline__ void neighborLoop(const Clu& cu, Stage&& stage, Load&& load, Compute&& compute,
                                             bool& resident)
{
    constexpr int NT = kB * SPLIT;
    constexpr int S  = (CH + NT - 1) / NT;
    auto          fill = [&](uint32_t b0, uint32_t b1) {
        uint32_t js[S];
#pragma unroll
        for (int s = 0; s < S; ++s)
        {
            const uint32_t u = b0 + threadIdx.x + s * NT;
            js[s]            = u < b1 ? cu.un[u] : 0u;
        }
#pragma unroll
        for (int s = 0; s < S; ++s)
        {
            const uint32_t u = b0 + threadIdx.x + s * NT;
            if (u < b1) stage(js[s], u - b0);
        }
    };

    if (cu.U <= (uint32_t)CH)
    {
        if (!resident)
        {
            fill(0, cu.U);
            __syncthreads();
            resident = true;
        }
        const uint32_t wBeg = cu.wBeg, wEnd = cu.wEnd;
        if (wBeg >= wEnd) return;
        const uint32_t* nl = cu.nl;
        if constexpr (LEAN)
        {
            // one record in flight while the other is computed: the LDS read latency (~100 cycles) is far below a
            // heavy pair's compute, and half the record registers let one more wave per SIMD in (momentum 152 -> 128
            // VGPRs).  List words beyond the share re-read its last word; their records are read, never computed.
            const uint32_t wLast = wEnd - 1;
            auto           ld    = [&](uint32_t w) { return nl[(size_t)min(w, wLast) * kWave]; };
            // list words prefetched SX_LEAN_DEPTH ahead (the list streams from HBM: a load's latency under load
            // spans several heavy pairs)
            constexpr int  D = SX_LEAN_DEPTH;
            uint32_t       q[D];
#pragma unroll
            for (int d = 0; d < D; ++d)
                q[d] = ld(wBeg + 1 + d);
            uint32_t       wd = nl[(size_t)wBeg * kWave];
            auto           ra = load(wd & 0xffffu);
            for (uint32_t w = wBeg;;)
            {
                const auto rb = load(wd >> 16);
                compute(ra);
                const bool odd = 2 * w + 1 < cu.cnt;
                wd             = q[0];
#pragma unroll
                for (int d = 0; d + 1 < D; ++d)
                    q[d] = q[d + 1];
                q[D - 1] = ld(w + 1 + D);
                ra             = load(wd & 0xffffu);
                if (odd) compute(rb);
                if (++w >= wEnd) break;
            }
            return;
        }
        // PF: list words beyond the share read the share's last word again (always in bounds) and every prefetch
        // below is unconditional, so the LDS reads of the next pair are issued on one path and the wait before a
        // computation covers only the records it consumes (a masked prefetch leaves a path on which the previous
        // pair's reads may still be outstanding, and the merged wait then also waits for the new reads).  Measured
        // (Sedov 64M): IAD -0.4 ms, AV -0.3 ms; momentum +0.3..0.7 ms (its records are 80 B: the extra registers of
        // the unmasked form cost more than the wait), so momentum takes the LEAN form above (22.5 -> 21.5 ms).
        const uint32_t  wLast = wEnd - 1;
        auto            ld    = [&](uint32_t w) {
            if constexpr (PF) return nl[(size_t)min(w, wLast) * kWave];
            else return w < wEnd ? nl[(size_t)w * kWave] : 0u;
        };
        // two record buffers used alternately (2x unrolled, no register copies); list words prefetched ahead
        uint32_t        q0 = ld(wBeg + 1), q1 = ld(wBeg + 2), q2 = ld(wBeg + 3);
        const uint32_t  w0 = nl[(size_t)wBeg * kWave];
        auto            a0 = load(w0 & 0xffffu); // slot 0 for a missing odd partner: valid, never computed
        auto            b0 = load(w0 >> 16);
        decltype(a0)    a1, b1;
        uint32_t        w = wBeg;
        while (true)
        {
            if (PF || w + 1 < wEnd) // past the share's end (PF): a valid slot that is never computed
            {
                a1 = load(q0 & 0xffffu);
                b1 = load(q0 >> 16);
                q0 = ld(w + 4);
            }
            compute(a0);
            if (2 * w + 1 < cu.cnt) compute(b0);
            if (++w >= wEnd) break;
            if (PF || w + 1 < wEnd)
            {
                a0 = load(q1 & 0xffffu);
                b0 = load(q1 >> 16);
                q1 = ld(w + 4);
            }
            compute(a1);
            if (2 * w + 1 < cu.cnt) compute(b1);
            if (++w >= wEnd) break;
            const uint32_t t = q0;
            q0 = q2, q2 = q1, q1 = t;
        }
    }
    else
    {
        resident         = false;
        uint32_t       k    = 2 * cu.wBeg;
        const uint32_t kEnd = min(cu.cnt, 2 * cu.wEnd);
        for (uint32_t b0 = 0; b0 < cu.U; b0 += CH)
        {
            const uint32_t b1 = min(cu.U, b0 + (uint32_t)CH);
            __syncthreads();
            fill(b0, b1);
            __syncthreads();
            while (k < kEnd)
            {
                const uint32_t w = cu.nl[(size_t)(k >> 1) * kWave];
                const uint32_t p = (k & 1) ? (w >> 16) : (w & 0xffffu);
                if (p >= b1) break;
                compute(load(p - b0));
                ++k;
            }
        }
    }
}

__device__ __forceinline__ void pbcRule(const Clu& cu, const DevBox& b, float r, float& x, float& y, float& z)
{
    if (cu.pbc) applyPBC(b, r, x, y, z);
}

/*! |(a, b, c)| scaled by the largest component: this file flushes denormals to zero, so the plain sum of squares
 *  would lose components below ~1e-19 (tiny velocity gradients) that the reference keeps */
__device__ __forceinline__ float norm3(float a, float b, float c)
{
    const float m = fmaxf(fabsf(a), fmaxf(fabsf(b), fabsf(c)));
    if (m == 0.0f) return 0.0f;
    const float r = 1.0f / m, x = a * r, y = b * r, z = c * r;
    return m * sqrtf(x * x + (y * y + z * z));
}

// ---- XMass: xmassJLoop (hydro_ve/xmass_kern.hpp:50-79) ----------------------------------------------------------

template<int CH, int SPLIT>
__global__ __launch_bounds__(kB * SPLIT) void xmassKernel(PairArgs a)
{
    __shared__ float4 sP[CH];
    __shared__ float  s_red[kClusterWaves * SPLIT];
    const Clu  cu = setup<SPLIT>(a, s_red);
    const RecX ri = a.rx[cu.iSafe];
    const float xi = relc(ri.x, cu.ox, a.box, 0), yi = relc(ri.y, cu.oy, a.box, 1), zi = relc(ri.z, cu.oz, a.box, 2);
    const float hInv = 1.0f / ri.h, hInv2 = hInv * hInv, h2 = 2.0f * ri.h;
    float       rho0 = cu.part == 0 ? ri.m : 0.0f;
    bool        res  = false;
    neighborLoop<CH, SPLIT>(
        cu,
        [&](uint32_t j, uint32_t slot) {
            const RecX r = a.rx[j];
            sP[slot] = make_float4(relc(r.x, cu.ox, a.box, 0), relc(r.y, cu.oy, a.box, 1), relc(r.z, cu.oz, a.box, 2), r.m);
        },
        [&](uint32_t p) { return sP[p]; },
        [&](const float4& q) {
            float rx = xi - q.x, ry = yi - q.y, rz = zi - q.z;
            pbcRule(cu, a.box, h2, rx, ry, rz);
            rho0 += kernelWt((rx * rx + ry * ry + rz * rz) * hInv2) * q.w;
        },
        res);
    float v[1] = {rho0};
    combineShares<SPLIT>(cu, v, reinterpret_cast<float*>(sP), 0u, true);
    if (cu.valid && cu.part == 0)
    {
        const float h3Inv = hInv * hInv * hInv;
        const float xm    = (float)((double)ri.m / ((double)v[0] * a.K * (double)h3Inv));
        a.xm[cu.i]        = xm;
        if (a.rtOut) a.rtOut[cu.i] = RecT{xm, 0.0f, 0.0f, 0.0f};
    }
}

// ---- VeDefGradh: veDefGradhJLoop (hydro_ve/ve_def_gradh_kern.hpp:43-90) -----------------------------------------
template<int CH, int SPLIT>
__global__ __launch_bounds__(kB * SPLIT) void veDefGradhKernel(PairArgs a)
{
    __shared__ float4 sP[CH];
    __shared__ float  sX[CH];
    __shared__ float  s_red[kClusterWaves * SPLIT];
    const Clu   cu     = setup<SPLIT>(a, s_red);
    const RecX  ri     = a.rx[cu.iSafe];
    const float xmassi = a.xm[cu.iSafe]; // the dense field (its RecT is rewritten by this kernel's EOS)
    const float xi = relc(ri.x, cu.ox, a.box, 0), yi = relc(ri.y, cu.oy, a.box, 1), zi = relc(ri.z, cu.oz, a.box, 2);
    const float hInv = 1.0f / ri.h, hInv2 = hInv * hInv, h2 = 2.0f * ri.h;
    const bool  own = cu.part == 0; // the self terms go to share 0
    float       kxi = own ? xmassi : 0.0f, whomegai = own ? -3.0f * xmassi : 0.0f, wrho0i = own ? -3.0f * ri.m : 0.0f;
    bool        res = false;
    neighborLoop<CH, SPLIT>(
        cu,
        [&](uint32_t j, uint32_t slot) {
            const RecX r = a.rx[j];
            sP[slot] = make_float4(relc(r.x, cu.ox, a.box, 0), relc(r.y, cu.oy, a.box, 1), relc(r.z, cu.oz, a.box, 2), r.m);
            sX[slot] = a.xm[j]; // the dense field (a union run of consecutive particles shares its sectors), not RecT
        },
        [&](uint32_t p) { return Rec5{sP[p], sX[p]}; },
        [&](const Rec5& r) {
            const float4& q      = r.a;
            const float   xmassj = r.s;
            float         rx = xi - q.x, ry = yi - q.y, rz = zi - q.z;
            pbcRule(cu, a.box, h2, rx, ry, rz);
            float w, vdw;
            kernelWvdWt((rx * rx + ry * ry + rz * rz) * hInv2, w, vdw);
            const float dterh = -(3.0f * w + vdw);
            kxi += w * xmassj;
            whomegai += dterh * xmassj;
            wrho0i += dterh * q.w;
        },
        res);
    {
        float v[3] = {kxi, whomegai, wrho0i};
        combineShares<SPLIT>(cu, v, reinterpret_cast<float*>(sP), 0u, true);
        kxi = v[0], whomegai = v[1], wrho0i = v[2];
    }
    if (cu.valid && cu.part == 0)
    {
        const double K     = a.K;
        const float  h3Inv = hInv * hInv * hInv;
        kxi                = (float)((double)kxi * (K * (double)h3Inv));
        whomegai           = (float)((double)whomegai * (K * (double)h3Inv * (double)hInv));
        wrho0i             = (float)((double)wrho0i * (K * (double)h3Inv * (double)hInv));
        whomegai           = (float)((double)(whomegai * ri.m / xmassi) +
                           ((double)kxi - K * (double)xmassi * (double)h3Inv) * (double)wrho0i);
        const float rhoi   = kxi * ri.m / xmassi;
        const float dhdrho = -ri.h / (rhoi * 3.0f);
        const float gradhi = 1.0f - dhdrho * whomegai;
        a.kx[cu.i]         = kxi;
        a.gradh[cu.i]      = gradhi;
        if (a.eos.temp)
        {
            // eosKernel's arithmetic (sx_hydro.hip: computeEOS_Impl, idealGasEOS) on the values just computed
            const EosFuse& e    = a.eos;
            const double   tmp  = e.cv * e.temp[cu.i] * (e.gamma - 1.0);
            const double   pi   = (double)rhoi * tmp;
            const double   ci   = sqrt(tmp);
            const float    prho = (float)(pi / (double)(kxi * ri.m * ri.m * gradhi));
            e.prho[cu.i]        = prho;
            e.c[cu.i]           = (float)ci;
            e.rvOut[cu.i]       = RecV{e.vx[cu.i], e.vy[cu.i], e.vz[cu.i], (float)ci};
            e.rtOut[cu.i]       = RecT{xmassi, kxi, prho, e.alpha[cu.i]};
        }
    }
}

// ---- IAD + divv/curlv: IADJLoop (iad_kern.hpp:43-109) + divV_curlVJLoop (divv_curlv_kern.hpp:43-123) -------------
//! STD: IADJLoopSTD (hydro_std/iad_kern.hpp:12-77), volumes m/rho and no velocity derivatives
template<int CH, int SPLIT, bool STD = false>
__global__ __launch_bounds__(kB * SPLIT) void iadDivvCurlvKernel(PairArgs a)
{
    __shared__ float4 sP[CH];               // x, y, z, vol = xm/kx (std: m/rho)
    __shared__ float4 sV[STD ? 1 : CH];     // vx, vy, vz, xm
    __shared__ float  s_red[kClusterWaves * SPLIT];
    __shared__ float  s_scr[SPLIT > 1 ? 9 * SPLIT * kCluster : 1];
    const Clu   cu  = setup<SPLIT>(a, s_red);
    const RecX  ri  = a.rx[cu.iSafe];
    const float xi = relc(ri.x, cu.ox, a.box, 0), yi = relc(ri.y, cu.oy, a.box, 1), zi = relc(ri.z, cu.oz, a.box, 2);
    const float hi = ri.h, hiInv = 1.0f / hi, hiInv2 = hiInv * hiInv, h2 = 2.0f * hi;
    auto        stage = [&](uint32_t j, uint32_t slot) {
        const RecX r = a.rx[j];
        if constexpr (STD)
            sP[slot] = make_float4(relc(r.x, cu.ox, a.box, 0), relc(r.y, cu.oy, a.box, 1), relc(r.z, cu.oz, a.box, 2),
                                   r.m / a.rs[j].rho);
        else
        {
            const RecV v = a.rv[j];
            const RecT t = a.rt[j];
            sP[slot]     = make_float4(relc(r.x, cu.ox, a.box, 0), relc(r.y, cu.oy, a.box, 1),
                                   relc(r.z, cu.oz, a.box, 2), t.xm / t.kx);
            sV[slot]     = make_float4(v.vx, v.vy, v.vz, t.xm);
        }
    };
    float t11 = 0, t12 = 0, t13 = 0, t22 = 0, t23 = 0, t33 = 0;
    bool  res = false;
    neighborLoop<CH, SPLIT>(
        cu, stage, [&](uint32_t p) { return sP[p]; },
        [&](const float4& q) {
            float rx = xi - q.x, ry = yi - q.y, rz = zi - q.z;
            pbcRule(cu, a.box, h2, rx, ry, rz);
            const float volj_w = q.w * kernelWt((rx * rx + ry * ry + rz * rz) * hiInv2);
            t11 += rx * rx * volj_w;
            t12 += rx * ry * volj_w;
            t13 += rx * rz * volj_w;
            t22 += ry * ry * volj_w;
            t23 += ry * rz * volj_w;
            t33 += rz * rz * volj_w;
        },
        res);
    {
        float v[6] = {t11, t12, t13, t22, t23, t33};
        combineShares<SPLIT>(cu, v, s_scr);
        t11 = v[0], t12 = v[1], t13 = v[2], t22 = v[3], t23 = v[4], t33 = v[5];
    }
    float cc[6];
    iadInvert(t11, t12, t13, t22, t23, t33, hi, a.K, cc);
    const float c11i = cc[0], c12i = cc[1], c13i = cc[2], c22i = cc[3], c23i = cc[4], c33i = cc[5];
    if constexpr (STD)
    {
        if (cu.valid && cu.part == 0)
        {
            const uint32_t i = cu.i;
            a.c11[i] = c11i, a.c12[i] = c12i, a.c13[i] = c13i, a.c22[i] = c22i, a.c23[i] = c23i, a.c33[i] = c33i;
        }
        return;
    }
    const RecV  vi  = a.rv[cu.iSafe];
    const RecT  ti  = a.rt[cu.iSafe];
    const float kxi = ti.kx;

    float dVx0 = 0, dVx1 = 0, dVx2 = 0, dVy0 = 0, dVy1 = 0, dVy2 = 0, dVz0 = 0, dVz1 = 0, dVz2 = 0;
    neighborLoop<CH, SPLIT>(
        cu, stage, [&](uint32_t p) { return Rec8{sP[p], sV[p]}; },
        [&](const Rec8& r) {
            const float4& q  = r.a;
            const float4& v  = r.b;
            float         rx = xi - q.x, ry = yi - q.y, rz = zi - q.z;
            pbcRule(cu, a.box, h2, rx, ry, rz);
            const float Wi   = kernelWt((rx * rx + ry * ry + rz * rz) * hiInv2);
            const float tA0  = -(c11i * rx + c12i * ry + c13i * rz) * Wi;
            const float tA1  = -(c12i * rx + c22i * ry + c23i * rz) * Wi;
            const float tA2  = -(c13i * rx + c23i * ry + c33i * rz) * Wi;
            const float fx = (v.x - vi.vx) * v.w, fy = (v.y - vi.vy) * v.w, fz = (v.z - vi.vz) * v.w;
            dVx0 += tA0 * fx;
            dVx1 += tA1 * fx;
            dVx2 += tA2 * fx;
            dVy0 += tA0 * fy;
            dVy1 += tA1 * fy;
            dVy2 += tA2 * fy;
            dVz0 += tA0 * fz;
            dVz1 += tA1 * fz;
            dVz2 += tA2 * fz;
        },
        res);
    {
        float v[9] = {dVx0, dVx1, dVx2, dVy0, dVy1, dVy2, dVz0, dVz1, dVz2};
        __syncthreads(); // s_scr still holds the tau shares being read
        combineShares<SPLIT>(cu, v, s_scr);
        dVx0 = v[0], dVx1 = v[1], dVx2 = v[2], dVy0 = v[3], dVy1 = v[4], dVy2 = v[5], dVz0 = v[6], dVz1 = v[7],
        dVz2 = v[8];
    }
    if (cu.valid && cu.part == 0)
    {
        const uint32_t i = cu.i;
        a.c11[i] = c11i, a.c12[i] = c12i, a.c13[i] = c13i, a.c22[i] = c22i, a.c23[i] = c23i, a.c33[i] = c33i;
        const float norm_kxi = (float)(a.K * (double)(hiInv * hiInv * hiInv) / (double)kxi);
        const float divv_i   = norm_kxi * (dVx0 + dVy1 + dVz2);
        a.divv[i]            = divv_i;
        if (a.rcOut) a.rcOut[i] = RecC{c11i, c12i, c13i, c22i, c23i, c33i, divv_i, ti.xm / ti.kx};
        if (a.curlv)
        {
            const float cv0 = dVz1 - dVy2, cv1 = dVx2 - dVz0, cv2 = dVy0 - dVx1;
            a.curlv[i]      = norm_kxi * norm3(cv0, cv1, cv2);
        }
        if (a.dV11) // doGradV (divv_curlv_kern.hpp:113-121)
        {
            a.dV11[i] = norm_kxi * dVx0;
            a.dV12[i] = norm_kxi * (dVx1 + dVy0);
            a.dV13[i] = norm_kxi * (dVx2 + dVz0);
            a.dV22[i] = norm_kxi * dVy1;
            a.dV23[i] = norm_kxi * (dVy2 + dVz1);
            a.dV33[i] = norm_kxi * dVz2;
        }
    }
}

/*! IAD + divv/curlv in ONE neighbor pass.  divV_curlVJLoop's terms are linear in the fresh c_i:
 *    dV_kb = sum_j -(c_i r)_k W_j f_jb = -sum_a c_ka M_ab,   M_ab = sum_j r_a W_j f_jb,  f_j = (v_j - v_i) xm_j,
 *  so the pass accumulates tau (6) and M (9) together and applies c_i after the inversion: one kernel evaluation
 *  and one record read per pair instead of two (same terms, different float summation order). */
template<int CH, int SPLIT>
__global__ __launch_bounds__(kB * SPLIT) void iadDivvCurlvFusedKernel(PairArgs a)
{
    __shared__ float4 sP[CH]; // x, y, z, vol = xm/kx
    __shared__ float4 sV[CH]; // vx, vy, vz, xm
    __shared__ float  s_red[kClusterWaves * SPLIT];
    static_assert(SPLIT == 1 || (6 * SPLIT * kCluster <= 4 * CH && 9 * SPLIT * kCluster <= 4 * CH),
                  "the share sums are combined in the record arrays");
    const Clu   cu  = setup<SPLIT>(a, s_red);
    const RecX  ri  = a.rx[cu.iSafe];
    const RecV  vi  = a.rv[cu.iSafe];
    const RecT  ti  = a.rt[cu.iSafe];
    const float kxi = ti.kx;
    const float xi = relc(ri.x, cu.ox, a.box, 0), yi = relc(ri.y, cu.oy, a.box, 1), zi = relc(ri.z, cu.oz, a.box, 2);
    const float hi = ri.h, hiInv = 1.0f / hi, hiInv2 = hiInv * hiInv, h2 = 2.0f * hi;
    float       t11 = 0, t12 = 0, t13 = 0, t22 = 0, t23 = 0, t33 = 0;
    float       M[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    bool        res = false;
    neighborLoop<CH, SPLIT>(
        cu,
        [&](uint32_t j, uint32_t slot) {
            const RecX r = a.rx[j];
            const RecV v = a.rv[j];
            const RecT t = a.rt[j];
            sP[slot]     = make_float4(relc(r.x, cu.ox, a.box, 0), relc(r.y, cu.oy, a.box, 1),
                                   relc(r.z, cu.oz, a.box, 2), t.xm / t.kx);
            sV[slot]     = make_float4(v.vx, v.vy, v.vz, t.xm);
        },
        [&](uint32_t p) { return Rec8{sP[p], sV[p]}; },
        [&](const Rec8& rec) {
            const float4& q  = rec.a;
            const float4& v  = rec.b;
            float         rx = xi - q.x, ry = yi - q.y, rz = zi - q.z;
            pbcRule(cu, a.box, h2, rx, ry, rz);
            const float W      = kernelWt((rx * rx + ry * ry + rz * rz) * hiInv2);
            const float rW[3] = {rx * W, ry * W, rz * W};
            // tau_ab += r_a r_b vol_j W: (r_a W vol_j) r_b, three products shared by the six sums
            const float px = rW[0] * q.w, py = rW[1] * q.w, pz = rW[2] * q.w;
            t11 = fmaf(px, rx, t11);
            t12 = fmaf(px, ry, t12);
            t13 = fmaf(px, rz, t13);
            t22 = fmaf(py, ry, t22);
            t23 = fmaf(py, rz, t23);
            t33 = fmaf(pz, rz, t33);
            const float f[3]  = {(v.x - vi.vx) * v.w, (v.y - vi.vy) * v.w, (v.z - vi.vz) * v.w};
#pragma unroll
            for (int aa = 0; aa < 3; ++aa)
#pragma unroll
                for (int b = 0; b < 3; ++b)
                    M[aa][b] = fmaf(rW[aa], f[b], M[aa][b]);
        },
        res);
    {
        // tau shares in sP's space, M shares in sV's (both read only by the neighbor loop, done at the first sync)
        float v[6] = {t11, t12, t13, t22, t23, t33};
        combineShares<SPLIT>(cu, v, reinterpret_cast<float*>(sP), 0u, true);
        t11 = v[0], t12 = v[1], t13 = v[2], t22 = v[3], t23 = v[4], t33 = v[5];
        float w[9] = {M[0][0], M[0][1], M[0][2], M[1][0], M[1][1], M[1][2], M[2][0], M[2][1], M[2][2]};
        combineShares<SPLIT>(cu, w, reinterpret_cast<float*>(sV));
#pragma unroll
        for (int k = 0; k < 9; ++k)
            M[k / 3][k % 3] = w[k];
    }
    float cc[6];
    iadInvert(t11, t12, t13, t22, t23, t33, hi, a.K, cc);
    const float c11i = cc[0], c12i = cc[1], c13i = cc[2], c22i = cc[3], c23i = cc[4], c33i = cc[5];
    // dV_kb = -(c_k0 M_0b + c_k1 M_1b + c_k2 M_2b), rows of the symmetric c_i
    float dV[3][3];
#pragma unroll
    for (int b = 0; b < 3; ++b)
    {
        dV[0][b] = -(c11i * M[0][b] + c12i * M[1][b] + c13i * M[2][b]);
        dV[1][b] = -(c12i * M[0][b] + c22i * M[1][b] + c23i * M[2][b]);
        dV[2][b] = -(c13i * M[0][b] + c23i * M[1][b] + c33i * M[2][b]);
    }
    // naming of divV_curlVJLoop: dVx{k} = dV[k][x], dVy{k} = dV[k][y], dVz{k} = dV[k][z]
    const float dVx0 = dV[0][0], dVx1 = dV[1][0], dVx2 = dV[2][0];
    const float dVy0 = dV[0][1], dVy1 = dV[1][1], dVy2 = dV[2][1];
    const float dVz0 = dV[0][2], dVz1 = dV[1][2], dVz2 = dV[2][2];
    if (cu.valid && cu.part == 0)
    {
        const uint32_t i = cu.i;
        a.c11[i] = c11i, a.c12[i] = c12i, a.c13[i] = c13i, a.c22[i] = c22i, a.c23[i] = c23i, a.c33[i] = c33i;
        const float norm_kxi = (float)(a.K * (double)(hiInv * hiInv * hiInv) / (double)kxi);
        const float divv_i   = norm_kxi * (dVx0 + dVy1 + dVz2);
        a.divv[i]            = divv_i;
        if (a.rcOut) a.rcOut[i] = RecC{c11i, c12i, c13i, c22i, c23i, c33i, divv_i, ti.xm / ti.kx};
        if (a.curlv)
        {
            const float cv0 = dVz1 - dVy2, cv1 = dVx2 - dVz0, cv2 = dVy0 - dVx1;
            a.curlv[i]      = norm_kxi * norm3(cv0, cv1, cv2);
        }
        if (a.dV11)
        {
            a.dV11[i] = norm_kxi * dVx0;
            a.dV12[i] = norm_kxi * (dVx1 + dVy0);
            a.dV13[i] = norm_kxi * (dVx2 + dVz0);
            a.dV22[i] = norm_kxi * dVy1;
            a.dV23[i] = norm_kxi * (dVy2 + dVz1);
            a.dV33[i] = norm_kxi * dVz2;
        }
    }
}

// ---- AV switches: AVswitchesJLoop (av_switches_kern.hpp:43-137) -------------------------------------------------
template<int CH, int SPLIT, int UMIN = 0, int UMAX = 0>
__global__ __launch_bounds__(kB * SPLIT) void avSwitchesKernel(PairArgs a)
{
    __shared__ float4 sP[CH]; // x, y, z, vol
    __shared__ float4 sV[CH]; // vx, vy, vz, c
    __shared__ float  sD[CH]; // divv
    __shared__ float  s_red[kClusterWaves * SPLIT];
    if constexpr (UMIN > 0 || UMAX > 0)
    {
        // one of the two capacity launches (avSwitches): this workgroup's cluster belongs to the other one
        const uint32_t blk = xcdBlock(blockIdx.x, gridDim.x);
        const uint32_t cc  = a.clusterList ? a.clusterList[blk] : blk;
        const uint32_t U   = listsB(a.lb, cc) ? a.lb.ucount[cc] : a.ucount[cc];
        if (U < (uint32_t)UMIN || (UMAX > 0 && U > (uint32_t)UMAX)) return;
    }
    const Clu   cu  = setup<SPLIT>(a, s_red);
    const RecX  ri  = a.rx[cu.iSafe];
    const RecV  vi  = a.rv[cu.iSafe];
    const RecC  ci6 = a.rc[cu.iSafe];
    const float xi = relc(ri.x, cu.ox, a.box, 0), yi = relc(ri.y, cu.oy, a.box, 1), zi = relc(ri.z, cu.oz, a.box, 2);
    const float hi = ri.h, ci = vi.c, hiInv = 1.0f / hi, hiInv2 = hiInv * hiInv, h2 = 2.0f * hi;
    const float hiInv3K     = (float)a.K * (hiInv * hiInv * hiInv);
    const float divv_i      = ci6.divv;
    float       vijsignal_i = 1.e-40f * ci;
    float       gx = 0, gy = 0, gz = 0;
    bool        res = false;
    auto        stage = [&](uint32_t j, uint32_t slot) {
        const RecX   r  = a.rx[j];
        const RecV   v  = a.rv[j];
        // {divv, vol = xm / kx}: the last 8 bytes of the neighbor's RecC (IAD / the halo pack wrote vol)
        const float2 dv = *reinterpret_cast<const float2*>(&a.rc[j].divv);
        sP[slot] = make_float4(relc(r.x, cu.ox, a.box, 0), relc(r.y, cu.oy, a.box, 1), relc(r.z, cu.oz, a.box, 2),
                               dv.y);
        sV[slot] = make_float4(v.vx, v.vy, v.vz, v.c);
        sD[slot] = dv.x;
    };
    auto loadRec = [&](uint32_t p) { return Rec9{sP[p], sV[p], sD[p]}; };
    neighborLoop<CH, SPLIT>(
        cu, stage, loadRec,
        [&](const Rec9& r) {
            const float4& q  = r.a;
            const float4& v  = r.b;
            float         rx = xi - q.x, ry = yi - q.y, rz = zi - q.z;
            pbcRule(cu, a.box, h2, rx, ry, rz);
            const float r2    = rx * rx + ry * ry + rz * rz;
            const float rinv  = rsqrtf(r2);
            const float vx_ij = vi.vx - v.x, vy_ij = vi.vy - v.y, vz_ij = vi.vz - v.z;
            const float rv    = rx * vx_ij + ry * vy_ij + rz * vz_ij;
            const float vsig  = rv < 0.0f ? ci + v.w - 3.0f * rv * rinv : 0.0f;
            vijsignal_i       = fmaxf(vijsignal_i, vsig);
            // termA_j = -(c_i r) K h_i^-3 W_j is linear in r with the target's c_i: the pass sums s = sum_j factor_j
            // W_j r and c_i is applied once after it (same terms, different float summation order)
            const float fw = kernelWt(r2 * hiInv2) * (q.w * (divv_i - r.s));
            gx = fmaf(fw, rx, gx);
            gy = fmaf(fw, ry, gy);
            gz = fmaf(fw, rz, gz);
        },
        res);
    {
        float v[4] = {gx, gy, gz, vijsignal_i};
        combineShares<SPLIT>(cu, v, reinterpret_cast<float*>(sP), 8u, true);
        gx = v[0], gy = v[1], gz = v[2], vijsignal_i = v[3];
    }
    if (!cu.valid || cu.part != 0) return;
    {
        const float sx = gx, sy = gy, sz = gz;
        gx = -hiInv3K * (ci6.c11 * sx + ci6.c12 * sy + ci6.c13 * sz);
        gy = -hiInv3K * (ci6.c12 * sx + ci6.c22 * sy + ci6.c23 * sz);
        gz = -hiInv3K * (ci6.c13 * sx + ci6.c23 * sy + ci6.c33 * sz);
    }
    const float graddivv = norm3(gx, gy, gz);
    float       alphaloc = 0.0f;
    if (divv_i < 0.0f)
    {
        const float a_const = hi * hi * graddivv;
        alphaloc            = a.alphamax * a_const / (a_const + hi * fabsf(divv_i) + 0.05f * ci);
    }
    float alpha_i = a.rt[cu.i].alpha;
    if (alphaloc >= alpha_i) { alpha_i = alphaloc; }
    else
    {
        const float decay    = hi / (a.decay_constant * vijsignal_i);
        const float alphadot = ((alphaloc >= a.alphamin) ? (alphaloc - alpha_i) : (a.alphamin - alpha_i)) / decay;
        const double dt      = a.dtPtr ? *a.dtPtr : a.dt;
        alpha_i              = (float)((double)alpha_i + (double)alphadot * dt);
    }
    a.alpha[cu.i] = alpha_i;
    if (a.rtOut)
    {
        // xm, kx and prho as they are (a concurrent reader of this record sees them unchanged either way)
        RecT t       = a.rt[cu.i];
        t.alpha      = alpha_i;
        a.rtOut[cu.i] = t;
    }
}

// ---- momentum + energy: momentumAndEnergyJLoop<avClean> (momentum_energy_kern.hpp:65-222) -------------------
//! Atwood-ramped momentum weights (momentum_energy_kern.hpp:178-195): xm_i^(2-s) xm_j^s and xm_j^(2-s) xm_i^s with
//! s = 0 below Atmin, 1 above Atmax (both exact products) and the ramp in between (exp2/log2 form)
__device__ __forceinline__ void atwoodWeights(float Atwood, float Atmin, float Atmax, float ramp, float xmi, float lxi,
                                              float xmj, float& a_mom, float& b_mom)
{
    if (Atwood < Atmin) { a_mom = xmi * xmi, b_mom = xmj * xmj; }
    else if (Atwood > Atmax) { a_mom = xmi * xmj, b_mom = a_mom; }
    else
    {
        const float sigma = ramp * (Atwood - Atmin);
        const float lxj   = __log2f(xmj);
        const float dl    = lxj - lxi;
        a_mom             = exp2f(fmaf(sigma, dl, 2.0f * lxi));
        b_mom             = exp2f(fmaf(-sigma, dl, 2.0f * lxj));
    }
}

//! LDS record of the momentum kernel: 80 B, + 24 B of velocity gradient with avClean
template<bool AVC>
struct RecM
{
    float4 p, v, t, a, b, g;
    float2 g2;
};

//! c11 .. c33 of a RecC without its divv and pad (two loads, 24 of its 32 bytes)
struct MeC
{
    float4 a; // c11, c12, c13, c22
    float2 b; // c23, c33
};
__device__ __forceinline__ MeC meLoadC(const RecC* rc, uint32_t j)
{
    const float* p = reinterpret_cast<const float*>(rc + j);
    return MeC{*reinterpret_cast<const float4*>(p), *reinterpret_cast<const float2*>(p + 4)};
}
//! a cluster's data the momentum kernel prefetches one cluster ahead: its union size and indices, each thread's own
//! target (list count, view flag, packed records) and, issued after the previous cluster's neighbor loop, the raw
//! records of the union entries this thread stages
template<int CH, int SPLIT, bool AVC>
struct MePre
{
    static constexpr int NT = kB * SPLIT, S = (CH + NT - 1) / NT;
    static constexpr int SP = S < 2 ? S : 2; // slots whose records are prefetched (registers); the rest load at staging
    uint32_t c, U;
    bool     lB; // the cluster's second set of lists is current (sx_device.hpp ListsB)
    uint32_t nc;
    uint8_t  act;
    RecX     o; // the cluster origin (its first particle)
    RecX     ri;
    RecV     vi;
    RecT     ti;
    MeC      ci;
    float    gi[AVC ? 6 : 1];
    uint32_t js[S];
};
template<bool AVC>
struct MeRaw
{
    RecX  x;
    RecV  v;
    RecT  t;
    MeC   c;
    float g[AVC ? 6 : 1];
};
template<bool AVC>
__device__ __forceinline__ MeRaw<AVC> meLoadRaw(const PairArgs& a, uint32_t j)
{
    MeRaw<AVC> r;
    r.x = a.rx[j], r.v = a.rv[j], r.t = a.rt[j], r.c = meLoadC(a.rc, j);
    if constexpr (AVC)
    {
        r.g[0] = a.dV11[j], r.g[1] = a.dV12[j], r.g[2] = a.dV13[j];
        r.g[3] = a.dV22[j], r.g[4] = a.dV23[j], r.g[5] = a.dV33[j];
    }
    return r;
}

/*! momentum + energy as a persistent kernel: the momentum records (80 B, 104 with avClean) fill the CU's LDS with one
 *  workgroup, so nothing overlaps a cluster's dependent load chain (targets -> union indices -> union records ->
 *  staging) but the loads of the next cluster: each workgroup walks its XCD's clusters and issues the next cluster's
 *  setup and union-index loads before the neighbor loop and its union records after it, so they land during the
 *  loop and the share combination.  Measured before this form (Sedov 64M): the kernel without its neighbor loop took
 *  7.9 of 21.4 ms. */
template<int CH, int SPLIT, bool AVC>
__global__ __launch_bounds__(kB * SPLIT) void momentumEnergyKernel(PairArgs a, uint32_t numClusters)
{
    __shared__ float4 sP[CH]; // x, y, z, 1/h
    __shared__ float4 sV[CH]; // vx, vy, vz, c
    __shared__ float4 sT[CH]; // m, xm, rho, m*prho
    __shared__ float4 sA[CH]; // alpha, c11, c12, c13
    __shared__ float4 sB[CH]; // c22, c23, c33, m/rho
    __shared__ float4 sG[AVC ? CH : 1];  // dV11, dV12, dV13, dV22 (avClean)
    __shared__ float2 sG2[AVC ? CH : 1]; // dV23, dV33
    __shared__ float  s_ext[kClusterWaves * SPLIT];
    __shared__ float  s_red[kClusterWaves * SPLIT];
    using Pre                  = MePre<CH, SPLIT, AVC>;
    constexpr int  NT          = Pre::NT, S = Pre::S, SP = Pre::SP;
    const int      wave        = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int      sub         = wave & (kClusterWaves - 1);
    const int      part        = wave / kClusterWaves;
    const int      tid         = sub * kWave + lane;
    const uint32_t ucapLoad    = min((uint32_t)CH, a.ucap);
    constexpr uint32_t kNone   = ~0u; // no further cluster (ids come from clusterList when given, not from [0, n))

    // t-th cluster of this workgroup: virtual block blockIdx.x + t * gridDim.x (gridDim a multiple of 8, so every
    // virtual block stays on this workgroup's XCD) through the XCD-contiguous mapping of the non-persistent kernels
    auto clusterAt = [&](uint32_t t) -> uint32_t {
        const uint64_t b = (uint64_t)blockIdx.x + (uint64_t)t * gridDim.x;
        if (b >= numClusters) return kNone;
        const uint32_t blk = xcdBlock((uint32_t)b, numClusters);
        return a.clusterList ? a.clusterList[blk] : blk;
    };
    auto prefetch = [&](uint32_t c) {
        Pre p;
        p.c = c;
        p.U = 0, p.nc = 1, p.act = 1, p.lB = false;
#pragma unroll
        for (int s = 0; s < S; ++s)
            p.js[s] = 0u;
        if (c == kNone) return p;
        const uint32_t c0 = __builtin_amdgcn_readfirstlane(a.first + c * kCluster), i = c0 + tid;
        const bool     in = c * kClusterWaves + sub < a.numGroups && i < a.last;
        const uint32_t iL = in ? i : c0;
        p.lB              = listsB(a.lb, c);
        p.U               = p.lB ? a.lb.ucount[c] : a.ucount[c];
        p.o               = a.rx[c0];
        p.nc              = in ? a.nc[i] : 1u;
        p.act             = (in && a.active) ? a.active[i] : (uint8_t)1;
        p.ri = a.rx[iL], p.vi = a.rv[iL], p.ti = a.rt[iL], p.ci = meLoadC(a.rc, iL);
        if constexpr (AVC)
        {
            p.gi[0] = a.dV11[iL], p.gi[1] = a.dV12[iL], p.gi[2] = a.dV13[iL];
            p.gi[3] = a.dV22[iL], p.gi[4] = a.dV23[iL], p.gi[5] = a.dV33[iL];
        }
        const uint32_t* un = a.uni + (size_t)c * a.ucap + (p.lB ? a.lb.uoff : 0u);
#pragma unroll
        for (int s = 0; s < S; ++s)
        {
            const uint32_t u = threadIdx.x + s * NT;
            p.js[s]          = u < ucapLoad ? un[u] : 0u; // in the cluster's union segment; entries >= U unused
        }
        return p;
    };
    // every slot is loaded (particle 0's records where nothing is staged): a load under a branch is merged with the
    // branch's alternative right after it, and that merge waited for the load there -- before the share combination
    // it is meant to overlap -- instead of at the next cluster's staging
    auto loadRecords = [&](const Pre& p, MeRaw<AVC> (&rr)[SP]) {
        const bool use = p.c != kNone && p.U <= (uint32_t)CH;
#pragma unroll
        for (int s = 0; s < SP; ++s)
        {
            const bool ok = use && threadIdx.x + s * NT < p.U;
            rr[s]         = meLoadRaw<AVC>(a, ok ? p.js[s] : 0u);
        }
    };

    float      waveMinDt = INFINITY;
    uint32_t   t         = 0;
    Pre        cur       = prefetch(clusterAt(0));
    MeRaw<AVC> rr[SP];
    loadRecords(cur, rr);
    while (cur.c != kNone)
    {
        // ---- cluster setup from the prefetched data (the same fields as setup<SPLIT>)
        Clu cu;
        cu.part            = part;
        cu.tid             = tid;
        cu.c               = cur.c;
        cu.gw              = cu.c * kClusterWaves + sub;
        const uint32_t c0  = a.first + cu.c * kCluster;
        cu.i               = c0 + tid;
        cu.valid           = cu.gw < a.numGroups && cu.i < a.last && cur.act != 0;
        cu.iSafe           = cu.valid ? cu.i : c0;
        cu.cnt             = 0;
        if (cu.valid)
        {
            const unsigned c1 = cur.nc - 1;
            cu.cnt            = c1 < a.ngmax ? c1 : a.ngmax;
        }
        const uint32_t nw = (cu.cnt + 1) >> 1;
        cu.wBeg           = nw * cu.part / SPLIT;
        cu.wEnd           = nw * (cu.part + 1) / SPLIT;
        cu.U              = cur.U;
        cu.un             = a.uni + (size_t)cu.c * a.ucap + (cur.lB ? a.lb.uoff : 0u);
        cu.nl             = (cur.lB ? a.lb.nloc : a.nloc) + (size_t)cu.gw * nlocWords(a.ngmax) * kWave + lane;
        const RecX o      = cur.o;
        cu.ox = o.x, cu.oy = o.y, cu.oz = o.z;
        // lanes outside the view read the cluster's first particle, as setup<SPLIT> does
        const RecX  ri  = cu.valid ? cur.ri : o;
        const RecV  vi  = cur.vi;
        const RecT  ti  = cur.ti;
        RecC ci6;
        ci6.c11 = cur.ci.a.x, ci6.c12 = cur.ci.a.y, ci6.c13 = cur.ci.a.z, ci6.c22 = cur.ci.a.w;
        ci6.c23 = cur.ci.b.x, ci6.c33 = cur.ci.b.y;
        {
            const float h2  = 2.0f * ri.h;
            float       ext = 0.0f;
            if (a.box.pbc[0]) ext = fmaxf(ext, (fabsf(relc(ri.x, cu.ox, a.box, 0)) + h2) * (float)a.box.il[0]);
            if (a.box.pbc[1]) ext = fmaxf(ext, (fabsf(relc(ri.y, cu.oy, a.box, 1)) + h2) * (float)a.box.il[1]);
            if (a.box.pbc[2]) ext = fmaxf(ext, (fabsf(relc(ri.z, cu.oz, a.box, 2)) + h2) * (float)a.box.il[2]);
            ext = waveMax(ext);
            if (lane == 0) s_ext[wave] = ext;
            __syncthreads(); // also: every thread is done with the previous cluster's records and share sums
            float e = s_ext[0];
            for (int w = 1; w < kClusterWaves * SPLIT; ++w)
                e = fmaxf(e, s_ext[w]);
            cu.pbc = __builtin_amdgcn_readfirstlane(e >= 0.49f ? 1 : 0);
        }

        auto stageRaw = [&](const MeRaw<AVC>& q, uint32_t slot) {
            const RecX& r   = q.x;
            const RecT& tq  = q.t;
            const MeC&  c6  = q.c;
            const float rho = tq.kx * r.m / tq.xm;
            sP[slot]        = make_float4(relc(r.x, cu.ox, a.box, 0), relc(r.y, cu.oy, a.box, 1),
                                   relc(r.z, cu.oz, a.box, 2), 1.0f / r.h);
            sV[slot]        = make_float4(q.v.vx, q.v.vy, q.v.vz, q.v.c);
            sT[slot]        = make_float4(r.m, tq.xm, rho, r.m * tq.prho);
            sA[slot]        = make_float4(tq.alpha, c6.a.x, c6.a.y, c6.a.z);
            sB[slot]        = make_float4(c6.a.w, c6.b.x, c6.b.y, r.m / rho);
            if constexpr (AVC)
            {
                sG[slot]  = make_float4(q.g[0], q.g[1], q.g[2], q.g[3]);
                sG2[slot] = make_float2(q.g[4], q.g[5]);
            }
        };
        bool res = false;
        if (cu.U <= (uint32_t)CH)
        {
#pragma unroll
            for (int s = 0; s < S; ++s)
            {
                const uint32_t u = threadIdx.x + s * NT;
                if (u < cu.U) stageRaw(s < SP ? rr[s < SP ? s : 0] : meLoadRaw<AVC>(a, cur.js[s]), u);
            }
            __syncthreads();
            res = true;
        }
        // the next cluster's setup and union indices load during this cluster's neighbor loop
        const Pre nxt = prefetch(clusterAt(++t));

        const float xi = relc(ri.x, cu.ox, a.box, 0), yi = relc(ri.y, cu.oy, a.box, 1), zi = relc(ri.z, cu.oz, a.box, 2);
        const float hi = ri.h, mi = ri.m, ci = vi.c, h2 = 2.0f * hi;
        const float alpha_i = ti.alpha, xmassi = ti.xm, prhoi = ti.prho;
        const float rhoi    = ti.kx * mi / xmassi;
        const float rhoiInv = 1.0f / rhoi;
        const float lxi     = __log2f(xmassi);
        const float xmi2    = xmassi * xmassi;
        const float hiInv   = 1.0f / hi;
        const float hiInv2  = hiInv * hiInv;
        const float hiInv3  = hiInv2 * hiInv;
        const float Atmin = a.Atmin, Atmax = a.Atmax, ramp = a.ramp, AtminLo = a.Atmin * (1.0f - 0x1p-20f);
        float maxvsignali = 0.0f;
        float mx = 0, my = 0, mz = 0, energy = 0, a_visc_energy = 0;
        float gradV_i[6] = {0, 0, 0, 0, 0, 0};
        float eta_crit   = 0.0f;
        if constexpr (AVC)
        {
#pragma unroll
            for (int k = 0; k < 6; ++k)
                gradV_i[k] = cur.gi[k];
            eta_crit = avEtaCrit(cu.cnt);
        }
        auto loadRec = [&](uint32_t p) {
                RecM<AVC> r;
                r.p = sP[p], r.v = sV[p], r.t = sT[p], r.a = sA[p], r.b = sB[p];
                if constexpr (AVC) r.g = sG[p], r.g2 = sG2[p];
                return r;
            };
        auto computeOne = [&](const RecM<AVC>& r) {
                const float4 &P = r.p, &V = r.v, &T = r.t, &A = r.a, &B = r.b;
                float         rx = xi - P.x, ry = yi - P.y, rz = zi - P.z;
                pbcRule(cu, a.box, h2, rx, ry, rz);
                const float r2     = rx * rx + ry * ry + rz * rz;
                const float rinv   = rsqrtf(r2);
                const float vx_ij  = vi.vx - V.x, vy_ij = vi.vy - V.y, vz_ij = vi.vz - V.z;
                const float hjInv  = P.w;
                const float hjInv2 = hjInv * hjInv;
                const float hjInv3 = hjInv2 * hjInv;
                const float t1 = r2 * hiInv2, t2 = r2 * hjInv2; // squares of v1 = r/h_i, v2 = r/h_j
                const float Wi     = hiInv3 * kernelWt(t1);
                const float Wj     = hjInv3 * kernelWt(t2);
                // IAD directions u = c r; the reference's termA = -u W (momentum_energy_kern.hpp:134-146) is applied
                // by folding -W into the per-side coefficients below
                const float u1i = ci6.c11 * rx + ci6.c12 * ry + ci6.c13 * rz;
                const float u2i = ci6.c12 * rx + ci6.c22 * ry + ci6.c23 * rz;
                const float u3i = ci6.c13 * rx + ci6.c23 * ry + ci6.c33 * rz;
                const float u1j = A.y * rx + A.z * ry + A.w * rz;
                const float u2j = A.z * rx + B.x * ry + B.y * rz;
                const float u3j = A.w * rx + B.y * ry + B.z * rz;
                const float mj = T.x, rhoj = T.z, cj = V.w;
                float       rv = rx * vx_ij + ry * vy_ij + rz * vz_ij;
                if constexpr (AVC)
                {
                    const float gj[6] = {r.g.x, r.g.y, r.g.z, r.g.w, r.g2.x, r.g2.y};
                    rv += avRvCorrection<false>(rx, ry, rz, r2 * rinv * fminf(hiInv, hjInv), eta_crit, gradV_i, gj);
                }
                const float wij = rv * rinv;
                // artificial_viscosity (kernels.hpp:70-84), halved for the a_visc average below
                const float vij_signal = (alpha_i + A.x) * 0.25f * (ci + cj) - 2.0f * wij;
                const float halfVisc   = wij < 0.0f ? -0.5f * vij_signal * wij : 0.0f;
                const float vijsignal  = 0.5f * (ci + cj) - 2.0f * wij;
                maxvsignali            = vijsignal > maxvsignali ? vijsignal : maxvsignali;
                // Atwood = |rho_i - rho_j| / (rho_i + rho_j); the wave-uniform test of the common case (below Atmin
                // everywhere) multiplies instead of dividing, against a threshold lowered by 2^-20 so that every lane
                // whose rounded quotient reaches Atmin takes the exact branch
                const float drho = fabsf(rhoi - rhoj), srho = rhoi + rhoj;
                float       a_mom, b_mom;
                if (__ballot(drho >= AtminLo * srho) == 0)
                {
                    a_mom = xmi2; // the common case: below Atmin in every lane
                    b_mom = T.y * T.y;
                }
                else atwoodWeights(drho * __frcp_rn(srho), Atmin, Atmax, ramp, xmassi, lxi, T.y, a_mom, b_mom);
                const float a_visc     = mj * rhoiInv * halfVisc;
                const float b_visc     = B.w * halfVisc;
                const float momentum_i = mj * prhoi * a_mom;
                const float momentum_j = T.w * b_mom;
                // v_ij . termA_i and v_ij . termA_j
                const float di = -Wi * (vx_ij * u1i + vy_ij * u2i + vz_ij * u3i);
                const float dj = -Wj * (vx_ij * u1j + vy_ij * u2j + vz_ij * u3j);
                energy += mj * a_mom * di;
                a_visc_energy += a_visc * di + b_visc * dj;
                // momentum_i termA_i + momentum_j termA_j + a_visc (a_visc termA_i + b_visc termA_j)
                const float ki = -(momentum_i + a_visc) * Wi, kj = -(momentum_j + b_visc) * Wj;
                mx += ki * u1i + kj * u1j;
                my += ki * u2i + kj * u2j;
                mz += ki * u3i + kj * u3j;
            };
        neighborLoop<CH, SPLIT, false, SX_ME_LEAN>(
            cu, [&](uint32_t j, uint32_t slot) { stageRaw(meLoadRaw<AVC>(a, j), slot); }, loadRec, computeOne,
            res);
        // the next cluster's union records load during the share combination and this cluster's stores
        loadRecords(nxt, rr);
        {
            float v[6] = {mx, my, mz, energy, a_visc_energy, maxvsignali};
            combineShares<SPLIT>(cu, v, reinterpret_cast<float*>(sP), 32u, true);
            mx = v[0], my = v[1], mz = v[2], energy = v[3], a_visc_energy = v[4], maxvsignali = v[5];
        }
        float dt_lane = INFINITY;
        if (cu.valid && cu.part == 0)
        {
            if (a_visc_energy < 0.0f) a_visc_energy = 0.0f;
            a.du[cu.i] = a.K * (double)(prhoi * energy + 0.5f * a_visc_energy);
            a.ax[cu.i] = (float)(-a.K * (double)mx);
            a.ay[cu.i] = (float)(-a.K * (double)my);
            a.az[cu.i] = (float)(-a.K * (double)mz);
            dt_lane    = tsKCourant(maxvsignali, hi, ci, a.Kcour);
            if (a.dtOut) a.dtOut[cu.i] = dt_lane;
        }
        // wave min -> per-group minimum, and the workgroup's running minimum (momentum_energy_gpu.cu:94-118)
        const float wmin = waveMin(dt_lane);
        if (a.groupDt != nullptr && lane == 0 && cu.part == 0 && cu.gw < a.numGroups)
        {
            float old        = a.groupDt[cu.gw];
            a.groupDt[cu.gw] = wmin < old ? wmin : old;
        }
        waveMinDt = fminf(waveMinDt, wmin);
        cur       = nxt;
    }
    if (lane == 0) s_red[wave] = waveMinDt;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        float m = s_red[0];
        for (int w = 1; w < kClusterWaves * SPLIT; ++w)
            m = s_red[w] < m ? s_red[w] : m;
        if (a.blockDt) a.blockDt[blockIdx.x] = m;
        else atomicMinPos(a.minDt, m);
    }
}

// ---- std momentum + energy: momentumAndEnergyJLoop (hydro_std/momentum_energy_kern.hpp:12-134) ----------------
struct RecMS
{
    float4 p, v, a, b;
    float  m;
};

template<int CH, int SPLIT>
__global__ __launch_bounds__(kB * SPLIT) void momentumStdKernel(PairArgs a)
{
    __shared__ float4 sP[CH]; // x, y, z, 1/h
    __shared__ float4 sV[CH]; // vx, vy, vz, c
    __shared__ float4 sA[CH]; // c11, c12, c13, m/rho
    __shared__ float4 sB[CH]; // c22, c23, c33, p/rho
    __shared__ float  sM[CH]; // m
    __shared__ float  s_red[kClusterWaves * SPLIT];
    const Clu   cu  = setup<SPLIT>(a, s_red);
    const RecX  ri  = a.rx[cu.iSafe];
    const RecV  vi  = a.rv[cu.iSafe];
    const RecS  si  = a.rs[cu.iSafe];
    const RecC  ci6 = a.rc[cu.iSafe];
    const float xi = relc(ri.x, cu.ox, a.box, 0), yi = relc(ri.y, cu.oy, a.box, 1), zi = relc(ri.z, cu.oz, a.box, 2);
    const float hi = ri.h, ci = vi.c, h2 = 2.0f * hi;
    const float roi    = si.rho;
    const float mi_roi = ri.m / roi;
    const float prr_i  = si.p / (roi * roi); // gradh_i = 1
    const float hiInv  = 1.0f / hi;
    const float hiInv3 = hiInv * hiInv * hiInv;
    float maxvsignali = 0.0f;
    float mx = 0, my = 0, mz = 0, energy = 0;
    bool  res = false;
    neighborLoop<CH, SPLIT, false>(
        cu,
        [&](uint32_t j, uint32_t slot) {
            const RecX r  = a.rx[j];
            const RecV v  = a.rv[j];
            const RecS s  = a.rs[j];
            const RecC c6 = a.rc[j];
            sP[slot]      = make_float4(relc(r.x, cu.ox, a.box, 0), relc(r.y, cu.oy, a.box, 1),
                                   relc(r.z, cu.oz, a.box, 2), 1.0f / r.h);
            sV[slot]      = make_float4(v.vx, v.vy, v.vz, v.c);
            sA[slot]      = make_float4(c6.c11, c6.c12, c6.c13, r.m / s.rho);
            sB[slot]      = make_float4(c6.c22, c6.c23, c6.c33, s.p / s.rho);
            sM[slot]      = r.m;
        },
        [&](uint32_t p) { return RecMS{sP[p], sV[p], sA[p], sB[p], sM[p]}; },
        [&](const RecMS& r) {
            const float4 &P = r.p, &V = r.v, &A = r.a, &B = r.b;
            float         rx = xi - P.x, ry = yi - P.y, rz = zi - P.z;
            pbcRule(cu, a.box, h2, rx, ry, rz);
            const float r2     = rx * rx + ry * ry + rz * rz;
            const float rinv   = rsqrtf(r2);
            const float vx_ij  = vi.vx - V.x, vy_ij = vi.vy - V.y, vz_ij = vi.vz - V.z;
            const float hjInv  = P.w, hjInv2 = hjInv * hjInv;
            const float Wi     = hiInv3 * kernelWt(r2 * (hiInv * hiInv));
            const float Wj     = hjInv2 * hjInv * kernelWt(r2 * hjInv2);
            const float tA1i   = ci6.c11 * rx + ci6.c12 * ry + ci6.c13 * rz;
            const float tA2i   = ci6.c12 * rx + ci6.c22 * ry + ci6.c23 * rz;
            const float tA3i   = ci6.c13 * rx + ci6.c23 * ry + ci6.c33 * rz;
            const float tA1j   = A.x * rx + A.y * ry + A.z * rz;
            const float tA2j   = A.y * rx + B.x * ry + B.y * rz;
            const float tA3j   = A.z * rx + B.y * ry + B.z * rz;
            const float cj     = V.w;
            const float wij    = (rx * vx_ij + ry * vy_ij + rz * vz_ij) * rinv;
            // 0.5 * artificial_viscosity(1, 1, ci, cj, wij) (kernels.hpp:70-84)
            const float visc   = wij < 0.0f ? -0.5f * (0.5f * (ci + cj) - 2.0f * wij) * wij : 0.0f;
            maxvsignali        = fmaxf(maxvsignali, ci + cj - 3.0f * wij);
            const float mj_pro_i  = r.m * prr_i;
            const float mj_roj_Wj = A.w * Wj;
            const float am        = Wi * fmaf(visc, mi_roi, mj_pro_i);
            const float bm        = mj_roj_Wj * (B.w + visc);
            mx += am * tA1i + bm * tA1j;
            my += am * tA2i + bm * tA2j;
            mz += am * tA3i + bm * tA3j;
            const float ae = Wi * fmaf(visc, mi_roi, 2.0f * mj_pro_i);
            const float be = visc * mj_roj_Wj;
            energy += ae * (vx_ij * tA1i + vy_ij * tA2i + vz_ij * tA3i) +
                      be * (vx_ij * tA1j + vy_ij * tA2j + vz_ij * tA3j);
        },
        res);
    {
        float v[5] = {mx, my, mz, energy, maxvsignali};
        combineShares<SPLIT>(cu, v, reinterpret_cast<float*>(sP), 16u, true);
        mx = v[0], my = v[1], mz = v[2], energy = v[3], maxvsignali = v[4];
    }
    float dt_lane = INFINITY;
    if (cu.valid && cu.part == 0)
    {
        a.du[cu.i] = -a.K * 0.5 * (double)energy;
        a.ax[cu.i] = (float)(a.K * (double)mx);
        a.ay[cu.i] = (float)(a.K * (double)my);
        a.az[cu.i] = (float)(a.K * (double)mz);
        dt_lane    = tsKCourant(maxvsignali, hi, ci, a.Kcour);
        if (a.dtOut) a.dtOut[cu.i] = dt_lane;
    }
    const float wmin = waveMin(dt_lane);
    const int   wave = threadIdx.x >> 6;
    __syncthreads(); // s_red is reused
    if ((threadIdx.x & 63) == 0) s_red[wave] = wmin;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        float m = s_red[0];
        for (int w = 1; w < kClusterWaves * SPLIT; ++w)
            m = s_red[w] < m ? s_red[w] : m;
        if (a.blockDt) a.blockDt[blockIdx.x] = m;
        else atomicMinPos(a.minDt, m);
    }
}

// LDS capacity per kernel (records of 16 / 20 / 32 / 36 / 80 B): the momentum union fills the CU's 160 KiB with
// one workgroup; the lighter kernels keep two or more workgroups per CU.  SPLIT waves share each group's lists so a
// CU holds enough waves to reach the VALU's two-cycle issue (one wave alone issues every four cycles).
#ifndef SX_CH_ME
#define SX_CH_ME 2000
#endif
#ifndef SX_SPLIT_XM
#define SX_SPLIT_XM 2
#endif
#ifndef SX_SPLIT_VD
#define SX_SPLIT_VD 2
#endif
#ifndef SX_SPLIT_IAD
#define SX_SPLIT_IAD 2
#endif
#ifndef SX_SPLIT_AV_LARGE
#define SX_SPLIT_AV_LARGE 3 // the 2048-record launch runs two workgroups per CU: three shares keep six waves per SIMD
#endif
#ifndef SX_SPLIT_AV
#define SX_SPLIT_AV 2
#endif
#ifndef SX_SPLIT_ME
#define SX_SPLIT_ME 3 // 12 waves on the CU's one (persistent) momentum workgroup: the loop's 104 VGPRs + the next cluster's prefetch
#endif
#ifndef SX_SPLIT_ME_AVC
#define SX_SPLIT_ME_AVC 2 // the avClean variant needs 190 VGPRs: two waves per SIMD
#endif
// kChVd = 2000: 40 KB of records, four VeDefGradh workgroups per CU (eight waves per SIMD)
#ifndef SX_CH_IAD
#define SX_CH_IAD 1660 // 53 KB: three IAD workgroups per CU (24 waves at 79 VGPRs; 2 at CH 1900: 10.3 -> 9.4 ms at 64M)
#endif
#ifndef SX_CH_AV
#define SX_CH_AV 1470 // 53 KB: three AV workgroups per CU (2048: two; Sedov 64M AV 10.0 -> 8.6 ms, step -1.2 ms)
#endif
constexpr int kChXm = 2048, kChVd = 2000, kChIad = SX_CH_IAD, kChAv = SX_CH_AV, kChAvLarge = 2048, kChMe = SX_CH_ME,
              kChMeAvc = 1536;

static inline unsigned clusters(const PairArgs& a)
{
    return a.clusterList ? a.listCount : (a.numGroups + kClusterWaves - 1) / kClusterWaves;
}

void xmass(const PairArgs& a, hipStream_t s)
{
    if (a.numGroups && clusters(a)) xmassKernel<kChXm, SX_SPLIT_XM><<<clusters(a), kB * SX_SPLIT_XM, 0, s>>>(a);
}
void veDefGradh(const PairArgs& a, hipStream_t s)
{
    if (a.numGroups && clusters(a)) veDefGradhKernel<kChVd, SX_SPLIT_VD><<<clusters(a), kB * SX_SPLIT_VD, 0, s>>>(a);
}
void iadDivvCurlv(const PairArgs& a, hipStream_t s)
{
    if (a.numGroups && clusters(a)) iadDivvCurlvFusedKernel<kChIad, SX_SPLIT_IAD><<<clusters(a), kB * SX_SPLIT_IAD, 0, s>>>(a);
}
//! AV switches in two launches by union size: clusters whose union fits 1470 records run three workgroups per CU (53
//! KB), larger ones (the lattice's 122-neighbor steps: ~1485 per cluster) two per CU with 2048 records instead of the
//! chunked path; each launch's workgroups of the other class exit after one load
void avSwitches(const PairArgs& a, hipStream_t s)
{
    if (!a.numGroups || !clusters(a)) return;
    avSwitchesKernel<kChAv, SX_SPLIT_AV, 0, kChAv><<<clusters(a), kB * SX_SPLIT_AV, 0, s>>>(a);
    if (a.unionMax == 0 || a.unionMax > (uint32_t)kChAv) // else every workgroup of it would exit after one load
        avSwitchesKernel<kChAvLarge, SX_SPLIT_AV_LARGE, kChAv + 1, 0><<<clusters(a), kB * SX_SPLIT_AV_LARGE, 0, s>>>(a);
}
//! min over the per-workgroup Courant time-steps of one launch -> *minDt (one atomic)
__global__ __launch_bounds__(1024) void reduceBlockDtKernel(const float* v, uint32_t n, float* minDt)
{
    __shared__ float s_m[16];
    float            m = INFINITY;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
        m = fminf(m, v[i]);
    m = waveMin(m);
    if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
            m = fminf(m, s_m[w]);
        atomicMinPos(minDt, m);
    }
}
static void reduceBlockDt(const PairArgs& a, hipStream_t s)
{
    if (a.blockDt) reduceBlockDtKernel<<<1, 1024, 0, s>>>(a.blockDt, clusters(a), a.minDt);
}

//! workgroups of the persistent momentum kernel: one per CU (its records fill the LDS), a multiple of 8 (XCDs)
static uint32_t momentumGrid(uint32_t numClusters)
{
    static int cus[64] = {};
    int        dev     = 0;
    (void)hipGetDevice(&dev);
    int& n = cus[dev & 63];
    if (n == 0)
    {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        n = std::max(8, n & ~7);
    }
    return std::min<uint32_t>(numClusters, (uint32_t)n);
}

void momentumEnergy(const PairArgs& a, hipStream_t s)
{
    const uint32_t ncl = clusters(a);
    if (!a.numGroups || !ncl) return;
    const uint32_t grid = momentumGrid(ncl);
    if (a.avClean) momentumEnergyKernel<kChMeAvc, SX_SPLIT_ME_AVC, true><<<grid, kB * SX_SPLIT_ME_AVC, 0, s>>>(a, ncl);
    else momentumEnergyKernel<kChMe, SX_SPLIT_ME, false><<<grid, kB * SX_SPLIT_ME, 0, s>>>(a, ncl);
    if (a.blockDt) reduceBlockDtKernel<<<1, 1024, 0, s>>>(a.blockDt, grid, a.minDt);
}
// std propagator: the IAD kernel without velocity derivatives (16 B records), momentum with 68 B records
constexpr int kChIadStd = 2048, kChMeStd = 2048;
void iadStd(const PairArgs& a, hipStream_t s)
{
    if (a.numGroups && clusters(a)) iadDivvCurlvKernel<kChIadStd, SX_SPLIT_IAD, true><<<clusters(a), kB * SX_SPLIT_IAD, 0, s>>>(a);
}
void momentumStd(const PairArgs& a, hipStream_t s)
{
    if (!a.numGroups || !clusters(a)) return;
    momentumStdKernel<kChMeStd, SX_SPLIT_ME><<<clusters(a), kB * SX_SPLIT_ME, 0, s>>>(a);
    reduceBlockDt(a, s);
}

} // namespace cluster
} // namespace sx
