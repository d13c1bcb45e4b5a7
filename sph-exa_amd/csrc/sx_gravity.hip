/*! @file sx_gravity.hip
 * @brief Self-gravity for gfx950: expansion centers + MAC radii, Cartesian quadrupole upsweep and the Barnes-Hut
 *        traversal with softened P2P (the ryoanji path of the reference, single rank, open box).
 *
 * Replaces MultipoleHolder::upsweep / compute (ryoanji/interface/multipole_holder.cuh:40-66, called from
 * ve_hydro.hpp:193-202) and the focus tree's expansion centers (octree_focus_mpi.hpp:325-459).  The arithmetic
 * follows the reference CPU functions (file compiled with -ffp-contract=off):
 *   upsweep   mass centers (source_center.hpp:69-97), setMac / computeVecMacR2 (macs.hpp:82-97, :130-143 of
 *             source_center.hpp), P2M (cartesian_qpole.hpp:88-126), M2M / addQuadrupole (:210-257): one thread
 *             per node in the reference's sequential order, so centers and multipoles are bit-identical;
 *   traverse  one wavefront per 64 consecutive targets = the reference's four target groups of 16
 *             (traversal_cpu.hpp:171): every 16-lane quarter keeps its own target box and MAC decisions
 *             (evaluateMac, macs.hpp:109-116), so each target sees exactly the reference's set of M2P nodes and P2P
 *             leaves.  The wave walks the union of the four opening sets 8 nodes x 8 octants at a time with a
 *             per-entry 4-bit quarter mask, collecting M2P nodes and P2P leaves into LDS lists that are evaluated
 *             in batches (node data by scalar loads, leaf sources staged through LDS).  M2P (cartesian_qpole.hpp:
 *             175-201) and P2P (kernel.hpp:514-535) in double with 1/sqrt like the reference's host path; only the
 *             summation order differs from the reference's depth-first walk.
 */
#include <type_traits>

#include "sx_gravity.hpp"

namespace sx
{

namespace
{

constexpr int kGStack = 320; //!< per-wave traversal stack (entries: node << 4 | quarter mask)
constexpr int kGList  = 176; //!< per-wave M2P / P2P interaction lists (LDS: 31 KB per workgroup, five per CU)

//! leaf index -> node index (the reference's leafToInternal + numInternalNodes)
__global__ void leafToNodeKernel(const int32_t* childOffsets, const int32_t* internalToLeaf, int numNodes,
                                 int32_t* leafToNode)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < numNodes && childOffsets[i] == 0) leafToNode[internalToLeaf[i]] = i;
}

//! cstone::massCenter<double> (source_center.hpp:69-81) per leaf, sequential like the reference
__global__ void leafCentersKernel(GravArgs a)
{
    int L = blockIdx.x * blockDim.x + threadIdx.x;
    if (L >= a.numLeaves) return;
    double c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    for (uint32_t i = a.layout[L]; i < a.layout[L + 1]; ++i)
    {
        double w = (double)a.m[i];
        c0 += w * a.x[i];
        c1 += w * a.y[i];
        c2 += w * a.z[i];
        c3 += w;
    }
    double invM = (c3 != 0.0) ? 1.0 / c3 : 0.0;
    double* c   = a.centers4 + 4 * (size_t)a.leafToNode[L];
    c[0] = c0 * invM, c[1] = c1 * invM, c[2] = c2 * invM, c[3] = c3;
}

//! CombineSourceCenter over the nodes of one level (cstone::upsweep, octree.hpp:584-602)
__global__ void upsweepCentersKernel(GravArgs a, int start, int end)
{
    int i = start + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= end) return;
    int c = a.childOffsets[i];
    if (!c) return;
    double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    for (int k = c; k < c + 8; ++k)
    {
        const double* q = a.centers4 + 4 * (size_t)k;
        double        w = q[3];
        s0 += w * q[0];
        s1 += w * q[1];
        s2 += w * q[2];
        s3 += w;
    }
    double  invM = (s3 != 0.0) ? 1.0 / s3 : 0.0;
    double* o    = a.centers4 + 4 * (size_t)i;
    o[0] = s0 * invM, o[1] = s1 * invM, o[2] = s2 * invM, o[3] = s3;
}

//! setMac: mac = 2 max(geo size) / theta + |com - geo center|, stored squared (0 for massless nodes)
__global__ void setMacKernel(GravArgs a)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.numNodes) return;
    double*       c  = a.centers4 + 4 * (size_t)i;
    const double* gc = a.geoCenters + 3 * (size_t)i;
    const double* gs = a.geoSizes + 3 * (size_t)i;
    double dx = c[0] - gc[0], dy = c[1] - gc[1], dz = c[2] - gc[2];
    double smax = gs[0] > gs[1] ? gs[0] : gs[1];
    smax        = smax > gs[2] ? smax : gs[2];
    double s    = sqrt(dx * dx + (dy * dy + dz * dz));
    double mac  = 2.0 * smax * (double)a.invTheta + s;
    c[3]        = (c[3] != 0.0) ? mac * mac : 0.0;
}

//! P2M<double, float, float> per leaf (float accumulators, each update formed in double)
__global__ void leafP2MKernel(GravArgs a)
{
    int L = blockIdx.x * blockDim.x + threadIdx.x;
    if (L >= a.numLeaves) return;
    const int     node = a.leafToNode[L];
    const double* cen  = a.centers4 + 4 * (size_t)node;
    float         gv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint32_t b = a.layout[L], e = a.layout[L + 1];
    if (b != e)
    {
        for (uint32_t i = b; i < e; ++i)
        {
            double m_i = (double)a.m[i];
            double rx = a.x[i] - cen[0], ry = a.y[i] - cen[1], rz = a.z[i] - cen[2];
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
    float* o = a.multipoles + 8 * (size_t)node;
    for (int k = 0; k < 8; ++k)
        o[k] = gv[k];
}

//! sum over each 16-lane group, in every lane of it
__device__ __forceinline__ double groupSumD(double v)
{
#pragma unroll
    for (int o = 8; o > 0; o >>= 1)
        v += __shfl_xor(v, o, 16);
    return v;
}

//! fast variant of leafCentersKernel + leafP2MKernel in one launch: 16 lanes per leaf, its particles across them, the
//! sums in double reduced over the group; the quadrupole's sums are rounded to float once instead of after every
//! particle.  A thread per leaf walked its
//! particles with every lane on another leaf, so the loads never coalesced (Evrard 14.1M: 0.75 + 0.76 ms per step;
//! 16 lanes per leaf in one launch: 0.16).  The leaves' multipoles need only their own centers, so they are formed before
//! the inner nodes' centers and MAC radii.  Same moments to double / float rounding; the exact variant keeps the
//! reference's sequential order (bit-identical upsweep).

__global__ __launch_bounds__(256) void leafMomentsWaveKernel(GravArgs a)
{
    // four leaves per wave, 16 lanes each: a leaf averages a few dozen particles, and the waves' dependent load chains
    // (leaf range -> particles -> reduction -> their second pass), not the arithmetic, set the time
    const int L    = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 4);
    const int t    = threadIdx.x & 15;
    const bool ok  = L < a.numLeaves;
    const uint32_t b = ok ? a.layout[L] : 0u, e = ok ? a.layout[L + 1] : 0u;
    // mass center (massCenter<double>): the sums reach every lane of the group (xor reduction)
    double c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    for (uint32_t i = b + t; i < e; i += 16)
    {
        const double w = (double)a.m[i];
        c0 += w * a.x[i];
        c1 += w * a.y[i];
        c2 += w * a.z[i];
        c3 += w;
    }
    c0 = groupSumD(c0), c1 = groupSumD(c1), c2 = groupSumD(c2), c3 = groupSumD(c3);
    const double invM = (c3 != 0.0) ? 1.0 / c3 : 0.0;
    const double cx = c0 * invM, cy = c1 * invM, cz = c2 * invM;
    // quadrupole about it (P2M; the leaf's particles are read again, from cache)
    double s[7] = {0, 0, 0, 0, 0, 0, 0};
    for (uint32_t i = b + t; i < e; i += 16)
    {
        const double m_i = (double)a.m[i];
        const double rx = a.x[i] - cx, ry = a.y[i] - cy, rz = a.z[i] - cz;
        s[0] += m_i;
        s[1] += rx * rx * m_i;
        s[2] += rx * ry * m_i;
        s[3] += rx * rz * m_i;
        s[4] += ry * ry * m_i;
        s[5] += ry * rz * m_i;
        s[6] += rz * rz * m_i;
    }
#pragma unroll
    for (int k = 0; k < 7; ++k)
        s[k] = groupSumD(s[k]);
    if (ok && t == 0)
    {
        const int node = a.leafToNode[L];
        double*   c    = a.centers4 + 4 * (size_t)node;
        c[0] = cx, c[1] = cy, c[2] = cz, c[3] = c3;
        float gv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (b != e)
        {
            for (int k = 0; k < 7; ++k)
                gv[k] = (float)s[k];
            const float traceQ = gv[1] + gv[4] + gv[6];
            gv[7]              = traceQ;
            gv[1]              = 3 * gv[1] - traceQ;
            gv[4]              = 3 * gv[4] - traceQ;
            gv[6]              = 3 * gv[6] - traceQ;
            gv[2] *= 3;
            gv[3] *= 3;
            gv[5] *= 3;
        }
        float* o = a.multipoles + 8 * (size_t)node;
        for (int k = 0; k < 8; ++k)
            o[k] = gv[k];
    }
}

//! M2M with addQuadrupole<float, double> over the nodes of one level (upsweepMultipoles, upsweep_cpu.hpp:71-86)
__global__ void upsweepMultipolesKernel(GravArgs a, int start, int end)
{
    int i = start + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= end) return;
    int c = a.childOffsets[i];
    if (!c) return;
    float         comp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const double* Xo      = a.centers4 + 4 * (size_t)i;
    for (int k = c; k < c + 8; ++k)
    {
        const double* Xi  = a.centers4 + 4 * (size_t)k;
        const float*  add = a.multipoles + 8 * (size_t)k;
        double rx = Xo[0] - Xi[0], ry = Xo[1] - Xi[1], rz = Xo[2] - Xi[2];
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
    float* o = a.multipoles + 8 * (size_t)i;
    for (int k = 0; k < 8; ++k)
        o[k] = comp[k];
}

//! M2P<double, double, float> (cartesian_qpole.hpp:175-201)
__device__ __forceinline__ void m2p(double (&acc)[4], double tx, double ty, double tz, const double* com, const float* M)
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
}

//! P2P<double, double, float, float> (kernel.hpp:514-535), softened with h_i + h_j
__device__ __forceinline__ void p2p(double (&acc)[4], double xi, double yi, double zi, double xj, double yj, double zj,
                                    float mj, float hi, float hj)
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
}

//! fast M2P on a staged record: r = t - c from float coordinates relative to the wave origin (for an accepted node
//! |c - o| is of the order of |r|, so the relative rounding stays ~2^-23), expansion in float with the raw v_rsq_f32
//! (rr > mac^2 > 0, never denormal).  A = {cx, cy, cz, M0}, B = {M1, M2, M3, M4}, C = {M5, M6}.
__device__ __forceinline__ void m2pRec(float (&acc)[4], float tx, float ty, float tz, const float4& A, const float4& B,
                                       const float2& C)
{
    const float r0 = tx - A.x, r1 = ty - A.y, r2 = tz - A.z;
    const float rr       = fmaf(r0, r0, fmaf(r1, r1, r2 * r2));
    const float r_minus1 = __builtin_amdgcn_rsqf(rr);
    const float r_minus2 = r_minus1 * r_minus1;
    const float r_minus5 = r_minus2 * r_minus2 * r_minus1;
    const float Qrx      = fmaf(r0, B.x, fmaf(r1, B.y, r2 * B.z));
    const float Qry      = fmaf(r0, B.y, fmaf(r1, B.w, r2 * C.x));
    const float Qrz      = fmaf(r0, B.z, fmaf(r1, C.x, r2 * C.y));
    const float rQr      = fmaf(r0, Qrx, fmaf(r1, Qry, r2 * Qrz));
#ifdef SX_M2P_V0
    const float rQrAndMonopole = (-2.5f * rQr * r_minus5 - A.w * r_minus1) * r_minus2;
    acc[0] -= fmaf(A.w, r_minus1, 0.5f * r_minus5 * rQr);
    acc[1] += fmaf(r_minus5, Qrx, rQrAndMonopole * r0);
    acc[2] += fmaf(r_minus5, Qry, rQrAndMonopole * r1);
    acc[3] += fmaf(r_minus5, Qrz, rQrAndMonopole * r2);
#else
    // the same expansion with the shared factors formed once (X = rQr r^-5, M0 r^-1) and every accumulation a fused
    // multiply-add into the running sum: 35 instead of 41 VALU per interaction (the reference's operation order is
    // kept by the exact variant, m2p(); this fast form agrees to float rounding)
    const float X    = rQr * r_minus5;
    const float M0r  = A.w * r_minus1;
    const float K    = fmaf(-2.5f, X, -M0r) * r_minus2; // rQrAndMonopole
    acc[0] -= fmaf(0.5f, X, M0r);
    acc[1] = fmaf(r_minus5, Qrx, fmaf(K, r0, acc[1]));
    acc[2] = fmaf(r_minus5, Qry, fmaf(K, r1, acc[2]));
    acc[3] = fmaf(r_minus5, Qrz, fmaf(K, r2, acc[3]));
#endif
}

typedef float v2f __attribute__((ext_vector_type(2)));

//! sum over the four 16-lane rows, in every lane: (r0 + r1) + (r2 + r3) by the gfx950 row-swap permutes (VALU, no
//! LDS crossbar round trip like __shfl_xor's ds_bpermute); the same sums in the same order as two xor shuffles
__device__ __forceinline__ float rowSum4(float v)
{
    const unsigned u = __float_as_uint(v);
    const auto     p = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    const float    a = __uint_as_float(p[0]) + __uint_as_float(p[1]);
    const unsigned w = __float_as_uint(a);
    const auto     q = __builtin_amdgcn_permlane32_swap(w, w, false, false);
    return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}

struct __attribute__((aligned(16))) GSrc
{
    double x, y, z;
    float  m, h;
};

#ifndef SX_GRAV_WPE
#define SX_GRAV_WPE 5 // 96 VGPRs: five waves per SIMD (a few spills, outside the evaluation loops)
#endif
//! COUNT: the per-target interaction counts (GravArgs::interactions, BhStats) -- a separate instantiation because the
//! counters' registers cost the traversal 9 SGPR and 4 VGPR spills and 3.6 ms at Evrard n=300 (A/B).  PBC: the walk
//! over the periodic images (GravArgs::numShells) -- likewise its own instantiation (the loop's state took the open
//! walk from 14 to 48 VGPR spills)
template<bool FAST, bool COUNT, bool PBC = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SX_GRAV_WPE))) void gravityTraverseKernel(GravArgs args)
{
    // the fields the traversal reads, as scalars: with the many closures below capturing the kernel argument by
    // reference, the compiler copied the whole struct to scratch and addressed it through flat pointers
    struct
    {
        const double *x, *y, *z, *centers4;
        const float * m, *h, *multipoles;
        const int32_t *childOffsets, *internalToLeaf;
        const uint32_t* layout;
        float *         ax, *ay, *az;
        double *        egrav, *waveE;
        uint32_t*       err;
        uint32_t        first, last;
        float           G;
        const uint8_t*  active;
        unsigned long long* inter;
    } const a{args.x, args.y, args.z, args.centers4, args.m, args.h, args.multipoles, args.childOffsets,
              args.internalToLeaf, args.layout, args.ax, args.ay, args.az, args.egrav, args.waveE, args.err, args.first,
              args.last,
              args.G, args.active, args.interactions};
    __shared__ int  s_stack[4][kGStack];
    __shared__ double s_tbox[4][4][6]; // per wave and quarter: target box center, half size
    __shared__ int  s_m2p[4][kGList];
    __shared__ int  s_p2p[4][kGList];
    __shared__ GSrc   s_src[FAST ? 1 : 4][kWave];
    __shared__ float4 s_srcF[FAST ? 4 : 1][2][kWave]; // fast P2P: source x, y, z relative to the wave origin, m
    __shared__ __attribute__((aligned(16))) float s_hF[FAST ? 4 : 1][2][kWave];
    __shared__ float4  s_tgt[4][kWave]; // the wave's targets relative to its origin, h
    __shared__ uint8_t s_idx[FAST ? 4 : 1][kWave]; // fast M2P: one quarter's accepted entries of the window
    __shared__ uint2   s_rng[FAST ? 4 : 1][FAST ? kGList : 1]; // fast P2P: particle range of each listed leaf

    const int      wave = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4;
    const uint32_t g    = xcdBlock(blockIdx.x, gridDim.x) * 4 + wave;
    const uint32_t i0   = a.first + g * kWave;
    if (i0 >= a.last) return; // whole wave
    const uint32_t i     = i0 + lane;
    // a group view's targets (the ve-bdt active rungs): the others are not traversed and keep their acceleration
    const bool     valid = i < a.last && (!a.active || a.active[i]);
    if (__ballot(valid) == 0ull)
    {
        if (lane == 0 && a.waveE) a.waveE[g] = 0.0;
        return;
    }
    const uint32_t iS    = valid ? i : i0;
    const double   xi = a.x[iS], yi = a.y[iS], zi = a.z[iS];
    const float    hi = a.h[iS];
    const uint64_t ltMask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    // fast variant: coordinates relative to the wave's first target, formed in double and rounded once
    const double ox = readfirstlaneD(xi), oy = readfirstlaneD(yi), oz = readfirstlaneD(zi); // lane 0's target
    const float  txr = (float)(xi - ox), tyr = (float)(yi - oy), tzr = (float)(zi - oz);

    // the quarters' target boxes (center, half size): wave-uniform, read by every node test; in LDS (broadcast reads)
    // -- as registers they did not stay scalar and were spilled to scratch inside the traversal loop
    double* const tb = &s_tbox[wave][0][0];
    // target box of each 16-lane quarter (computeCenterAndSize, traversal_cpu.hpp:43-59), over its valid targets
    // shifted by -(sx, sy, sz) (a periodic image, traversal_cpu.hpp:205-212)
    auto setBoxes = [&](double sx, double sy, double sz) {
        const double t0 = xi - sx, t1 = yi - sy, t2 = zi - sz;
        double       lo[3]  = {valid ? t0 : INFINITY, valid ? t1 : INFINITY, valid ? t2 : INFINITY};
        double       hiB[3] = {valid ? t0 : -INFINITY, valid ? t1 : -INFINITY, valid ? t2 : -INFINITY};
#pragma unroll
        for (int o = 8; o > 0; o >>= 1)
            for (int d = 0; d < 3; ++d)
            {
                lo[d]  = fmin(lo[d], __shfl_xor(lo[d], o, 16));
                hiB[d] = fmax(hiB[d], __shfl_xor(hiB[d], o, 16));
            }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
            for (int d = 0; d < 3; ++d)
            {
                const double l = __shfl(lo[d], 16 * qq), h = __shfl(hiB[d], 16 * qq);
                if (lane == 0) tb[6 * qq + d] = (h + l) * 0.5, tb[6 * qq + 3 + d] = (h - l) * 0.5;
            }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
    };
    if constexpr (!PBC) // the box itself, once (inline: as a call of the lambda the open walk took two more spills)
    {
        double lo[3]  = {valid ? xi : INFINITY, valid ? yi : INFINITY, valid ? zi : INFINITY};
        double hiB[3] = {valid ? xi : -INFINITY, valid ? yi : -INFINITY, valid ? zi : -INFINITY};
#pragma unroll
        for (int o = 8; o > 0; o >>= 1)
            for (int d = 0; d < 3; ++d)
            {
                lo[d]  = fmin(lo[d], __shfl_xor(lo[d], o, 16));
                hiB[d] = fmax(hiB[d], __shfl_xor(hiB[d], o, 16));
            }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
            for (int d = 0; d < 3; ++d)
            {
                const double l = __shfl(lo[d], 16 * qq), h = __shfl(hiB[d], 16 * qq);
                if (lane == 0) tb[6 * qq + d] = (h + l) * 0.5, tb[6 * qq + 3 + d] = (h - l) * 0.5;
            }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
    }
    // the image being walked: the targets' coordinates and the fast variant's origin, shifted
    using Shifted = std::conditional_t<PBC, double, const double>; // the open walk: plain copies of xi, ox
    Shifted xs = xi, ys = yi, zs = zi, oxs = ox, oys = oy, ozs = oz;
    const uint64_t bv     = __ballot(valid); // quarters with at least one valid target (lanes fill in order)
    const unsigned qValid = ((bv & 0xffffull) ? 1u : 0u) | (((bv >> 16) & 0xffffull) ? 2u : 0u) |
                            (((bv >> 32) & 0xffffull) ? 4u : 0u) | (((bv >> 48) & 0xffffull) ? 8u : 0u);
    // interaction statistics as the reference counts them (per target: sources evaluated by P2P, nodes by M2P), only
    // for the valid targets of a quarter (the lanes the evaluation pads with do not count); wave-uniform scalars
    const unsigned qn[4] = {(unsigned)__popcll(bv & 0xffffull), (unsigned)__popcll((bv >> 16) & 0xffffull),
                            (unsigned)__popcll((bv >> 32) & 0xffffull), (unsigned)__popcll(bv >> 48)};
    auto targetsOf = [&](unsigned mask) -> unsigned {
        return ((mask & 1u) ? qn[0] : 0u) + ((mask & 2u) ? qn[1] : 0u) + ((mask & 4u) ? qn[2] : 0u) +
               ((mask & 8u) ? qn[3] : 0u);
    };
    unsigned long long numP2P = 0, numM2P = 0;

    // evaluateMac: true = the target box is inside the node's acceptance radius (descend / P2P).  Massless nodes
    // (mac^2 = 0, setMac) never violate and are dropped by the caller: their M2P adds exactly zero, and skipping it
    // avoids 0 * inf when a target sits on the zero expansion center of an empty node.
    auto violates = [&](int node, unsigned mask, bool& massless) -> unsigned {
        const double* com = a.centers4 + 4 * (size_t)node;
        const double  c0 = com[0], c1 = com[1], c2 = com[2], mac2 = fabs(com[3]);
        massless          = mac2 == 0.0;
        unsigned      v   = 0;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
        {
            if (!((mask >> qq) & 1u)) continue;
            const double* bq = tb + 6 * qq;
            double d0 = fabs(bq[0] - c0) - bq[3], d1 = fabs(bq[1] - c1) - bq[4], d2 = fabs(bq[2] - c2) - bq[5];
            d0 += fabs(d0);
            d1 += fabs(d1);
            d2 += fabs(d2);
            d0 *= 0.5;
            d1 *= 0.5;
            d2 *= 0.5;
            if (d0 * d0 + (d1 * d1 + d2 * d2) < mac2) v |= 1u << qq;
        }
        return v;
    };

    double acc[4] = {0, 0, 0, 0};
    int    nM = 0, nP = 0, sp = 0;
    bool   overflow = false;

    // fast evaluation layout: lane 16 * sub + t evaluates target t of EVERY quarter qq against the sub-th of each
    // group of four interaction entries that quarter needs, so no lane idles on an entry its quarter did not accept.
    // Per quarter the lanes fetch that quarter's targets (qx..qh), sum into fq, and the four partial sums of a target
    // are added across subs into the target's own lane (sub == qq), which accumulates fo and, per flush, acc.
    const int sub = lane >> 4, tq = lane & 15;
    s_tgt[wave][lane] = make_float4(txr, tyr, tzr, hi); // SX_LOAD_QUARTER: one LDS read instead of five bpermutes
    float qx = 0, qy = 0, qz = 0, qh = 0;
    bool  qok = false;
    // per quarter its partial sums, folded across the four subs once per flush (not once per window / chunk)
    float fq[4][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}}, fo[4] = {0, 0, 0, 0};
#define SX_LOAD_QUARTER(qq)                                                                                            \
    {                                                                                                                  \
        const float4 t_ = s_tgt[wave][16 * (qq) + tq];                                                                 \
        qx = t_.x, qy = t_.y, qz = t_.z, qh = t_.w;                                                                    \
        qok = i0 + (uint32_t)(16 * (qq) + tq) < a.last;                                                                \
    }
#define SX_FOLD_QUARTER(qq)                                                                                            \
    _Pragma("unroll") for (int c_ = 0; c_ < 4; ++c_)                                                                  \
    {                                                                                                                  \
        const float v_ = rowSum4(fq[qq][c_]);                                                                          \
        if (sub == (qq)) fo[c_] += v_;                                                                                 \
        fq[qq][c_] = 0.0f;                                                                                             \
    }
#define SX_FOLD_ALL() SX_FOLD_QUARTER(0) SX_FOLD_QUARTER(1) SX_FOLD_QUARTER(2) SX_FOLD_QUARTER(3)
#define SX_FLUSH_FO()                                                                                                  \
    _Pragma("unroll") for (int c_ = 0; c_ < 4; ++c_) acc[c_] += (double)fo[c_], fo[c_] = 0.0f;
    auto flushM2P = [&]() {
        if constexpr (FAST)
        {
            // windows of 64 entries: each lane stages one node (center relative to the wave origin, multipole) into
            // LDS -- one load round trip per window instead of one per node -- then every quarter walks the entries
            // it accepted four at a time
            float4* sA = &s_srcF[wave][0][0];
            float4* sB = &s_srcF[wave][1][0];
            float2* sC = reinterpret_cast<float2*>(&s_hF[wave][0][0]);
            for (int b0 = 0; b0 < nM; b0 += kWave)
            {
                const int nw = min(kWave, nM - b0);
                unsigned  em = 0;
                __builtin_amdgcn_wave_barrier(); // the previous window's records have been read
                if (lane < nw)
                {
                    const int     e    = s_m2p[wave][b0 + lane];
                    const int     node = e >> 4;
                    const double* c    = a.centers4 + 4 * (size_t)node;
                    const float*  M    = a.multipoles + 8 * (size_t)node;
                    em                 = (unsigned)(e & 15);
                    sA[lane] = make_float4((float)(c[0] - oxs), (float)(c[1] - oys), (float)(c[2] - ozs), M[0]);
                    sB[lane] = make_float4(M[1], M[2], M[3], M[4]);
                    sC[lane] = make_float2(M[5], M[6]);
                }
                __builtin_amdgcn_s_waitcnt(0xc07f);
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int qq = 0; qq < 4; ++qq)
                {
                    // the window's entries this quarter accepted, compacted in LDS; lanes take them four at a time
                    const bool     mine = (em >> qq) & 1u;
                    const uint64_t W    = __ballot(mine);
                    const int      cnt  = __popcll(W);
                    if (cnt == 0) continue;
                    if constexpr (COUNT) numM2P += (unsigned long long)cnt * qn[qq];
                    SX_LOAD_QUARTER(qq)
                    __builtin_amdgcn_wave_barrier(); // the previous quarter's reads of s_idx are done
                    if (mine) s_idx[wave][__popcll(W & ltMask)] = (uint8_t)lane;
                    __builtin_amdgcn_s_waitcnt(0xc07f);
                    __builtin_amdgcn_wave_barrier();
                    if (qok)
                        for (int k = sub; k < cnt; k += 4)
                        {
                            const int e = s_idx[wave][k];
                            m2pRec(fq[qq], qx, qy, qz, sA[e], sB[e], sC[e]);
                        }
                }
            }
            SX_FOLD_ALL()
            SX_FLUSH_FO()
        }
        else
            for (int k = 0; k < nM; ++k)
            {
                const int e    = __builtin_amdgcn_readfirstlane(s_m2p[wave][k]);
                const int node = e >> 4;
                if constexpr (COUNT) numM2P += targetsOf((unsigned)(e & 15));
                if (valid && (((e & 15) >> q) & 1))
                    m2p(acc, xs, ys, zs, a.centers4 + 4 * (size_t)node, a.multipoles + 8 * (size_t)node);
            }
        nM = 0;
    };
    // fast P2P: leaf sources converted to float relative coordinates while staged; the next leaf chunk (<= 64
    // sources, one per lane) is loaded into registers while the current one is evaluated from LDS
    auto flushP2PFast = [&]() {
        // the particle ranges of all listed leaves are resolved first, one leaf per lane (two dependent loads per
        // 64 leaves instead of per leaf), into s_rng
        for (int b0 = 0; b0 < nP; b0 += kWave)
            if (b0 + lane < nP)
            {
                const int lidx              = a.internalToLeaf[s_p2p[wave][b0 + lane] >> 4];
                s_rng[wave][b0 + lane] = make_uint2(a.layout[lidx], a.layout[lidx + 1]);
            }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        int      ek = 0;
        uint32_t ec0 = 0, js = 0, jn = 0;
        unsigned jm = 0;
        auto     nextChunk = [&]() -> bool {
            while (ek < nP)
            {
                const int      e  = __builtin_amdgcn_readfirstlane(s_p2p[wave][ek]);
                const uint32_t s0 = __builtin_amdgcn_readfirstlane(s_rng[wave][ek].x);
                const uint32_t s1 = __builtin_amdgcn_readfirstlane(s_rng[wave][ek].y);
                if (s0 + ec0 < s1)
                {
                    js = s0 + ec0;
                    jn = min((uint32_t)kWave, s1 - js);
                    jm = (unsigned)(e & 15);
                    ec0 += kWave;
                    if (s0 + ec0 >= s1) ++ek, ec0 = 0;
                    // following list leaves with the same quarter mask whose particles continue this range (siblings
                    // of one node, appended together in SFC order) join the chunk up to 64 sources
                    while (ec0 == 0 && jn < (uint32_t)kWave && ek < nP)
                    {
                        const int      e2 = __builtin_amdgcn_readfirstlane(s_p2p[wave][ek]);
                        const uint32_t r0 = __builtin_amdgcn_readfirstlane(s_rng[wave][ek].x);
                        const uint32_t r1 = __builtin_amdgcn_readfirstlane(s_rng[wave][ek].y);
                        if ((unsigned)(e2 & 15) != jm || r0 != js + jn) break;
                        const uint32_t take = min((uint32_t)kWave - jn, r1 - r0);
                        jn += take;
                        if (take == r1 - r0) ++ek;
                        else ec0 = take;
                    }
                    return true;
                }
                ++ek, ec0 = 0;
            }
            return false;
        };
        // the next chunk's sources stay raw (double coordinates) until they are staged: a conversion right after
        // the loads would wait for them there, before the current chunk's evaluation they are meant to overlap
        double px = 0.0, py = 0.0, pz = 0.0;
        float  pm = 0.f, ph = 0.f;
        auto   loadRegs = [&]() {
            if ((uint32_t)lane < jn)
            {
                const uint32_t j = js + lane;
                px = a.x[j], py = a.y[j], pz = a.z[j], pm = a.m[j], ph = a.h[j];
            }
        };
        bool have = nextChunk();
        if (have) loadRegs();
        int buf = 0;
        while (have)
        {
            const uint32_t cn = jn;
            const unsigned cm = jm;
            if constexpr (COUNT) numP2P += (unsigned long long)cn * targetsOf(cm);
            __builtin_amdgcn_wave_barrier();
            {
                // source l goes to pair P = 4 (l / 8) + l % 4 as half (l / 4) % 2: the lane of sub s evaluates sources
                // s + 8j and s + 8j + 4 together; lanes [cn, roundup8(cn)) write massless far-away padding
                const uint32_t pad = (cn + 7u) & ~7u;
                if ((uint32_t)lane < pad)
                {
                    const bool  in = (uint32_t)lane < cn;
                    const int   P = (lane >> 3) * 4 + (lane & 3), hf = (lane >> 2) & 1;
                    float*      d = reinterpret_cast<float*>(&s_srcF[wave][buf][0]) + P * 8 + hf;
                    d[0] = in ? (float)(px - oxs) : 1e18f, d[2] = in ? (float)(py - oys) : 1e18f;
                    d[4] = in ? (float)(pz - ozs) : 1e18f, d[6] = in ? pm : 0.0f;
                    s_hF[wave][buf][P * 2 + hf] = in ? ph : 0.0f;
                }
            }
            have = nextChunk();
            if (have) loadRegs();
            __builtin_amdgcn_s_waitcnt(0xc07f); // lgkmcnt(0): the staged chunk has landed
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int qq = 0; qq < 4; ++qq)
            {
                if (!((cm >> qq) & 1u)) continue;
                SX_LOAD_QUARTER(qq)
                if (qok)
                {
                    // two sources per iteration in packed FP32 (v_pk_add/mul/fma_f32), the padding adds exact zeros
                    const float* sp = reinterpret_cast<const float*>(&s_srcF[wave][buf][0]);
                    const v2f    tx = {qx, qx}, ty = {qy, qy}, tz = {qz, qz}, th = {qh, qh};
                    v2f          f2[4] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
                    for (uint32_t s = sub, P = sub; s < cn; s += 8, P += 4)
                    {
                        const float4 A = *reinterpret_cast<const float4*>(sp + P * 8);
                        const float4 B = *reinterpret_cast<const float4*>(sp + P * 8 + 4);
                        const float2 H = *reinterpret_cast<const float2*>(&s_hF[wave][buf][P * 2]);
                        const v2f    dx = v2f{A.x, A.y} - tx, dy = v2f{A.z, A.w} - ty, dz = v2f{B.x, B.y} - tz;
                        const v2f    R2 = __builtin_elementwise_fma(dx, dx, __builtin_elementwise_fma(dy, dy, dz * dz));
                        const v2f    h_ij = th + v2f{H.x, H.y};
                        const v2f    hh   = h_ij * h_ij;
                        const v2f    invR = {__builtin_amdgcn_rsqf(fmaxf(R2.x, hh.x)),
                                             __builtin_amdgcn_rsqf(fmaxf(R2.y, hh.y))}; // >= h^2: no denormals
                        const v2f    invR3m = v2f{B.z, B.w} * invR * invR * invR;
                        f2[0] = __builtin_elementwise_fma(-invR3m, R2, f2[0]);
                        f2[1] = __builtin_elementwise_fma(dx, invR3m, f2[1]);
                        f2[2] = __builtin_elementwise_fma(dy, invR3m, f2[2]);
                        f2[3] = __builtin_elementwise_fma(dz, invR3m, f2[3]);
                    }
#pragma unroll
                    for (int c_ = 0; c_ < 4; ++c_)
                        fq[qq][c_] += f2[c_].x + f2[c_].y;
                }
            }
            buf ^= 1;
        }
        SX_FOLD_ALL()
        SX_FLUSH_FO()
        nP = 0;
    };
    auto flushP2P = [&]() {
        if constexpr (FAST) return flushP2PFast();
        for (int k = 0; k < nP; ++k)
        {
            const int      e    = __builtin_amdgcn_readfirstlane(s_p2p[wave][k]);
            const int      node = e >> 4;
            const bool     mine = valid && (((e & 15) >> q) & 1);
            const int      lidx = a.internalToLeaf[node];
            const uint32_t s0 = a.layout[lidx], s1 = a.layout[lidx + 1];
            if constexpr (COUNT) numP2P += (unsigned long long)(s1 - s0) * targetsOf((unsigned)(e & 15));
            for (uint32_t c0 = s0; c0 < s1; c0 += kWave)
            {
                const uint32_t cnt = min((uint32_t)kWave, s1 - c0);
                __builtin_amdgcn_wave_barrier();
                if ((uint32_t)lane < cnt)
                {
                    const uint32_t j = c0 + lane;
                    s_src[wave][lane] = GSrc{a.x[j], a.y[j], a.z[j], a.m[j], a.h[j]};
                }
                __builtin_amdgcn_s_waitcnt(0xc07f);
                __builtin_amdgcn_wave_barrier();
                if (mine)
                    for (uint32_t s = 0; s < cnt; ++s)
                    {
                        const GSrc src = s_src[wave][s];
                        p2p(acc, xs, ys, zs, src.x, src.y, src.z, src.m, hi, src.h);
                    }
            }
        }
        nP = 0;
    };
    // append the entries of the lanes with `want` to a list (ballot compaction)
    auto append = [&](int* list, int& n, bool want, int entry) {
        const uint64_t b = __ballot(want);
        if (want) list[n + __popcll(b & ltMask)] = entry;
        n += __popcll(b);
    };

    // periodic images (computeGravity with numShells, traversal_cpu.hpp:200-216: iz, iy, ix; the targets shifted by
    // -(ix Lx, iy Ly, iz Lz)); numShells 0: the box itself
    const int ns = PBC ? args.numShells : 0;
    for (int iz = -ns; iz <= ns; ++iz)
    for (int iy = -ns; iy <= ns; ++iy)
    for (int ix = -ns; ix <= ns; ++ix)
    {
    if constexpr (PBC)
    {
        const double sx = ix * args.boxL[0], sy = iy * args.boxL[1], sz = iz * args.boxL[2];
        xs = xi - sx, ys = yi - sy, zs = zi - sz;
        oxs = ox - sx, oys = oy - sy, ozs = oz - sz;
        setBoxes(sx, sy, sz);
    }
    // root (singleTraversal, traversal.hpp:69-80)
    {
        bool           massless;
        const unsigned v = violates(0, qValid, massless);
        if ((qValid & ~v) && !massless) { s_m2p[wave][0] = (0 << 4) | (int)(qValid & ~v), nM = 1; }
        if (v)
        {
            if (a.childOffsets[0] == 0) { s_p2p[wave][0] = (int)v, nP = 1; }
            else { s_stack[wave][0] = (int)v, sp = 1; }
        }
        __builtin_amdgcn_wave_barrier();
    }
    // one call site per flush (the closures are then inlined and their captures stay in registers)
    while (true)
    {
        const bool done = sp == 0 || overflow;
        if (done || nM > kGList - kWave) flushM2P();
        if (done || nP > kGList - kWave) flushP2P();
        if (done) break;
        const int take = min(8, sp);
        sp -= take;
        const int  slot = lane >> 3, oct = lane & 7;
        const bool ok   = slot < take;
        const int  e    = ok ? s_stack[wave][sp + slot] : 0;
        __builtin_amdgcn_wave_barrier();
        const int      parent = e >> 4;
        const unsigned pmask  = ok ? (unsigned)(e & 15) : 0u;
        const int      child  = ok ? a.childOffsets[parent] + oct : 0;
        bool           massless = true;
        const unsigned v        = ok ? violates(child, pmask, massless) : 0u;
        const unsigned accept   = massless ? 0u : pmask & ~v;
        const bool     leaf   = ok && a.childOffsets[child] == 0;
        append(s_m2p[wave], nM, accept != 0, (child << 4) | (int)accept);
        append(s_p2p[wave], nP, v != 0 && leaf, (child << 4) | (int)v);
        {
            const bool     push = v != 0 && !leaf;
            const uint64_t b    = __ballot(push);
            if (sp + __popcll(b) > kGStack) overflow = true;
            else
            {
                if (push) s_stack[wave][sp + __popcll(b & ltMask)] = (child << 4) | (int)v;
                sp += __popcll(b);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    } // images
    if (overflow && lane == 0) atomicOr(a.err, 1u);

    // output: ax += G * acc (computeGravity, traversal_cpu.hpp:218-228), egrav = 0.5 sum G m_i phi_i
    double u = 0.0;
    if (valid)
    {
        const double G = (double)a.G;
        u              = (double)(a.G * a.m[i]) * acc[0];
        a.ax[i]        = (float)((double)a.ax[i] + G * acc[1]);
        a.ay[i]        = (float)((double)a.ay[i] + G * acc[2]);
        a.az[i]        = (float)((double)a.az[i] + G * acc[3]);
    }
    if (COUNT && lane == 0 && a.inter)
    {
        atomicAdd(a.inter, numP2P);
        atomicAdd(a.inter + 1, numM2P);
    }
    u = waveSum(u);
    if (lane == 0 && a.waveE) a.waveE[g] = 0.5 * u;
    else if (lane == 0 && a.egrav) atomicAdd(a.egrav, 0.5 * u);
#undef SX_LOAD_QUARTER
#undef SX_FOLD_QUARTER
#undef SX_FOLD_ALL
#undef SX_FLUSH_FO
}

inline unsigned grid(size_t n, int b = 256) { return (unsigned)((n + b - 1) / b); }

// ---- multi-rank gravity: level-6 cell multipoles, near/far classification, far tree --------------------------

//! mass center, MAC radius (setMac with the cell's geometry from the far tree) and quadrupole of each local cell
__global__ void cellMomentsKernel(const double* x, const double* y, const double* z, const float* m,
                                  const uint32_t* cellBeg, const uint32_t* cellIds, int nCells,
                                  const int32_t* farLeafToNode, const double* geoC, const double* geoS, float invTheta,
                                  GCell* out, int drift)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nCells) return;
    const uint32_t b = cellBeg[k], e = cellBeg[k + 1];
    double         c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    for (uint32_t i = b; i < e; ++i)
    {
        const double w = (double)m[i];
        c0 += w * x[i];
        c1 += w * y[i];
        c2 += w * z[i];
        c3 += w;
    }
    const double invM = c3 != 0.0 ? 1.0 / c3 : 0.0;
    GCell        g{};
    g.com[0] = c0 * invM, g.com[1] = c1 * invM, g.com[2] = c2 * invM;
    const int     node = farLeafToNode[cellIds[k]];
    const double* gc   = geoC + 3 * (size_t)node;
    const double* gs   = geoS + 3 * (size_t)node;
    // the MAC box: the cell (a sync's cells hold their particles), or the cell and its drifted particles
    double off[3] = {0.0, 0.0, 0.0}, hs[3] = {gs[0], gs[1], gs[2]};
    if (drift)
    {
        double lo[3] = {-gs[0], -gs[1], -gs[2]}, hi[3] = {gs[0], gs[1], gs[2]};
        for (uint32_t i = b; i < e; ++i)
        {
            const double r[3] = {x[i] - gc[0], y[i] - gc[1], z[i] - gc[2]};
            for (int d = 0; d < 3; ++d)
                lo[d] = fmin(lo[d], r[d]), hi[d] = fmax(hi[d], r[d]);
        }
        for (int d = 0; d < 3; ++d)
        {
            off[d] = 0.5 * (lo[d] + hi[d]);
            // the float copy in GCell::box (far-tree refresh) rounded outwards
            hs[d]  = (double)(float)(0.5 * (hi[d] - lo[d])) * (1.0 + 0x1p-20) + fabs((double)(float)off[d] - off[d]);
        }
    }
    for (int d = 0; d < 3; ++d)
        g.box[d] = (float)off[d], g.box[3 + d] = (float)hs[d];
    const double  dx = g.com[0] - (gc[0] + off[0]), dy = g.com[1] - (gc[1] + off[1]), dz = g.com[2] - (gc[2] + off[2]);
    const double  smax = fmax(fmax(hs[0], hs[1]), hs[2]);
    const double  mac  = 2.0 * smax * (double)invTheta + sqrt(dx * dx + (dy * dy + dz * dz));
    g.mac2             = c3 != 0.0 ? mac * mac : 0.0;
    float gv[8]        = {0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t i = b; i < e; ++i)
    {
        const double m_i = (double)m[i];
        const double rx = x[i] - g.com[0], ry = y[i] - g.com[1], rz = z[i] - g.com[2];
        gv[0] = (float)((double)gv[0] + m_i);
        gv[1] = (float)((double)gv[1] + rx * rx * m_i);
        gv[2] = (float)((double)gv[2] + rx * ry * m_i);
        gv[3] = (float)((double)gv[3] + rx * rz * m_i);
        gv[4] = (float)((double)gv[4] + ry * ry * m_i);
        gv[5] = (float)((double)gv[5] + ry * rz * m_i);
        gv[6] = (float)((double)gv[6] + rz * rz * m_i);
    }
    const float traceQ = gv[1] + gv[4] + gv[6];
    gv[7]              = traceQ;
    gv[1]              = 3 * gv[1] - traceQ;
    gv[4]              = 3 * gv[4] - traceQ;
    gv[6]              = 3 * gv[6] - traceQ;
    gv[2] *= 3;
    gv[3] *= 3;
    gv[5] *= 3;
    for (int q = 0; q < 8; ++q)
        g.q[q] = gv[q];
    g.cell  = cellIds[k];
    g.count = e - b;
    out[k]  = g;
}

//! one wave per remote cell: near[k] = 1 if the cell violates the vector MAC for any target box (c, s: center and
//! half-size, stride 8 doubles) -- such a cell's particles are needed as gravity halos.  PBC: the smallest distance
//! over the images shifted by -1, 0, +1 box lengths is taken per axis (the squared distance is a sum of per-axis
//! terms, so this is the minimum over all 27 images), and the MAC radius is widened by a relative 1e-9: a cell at
//! the acceptance boundary becomes near, never a far leaf that the image walk's own test (other rounding) opens
__global__ void cellNearKernel(const GCell* cells, int nCells, const double* boxes, int nBoxes, uint32_t* near,
                               double L0, double L1, double L2, int pbc)
{
    const int k    = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (k >= nCells) return;
    const GCell& g   = cells[k];
    bool         hit = false;
    const double mac2 = pbc ? g.mac2 * (1.0 + 1e-9) : g.mac2;
    if (g.mac2 != 0.0)
        for (int b = lane; b < nBoxes && !hit; b += 64)
        {
            const double* B  = boxes + 8 * (size_t)b;
            double        a0 = fabs(B[0] - g.com[0]), a1 = fabs(B[1] - g.com[1]), a2 = fabs(B[2] - g.com[2]);
            if (pbc)
            {
                a0 = fmin(a0, fabs(L0 - a0));
                a1 = fmin(a1, fabs(L1 - a1));
                a2 = fmin(a2, fabs(L2 - a2));
            }
            double d0 = a0 - B[3], d1 = a1 - B[4], d2 = a2 - B[5];
            d0 = d0 > 0 ? d0 : 0;
            d1 = d1 > 0 ? d1 : 0;
            d2 = d2 > 0 ? d2 : 0;
            hit = d0 * d0 + (d1 * d1 + d2 * d2) < mac2;
        }
    const bool any = __ballot(hit) != 0;
    if (lane == 0) near[k] = any ? 1u : 0u;
}

//! far-tree leaf boxes between syncs: a far cell's leaf takes the cell's MAC box (GCell::box, relative to the leaf's
//! geometric center)
__global__ void farLeafBoxKernel(GravArgs a, const GCell* cells, const uint32_t* far, int nCells, double* outC,
                                 double* outS)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nCells || !far[k]) return;
    const GCell& g    = cells[k];
    const int    node = a.leafToNode[g.cell];
    for (int d = 0; d < 3; ++d)
    {
        outC[3 * (size_t)node + d] = a.geoCenters[3 * (size_t)node + d] + (double)g.box[d];
        outS[3 * (size_t)node + d] = (double)g.box[3 + d];
    }
}

//! inner nodes of one level: the box holding their eight children's boxes (open box: no minimum image)
__global__ void unionBoxKernel(const int32_t* childOffsets, int b, int e, double* c, double* sz)
{
    const int node = b + blockIdx.x * blockDim.x + threadIdx.x;
    if (node >= e) return;
    const int c0 = childOffsets[node];
    if (c0 == 0) return;
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int k = c0; k < c0 + 8; ++k)
        for (int d = 0; d < 3; ++d)
        {
            lo[d] = fmin(lo[d], c[3 * (size_t)k + d] - sz[3 * (size_t)k + d]);
            hi[d] = fmax(hi[d], c[3 * (size_t)k + d] + sz[3 * (size_t)k + d]);
        }
    for (int d = 0; d < 3; ++d)
    {
        // rounded outwards: the union must hold every child box
        c[3 * (size_t)node + d]  = 0.5 * (lo[d] + hi[d]);
        sz[3 * (size_t)node + d] = 0.5 * (hi[d] - lo[d]) * (1.0 + 0x1p-40);
    }
}

//! far-tree leaves: cells with far[k] set get their mass center / mass and quadrupole, all other leaves are massless
__global__ void farLeavesKernel(GravArgs a, const GCell* cells, const uint32_t* far, int nCells)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nCells || !far[k]) return;
    const GCell& g    = cells[k];
    const int    node = a.leafToNode[g.cell];
    double*      c    = a.centers4 + 4 * (size_t)node;
    c[0] = g.com[0], c[1] = g.com[1], c[2] = g.com[2], c[3] = (double)g.q[0];
    float* o = a.multipoles + 8 * (size_t)node;
    for (int q = 0; q < 8; ++q)
        o[q] = g.q[q];
}

} // namespace

hipError_t cellMoments(const double* x, const double* y, const double* z, const float* m, const uint32_t* cellBeg,
                       const uint32_t* cellIds, int nCells, const int32_t* farLeafToNode, const double* geoC,
                       const double* geoS, float invTheta, GCell* out, hipStream_t s, bool drift)
{
    if (nCells > 0)
        cellMomentsKernel<<<grid(nCells), 256, 0, s>>>(x, y, z, m, cellBeg, cellIds, nCells, farLeafToNode, geoC, geoS,
                                                       invTheta, out, drift ? 1 : 0);
    return hipGetLastError();
}

hipError_t farRefreshBoxes(const GravArgs& a, const GCell* cells, const uint32_t* far, int nCells,
                           const int32_t* levelRangeHost, double* outC, double* outS, hipStream_t s)
{
    if (a.numNodes <= 0) return hipSuccess;
    (void)hipMemcpyAsync(outC, a.geoCenters, sizeof(double) * 3 * (size_t)a.numNodes, hipMemcpyDeviceToDevice, s);
    (void)hipMemcpyAsync(outS, a.geoSizes, sizeof(double) * 3 * (size_t)a.numNodes, hipMemcpyDeviceToDevice, s);
    if (nCells > 0) farLeafBoxKernel<<<grid(nCells), 256, 0, s>>>(a, cells, far, nCells, outC, outS);
    for (int level = kMaxLevel; level >= 0; --level)
    {
        const int b = levelRangeHost[level], e = levelRangeHost[level + 1];
        if (e > b) unionBoxKernel<<<grid(e - b), 256, 0, s>>>(a.childOffsets, b, e, outC, outS);
    }
    return hipGetLastError();
}

hipError_t cellNearFlags(const GCell* cells, int nCells, const double* boxes, int nBoxes, uint32_t* near, hipStream_t s,
                         const double* boxL)
{
    if (nCells > 0)
        cellNearKernel<<<grid((size_t)nCells * 64), 256, 0, s>>>(cells, nCells, boxes, nBoxes, near,
                                                                 boxL ? boxL[0] : 0.0, boxL ? boxL[1] : 0.0,
                                                                 boxL ? boxL[2] : 0.0, boxL ? 1 : 0);
    return hipGetLastError();
}

void combineRoots(const double cN[4], const float mN[8], const double cF[4], const float mF[8], double c[4], float m[8])
{
    // CombineSourceCenter over the two roots (weights: their masses), then the M2M of upsweepMultipolesKernel
    const double  wN = (double)mN[0], wF = (double)mF[0], W = wN + wF;
    const double  inv = W != 0.0 ? 1.0 / W : 0.0;
    for (int d = 0; d < 3; ++d)
        c[d] = (wN * cN[d] + wF * cF[d]) * inv;
    c[3] = W;
    float         comp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const double* Xi[2]   = {cN, cF};
    const float*  add[2]  = {mN, mF};
    for (int k = 0; k < 2; ++k)
    {
        if (add[k][0] == 0.0f) continue; // an empty tree (all cells near, or no locals): its center is meaningless
        const float* q  = add[k];
        double       rx = c[0] - Xi[k][0], ry = c[1] - Xi[k][1], rz = c[2] - Xi[k][2];
        double       rx_2 = rx * rx, ry_2 = ry * ry, rz_2 = rz * rz;
        double       r_2  = (rx_2 + ry_2 + rz_2) * (1.0 / 3.0);
        double       ml   = (double)(q[0] * 3);
        comp[7]           = (float)((double)(comp[7] + q[7]) + ml * r_2);
        comp[0] += q[0];
        comp[1] = (float)((double)comp[1] + ((double)q[1] + ml * (rx_2 - r_2)));
        comp[2] = (float)((double)comp[2] + ((double)q[2] + ml * rx * ry));
        comp[3] = (float)((double)comp[3] + ((double)q[3] + ml * rx * rz));
        comp[4] = (float)((double)comp[4] + ((double)q[4] + ml * (ry_2 - r_2)));
        comp[5] = (float)((double)comp[5] + ((double)q[5] + ml * ry * rz));
        comp[6] = (float)((double)comp[6] + ((double)q[6] + ml * (rz_2 - r_2)));
    }
    for (int k = 0; k < 8; ++k)
        m[k] = comp[k];
}

hipError_t farTreeLeafMap(const GravArgs& a, hipStream_t s)
{
    leafToNodeKernel<<<grid(a.numNodes), 256, 0, s>>>(a.childOffsets, a.internalToLeaf, a.numNodes, a.leafToNode);
    return hipGetLastError();
}

hipError_t farUpsweep(const GravArgs& a, const GCell* cells, const uint32_t* far, int nCells,
                      const int32_t* levelRangeHost, hipStream_t s)
{
    if (a.numNodes <= 0) return hipSuccess;
    (void)hipMemsetAsync(a.centers4, 0, sizeof(double) * 4 * (size_t)a.numNodes, s);
    (void)hipMemsetAsync(a.multipoles, 0, sizeof(float) * 8 * (size_t)a.numNodes, s);
    if (nCells > 0) farLeavesKernel<<<grid(nCells), 256, 0, s>>>(a, cells, far, nCells);
    for (int level = kMaxLevel; level >= 0; --level)
    {
        const int b = levelRangeHost[level], e = levelRangeHost[level + 1];
        if (e > b) upsweepCentersKernel<<<grid(e - b), 256, 0, s>>>(a, b, e);
    }
    setMacKernel<<<grid(a.numNodes), 256, 0, s>>>(a);
    for (int level = kMaxLevel; level >= 0; --level)
    {
        const int b = levelRangeHost[level], e = levelRangeHost[level + 1];
        if (e > b) upsweepMultipolesKernel<<<grid(e - b), 256, 0, s>>>(a, b, e);
    }
    return hipGetLastError();
}

hipError_t gravityUpsweep(const GravArgs& a, const int32_t* levelRangeHost, hipStream_t s)
{
    if (a.numNodes <= 0) return hipSuccess;
    leafToNodeKernel<<<grid(a.numNodes), 256, 0, s>>>(a.childOffsets, a.internalToLeaf, a.numNodes, a.leafToNode);
    if (a.fast) leafMomentsWaveKernel<<<grid((size_t)a.numLeaves * 16), 256, 0, s>>>(a); // centers + P2M
    else leafCentersKernel<<<grid(a.numLeaves), 256, 0, s>>>(a);
    for (int level = kMaxLevel; level >= 0; --level)
    {
        const int b = levelRangeHost[level], e = levelRangeHost[level + 1];
        if (e > b) upsweepCentersKernel<<<grid(e - b), 256, 0, s>>>(a, b, e);
    }
    setMacKernel<<<grid(a.numNodes), 256, 0, s>>>(a);
    if (!a.fast) leafP2MKernel<<<grid(a.numLeaves), 256, 0, s>>>(a);
    for (int level = kMaxLevel; level >= 0; --level)
    {
        const int b = levelRangeHost[level], e = levelRangeHost[level + 1];
        if (e > b) upsweepMultipolesKernel<<<grid(e - b), 256, 0, s>>>(a, b, e);
    }
    return hipGetLastError();
}

//! sum of the per-wave energies of one traversal -> *egrav (one atomic)
__global__ __launch_bounds__(1024) void reduceWaveEnergyKernel(const double* v, uint32_t n, double* egrav)
{
    __shared__ double s_e[16];
    double            e = 0.0;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
        e += v[i];
    e = waveSum(e);
    if ((threadIdx.x & 63) == 0) s_e[threadIdx.x >> 6] = e;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
            e += s_e[w];
        atomicAdd(egrav, e);
    }
}

hipError_t gravityTraverse(const GravArgs& a, hipStream_t s)
{
    if (a.last <= a.first) return hipSuccess;
    const uint32_t waves = (a.last - a.first + kWave - 1) / kWave;
    const unsigned g = (waves + 3) / 4;
    if (a.numShells > 0)
    {
        // periodic images: counting (BhStats) is not provided on this path
        if (a.fast) gravityTraverseKernel<true, false, true><<<g, 256, 0, s>>>(a);
        else gravityTraverseKernel<false, false, true><<<g, 256, 0, s>>>(a);
    }
    else if (a.interactions)
    {
        if (a.fast) gravityTraverseKernel<true, true><<<g, 256, 0, s>>>(a);
        else gravityTraverseKernel<false, true><<<g, 256, 0, s>>>(a);
    }
    else if (a.fast) gravityTraverseKernel<true, false><<<g, 256, 0, s>>>(a);
    else gravityTraverseKernel<false, false><<<g, 256, 0, s>>>(a);
    if (a.waveE && a.egrav) reduceWaveEnergyKernel<<<1, 1024, 0, s>>>(a.waveE, waves, a.egrav);
    return hipGetLastError();
}

} // namespace sx
