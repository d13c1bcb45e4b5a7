/*! @file sx_hydro.hip
 * @brief VE hydro kernels for gfx950: XMass, VeDefGradh, IAD + divv/curlv, AV switches, momentum + energy,
 *        EOS, position/energy integration and h update.
 *
 * Gather kernels: one wavefront per 64-particle SFC block, one lane per target particle; each lane walks its own
 * neighbor list (lane-interleaved, nidx[(block*ngmax + k)*64 + lane], coalesced 256 B per k, or the cluster
 * union positions of sx_neighbors.hip resolved through uni[]) and gathers the
 * neighbor's packed 16-byte-aligned records (RecX 32 B, RecV/RecT 16 B, RecC 32 B) -- 1-2 dwordx4 per record
 * instead of one dword gather per SoA field.  Tables are {t[i], t[i+1]-t[i]} pairs: one 8-byte gather per lookup.
 *
 * The per-pair arithmetic is the reference's, expression by expression (citations per kernel; the CPU
 * restatement with identical structure is oracle/sph_oracle.c).  Compiled twice, see sx_hydro.hpp.  The exact
 * variant always runs these kernels; the fast variant runs them only on global (imported) lists and otherwise the
 * LDS-staged cluster kernels of sx_hydro_cluster.hip.
 */
#include "sx_hydro.hpp"
#include "sx_sfc.hpp"

#ifndef SX_VARIANT
#error "SX_VARIANT must be exact or fast"
#endif

namespace sx
{
namespace SX_VARIANT
{

constexpr int kBlock = 256;
#define SX_STR2(x) #x
#define SX_STR(x) SX_STR2(x)
constexpr bool kFastClusters = SX_STR(SX_VARIANT)[0] == 'f';

#define SX_PAIR_PROLOGUE                                                                                               \
    const uint32_t gw   = (xcdBlock(blockIdx.x, gridDim.x) * kBlock + threadIdx.x) >> 6;                               \
    const uint32_t lane = threadIdx.x & 63;                                                                            \
    const uint32_t i     = a.first + gw * kGroupSize + lane;                                                           \
    const bool     valid = gw < a.numGroups && i < a.last && (!a.active || a.active[i]); /* no early return: barrier */\
    unsigned       cnt   = 0;                                                                                          \
    if (valid)                                                                                                         \
    {                                                                                                                  \
        unsigned c1 = a.nc[i] - 1;                                                                                     \
        cnt         = c1 < a.ngmax ? c1 : a.ngmax;                                                                     \
    }                                                                                                                  \
    const bool      lB = a.localLists && gw < a.numGroups && listsB(a.lb, gw / kClusterWaves);                       \
    const uint32_t* nb = a.localLists ? (lB ? a.lb.nloc : a.nloc) + (size_t)gw * nlocWords(a.ngmax) * kWave + lane    \
                                      : a.nidx + (size_t)gw * a.ngmax * kWave + lane;                                 \
    const uint32_t* un = a.localLists ? a.uni + (size_t)(gw / kClusterWaves) * a.ucap + (lB ? a.lb.uoff : 0u)        \
                                      : nullptr;                                                                       \
    auto nbj = [&](unsigned k) -> uint32_t {                                                                           \
        if (!a.localLists) return nb[(size_t)k * kWave];                                                               \
        uint32_t w = nb[(size_t)(k >> 1) * kWave];                                                                     \
        return un[(k & 1) ? (w >> 16) : (w & 0xffffu)];                                                                \
    };

//! xmassJLoop (hydro_ve/xmass_kern.hpp:50-79)
__global__ __launch_bounds__(kBlock) void xmassKernel(PairArgs a)
{
    SX_PAIR_PROLOGUE
    if (!valid) return;
    const RecX ri    = a.rx[i];
    float      hInv  = (float)(1.0 / ri.h);
    float      h3Inv = hInv * hInv * hInv;
    float      rho0i = ri.m;
    for (unsigned k = 0; k < cnt; ++k)
    {
        uint32_t   j  = nbj(k);
        const RecX rj = a.rx[j];
        float      xx = (float)(ri.x - rj.x);
        float      yy = (float)(ri.y - rj.y);
        float      zz = (float)(ri.z - rj.z);
        applyPBC(a.box, 2.0f * ri.h, xx, yy, zz);
        float dist = sqrtf(xx * xx + yy * yy + zz * zz);
        float vloc = dist * hInv;
        float w    = lookup(a.wh, vloc);
        rho0i += w * rj.m;
    }
    a.xm[i] = (float)((double)ri.m / ((double)rho0i * a.K * (double)h3Inv));
}

//! veDefGradhJLoop (hydro_ve/ve_def_gradh_kern.hpp:43-90)
__global__ __launch_bounds__(kBlock) void veDefGradhKernel(PairArgs a)
{
    SX_PAIR_PROLOGUE
    if (!valid) return;
    const RecX ri       = a.rx[i];
    const float xmassi  = a.rt[i].xm;
    float      hInv     = 1.0f / ri.h;
    float      h3Inv    = hInv * hInv * hInv;
    float      kxi      = xmassi;
    float      whomegai = -3.0f * xmassi;
    float      wrho0i   = -3.0f * ri.m;
    for (unsigned k = 0; k < cnt; ++k)
    {
        uint32_t   j  = nbj(k);
        const RecX rj = a.rx[j];
        float      xmassj = a.rt[j].xm;
        float      xx = (float)(ri.x - rj.x);
        float      yy = (float)(ri.y - rj.y);
        float      zz = (float)(ri.z - rj.z);
        applyPBC(a.box, 2.0f * ri.h, xx, yy, zz);
        float dist  = sqrtf(xx * xx + yy * yy + zz * zz);
        float vloc  = dist * hInv;
        float w     = lookup(a.wh, vloc);
        float dw    = lookup(a.whd, vloc);
        float dterh = -(3.0f * w + vloc * dw);
        kxi += w * xmassj;
        whomegai += dterh * xmassj;
        wrho0i += dterh * rj.m;
    }
    const double K = a.K;
    kxi            = (float)((double)kxi * (K * (double)h3Inv));
    whomegai       = (float)((double)whomegai * (K * (double)h3Inv * (double)hInv));
    wrho0i         = (float)((double)wrho0i * (K * (double)h3Inv * (double)hInv));
    whomegai       = (float)((double)(whomegai * ri.m / xmassi) +
                       ((double)kxi - K * (double)xmassi * (double)h3Inv) * (double)wrho0i);
    float rhoi     = kxi * ri.m / xmassi;
    float dhdrho   = -ri.h / (rhoi * 3.0f);
    a.kx[i]        = kxi;
    a.gradh[i]     = 1.0f - dhdrho * whomegai;
}

//! IADJLoop (hydro_ve/iad_kern.hpp:43-109) fused with divV_curlVJLoop (divv_curlv_kern.hpp:43-123), doGradV off
__global__ __launch_bounds__(kBlock) void iadDivvCurlvKernel(PairArgs a)
{
    SX_PAIR_PROLOGUE
    if (!valid) return;
    const RecX ri    = a.rx[i];
    const RecV vi    = a.rv[i];
    const float kxi  = a.rt[i].kx;
    float      hi    = ri.h;
    float      hiInv = 1.0f / hi;
    float      t11 = 0, t12 = 0, t13 = 0, t22 = 0, t23 = 0, t33 = 0;
    for (unsigned k = 0; k < cnt; ++k)
    {
        uint32_t   j  = nbj(k);
        const RecX rj = a.rx[j];
        const RecT tj = a.rt[j];
        float      rx = (float)(ri.x - rj.x);
        float      ry = (float)(ri.y - rj.y);
        float      rz = (float)(ri.z - rj.z);
        applyPBC(a.box, 2.0f * hi, rx, ry, rz);
        float dist   = sqrtf(rx * rx + ry * ry + rz * rz);
        float vloc   = dist * hiInv;
        float w      = lookup(a.wh, vloc);
        float volj_w = tj.xm / tj.kx * w;
        t11 += rx * rx * volj_w;
        t12 += rx * ry * volj_w;
        t13 += rx * rz * volj_w;
        t22 += ry * ry * volj_w;
        t23 += ry * rz * volj_w;
        t33 += rz * rz * volj_w;
    }
    float cc[6];
    iadInvert(t11, t12, t13, t22, t23, t33, hi, a.K, cc);
    const float c11i = cc[0], c12i = cc[1], c13i = cc[2], c22i = cc[3], c23i = cc[4], c33i = cc[5];
    a.c11[i]         = c11i;
    a.c12[i]         = c12i;
    a.c13[i]         = c13i;
    a.c22[i]         = c22i;
    a.c23[i]         = c23i;
    a.c33[i]         = c33i;

    // divV_curlVJLoop with the freshly computed c_ij of particle i (the CPU loop writes c_ij first, then reads them)
    float hiInv3 = hiInv * hiInv * hiInv;
    float dVx0 = 0, dVx1 = 0, dVx2 = 0, dVy0 = 0, dVy1 = 0, dVy2 = 0, dVz0 = 0, dVz1 = 0, dVz2 = 0;
    for (unsigned k = 0; k < cnt; ++k)
    {
        uint32_t   j  = nbj(k);
        const RecX rj = a.rx[j];
        const RecV vj = a.rv[j];
        float      xmassj = a.rt[j].xm;
        float      rx = (float)(ri.x - rj.x);
        float      ry = (float)(ri.y - rj.y);
        float      rz = (float)(ri.z - rj.z);
        applyPBC(a.box, 2.0f * hi, rx, ry, rz);
        float r2    = rx * rx + ry * ry + rz * rz;
        float dist  = sqrtf(r2);
        float vx_ji = vj.vx - vi.vx;
        float vy_ji = vj.vy - vi.vy;
        float vz_ji = vj.vz - vi.vz;
        float v1    = dist * hiInv;
        float Wi    = lookup(a.wh, v1);
        float tA0   = -(c11i * rx + c12i * ry + c13i * rz) * Wi;
        float tA1   = -(c12i * rx + c22i * ry + c23i * rz) * Wi;
        float tA2   = -(c13i * rx + c23i * ry + c33i * rz) * Wi;
        float fx = vx_ji * xmassj, fy = vy_ji * xmassj, fz = vz_ji * xmassj;
        dVx0 = dVx0 + tA0 * fx;
        dVx1 = dVx1 + tA1 * fx;
        dVx2 = dVx2 + tA2 * fx;
        dVy0 = dVy0 + tA0 * fy;
        dVy1 = dVy1 + tA1 * fy;
        dVy2 = dVy2 + tA2 * fy;
        dVz0 = dVz0 + tA0 * fz;
        dVz1 = dVz1 + tA1 * fz;
        dVz2 = dVz2 + tA2 * fz;
    }
    float norm_kxi = (float)(a.K * (double)hiInv3 / (double)kxi);
    a.divv[i]      = norm_kxi * (dVx0 + dVy1 + dVz2);
    if (a.curlv)
    {
        float cv0 = dVz1 - dVy2, cv1 = dVx2 - dVz0, cv2 = dVy0 - dVx1;
        a.curlv[i] = norm_kxi * sqrtf(cv0 * cv0 + (cv1 * cv1 + cv2 * cv2));
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

//! AVswitchesJLoop (hydro_ve/av_switches_kern.hpp:43-137); alpha is read-modify-write
__global__ __launch_bounds__(kBlock) void avSwitchesKernel(PairArgs a)
{
    SX_PAIR_PROLOGUE
    if (!valid) return;
    const RecX ri = a.rx[i];
    const RecV vi = a.rv[i];
    const RecC ci6 = a.rc[i];
    float      hi = ri.h, ci = vi.c;
    float      vijsignal_i = 1.e-40f * ci;
    float      hiInv       = 1.0f / hi;
    float      hiInv3      = hiInv * hiInv * hiInv;
    float      divv_i      = ci6.divv;
    float      gx = 0, gy = 0, gz = 0;
    for (unsigned k = 0; k < cnt; ++k)
    {
        uint32_t   j  = nbj(k);
        const RecX rj = a.rx[j];
        const RecV vj = a.rv[j];
        const RecT tj = a.rt[j];
        float      divvj = a.rc[j].divv;
        float      rx = (float)(ri.x - rj.x);
        float      ry = (float)(ri.y - rj.y);
        float      rz = (float)(ri.z - rj.z);
        applyPBC(a.box, 2.0f * hi, rx, ry, rz);
        float r2           = rx * rx + ry * ry + rz * rz;
        float dist         = sqrtf(r2);
        float vx_ij        = vi.vx - vj.vx;
        float vy_ij        = vi.vy - vj.vy;
        float vz_ij        = vi.vz - vj.vz;
        float rv           = rx * vx_ij + ry * vy_ij + rz * vz_ij;
        float vijsignal_ij = 0.0f;
        if (rv < 0.0f) { vijsignal_ij = ci + vj.c - 3.0f * rv / dist; }
        if (vijsignal_i < vijsignal_ij) vijsignal_i = vijsignal_ij;
        float v1     = dist * hiInv;
        float Wi     = (float)(a.K * (double)hiInv3 * (double)lookup(a.wh, v1));
        float termA1 = -(ci6.c11 * rx + ci6.c12 * ry + ci6.c13 * rz) * Wi;
        float termA2 = -(ci6.c12 * rx + ci6.c22 * ry + ci6.c23 * rz) * Wi;
        float termA3 = -(ci6.c13 * rx + ci6.c23 * ry + ci6.c33 * rz) * Wi;
        float volj   = tj.xm / tj.kx;
        float factor = volj * (divv_i - divvj);
        gx += factor * termA1;
        gy += factor * termA2;
        gz += factor * termA3;
    }
    float graddivv = sqrtf(gx * gx + gy * gy + gz * gz);
    float alphaloc = 0.0f;
    if (divv_i < 0.0f)
    {
        float a_const = hi * hi * graddivv;
        alphaloc      = a.alphamax * a_const / (a_const + hi * fabsf(divv_i) + 0.05f * ci);
    }
    float alpha_i = a.rt[i].alpha;
    if (alphaloc >= alpha_i) { alpha_i = alphaloc; }
    else
    {
        float decay    = hi / (a.decay_constant * vijsignal_i);
        float alphadot = 0.0f;
        if (alphaloc >= a.alphamin) { alphadot = (alphaloc - alpha_i) / decay; }
        else { alphadot = (a.alphamin - alpha_i) / decay; }
        const double dt = a.dtPtr ? *a.dtPtr : a.dt;
        alpha_i         = (float)((double)alpha_i + (double)alphadot * dt);
    }
    a.alpha[i] = alpha_i;
}

//! momentumAndEnergyJLoop<avClean> (hydro_ve/momentum_energy_kern.hpp:65-222) + Courant time-step
//! reduction (momentum_energy_gpu.cu:94-118).  tdpdTrho == nullptr => eCoeff = prho_i.
template<bool AVC>
__global__ __launch_bounds__(kBlock) void momentumEnergyKernel(PairArgs a)
{
    SX_PAIR_PROLOGUE
    float dt_lane = INFINITY;
    if (valid)
    {
        const RecX ri  = a.rx[i];
        const RecV vi  = a.rv[i];
        const RecT ti  = a.rt[i];
        const RecC ci6 = a.rc[i];
        float      hi = ri.h, mi = ri.m, ci = vi.c, kxi = ti.kx;
        float      alpha_i = ti.alpha;
        float      xmassi  = ti.xm;
        float      rhoi    = kxi * mi / xmassi;
        float      prhoi   = ti.prho;
        float      hiInv   = 1.0f / hi;
        float      hiInv3  = hiInv * hiInv * hiInv;
        float      maxvsignali = 0.0f;
        float      mx = 0, my = 0, mz = 0, energy = 0, a_visc_energy = 0;
        float      gradV_i[6] = {0, 0, 0, 0, 0, 0};
        float      eta_crit   = 0.0f;
        if constexpr (AVC)
        {
            gradV_i[0] = a.dV11[i], gradV_i[1] = a.dV12[i], gradV_i[2] = a.dV13[i];
            gradV_i[3] = a.dV22[i], gradV_i[4] = a.dV23[i], gradV_i[5] = a.dV33[i];
            eta_crit   = avEtaCrit(cnt);
        }
        for (unsigned k = 0; k < cnt; ++k)
        {
            uint32_t   j  = nbj(k);
            const RecX rj = a.rx[j];
            const RecV vj = a.rv[j];
            const RecT tj = a.rt[j];
            const RecC cj6 = a.rc[j];
            float      rx = (float)(ri.x - rj.x);
            float      ry = (float)(ri.y - rj.y);
            float      rz = (float)(ri.z - rj.z);
            applyPBC(a.box, 2.0f * hi, rx, ry, rz);
            float r2     = rx * rx + ry * ry + rz * rz;
            float dist   = sqrtf(r2);
            float vx_ij  = vi.vx - vj.vx;
            float vy_ij  = vi.vy - vj.vy;
            float vz_ij  = vi.vz - vj.vz;
            float hj     = rj.h;
            float hjInv  = 1.0f / hj;
            float v1     = dist * hiInv;
            float v2     = dist * hjInv;
            float hjInv3 = hjInv * hjInv * hjInv;
            float Wi     = hiInv3 * lookup(a.wh, v1);
            float Wj     = hjInv3 * lookup(a.wh, v2);
            float tA1i   = -(ci6.c11 * rx + ci6.c12 * ry + ci6.c13 * rz) * Wi;
            float tA2i   = -(ci6.c12 * rx + ci6.c22 * ry + ci6.c23 * rz) * Wi;
            float tA3i   = -(ci6.c13 * rx + ci6.c23 * ry + ci6.c33 * rz) * Wi;
            float tA1j   = -(cj6.c11 * rx + cj6.c12 * ry + cj6.c13 * rz) * Wj;
            float tA2j   = -(cj6.c12 * rx + cj6.c22 * ry + cj6.c23 * rz) * Wj;
            float tA3j   = -(cj6.c13 * rx + cj6.c23 * ry + cj6.c33 * rz) * Wj;
            float mj     = rj.m;
            float cj     = vj.c;
            float xmassj = tj.xm;
            float rhoj   = tj.kx * mj / xmassj;
            float rv     = rx * vx_ij + ry * vy_ij + rz * vz_ij;
            if constexpr (AVC)
            {
                const float gradV_j[6] = {a.dV11[j], a.dV12[j], a.dV13[j], a.dV22[j], a.dV23[j], a.dV33[j]};
                rv += avRvCorrection<!kFastClusters>(rx, ry, rz, v2 < v1 ? v2 : v1, eta_crit, gradV_i, gradV_j);
            }
            float wij    = rv / dist;
            // artificial_viscosity<float> (kernels.hpp:70-84): (alpha_i + alpha_j) / 4.0 is evaluated in double
            float viscosity_ij = 0.0f;
            if (wij < 0.0f)
            {
                float vij_signal =
                    (float)((double)(alpha_i + tj.alpha) / 4.0 * (double)(ci + cj) - (double)(2.0f * wij));
                viscosity_ij = -vij_signal * wij;
            }
            float vijsignal = 0.5f * (ci + cj) - 2.0f * wij;
            maxvsignali     = (vijsignal > maxvsignali) ? vijsignal : maxvsignali;
            float a_mom, b_mom;
            float Atwood = fabsf(rhoi - rhoj) / (rhoi + rhoj);
            if (Atwood < a.Atmin)
            {
                a_mom = xmassi * xmassi;
                b_mom = xmassj * xmassj;
            }
            else if (Atwood > a.Atmax)
            {
                a_mom = xmassi * xmassj;
                b_mom = a_mom;
            }
            else
            {
                // unqualified pow(float,float) in namespace sph resolves to ::pow(double,double)
                float sigma_ij = a.ramp * (Atwood - a.Atmin);
                a_mom = (float)(pow((double)xmassi, (double)(2.0f - sigma_ij)) * pow((double)xmassj, (double)sigma_ij));
                b_mom = (float)(pow((double)xmassj, (double)(2.0f - sigma_ij)) * pow((double)xmassi, (double)sigma_ij));
            }
            float a_visc   = mj / rhoi * viscosity_ij;
            float b_visc   = mj / rhoj * viscosity_ij;
            float a_visc_x = 0.5f * (a_visc * tA1i + b_visc * tA1j);
            float a_visc_y = 0.5f * (a_visc * tA2i + b_visc * tA2j);
            float a_visc_z = 0.5f * (a_visc * tA3i + b_visc * tA3j);
            a_visc_energy += a_visc_x * vx_ij + a_visc_y * vy_ij + a_visc_z * vz_ij;
            energy += mj * a_mom * (vx_ij * tA1i + vy_ij * tA2i + vz_ij * tA3i);
            float momentum_i = mj * prhoi * a_mom;
            float momentum_j = mj * tj.prho * b_mom;
            mx += momentum_i * tA1i + momentum_j * tA1j + a_visc_x;
            my += momentum_i * tA2i + momentum_j * tA2j + a_visc_y;
            mz += momentum_i * tA3i + momentum_j * tA3j + a_visc_z;
        }
        if (a_visc_energy < 0.0f) a_visc_energy = 0.0f;
        a.du[i] = a.K * (double)(prhoi * energy + 0.5f * a_visc_energy);
        a.ax[i] = (float)(-a.K * (double)mx);
        a.ay[i] = (float)(-a.K * (double)my);
        a.az[i] = (float)(-a.K * (double)mz);
        dt_lane = tsKCourant(maxvsignali, hi, ci, a.Kcour);
        if (a.dtOut) a.dtOut[i] = dt_lane;
    }
    // wave min -> block min -> one atomic per block (momentum_energy_gpu.cu:94-118)
    float wmin = waveMin(dt_lane);
    if (a.groupDt != nullptr && lane == 0 && gw < a.numGroups)
    {
        float old = a.groupDt[gw];
        a.groupDt[gw] = wmin < old ? wmin : old;
    }
    __shared__ float smin[kBlock / kWave];
    if (lane == 0) smin[threadIdx.x >> 6] = wmin;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        float m = smin[0];
        for (int w = 1; w < kBlock / kWave; ++w)
            m = smin[w] < m ? smin[w] : m;
        atomicMinPos(a.minDt, m);
    }
}

//! computeEOS_Impl (hydro_ve/eos.hpp:52-77), idealGasEOS (sph/eos.hpp:32-40)
__global__ void eosKernel(EosArgs a)
{
    uint32_t i = a.first + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.last) return;
    float  rho = a.kx[i] * a.m[i] / a.xm[i];
    double tmp = (double)idealGasCv(a.mui, a.gamma) * a.temp[i] * (a.gamma - 1.0);
    double pi  = (double)rho * tmp;
    double ci  = sqrt(tmp);
    const float prho = (float)(pi / (double)(a.kx[i] * a.m[i] * a.m[i] * a.gradh[i]));
    a.prho[i]        = prho;
    a.c[i]           = (float)ci;
    if (a.rho) a.rho[i] = rho;
    if (a.p) a.p[i] = (float)pi;
    if (a.rvOut) a.rvOut[i] = RecV{a.vx[i], a.vy[i], a.vz[i], (float)ci};
    if (a.rtOut) a.rtOut[i] = RecT{a.xm[i], a.kx[i], prho, a.alpha[i]};
}

// ---- std propagator (HydroProp, std_hydro.hpp:124-184) ----------------------------------------------------------

//! markRampJLoop (hydro_ve/additional_fields_kern.hpp:38-58) on the step's neighbor lists; rho = kx m / xm from
//! the field arrays (m from the packed RecX records)
__global__ __launch_bounds__(kBlock) void markRampKernel(PairArgs a)
{
    SX_PAIR_PROLOGUE
    if (!valid) return;
    const float rhoi = a.kx[i] * a.rx[i].m / a.xm[i];
    float       mark = 0.0f;
    for (unsigned k = 0; k < cnt; ++k)
    {
        const uint32_t j      = nbj(k);
        const float    rhoj   = a.kx[j] * a.rx[j].m / a.xm[j];
        const float    Atwood = fabsf(rhoi - rhoj) / (rhoi + rhoj);
        if (Atwood > a.Atmax) { mark += 1.0f; }
        else if (Atwood >= a.Atmin) { mark += a.ramp * (Atwood - a.Atmin); }
    }
    a.markRamp[i] = mark / (float)cnt;
}

//! convertXmassToRho (hydro_ve/xmass_gpu.cu:134-148): the xmass kernel wrote m / rho0 into rho
__global__ void xmassToRhoKernel(uint32_t first, uint32_t last, const float* m, float* rho)
{
    uint32_t i = first + blockIdx.x * blockDim.x + threadIdx.x;
    if (i < last) rho[i] = m[i] / rho[i];
}

//! cudaEOS_HydroStd (hydro_std/eos_gpu.cu:43-52): idealGasEOS(temp, rho, mui, gamma) in double (sph/eos.hpp:31-40)
__global__ void eosStdKernel(EosArgs a)
{
    uint32_t i = a.first + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.last) return;
    double tmp = (double)idealGasCv(a.mui, a.gamma) * a.temp[i] * (a.gamma - 1.0);
    a.p[i]     = (float)((double)a.rho[i] * tmp);
    a.c[i]     = (float)sqrt(tmp);
}

//! IADJLoopSTD (hydro_std/iad_kern.hpp:12-77): the IAD tensor with volumes m_j / rho_j
__global__ __launch_bounds__(kBlock) void iadStdKernel(PairArgs a)
{
    SX_PAIR_PROLOGUE
    if (!valid) return;
    const RecX ri    = a.rx[i];
    const float hi    = ri.h;
    const float hiInv = 1.0f / hi;
    float       t11 = 0, t12 = 0, t13 = 0, t22 = 0, t23 = 0, t33 = 0;
    for (unsigned k = 0; k < cnt; ++k)
    {
        uint32_t   j  = nbj(k);
        const RecX rj = a.rx[j];
        float      rx = (float)(ri.x - rj.x);
        float      ry = (float)(ri.y - rj.y);
        float      rz = (float)(ri.z - rj.z);
        applyPBC(a.box, 2.0f * hi, rx, ry, rz);
        float dist     = sqrtf(rx * rx + ry * ry + rz * rz);
        float w        = lookup(a.wh, dist * hiInv);
        float mj_roj_w = rj.m / a.rs[j].rho * w;
        t11 += rx * rx * mj_roj_w;
        t12 += rx * ry * mj_roj_w;
        t13 += rx * rz * mj_roj_w;
        t22 += ry * ry * mj_roj_w;
        t23 += ry * rz * mj_roj_w;
        t33 += rz * rz * mj_roj_w;
    }
    float cc[6];
    iadInvert(t11, t12, t13, t22, t23, t33, hi, a.K, cc);
    a.c11[i] = cc[0], a.c12[i] = cc[1], a.c13[i] = cc[2], a.c22[i] = cc[3], a.c23[i] = cc[4], a.c33[i] = cc[5];
}

//! momentumAndEnergyJLoop of the std propagator (hydro_std/momentum_energy_kern.hpp:12-134): gradh = 1, alpha = 1
//! with the halved AV; Courant time-step reduced as in cudaGradP (hydro_std/momentum_energy_gpu.cu:64-107)
__global__ __launch_bounds__(kBlock) void momentumStdKernel(PairArgs a)
{
    SX_PAIR_PROLOGUE
    float dt_lane = INFINITY;
    if (valid)
    {
        const RecX ri  = a.rx[i];
        const RecV vi  = a.rv[i];
        const RecS si  = a.rs[i];
        const RecC ci6 = a.rc[i];
        const float hi = ri.h, roi = si.rho, pri = si.p, ci = vi.c;
        const float mi_roi = ri.m / roi;
        const float hiInv  = 1.0f / hi;
        const float hiInv3 = hiInv * hiInv * hiInv;
        float       maxvsignali = 0.0f;
        float       mx = 0, my = 0, mz = 0, energy = 0;
        for (unsigned k = 0; k < cnt; ++k)
        {
            uint32_t   j   = nbj(k);
            const RecX rj  = a.rx[j];
            const RecV vj  = a.rv[j];
            const RecS sj  = a.rs[j];
            const RecC cj6 = a.rc[j];
            float      rx  = (float)(ri.x - rj.x);
            float      ry  = (float)(ri.y - rj.y);
            float      rz  = (float)(ri.z - rj.z);
            applyPBC(a.box, 2.0f * hi, rx, ry, rz);
            float r2     = rx * rx + ry * ry + rz * rz;
            float dist   = sqrtf(r2);
            float vx_ij  = vi.vx - vj.vx;
            float vy_ij  = vi.vy - vj.vy;
            float vz_ij  = vi.vz - vj.vz;
            float hjInv  = 1.0f / rj.h;
            float v1     = dist * hiInv;
            float v2     = dist * hjInv;
            float rv     = rx * vx_ij + ry * vy_ij + rz * vz_ij;
            float hjInv3 = hjInv * hjInv * hjInv;
            float Wi     = hiInv3 * lookup(a.wh, v1);
            float Wj     = hjInv3 * lookup(a.wh, v2);
            float tA1i   = ci6.c11 * rx + ci6.c12 * ry + ci6.c13 * rz;
            float tA2i   = ci6.c12 * rx + ci6.c22 * ry + ci6.c23 * rz;
            float tA3i   = ci6.c13 * rx + ci6.c23 * ry + ci6.c33 * rz;
            float tA1j   = cj6.c11 * rx + cj6.c12 * ry + cj6.c13 * rz;
            float tA2j   = cj6.c12 * rx + cj6.c22 * ry + cj6.c23 * rz;
            float tA3j   = cj6.c13 * rx + cj6.c23 * ry + cj6.c33 * rz;
            float roj    = sj.rho;
            float cj     = vj.c;
            float wij    = rv / dist;
            // 0.5 * artificial_viscosity(1, 1, ci, cj, wij) (kernels.hpp:70-84): (1 + 1) / 4.0 is a double
            float visc = 0.0f;
            if (wij < 0.0f)
            {
                float vij_signal = (float)((double)(1.0f + 1.0f) / 4.0 * (double)(ci + cj) - (double)(2.0f * wij));
                visc             = -vij_signal * wij;
            }
            const float viscosity_ij = 0.5f * visc;
            const float vijsignal    = ci + cj - 3.0f * wij;
            maxvsignali              = (vijsignal > maxvsignali) ? vijsignal : maxvsignali;
            const float mj        = rj.m;
            const float mj_roj_Wj = mj / roj * Wj;
            const float mj_pro_i  = mj * pri / (roi * roi); // gradh_i = 1
            const float am        = Wi * (mj_pro_i + viscosity_ij * mi_roi);
            const float bm        = mj_roj_Wj * (sj.p / roj + viscosity_ij); // gradh_j = 1
            mx += am * tA1i + bm * tA1j;
            my += am * tA2i + bm * tA2j;
            mz += am * tA3i + bm * tA3j;
            const float ae = Wi * (2.0f * mj_pro_i + viscosity_ij * mi_roi);
            const float be = viscosity_ij * mj_roj_Wj;
            energy += vx_ij * (ae * tA1i + be * tA1j) + vy_ij * (ae * tA2i + be * tA2j) + vz_ij * (ae * tA3i + be * tA3j);
        }
        a.du[i] = -a.K * 0.5 * (double)energy;
        a.ax[i] = (float)(a.K * (double)mx);
        a.ay[i] = (float)(a.K * (double)my);
        a.az[i] = (float)(a.K * (double)mz);
        dt_lane = tsKCourant(maxvsignali, hi, ci, a.Kcour);
        if (a.dtOut) a.dtOut[i] = dt_lane;
    }
    float wmin = waveMin(dt_lane);
    __shared__ float smin[kBlock / kWave];
    if (lane == 0) smin[threadIdx.x >> 6] = wmin;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        float m = smin[0];
        for (int w = 1; w < kBlock / kWave; ++w)
            m = smin[w] < m ? smin[w] : m;
        atomicMinPos(a.minDt, m);
    }
}

//! positionUpdate + putInBox + energyUpdate (positions.hpp:54-139, F2-correct as positions_gpu.cu:118-165)
__global__ void positionsKernel(PosArgs a)
{
    uint32_t i = a.first + blockIdx.x * blockDim.x + threadIdx.x;
    float    dv[3] = {0.0f, 0.0f, 0.0f}; // this step's displacement for the grid (every lane reaches it below)
    double   pc[3] = {0.0, 0.0, 0.0};
    bool     moved = false;
    if (i < a.last)
    {
        const DevBox& b    = a.box;
        bool          skip = false;
        if ((b.fbc[0] || b.fbc[1] || b.fbc[2]) && a.vx[i] == 0.0f && a.vy[i] == 0.0f && a.vz[i] == 0.0f)
        {
            double X[3] = {a.x[i], a.y[i], a.z[i]};
            for (int d = 0; d < 3; ++d)
            {
                double top = b.lim[2 * d + 1], bot = b.lim[2 * d];
                if (b.fbc[d] && (fabs(top - X[d]) < 2.0f * a.h[i] || fabs(bot - X[d]) < 2.0f * a.h[i])) skip = true;
            }
        }
        const double dt = a.dtPtr ? a.dtPtr[0] : a.dt, dt_m1 = a.dtPtr ? a.dtPtr[1] : a.dt_m1;
        if (!skip)
        {
            double A[3]  = {a.ax[i], a.ay[i], a.az[i]};
            double X[3]  = {a.x[i], a.y[i], a.z[i]};
            double dX[3] = {a.x_m1[i], a.y_m1[i], a.z_m1[i]};
            double Xn[3], Vn1[3], dXn1[3];
            double inv = 1.0 / dt_m1, hdm1 = 0.5 * dt_m1, adt = fabs(dt);
    #pragma unroll
            for (int k = 0; k < 3; ++k)
            {
                double Vnmhalf = dX[k] * inv;
                double Vn      = Vnmhalf + A[k] * hdm1;
                Vn1[k]         = Vn + A[k] * dt;
                dXn1[k]        = (Vn + (A[k] * 0.5) * adt) * dt;
                Xn[k]          = X[k] + dXn1[k];
            }
    #pragma unroll
            for (int d = 0; d < 3; ++d)
            {
                if (b.pbc[d] && Xn[d] > b.lim[2 * d + 1]) Xn[d] -= b.l[d];
                else if (b.pbc[d] && Xn[d] < b.lim[2 * d]) Xn[d] += b.l[d];
            }
            a.x[i]    = Xn[0];
            a.y[i]    = Xn[1];
            a.z[i]    = Xn[2];
            a.x_m1[i] = (float)dXn1[0];
            a.y_m1[i] = (float)dXn1[1];
            a.z_m1[i] = (float)dXn1[2];
            a.vx[i]   = (float)Vn1[0];
            a.vy[i]   = (float)Vn1[1];
            a.vz[i]   = (float)Vn1[2];
            if (a.keys) a.keys[i] = sfcKey(Xn[0], Xn[1], Xn[2], b);
            if (a.dispX)
            {
                // the move without the periodic wrap above (float; the filter's bounds allow for its rounding)
                dv[0] = (float)dXn1[0], dv[1] = (float)dXn1[1], dv[2] = (float)dXn1[2];
                a.dispX[i] = dv[0], a.dispY[i] = dv[1], a.dispZ[i] = dv[2];
                pc[0] = Xn[0], pc[1] = Xn[1], pc[2] = Xn[2];
                moved = true;
            }
        }
        else
        {
            if (a.keys) a.keys[i] = sfcKey(a.x[i], a.y[i], a.z[i], b);
            if (a.dispX) a.dispX[i] = 0.0f, a.dispY[i] = 0.0f, a.dispZ[i] = 0.0f;
            if (a.dispX) pc[0] = a.x[i], pc[1] = a.y[i], pc[2] = a.z[i], moved = true;
        }
        double u_old = (double)a.constCv * a.temp[i];
        double du = a.du[i], du_m1 = (double)a.du_m1[i];
        double u_new = u_old + du * dt + 0.5 * (du - du_m1) / dt_m1 * fabs(dt) * dt;
        if (u_new < 0.) { u_new = u_old * exp(u_new * dt / u_old); }
        a.temp[i]  = u_new / (double)a.constCv;
        a.du_m1[i] = (float)du;
    }
    if (a.cells) gridRangeAtomic(a.cells, a.grid, pc[0], pc[1], pc[2], dv[0], dv[1], dv[2], moved);
}

//! updateSmoothingLengthGpuKernel (update_h_gpu.cu:39-46)
__global__ void updateHKernel(uint32_t first, uint32_t last, uint32_t ng0, const uint32_t* nc, float* h,
                              const float* powTab)
{
    uint32_t i = first + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= last) return;
    h[i] = updateH(ng0, nc[i], h[i], powTab);
}

static inline unsigned pairGrid(const PairArgs& a) { return (a.numGroups * kWave + kBlock - 1) / kBlock; }

static void launchXmass(const PairArgs& a, hipStream_t s)
{
    if (kFastClusters && a.localLists) return cluster::xmass(a, s);
    if (a.numGroups) xmassKernel<<<pairGrid(a), kBlock, 0, s>>>(a);
}
static void launchVeDefGradh(const PairArgs& a, hipStream_t s)
{
    if (kFastClusters && a.localLists) return cluster::veDefGradh(a, s);
    if (a.numGroups) veDefGradhKernel<<<pairGrid(a), kBlock, 0, s>>>(a);
}
static void launchIad(const PairArgs& a, hipStream_t s)
{
    if (kFastClusters && a.localLists) return cluster::iadDivvCurlv(a, s);
    if (a.numGroups) iadDivvCurlvKernel<<<pairGrid(a), kBlock, 0, s>>>(a);
}
static void launchAv(const PairArgs& a, hipStream_t s)
{
    if (kFastClusters && a.localLists) return cluster::avSwitches(a, s);
    if (a.numGroups) avSwitchesKernel<<<pairGrid(a), kBlock, 0, s>>>(a);
}
static void launchMomentum(const PairArgs& a, hipStream_t s)
{
    if (kFastClusters && a.localLists) return cluster::momentumEnergy(a, s);
    if (!a.numGroups) return;
    if (a.avClean) momentumEnergyKernel<true><<<pairGrid(a), kBlock, 0, s>>>(a);
    else momentumEnergyKernel<false><<<pairGrid(a), kBlock, 0, s>>>(a);
}
static void launchEos(const EosArgs& a, hipStream_t s)
{
    uint32_t n = a.last - a.first;
    if (n) eosKernel<<<(n + 255) / 256, 256, 0, s>>>(a);
}
static void launchPositions(const PosArgs& a, hipStream_t s)
{
    uint32_t n = a.last - a.first;
    if (n) positionsKernel<<<(n + 255) / 256, 256, 0, s>>>(a);
}
static void launchUpdateH(uint32_t first, uint32_t last, uint32_t ng0, const uint32_t* nc, float* h,
                          const float* powTab, hipStream_t s)
{
    uint32_t n = last - first;
    if (n) updateHKernel<<<(n + 255) / 256, 256, 0, s>>>(first, last, ng0, nc, h, powTab);
}

static void launchXmassToRho(uint32_t first, uint32_t last, const float* m, float* rho, hipStream_t s)
{
    uint32_t n = last - first;
    if (n) xmassToRhoKernel<<<(n + 255) / 256, 256, 0, s>>>(first, last, m, rho);
}
static void launchEosStd(const EosArgs& a, hipStream_t s)
{
    uint32_t n = a.last - a.first;
    if (n) eosStdKernel<<<(n + 255) / 256, 256, 0, s>>>(a);
}
static void launchIadStd(const PairArgs& a, hipStream_t s)
{
    if (kFastClusters && a.localLists) return cluster::iadStd(a, s);
    if (a.numGroups) iadStdKernel<<<pairGrid(a), kBlock, 0, s>>>(a);
}
static void launchMarkRamp(const PairArgs& a, hipStream_t s)
{
    if (a.numGroups) markRampKernel<<<pairGrid(a), kBlock, 0, s>>>(a);
}
static void launchMomentumStd(const PairArgs& a, hipStream_t s)
{
    if (kFastClusters && a.localLists) return cluster::momentumStd(a, s);
    if (a.numGroups) momentumStdKernel<<<pairGrid(a), kBlock, 0, s>>>(a);
}

} // namespace SX_VARIANT

#define SX_CAT2(a, b) a##b
#define SX_CAT(a, b) SX_CAT2(a, b)

const HydroLaunch& SX_CAT(hydro_, SX_VARIANT)()
{
    static const HydroLaunch t{SX_VARIANT::launchXmass,     SX_VARIANT::launchVeDefGradh, SX_VARIANT::launchIad,
                               SX_VARIANT::launchAv,        SX_VARIANT::launchMomentum,   SX_VARIANT::launchEos,
                               SX_VARIANT::launchPositions, SX_VARIANT::launchUpdateH,
                               SX_VARIANT::launchXmassToRho, SX_VARIANT::launchEosStd,
                               SX_VARIANT::launchIadStd,    SX_VARIANT::launchMomentumStd,
                               SX_VARIANT::launchMarkRamp,
                               SX_VARIANT::kFastClusters};
    return t;
}

} // namespace sx
