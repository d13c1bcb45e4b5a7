/*! @file sx_timestep.hip
 * @brief Block time-step (ve-bdt) seam on gfx950: group time-steps, rung bookkeeping, the rung-aware position
 *        update and the drift of inactive rungs.  Compiled -ffp-contract=off: the formulas round exactly like the
 *        reference's (positions.hpp:54-88 energyUpdate / positionUpdate, eos.hpp:13-18 idealGasCv).
 *
 * Replaces sph/include/sph/ts_groups.cu:17-108 (groupDivvTimestepGpu, groupAccTimestepGpu, storeRungGpu),
 * sph/include/sph/positions_gpu.cu:45-179 (driftPositionsGpu, computePositionsGpu with dt_m1 per rung) and the device
 * work of the rung bookkeeping in sph/include/sph/ts_rungs.hpp:67-157 (sortGroupDt, the fast-fraction pick,
 * findRungRanges' lower bounds) and sph/include/sph/groups.hpp:31-48 (extractGroupGpu).
 *
 * Target groups: one wavefront per group (the reference's warp on AMD, 64 lanes), groups given as
 * [groupStart[g], groupEnd[g]) (computeSpatialGroups / sliced rung views) or, with groupStart == nullptr, the
 * fixed 64-particle blocks of [first, last).
 */
#include <hipcub/hipcub.hpp>

#include "sx_timestep.hpp"

namespace sx
{

__device__ __forceinline__ bool groupBounds(const GroupArgs& g, uint32_t w, uint32_t& s, uint32_t& e)
{
    if (w >= g.numGroups) return false;
    if (g.start)
    {
        s = g.start[w];
        e = g.end[w];
    }
    else
    {
        s = g.first + w * 64u;
        e = min(s + 64u, g.last);
    }
    return true;
}

//! idealGasCv<float, double> (eos.hpp:13-18): R / mui in float, divided by (gamma - 1) in double, stored as float
__device__ __forceinline__ float idealGasCvF(float mui, double gamma)
{
    const float R = 8.317e7f;
    return (float)((double)(R / mui) / (gamma - 1.0f));
}

//! energyUpdate<double, double> (positions.hpp:54-61)
__device__ __forceinline__ double energyUpdate(double u_old, double dt, double dt_m1, double du, double du_m1)
{
    double u_new = u_old + du * dt + 0.5 * (du - du_m1) / dt_m1 * fabs(dt) * dt;
    if (u_new < 0.) { u_new = u_old * exp(u_new * dt / u_old); }
    return u_new;
}

//! positionUpdate<double> (positions.hpp:77-88); pbc: putInBox on the periodic axes (box.hpp:209-230)
__device__ __forceinline__ void positionUpdate(double dt, double dt_m1, const double X[3], const double A[3],
                                               const double dX[3], const DevBox* pbc, double Xn[3], double Vn1[3],
                                               double dXn1[3])
{
    const double inv = 1.0 / dt_m1, hdm1 = 0.5 * dt_m1, adt = fabs(dt);
#pragma unroll
    for (int k = 0; k < 3; ++k)
    {
        const double Vnmhalf = dX[k] * inv;
        const double Vn      = Vnmhalf + A[k] * hdm1;
        Vn1[k]               = Vn + A[k] * dt;
        dXn1[k]              = (Vn + (A[k] * 0.5) * adt) * dt;
        Xn[k]                = X[k] + dXn1[k];
    }
    if (pbc)
#pragma unroll
        for (int d = 0; d < 3; ++d)
        {
            if (pbc->pbc[d] && Xn[d] > pbc->lim[2 * d + 1]) Xn[d] -= pbc->l[d];
            else if (pbc->pbc[d] && Xn[d] < pbc->lim[2 * d]) Xn[d] += pbc->l[d];
        }
}

__device__ __forceinline__ float rungDtM1(const RungPosArgs& a, uint32_t i)
{
    return a.rung ? a.dt_m1[a.rung[i]] : a.dt_m1[0];
}

//! computePositionsKernel (positions_gpu.cu:110-160)
__global__ void rungPositionsKernel(RungPosArgs a)
{
    const uint32_t w    = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t       s, e;
    if (!groupBounds(a.grp, w, s, e)) return;
    const uint32_t i = s + lane;
    if (i >= e) return;
    const DevBox& b = a.box;
    if ((b.fbc[0] || b.fbc[1] || b.fbc[2]) && a.vx[i] == 0.0f && a.vy[i] == 0.0f && a.vz[i] == 0.0f)
    {
        const double X[3] = {a.x[i], a.y[i], a.z[i]};
        for (int d = 0; d < 3; ++d)
        {
            const double top = b.lim[2 * d + 1], bot = b.lim[2 * d];
            if (b.fbc[d] && (fabs(top - X[d]) < 2.0f * a.h[i] || fabs(bot - X[d]) < 2.0f * a.h[i])) return;
        }
    }
    const double dt_m1 = rungDtM1(a, i);
    const double A[3] = {a.ax[i], a.ay[i], a.az[i]}, X[3] = {a.x[i], a.y[i], a.z[i]},
                 dX[3] = {a.x_m1[i], a.y_m1[i], a.z_m1[i]};
    double Xn[3], V[3], dXn[3];
    positionUpdate(a.dt, dt_m1, X, A, dX, &b, Xn, V, dXn);
    a.x[i] = Xn[0], a.y[i] = Xn[1], a.z[i] = Xn[2];
    a.x_m1[i] = (float)dXn[0], a.y_m1[i] = (float)dXn[1], a.z_m1[i] = (float)dXn[2];
    a.vx[i] = (float)V[0], a.vy[i] = (float)V[1], a.vz[i] = (float)V[2];
    if (a.temp)
    {
        const float cv = a.constCv < 0 ? idealGasCvF(a.mui[i], a.gamma) : (float)a.constCv;
        a.temp[i]      = energyUpdate(a.temp[i] * cv, a.dt, dt_m1, a.du[i], (double)a.du_m1[i]) / cv;
    }
    else if (a.u) { a.u[i] = energyUpdate(a.u[i], a.dt, dt_m1, a.du[i], (double)a.du_m1[i]); }
    a.du_m1[i] = (float)a.du[i];
}

//! driftKernel (positions_gpu.cu:45-86): back to the start of the hierarchy by dt_back, then forward by dt, on an
//! open box (no PBC: drifting must not invalidate the octree); x_m1 and du_m1 are kept
__global__ void driftKernel(RungPosArgs a)
{
    const uint32_t w    = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t       s, e;
    if (!groupBounds(a.grp, w, s, e)) return;
    const uint32_t i = s + lane;
    if (i >= e) return;
    const double dt_m1 = rungDtM1(a, i);
    const double A[3] = {a.ax[i], a.ay[i], a.az[i]}, Xb[3] = {a.x[i], a.y[i], a.z[i]},
                 dX[3] = {a.x_m1[i], a.y_m1[i], a.z_m1[i]};
    double X0[3], V[3], dXn[3], X1[3];
    positionUpdate(-a.dtBack, dt_m1, Xb, A, dX, nullptr, X0, V, dXn);
    positionUpdate(a.dt, dt_m1, X0, A, dX, nullptr, X1, V, dXn);
    a.x[i] = X1[0], a.y[i] = X1[1], a.z[i] = X1[2];
    a.vx[i] = (float)V[0], a.vy[i] = (float)V[1], a.vz[i] = (float)V[2];
    if (a.temp)
    {
        const float  cv      = a.constCv < 0 ? idealGasCvF(a.mui[i], a.gamma) : (float)a.constCv;
        const double u_recov = energyUpdate(a.temp[i] * cv, -a.dtBack, dt_m1, a.du[i], (double)a.du_m1[i]);
        a.temp[i]            = energyUpdate(u_recov, a.dt, dt_m1, a.du[i], (double)a.du_m1[i]) / cv;
    }
    else if (a.u)
    {
        const double u_recov = energyUpdate(a.u[i], -a.dtBack, dt_m1, a.du[i], (double)a.du_m1[i]);
        a.u[i]               = energyUpdate(u_recov, a.dt, dt_m1, a.du[i], (double)a.du_m1[i]);
    }
}

//! groupDivvKernel (ts_groups.cu:17-36): groupDt = min(groupDt, Krho / |max divv|), one thread per group
__global__ void groupDivvKernel(float Krho, GroupArgs g, const float* divv, float* groupDt)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t       s, e;
    if (!groupBounds(g, t, s, e)) return;
    float localMax = -INFINITY;
    for (uint32_t i = s; i < e; ++i)
        localMax = fmaxf(localMax, divv[i]);
    groupDt[t] = fminf(groupDt[t], Krho / fabsf(localMax));
}

//! groupAccKernel (ts_groups.cu:49-68): groupDt = min(groupDt, etaAcc / |a|max^(1/2)^(1/2))
__global__ void groupAccKernel(float etaAcc, GroupArgs g, const float* ax, const float* ay, const float* az,
                               float* groupDt)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t       s, e;
    if (!groupBounds(g, t, s, e)) return;
    float maxAcc = 0;
    for (uint32_t i = s; i < e; ++i)
        maxAcc = fmaxf(maxAcc, ax[i] * ax[i] + (ay[i] * ay[i] + az[i] * az[i])); // norm2, right-fold dot
    groupDt[t] = fminf(groupDt[t], etaAcc / sqrtf(sqrtf(maxAcc)));
}

//! storeRungKernel (ts_groups.cu:84-96)
__global__ void storeRungKernel(GroupArgs g, uint8_t rung, uint8_t* rungs)
{
    const uint32_t w    = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t       s, e;
    if (!groupBounds(g, w, s, e)) return;
    if (s + lane < e) rungs[s + lane] = rung;
}

// ---- group views of the pair kernels (ve-bdt active rungs: a slice of the rung-sorted groups) ---------------------

//! marks the targets of the view's groups in active[] and reduces [min start, max end) into mm[0], mm[1]
//! (mm preset to {UINT32_MAX, 0}); one atomic pair per workgroup
__global__ void viewRangeKernel(GroupArgs g, uint8_t* active, uint32_t* mm)
{
    uint32_t lo = 0xffffffffu, hi = 0;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < g.numGroups; t += gridDim.x * blockDim.x)
    {
        uint32_t s, e;
        groupBounds(g, t, s, e);
        for (uint32_t i = s; i < e; ++i)
            active[i] = 1;
        if (s < e) lo = min(lo, s), hi = max(hi, e);
    }
    lo = waveMin(lo), hi = waveMax(hi);
    __shared__ uint32_t s_lo[4], s_hi[4];
    if ((threadIdx.x & 63) == 0) s_lo[threadIdx.x >> 6] = lo, s_hi[threadIdx.x >> 6] = hi;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        for (int w = 1; w < 4; ++w)
            lo = min(lo, s_lo[w]), hi = max(hi, s_hi[w]);
        atomicMin(mm, lo);
        atomicMax(mm + 1, hi);
    }
}

//! groupDt[t] = min(groupDt[t], min over group t of v) -- the per-group Courant minimum of momentumEnergyGpu
//! (momentum_energy_gpu.cu:98-104: warpMin of the group's targets into groupDt[targetIdx])
__global__ void groupMinKernel(GroupArgs g, const float* v, float* groupDt)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t       s, e;
    if (!groupBounds(g, t, s, e)) return;
    float m = INFINITY;
    for (uint32_t i = s; i < e; ++i)
        m = fminf(m, v[i]);
    groupDt[t] = fminf(groupDt[t], m);
}

//! updateSmoothingLengthGpu over the targets of a group view (update_h_gpu.cu:49-60)
__global__ void updateHGroupsKernel(GroupArgs g, uint32_t ng0, const uint32_t* nc, float* h, const float* powTab)
{
    const uint32_t w    = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t       s, e;
    if (!groupBounds(g, w, s, e)) return;
    for (uint32_t i = s + lane; i < e; i += 64)
        h[i] = updateH(ng0, nc[i], h[i], powTab);
}

static unsigned waveGrid(uint32_t numGroups) { return (numGroups + 3) / 4; }

hipError_t viewRange(const GroupArgs& g, uint8_t* active, uint32_t* mm, hipStream_t s)
{
    if (g.numGroups)
        viewRangeKernel<<<(g.numGroups + 255) / 256 < 1024u ? (g.numGroups + 255) / 256 : 1024u, 256, 0, s>>>(g, active, mm);
    return hipGetLastError();
}

hipError_t groupMin(const GroupArgs& g, const float* v, float* groupDt, hipStream_t s)
{
    if (g.numGroups) groupMinKernel<<<(g.numGroups + 255) / 256, 256, 0, s>>>(g, v, groupDt);
    return hipGetLastError();
}

hipError_t updateHGroups(const GroupArgs& g, uint32_t ng0, const uint32_t* nc, float* h, const float* powTab,
                         hipStream_t s)
{
    if (g.numGroups) updateHGroupsKernel<<<waveGrid(g.numGroups), 256, 0, s>>>(g, ng0, nc, h, powTab);
    return hipGetLastError();
}

hipError_t rungPositions(const RungPosArgs& a, hipStream_t s)
{
    if (a.grp.numGroups) rungPositionsKernel<<<waveGrid(a.grp.numGroups), 256, 0, s>>>(a);
    return hipGetLastError();
}

hipError_t driftPositions(const RungPosArgs& a, hipStream_t s)
{
    if (a.grp.numGroups) driftKernel<<<waveGrid(a.grp.numGroups), 256, 0, s>>>(a);
    return hipGetLastError();
}

hipError_t groupDivvTimestep(float Krho, const GroupArgs& g, const float* divv, float* groupDt, hipStream_t s)
{
    if (g.numGroups) groupDivvKernel<<<(g.numGroups + 255) / 256, 256, 0, s>>>(Krho, g, divv, groupDt);
    return hipGetLastError();
}

hipError_t groupAccTimestep(float etaAcc, const GroupArgs& g, const float* ax, const float* ay, const float* az,
                            float* groupDt, hipStream_t s)
{
    if (g.numGroups) groupAccKernel<<<(g.numGroups + 255) / 256, 256, 0, s>>>(etaAcc, g, ax, ay, az, groupDt);
    return hipGetLastError();
}

hipError_t storeRung(const GroupArgs& g, uint8_t rung, uint8_t* rungs, hipStream_t s)
{
    if (g.numGroups) storeRungKernel<<<waveGrid(g.numGroups), 256, 0, s>>>(g, rung, rungs);
    return hipGetLastError();
}

// ---- rung bookkeeping (ts_rungs.hpp:67-157, groups.hpp:31-48) ----------------------------------------------------

__global__ void sequenceKernel(uint32_t* v, uint32_t n, uint32_t start)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = start + i;
}

hipError_t sortGroupDt(float* groupDt, uint32_t* groupIndices, uint32_t numGroups, uint32_t numGroupsTot,
                       RungScratch& sc, hipStream_t s)
{
    if (numGroups)
    {
        sequenceKernel<<<(numGroups + 255) / 256, 256, 0, s>>>(groupIndices, numGroups, 0u);
        size_t bytes = 0;
        hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, groupDt, sc.keys, groupIndices, sc.vals, (int)numGroups, 0,
                                           32, s);
        if (bytes > sc.tmpBytes) return hipErrorOutOfMemory;
        if (hipError_t e = hipcub::DeviceRadixSort::SortPairs(sc.tmp, bytes, groupDt, sc.keys, groupIndices, sc.vals,
                                                              (int)numGroups, 0, 32, s))
            return e;
        if (hipError_t e = hipMemcpyAsync(groupDt, sc.keys, 4ull * numGroups, hipMemcpyDeviceToDevice, s)) return e;
        if (hipError_t e = hipMemcpyAsync(groupIndices, sc.vals, 4ull * numGroups, hipMemcpyDeviceToDevice, s))
            return e;
    }
    if (numGroupsTot > numGroups)
        sequenceKernel<<<(numGroupsTot - numGroups + 255) / 256, 256, 0, s>>>(groupIndices + numGroups,
                                                                            numGroupsTot - numGroups, numGroups);
    return hipGetLastError();
}

size_t sortGroupDtTmpBytes(uint32_t numGroups)
{
    size_t bytes = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (float*)nullptr, (float*)nullptr, (uint32_t*)nullptr,
                                       (uint32_t*)nullptr, (int)numGroups, 0, 32);
    return bytes;
}

//! {groupDt[0], groupDt[k]} as doubles (the values the reference copies to the host, then min-reduces over ranks)
__global__ void pickDtKernel(const float* groupDt, uint32_t k, double* out)
{
    if (threadIdx.x == 0) out[0] = groupDt[0], out[1] = groupDt[k];
}

hipError_t pickDt(const float* groupDt, uint32_t k, double* out, hipStream_t s)
{
    pickDtKernel<<<1, 64, 0, s>>>(groupDt, k, out);
    return hipGetLastError();
}

//! findRungRanges (ts_rungs.hpp:116-130): out[0] = 0, out[r] = lower_bound((1 << r) * minDt) for 0 < r < numRungs,
//! numGroups for the others
__global__ void rungRangesKernel(const float* groupDt, uint32_t numGroups, float minDt, int numRungs, uint32_t* out)
{
    const int r = threadIdx.x;
    if (r > kMaxNumRungs) return;
    uint32_t v = r == 0 ? 0u : numGroups;
    if (r >= 1 && r < numRungs)
    {
        const float maxDtRung = (float)(1 << r) * minDt;
        uint32_t    lo = 0, hi = numGroups;
        while (lo < hi)
        {
            const uint32_t mid = (lo + hi) >> 1;
            if (groupDt[mid] < maxDtRung) lo = mid + 1;
            else hi = mid;
        }
        v = lo;
    }
    out[r] = v;
}

hipError_t rungRanges(const float* groupDt, uint32_t numGroups, float minDt, int numRungs, uint32_t* out,
                      hipStream_t s)
{
    rungRangesKernel<<<1, 64, 0, s>>>(groupDt, numGroups, minDt, numRungs, out);
    return hipGetLastError();
}

//! extractGroupGpu (groups.hpp:31-48): out group k = group indices[first + k] of grp
__global__ void extractGroupsKernel(GroupArgs g, const uint32_t* indices, uint32_t first, uint32_t n, uint32_t* outStart,
                                    uint32_t* outEnd)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t j = indices[first + k];
    uint32_t       s = 0, e = 0;
    groupBounds(g, j, s, e);
    outStart[k] = s;
    outEnd[k]   = e;
}

hipError_t extractGroups(const GroupArgs& g, const uint32_t* indices, uint32_t first, uint32_t last,
                         uint32_t* outStart, uint32_t* outEnd, hipStream_t s)
{
    if (last > first)
        extractGroupsKernel<<<(last - first + 255) / 256, 256, 0, s>>>(g, indices, first, last - first, outStart,
                                                                       outEnd);
    return hipGetLastError();
}

} // namespace sx
