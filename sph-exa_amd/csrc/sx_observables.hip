/*! @file sx_observables.hip
 * @brief Conserved quantities of the locally owned particles on the GPU (replaces conservedQuantitiesGpu,
 *        main/src/observables/conserved_gpu.cu:71-94, and the nc reduction of computeConservedQuantities,
 *        conserved_quantities.hpp:118-131).
 *
 * One pass over [first, last): kinetic energy sum m |v|^2 (halved at the end), internal energy sum u m (or
 * cv T m), linear momentum sum m v, angular momentum sum m (x cross v) and sum nc, all in double.  Each workgroup
 * reduces its 256 particles with wave shuffles and writes one partial per quantity; a second one-workgroup pass sums
 * the partials in a fixed order, so the result is deterministic (independent of scheduling).
 */
#include "sx_observables.hpp"

namespace sx
{

namespace
{

constexpr int kQ = 10; // eKin, eInt, linmom xyz, angmom xyz, ncsum, (spare)

template<class T>
__device__ __forceinline__ T blockSum(T v, T* s)
{
    v = waveSum(v);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
    __syncthreads();
    T r = 0;
    if (threadIdx.x == 0)
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w)
            r += s[w];
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(256) void conservedPartialKernel(ConservedArgs a, double* partial)
{
    __shared__ double s[4];
    const size_t i = a.first + blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    double q[kQ] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (i < a.last)
    {
        const double m  = a.m[i];
        const double X0 = a.x[i], X1 = a.y[i], X2 = a.z[i];
        const double V0 = a.vx[i], V1 = a.vy[i], V2 = a.vz[i];
        q[0]            = m * (V0 * V0 + V1 * V1 + V2 * V2);
        q[1]            = a.u ? a.u[i] * m : (a.temp ? a.cv * a.temp[i] * m : 0.0);
        q[2] = m * V0, q[3] = m * V1, q[4] = m * V2;
        q[5] = m * (X1 * V2 - X2 * V1);
        q[6] = m * (X2 * V0 - X0 * V2);
        q[7] = m * (X0 * V1 - X1 * V0);
        q[8] = a.nc ? (double)a.nc[i] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < kQ; ++k)
    {
        const double v = blockSum(q[k], s);
        if (threadIdx.x == 0) partial[(size_t)k * gridDim.x + blockIdx.x] = v;
    }
}

__global__ __launch_bounds__(256) void conservedFinalKernel(const double* partial, int nb, double* out)
{
    __shared__ double s[4];
    for (int k = 0; k < kQ; ++k)
    {
        double acc = 0;
        for (int b = threadIdx.x; b < nb; b += blockDim.x)
            acc += partial[(size_t)k * nb + b];
        acc = blockSum(acc, s);
        if (threadIdx.x == 0) out[k] = k == 0 ? 0.5 * acc : acc;
    }
}

} // namespace

size_t conservedScratch(size_t n) { return (size_t)kQ * std::max<size_t>(1, (n + 255) / 256); }

hipError_t conservedQuantities(const ConservedArgs& a, double* scratch, double* out, hipStream_t s)
{
    const size_t n  = a.last > a.first ? a.last - a.first : 0;
    const int    nb = (int)std::max<size_t>(1, (n + 255) / 256);
    conservedPartialKernel<<<nb, 256, 0, s>>>(a, scratch);
    conservedFinalKernel<<<1, 256, 0, s>>>(scratch, nb, out);
    return hipGetLastError();
}

} // namespace sx
