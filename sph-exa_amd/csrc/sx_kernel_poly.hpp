/*! @file sx_kernel_poly.hpp
 * @brief The SPH kernel W(v) = sinc(pi v / 2)^6 and dW/dv evaluated in registers (fast variant's LDS-staged pair
 *        kernels, sx_hydro_cluster.hip) instead of the reference's 20000-point lookup tables
 *        (sph/sph_kernel_tables.hpp:27-101, table_lookup.hpp:14-26).
 *
 * sinc(pi v / 2) and (d/dv sinc(pi v / 2)) / v are least-squares polynomials of degree 6 in t = v^2 on [0, 2]
 * (coefficients fitted in double, stored as float).  Evaluated in float with FMA, |W - sinc6| < 3.1e-7 and
 * |dW - sinc6d| < 8e-7 over [0, 2) (the float-interpolated tables: 1.1e-7 and 2.2e-7) -- a few float ulps of W(0) = 1
 * (tests/test_capi_cpu.py::test_kernel_poly_matches_sinc6_and_tables checks this against the exact function and the tables, through
 * sx_kernel_poly()).  Both are 0 for v >= 2, like lt::lookup's last interval.
 */
#pragma once

#include <hip/hip_runtime.h>

namespace sx
{

//! sinc(pi v / 2) as a polynomial in t = v^2 on [0, 2] (least squares, see the file header)
__host__ __device__ __forceinline__ float sincPoly(float t)
{
    float s = 3.08339593857454e-08f;
    s       = fmaf(s, t, -2.262898533444968e-06f);
    s       = fmaf(s, t, 0.00010206655861111358f);
    s       = fmaf(s, t, -0.0029803994111716747f);
    s       = fmaf(s, t, 0.050733841955661774f);
    s       = fmaf(s, t, -0.411233514547348f);
    return fmaf(s, t, 1.0f);
}
//! (d/dv sinc(pi v / 2)) / v as a polynomial in t = v^2
__host__ __device__ __forceinline__ float dsincPolyOverV(float t)
{
    float s = 5.004272196629245e-08f;
    s       = fmaf(s, t, -2.7139270741827204e-07f);
    s       = fmaf(s, t, -1.9479362890706398e-05f);
    s       = fmaf(s, t, 0.0008091478957794607f);
    s       = fmaf(s, t, -0.01787404529750347f);
    s       = fmaf(s, t, 0.20293137431144714f);
    return fmaf(s, t, -0.8224664926528931f);
}
//! W(v) = sinc6 (sph_kernel_tables.hpp:27-40); 0 beyond the support like lt::lookup's last interval: t = v^2 is
//! clamped to 4, where sincPoly evaluates to exactly 0.0f (with or without FMA), so no compare/select is needed
__host__ __device__ __forceinline__ float kernelW(float v)
{
    float s  = sincPoly(fminf(v * v, 4.0f));
    float s2 = s * s;
    return s2 * s2 * s2;
}
//! W as a function of t = v^2 = r^2 / h^2: the pair kernels that need no |r| skip the square root
__host__ __device__ __forceinline__ float kernelWt(float t)
{
    float s  = sincPoly(fminf(t, 4.0f));
    float s2 = s * s;
    return s2 * s2 * s2;
}
//! W and v dW/dv = 6 sinc^5 t sinc'/v as functions of t = v^2
__host__ __device__ __forceinline__ void kernelWvdWt(float t, float& w, float& vdw)
{
    t        = fminf(t, 4.0f);
    float s  = sincPoly(t);
    float s2 = s * s;
    float s4 = s2 * s2;
    w        = s4 * s2;
    vdw      = 6.0f * s4 * s * t * dsincPolyOverV(t);
}
//! W and dW/dv = 6 sinc^5 sinc' (sinc6d); both exactly 0 for v >= 2 through the same clamp (s = 0)
__host__ __device__ __forceinline__ void kernelWdW(float v, float& w, float& dw)
{
    float t  = fminf(v * v, 4.0f);
    float s  = sincPoly(t);
    float s2 = s * s;
    float s4 = s2 * s2;
    w        = s4 * s2;
    dw       = 6.0f * s4 * s * v * dsincPolyOverV(t);
}

} // namespace sx
