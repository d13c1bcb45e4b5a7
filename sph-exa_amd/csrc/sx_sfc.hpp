/*! @file sx_sfc.hpp
 * @brief Hilbert SFC keys of particle coordinates, shared by the key kernel (sx_tree.hip) and the position update
 *        (sx_hydro.hip), which writes the next step's keys while it has the new coordinates in registers.
 *        Rounding is explicit (__dmul_rn / __dsub_rn), so the keys are bit-identical under any -ffp-contract.
 */
#pragma once
#include "sx_device.hpp"

namespace sx
{

//! iHilbert<uint64_t> (sfc/hilbert.hpp:60-105), branch-free: per Morton octant one byte of a 64-bit constant holds the
//! Hilbert digit, the x/y/z reflections and the axis permutation the reference applies at that level (built from the
//! reference's expressions at compile time), and the digits go straight to their bit positions (32-bit halves).
//! Checked equal to the reference's loop on 2e7 random coordinates; keys are bit-exact in tests/test_gpu_parity.py.
__device__ __forceinline__ uint64_t iHilbert(unsigned px, unsigned py, unsigned pz)
{
    constexpr uint64_t T = [] {
        constexpr unsigned m2h[8] = {0, 1, 3, 2, 7, 6, 4, 5}; // mortonToHilbert
        uint64_t           t      = 0;
        for (unsigned o = 0; o < 8; ++o)
        {
            const unsigned xi = o >> 2, yi = (o >> 1) & 1u, zi = o & 1u;
            const unsigned fx = xi & ((!yi) | zi), fy = (xi & (yi | zi)) | (yi & (!zi)), fz = (xi & (!yi) & (!zi)) | (yi & (!zi));
            const unsigned perm = zi ? 1u : (!yi ? 2u : 0u); // 1: (x,y,z) <- (y,z,x), 2: x <-> z
            t |= (uint64_t)(m2h[o] | (fx << 3) | (fy << 4) | (fz << 5) | (perm << 6)) << (8 * o);
        }
        return t;
    }();
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int level = kMaxLevel - 1; level >= 0; --level)
    {
        const unsigned o = (((px >> level) & 1u) << 2) | (((py >> level) & 1u) << 1) | ((pz >> level) & 1u);
        const unsigned e = (unsigned)(T >> (8 * o)) & 0xffu;
        const int      s = 3 * level;
        if (s >= 32) hi |= (e & 7u) << (s - 32);
        else
        {
            lo |= (e & 7u) << s;
            if (s > 29) hi |= (e & 7u) >> (32 - s);
        }
        px ^= 0u - ((e >> 3) & 1u);
        py ^= 0u - ((e >> 4) & 1u);
        pz ^= 0u - ((e >> 5) & 1u);
        const unsigned perm = e >> 6;
        const unsigned nx = perm == 1u ? py : (perm == 2u ? pz : px);
        const unsigned ny = perm == 1u ? pz : py;
        const unsigned nz = perm == 0u ? pz : px;
        px = nx, py = ny, pz = nz;
    }
    return ((uint64_t)hi << 32) | lo;
}

//! computeSfcKeys / sfc3D<HilbertKey<uint64_t>> (sfc/sfc.hpp:157-194, 284-291): box-normalised integer coordinates,
//! clamped to the last cell, then iHilbert
__device__ __forceinline__ uint64_t sfcKey(double x, double y, double z, const DevBox& b)
{
    constexpr unsigned cubeLength = 1u << kMaxLevel;
    constexpr int      mcoord     = (1 << kMaxLevel) - 1;
    const double       mx = __dmul_rn((double)cubeLength, b.il[0]), my = __dmul_rn((double)cubeLength, b.il[1]),
                 mz = __dmul_rn((double)cubeLength, b.il[2]);
    int ix = (int)__dsub_rn(floor(__dmul_rn(x, mx)), __dmul_rn(b.lim[0], mx));
    int iy = (int)__dsub_rn(floor(__dmul_rn(y, my)), __dmul_rn(b.lim[2], my));
    int iz = (int)__dsub_rn(floor(__dmul_rn(z, mz)), __dmul_rn(b.lim[4], mz));
    ix     = ix < mcoord ? ix : mcoord;
    iy     = iy < mcoord ? iy : mcoord;
    iz     = iz < mcoord ? iz : mcoord;
    return iHilbert((unsigned)ix, (unsigned)iy, (unsigned)iz);
}

} // namespace sx
