/*! @file sx_ewald.hip
 * @brief Ewald correction of periodic self-gravity on gfx950 (ryoanji/src/ryoanji/nbody/ewald.hpp, the GPU seam
 *        computeGravityEwaldGpu of ryoanji/interface/ewald.cu:60-95).
 *
 * The tree walk (sx_gravity.hip) evaluates the central image; this adds, per target, the real-space image sum of the
 * root's quadrupole expansion (erfc-screened, -erf inside the replica shells the walk covered) and the k-space sum,
 * with the reference's types: double coordinates and sums, float gamma coefficients and multipole (EwaldParameters<
 * double, float>).  One thread per target; the k-space table (ewaldInitParameters, built on the host in the same
 * arithmetic) is read by every thread at the same index: scalar loads.  Compiled with -ffp-contract=off so that every
 * product rounds as in the reference; the remaining difference is the device's exp/erf/erfc/sin/cos (a few ulp in
 * double, usually absorbed by the float gammas).
 */
#include <cmath>

#include "sx_device.hpp"
#include "sx_gravity.hpp"

namespace sx
{

namespace
{

constexpr int kEwaldBlock = 256;

__global__ __launch_bounds__(kEwaldBlock) void ewaldKernel(EwaldArgs a)
{
    __shared__ double s_red[kEwaldBlock / kWave];
    const uint32_t    i     = a.first + blockIdx.x * kEwaldBlock + threadIdx.x;
    const bool        valid = i < a.last && (!a.active || a.active[i]);
    double            u     = 0.0;
    if (valid)
    {
        const EwaldParams& p = a.p;
        const float*       M = p.M;
        // ewaldEvalMultipoleComplete<double, double, float> (ewald.hpp:106-131): the moments / 3 in float
        const float  qxx = (M[1] + M[7]) / 3.0f, qyy = (M[4] + M[7]) / 3.0f, qzz = (M[6] + M[7]) / 3.0f;
        const float  qxy = M[2] / 3.0f, qxz = M[3] / 3.0f, qyz = M[5] / 3.0f;
        const double Qtr = 0.5 * (double)M[7];
        const double rx = a.x[i] - p.cx, ry = a.y[i] - p.cy, rz = a.z[i] - p.cz;

        // ---- real space (computeEwaldRealSpace, ewald.hpp:224-325)
        double pot = p.k1 * (double)M[0], ax = 0, ay = 0, az = 0;
        const int nE = p.numEwaldShells, nR = p.numReplicaShells;
        for (int ix = -nE; ix <= nE; ++ix)
            for (int iy = -nE; iy <= nE; ++iy)
                for (int iz = -nE; iz <= nE; ++iz)
                {
                    const bool   pre = ix >= -nR && ix <= nR && iy >= -nR && iy <= nR && iz >= -nR && iz <= nR;
                    const double Rx = rx + ix * p.L, Ry = ry + iy * p.L, Rz = rz + iz * p.L;
                    const double R2 = Rx * Rx + (Ry * Ry + Rz * Rz); // norm2: a right fold (util/array.hpp:255)
                    if (R2 > p.lCut2 && !pre) continue;
                    float g0, g1, g2, g3;
                    if (R2 < p.smallR2 && p.ka > 0)
                    {
                        // series about the origin (ewald.hpp:270-291); gamma[4], gamma[5] unused by the quadrupole
                        double       c0   = p.ka;
                        const double R2a2 = R2 * p.alpha2;
                        g0                = (float)(c0 * (R2a2 / 3.0 - 1.0));
                        c0 *= 2 * p.alpha2;
                        g1 = (float)(c0 * (R2a2 / 5.0 - 1.0 / 3.0));
                        c0 *= 2 * p.alpha2;
                        g2 = (float)(c0 * (R2a2 / 7.0 - 1.0 / 5.0));
                        c0 *= 2 * p.alpha2;
                        g3 = (float)(c0 * (R2a2 / 9.0 - 1.0 / 7.0));
                    }
                    else
                    {
                        const double Rmag   = sqrt(R2);
                        const double invR   = 1.0 / Rmag;
                        const double invR2  = invR * invR;
                        const double ea     = exp(-R2 * p.alpha2) * p.ka * invR2;
                        double       alphan = 1.0;
                        const double fn     = pre ? -erf(p.alpha * Rmag) : erfc(p.alpha * Rmag);
                        g0                  = (float)(fn * invR);
                        g1                  = (float)((double)g0 * invR2 + ea);
                        alphan *= 2 * p.alpha2;
                        g2 = (float)((double)(3 * g1) * invR2 + alphan * ea);
                        alphan *= 2 * p.alpha2;
                        g3 = (float)((double)(5 * g2) * invR2 + alphan * ea);
                    }
                    const double Qr0 = Rx * (double)qxx + Ry * (double)qxy + Rz * (double)qxz;
                    const double Qr1 = Rx * (double)qxy + Ry * (double)qyy + Rz * (double)qyz;
                    const double Qr2 = Rx * (double)qxz + Ry * (double)qyz + Rz * (double)qzz;
                    const double rQr = 0.5 * (Rx * Qr0 + (Ry * Qr1 + Rz * Qr2));
                    pot += (double)(-g0 * M[0]) + (double)g1 * Qtr - (double)g2 * rQr;
                    const double inner = (double)(g1 * M[0]) - (double)g2 * Qtr + (double)g3 * rQr;
                    ax += (double)g2 * Qr0 - Rx * inner;
                    ay += (double)g2 * Qr1 - Ry * inner;
                    az += (double)g2 * Qr2 - Rz * inner;
                }

        // ---- k space (computeEwaldKSpace, ewald.hpp:327-351)
        double kp = 0, kx = 0, ky = 0, kz = 0;
        for (int k = 0; k < p.numH; ++k)
        {
            const double* h     = a.hsum + 5 * k; // hr_scaled x, y, z, hfac_cos, hfac_sin
            const double  hdotx = h[0] * rx + (h[1] * ry + h[2] * rz);
            const double  c = cos(hdotx), s = sin(hdotx);
            const double  csSum = h[3] * c + h[4] * s, csDiff = h[3] * s - h[4] * c;
            kp -= csSum;
            kx += csDiff * h[0];
            ky += csDiff * h[1];
            kz += csDiff * h[2];
        }
        // computeGravityEwald (ewald.hpp:396-410): potAcc = real + k
        pot += kp, ax += kx, ay += ky, az += kz;
        a.ax[i] = (float)((double)a.ax[i] + (double)a.G * ax);
        a.ay[i] = (float)((double)a.ay[i] + (double)a.G * ay);
        a.az[i] = (float)((double)a.az[i] + (double)a.G * az);
        u       = pot * (double)a.m[i];
    }
    // sum m phi: wave, then block, then one atomic per block
    for (int o = kWave / 2; o > 0; o >>= 1)
        u += __shfl_xor(u, o, kWave);
    if ((threadIdx.x & (kWave - 1)) == 0) s_red[threadIdx.x / kWave] = u;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        double t = 0;
        for (int w = 0; w < kEwaldBlock / kWave; ++w)
            t += s_red[w];
        atomicAdd(a.usum, a.uscale * t);
    }
}

//! ewaldEvalMultipoleComplete<float, double, float>(...)[0] (ewald.hpp:106-131), the k-space coefficients' form
float evalPotentialF(const double hr[3], const float g[6], const float M[8])
{
    const float r0 = (float)hr[0], r1 = (float)hr[1], r2 = (float)hr[2];
    const float qxx = (M[1] + M[7]) / 3.0f, qyy = (M[4] + M[7]) / 3.0f, qzz = (M[6] + M[7]) / 3.0f;
    const float qxy = M[2] / 3.0f, qxz = M[3] / 3.0f, qyz = M[5] / 3.0f;
    const float Q0 = r0 * qxx + r1 * qxy + r2 * qxz, Q1 = r0 * qxy + r1 * qyy + r2 * qyz,
                Q2 = r0 * qxz + r1 * qyz + r2 * qzz;
    const float rQr = (float)(0.5 * (double)(r0 * Q0 + (r1 * Q1 + r2 * Q2)));
    const float Qtr = (float)(0.5 * (double)M[7]);
    return -g[0] * M[0] + g[1] * Qtr - g[2] * rQr;
}

} // namespace

int ewaldInit(EwaldParams& p, std::vector<double>& hsum, const double center[3], const float Mroot[8], double L,
              int numReplicaShells, double lCut, double hCut, double alphaScale, double smallR)
{
    // ewaldInitParameters (ewald.hpp:149-214)
    if (lCut == 0 && hCut == 0 && alphaScale == 0) numReplicaShells = 0;
    p                  = EwaldParams{};
    p.cx = center[0], p.cy = center[1], p.cz = center[2];
    for (int k = 0; k < 8; ++k)
        p.M[k] = Mroot[k];
    p.numReplicaShells = numReplicaShells;
    p.numEwaldShells   = std::max((int)std::ceil(lCut), numReplicaShells);
    p.L                = L;
    hsum.clear();
    p.numH = 0;
    if (p.numEwaldShells == 0) return 0;
    const int    hReps = (int)std::ceil(hCut);
    if (hReps > 3) return -1; // EwaldParameters::maxCeilHcut
    const double alpha = alphaScale / L;
    const double k4    = M_PI * M_PI / (alpha * alpha * L * L);
    const double hCut2 = hCut * hCut;
    for (int hx = -hReps; hx <= hReps; hx++)
        for (int hy = -hReps; hy <= hReps; hy++)
            for (int hz = -hReps; hz <= hReps; hz++)
            {
                const double hr[3] = {(double)hx, (double)hy, (double)hz};
                const double h2    = hr[0] * hr[0] + (hr[1] * hr[1] + hr[2] * hr[2]);
                if (h2 == 0 || h2 > hCut2) continue;
                const float g0 = (float)(std::exp(-k4 * h2) / (M_PI * h2 * L));
                const float g1 = (float)(2 * M_PI / L * g0);
                const float g2 = (float)(-2 * M_PI / L * g1);
                const float g3 = (float)(2 * M_PI / L * g2);
                const float g4 = (float)(-2 * M_PI / L * g3);
                const float g5 = (float)(2 * M_PI / L * g4);
                const float gc[6] = {g0, 0.0f, g2, 0.0f, g4, 0.0f}, gs[6] = {0.0f, g1, 0.0f, g3, 0.0f, g5};
                const double s = 2 * M_PI / L;
                hsum.insert(hsum.end(), {s * hr[0], s * hr[1], s * hr[2], (double)evalPotentialF(hr, gc, Mroot),
                                         (double)evalPotentialF(hr, gs, Mroot)});
                p.numH++;
            }
    // computeEwaldRealSpace's constants (ewald.hpp:235-240), in the reference's operand order
    p.lCut2   = lCut * lCut * L * L;
    p.alpha   = alphaScale / L;
    p.alpha2  = p.alpha * p.alpha;
    p.k1      = M_PI / (p.alpha2 * L * L * L);
    p.ka      = 2.0 * p.alpha / std::sqrt(M_PI);
    p.smallR2 = smallR * L * L;
    return 0;
}

hipError_t ewaldCorrection(const EwaldArgs& a, hipStream_t s)
{
    if (a.last <= a.first || a.p.numEwaldShells == 0) return hipSuccess;
    const uint32_t n = a.last - a.first;
    ewaldKernel<<<(n + kEwaldBlock - 1) / kEwaldBlock, kEwaldBlock, 0, s>>>(a);
    return hipGetLastError();
}

} // namespace sx
