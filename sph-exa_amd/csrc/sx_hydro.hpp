/*! @file sx_hydro.hpp
 * @brief Argument blocks and launch table of the VE pair kernels (sx_hydro.hip).
 *
 * sx_hydro.hip is compiled twice: SX_VARIANT=exact with -ffp-contract=off (bit-reproducible against the CPU
 * reference for an identical neighbor order) and SX_VARIANT=fast with FMA contraction (production).
 */
#pragma once

#include "sx_device.hpp"

namespace sx
{

//! arguments shared by the neighbor-list pair kernels (one wavefront per 64-particle block of [first,last))
//! computeEOS_Impl (hydro_ve/eos.hpp:52-77) fused into the producer of kx and gradh (cluster VeDefGradh): the same
//! arithmetic as eosKernel per computed target, its records included; temp == nullptr: not fused
struct EosFuse
{
    const double* temp;
    double        cv;    // (double)idealGasCv(mui, gamma)
    double        gamma;
    float *       prho, *c;
    const float * vx, *vy, *vz, *alpha;
    RecV*         rvOut;
    RecT*         rtOut;
};

struct PairArgs
{
    uint32_t first, last, numGroups, ngmax;
    // neighbor lists (NbLists, sx_tree.hpp): global nidx[group][k][lane], or, with localLists, the cluster unions
    // uni[cluster*ucap + u] (ucount[cluster] entries) and u16 positions nloc[group][k/2][lane]
    int             localLists;
    const uint32_t* nidx;
    const uint32_t* nloc;
    const uint32_t* uni;
    const uint32_t* ucount;
    uint32_t        ucap;
    ListsB          lb;   // the second set of cluster lists (sx_device.hpp); lb.sel == nullptr: none
    const uint32_t* nc;   // includes self
    const RecX*     rx;
    const RecV*     rv;
    const RecT*     rt;
    const RecC*     rc;
    const float2*   wh;
    const float2*   whd;
    DevBox          box;
    double          K;
    // outputs
    float *  xm, *kx, *gradh;
    float *  c11, *c12, *c13, *c22, *c23, *c33, *divv, *curlv;
    float*   alpha;
    float *  ax, *ay, *az;
    double*  du;
    float*   minDt;   // device scalar, atomic min (Courant)
    float*   blockDt; // cluster kernels, nullable: per-workgroup Courant minima (one per launched workgroup),
                      // reduced into *minDt by one small kernel after the launch instead of one atomic per workgroup
    float*   groupDt; // nullable, per 64-block min
    // params
    float  alphamin, alphamax, decay_constant;
    double        dt;    // AV switches time-step (d.minDt)
    const double* dtPtr; // if non-null, *dtPtr replaces dt (device-resident time-step)
    float  Atmin, Atmax, ramp, Kcour;
    // avClean (HydroVeProp<true>, ve_hydro.hpp:50-85): the IAD kernel writes the velocity gradient (GradVFields)
    // when dV11 != nullptr (doGradV, iad_divv_curlv_gpu.cu:96-97); momentum reads it when avClean != 0
    float *dV11, *dV12, *dV13, *dV22, *dV23, *dV33;
    int    avClean;
    // std propagator (HydroProp, std_hydro.hpp:124-184): rho and p of every particle (IAD, momentumEnergySTD)
    const RecS* rs;
    // markRampJLoop (hydro_ve/additional_fields_kern.hpp:38-58): fraction of the Atwood ramp over the neighbors
    float* markRamp;
    // cluster kernels only: process the listCount clusters clusterList[0..listCount) instead of all of them (the
    // interior / boundary split that overlaps a halo exchange with the interior clusters, sx_sim.cpp)
    const uint32_t* clusterList;
    uint32_t        listCount;
    // group views (ve-bdt active rungs): targets with active[i] == 0 are skipped -- not computed, not written, as the
    // reference's kernels visit only the view's groups; nullable = every target of [first, last)
    const uint8_t* active;
    // nullable: each computed target's Courant time-step (momentum kernels), for the per-view-group minimum
    float* dtOut;
    // nullable (cluster kernels, full views): the producing kernel also writes the targets' records for the next
    // kernels, so only the halos need a packing pass: XMass rtOut = {xm, 0, 0, 0}, IAD rcOut = {c_ij, divv},
    // AV switches rtOut = the target's record with the new alpha
    RecT* rtOut;
    RecC* rcOut;
    // cluster kernels, 0 = unknown: an upper bound of every cluster's union size (the search's statistics, read by
    // the host once the search has finished); AV switches skips its large-union launch when no union needs it
    uint32_t unionMax;
    // cluster VeDefGradh only (full views): EOS of every computed target in its epilogue
    EosFuse eos;
};

//! IAD tail shared by the VE and std IAD kernels (iad_kern.hpp:84-108, hydro_std/iad_kern.hpp:54-76): exponent
//! normalisation of tau, then the cofactor inverse scaled by h^3 / K
__device__ __forceinline__ void iadInvert(float t11, float t12, float t13, float t22, float t23, float t33, float hi,
                                          double K, float (&c)[6])
{
    auto getExp    = [](float v) { return v == 0.0f ? 0 : ilogbf(v); };
    int  tauExpSum = getExp(t11) + getExp(t12) + getExp(t13) + getExp(t22) + getExp(t23) + getExp(t33);
    const float nrm = ldexpf(1.0f, -tauExpSum / 6);
    t11 *= nrm, t12 *= nrm, t13 *= nrm, t22 *= nrm, t23 *= nrm, t33 *= nrm;
    const float det    = t11 * t22 * t33 + 2.0f * t12 * t23 * t13 - t11 * t23 * t23 - t22 * t13 * t13 - t33 * t12 * t12;
    const float factor = (float)((double)(nrm * (hi * hi * hi)) / ((double)det * K));
    c[0]               = (t22 * t33 - t23 * t23) * factor;
    c[1]               = (t13 * t23 - t33 * t12) * factor;
    c[2]               = (t12 * t23 - t22 * t13) * factor;
    c[3]               = (t11 * t33 - t13 * t13) * factor;
    c[4]               = (t13 * t12 - t11 * t23) * factor;
    c[5]               = (t11 * t22 - t12 * t12) * factor;
}

//! eta_crit of momentumAndEnergyJLoop<avClean> (momentum_energy_kern.hpp:112): formed in double, stored as float
__device__ __forceinline__ float avEtaCrit(unsigned cnt)
{
    return (float)cbrt((double)32.0f * 3.14159265358979323846 / 3.0 / (double)(float)(cnt + 1));
}

/*! avRvCorrection<float, float> (momentum_energy_kern.hpp:43-63): symv is the upper-triangle product
 *  (kernels.hpp:88-95), dot the right fold a0*b0 + (a1*b1 + a2*b2) (util/array.hpp:253-256), stl::min/max
 *  (primitives/stl.hpp:53-65).  EXACT evaluates exp in double and rounds once (glibc's expf wherever that is
 *  correctly rounded); the fast variant uses expf. */
template<bool EXACT>
__device__ __forceinline__ float avRvCorrection(float rx, float ry, float rz, float eta_ab, float eta_crit,
                                                const float (&gi)[6], const float (&gj)[6])
{
    const float dmy1 = rx * (gi[0] * rx + gi[1] * ry + gi[2] * rz) + (ry * (gi[3] * ry + gi[4] * rz) + rz * (gi[5] * rz));
    const float dmy2 = rx * (gj[0] * rx + gj[1] * ry + gj[2] * rz) + (ry * (gj[3] * ry + gj[4] * rz) + rz * (gj[5] * rz));
    float       dmy3 = 1.0f;
    if (eta_ab < eta_crit)
    {
        const float etaDiff = 5.0f * (eta_ab - eta_crit);
        const float arg     = -etaDiff * etaDiff;
        dmy3                = EXACT ? (float)exp((double)arg) : expf(arg);
    }
    const float A_ab   = (dmy2 != 0.0f) ? dmy1 / dmy2 : 0.0f;
    const float A_abp1 = 1.0f + A_ab;
    float       q      = 4.0f * A_ab / (A_abp1 * A_abp1);
    q                  = q < 1.0f ? q : 1.0f;
    q                  = 0.0f < q ? q : 0.0f;
    const float phi_ab = 0.5f * dmy3 * q;
    return -phi_ab * (dmy1 + dmy2);
}

struct EosArgs
{
    uint32_t      first, last;
    float         mui;
    double        gamma;
    const double* temp;
    const float * m, *kx, *xm, *gradh;
    float *       prho, *c, *rho, *p;
    // nullable: also write the records {vx, vy, vz, c} and {xm, kx, prho, alpha} of [first, last)
    const float * vx, *vy, *vz, *alpha;
    RecV*         rvOut;
    RecT*         rtOut;
};

struct PosArgs
{
    uint32_t first, last;
    double        dt, dt_m1;
    const double* dtPtr; // if non-null: dt = dtPtr[0], dt_m1 = dtPtr[1]
    DevBox        box;
    double*  x, *y, *z;
    float *  x_m1, *y_m1, *z_m1, *vx, *vy, *vz;
    const float *ax, *ay, *az;
    double*      temp;
    const double* du;
    float*        du_m1;
    const float*  h;
    float         constCv;
    // nullable: the next sync's SFC keys of the updated coordinates (sfcKey, box `box`), written in the same pass
    uint64_t*     keys;
    // nullable (skin lists, sx_skin.hpp): this step's displacement vector (unwrapped), per particle, and its
    // component ranges by cell of the updated position (gridRangeAtomic; initialised by the caller), so the next
    // step's filter needs no pass over the particles
    float *       dispX, *dispY, *dispZ;
    uint32_t*     cells;
    DispGrid      grid;
};

struct HydroLaunch
{
    void (*xmass)(const PairArgs&, hipStream_t);
    void (*veDefGradh)(const PairArgs&, hipStream_t);
    void (*iadDivvCurlv)(const PairArgs&, hipStream_t);
    void (*avSwitches)(const PairArgs&, hipStream_t);
    void (*momentumEnergy)(const PairArgs&, hipStream_t);
    void (*eos)(const EosArgs&, hipStream_t);
    void (*positions)(const PosArgs&, hipStream_t);
    void (*updateH)(uint32_t first, uint32_t last, uint32_t ng0, const uint32_t* nc, float* h, const float* powTab,
                    hipStream_t);
    // std propagator (HydroProp): density = xmass written to rho then rho = m / rho (xmass_gpu.cu:134-164),
    // EOS_HydroStd, IAD with m/rho volumes, momentumEnergySTD
    void (*xmassToRho)(uint32_t first, uint32_t last, const float* m, float* rho, hipStream_t);
    void (*eosStd)(const EosArgs&, hipStream_t);
    void (*iadStd)(const PairArgs&, hipStream_t);
    void (*momentumStd)(const PairArgs&, hipStream_t);
    // diagnostic field of the KH ramp (hydro_ve/additional_fields.cu:47-98): a.markRamp from xm, kx and m
    void (*markRamp)(const PairArgs&, hipStream_t);
    // the pair launchers honour PairArgs::clusterList (cluster kernels on local lists); false for the exact variant
    bool clusterLists;
};

const HydroLaunch& hydro_exact();
const HydroLaunch& hydro_fast();

//! fast-variant pair kernels on cluster lists (sx_hydro_cluster.hip): one workgroup per 256-particle cluster, the
//! cluster's neighbor union staged in LDS, the kernel W evaluated in registers
namespace cluster
{
void xmass(const PairArgs&, hipStream_t);
void veDefGradh(const PairArgs&, hipStream_t);
void iadDivvCurlv(const PairArgs&, hipStream_t);
void avSwitches(const PairArgs&, hipStream_t);
void momentumEnergy(const PairArgs&, hipStream_t);
void iadStd(const PairArgs&, hipStream_t);
void momentumStd(const PairArgs&, hipStream_t);
} // namespace cluster

} // namespace sx
