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
    float*   groupDt; // nullable, per 64-block min
    // params
    float  alphamin, alphamax, decay_constant;
    double        dt;    // AV switches time-step (d.minDt)
    const double* dtPtr; // if non-null, *dtPtr replaces dt (device-resident time-step)
    float  Atmin, Atmax, ramp, Kcour;
};

struct EosArgs
{
    uint32_t      first, last;
    float         mui;
    double        gamma;
    const double* temp;
    const float * m, *kx, *xm, *gradh;
    float *       prho, *c, *rho, *p;
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
} // namespace cluster

} // namespace sx
