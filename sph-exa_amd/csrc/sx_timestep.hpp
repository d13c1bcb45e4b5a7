/*! @file sx_timestep.hpp
 * @brief host launchers of the block time-step seam (sx_timestep.hip): group time-steps, rungs, rung-aware
 *        positions and drift.
 */
#pragma once

#include "sx_device.hpp"

namespace sx
{

//! a GroupView (traversal/groups.hpp:19-55): explicit [start[g], end[g]) or, with start == nullptr, fixed
//! 64-particle blocks of [first, last)
struct GroupArgs
{
    uint32_t        first, last, numGroups;
    const uint32_t* start;
    const uint32_t* end;
};

constexpr int kMaxNumRungs = 4; //!< sph::Timestep::maxNumRungs (timestep.h:42)

struct RungPosArgs
{
    GroupArgs      grp;
    double         dt, dtBack; // dtBack: drift only
    float          dt_m1[kMaxNumRungs];
    const uint8_t* rung; // nullable: dt_m1[0] for everyone
    DevBox         box;
    double *       x, *y, *z;
    float *        x_m1, *y_m1, *z_m1, *vx, *vy, *vz;
    const float *  ax, *ay, *az;
    double*        temp; // temp or u (the other nullptr)
    double*        u;
    const double*  du;
    float*         du_m1;
    const float*   h;
    const float*   mui;   // per-particle mean molecular weight when constCv < 0
    double         gamma, constCv;
};

hipError_t rungPositions(const RungPosArgs& a, hipStream_t s);
hipError_t driftPositions(const RungPosArgs& a, hipStream_t s);
hipError_t groupDivvTimestep(float Krho, const GroupArgs& g, const float* divv, float* groupDt, hipStream_t s);
hipError_t groupAccTimestep(float etaAcc, const GroupArgs& g, const float* ax, const float* ay, const float* az,
                            float* groupDt, hipStream_t s);
hipError_t storeRung(const GroupArgs& g, uint8_t rung, uint8_t* rungs, hipStream_t s);
//! group views of the pair kernels: active[] marks for the view's targets and [min start, max end) into mm
//! (preset {UINT32_MAX, 0}); per-group minimum of per-target values; h update over the view's targets
hipError_t viewRange(const GroupArgs& g, uint8_t* active, uint32_t* mm, hipStream_t s);
hipError_t groupMin(const GroupArgs& g, const float* v, float* groupDt, hipStream_t s);
hipError_t updateHGroups(const GroupArgs& g, uint32_t ng0, const uint32_t* nc, float* h, const float* powTab,
                         hipStream_t s);

//! rung bookkeeping (ts_rungs.hpp:67-157): sort buffers of numGroups keys / values and the radix-sort temp storage
struct RungScratch
{
    float*    keys;
    uint32_t* vals;
    void*     tmp;
    size_t    tmpBytes;
};
size_t     sortGroupDtTmpBytes(uint32_t numGroups);
//! sortGroupDt (ts_rungs.hpp:67-78) + the index sequence past numGroups (computeMinTimestep, :98)
hipError_t sortGroupDt(float* groupDt, uint32_t* groupIndices, uint32_t numGroups, uint32_t numGroupsTot,
                       RungScratch& sc, hipStream_t s);
hipError_t pickDt(const float* groupDt, uint32_t k, double* out, hipStream_t s);
hipError_t rungRanges(const float* groupDt, uint32_t numGroups, float minDt, int numRungs, uint32_t* out,
                      hipStream_t s);
hipError_t extractGroups(const GroupArgs& g, const uint32_t* indices, uint32_t first, uint32_t last,
                         uint32_t* outStart, uint32_t* outEnd, hipStream_t s);

} // namespace sx
