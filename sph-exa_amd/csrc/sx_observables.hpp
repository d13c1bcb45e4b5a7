/*! @file sx_observables.hpp
 * @brief Conserved-quantity reduction (sx_observables.hip).
 */
#pragma once

#include "sx_device.hpp"

#include <algorithm>

namespace sx
{

struct ConservedArgs
{
    size_t          first, last;
    const double *  x, *y, *z;
    const float *   vx, *vy, *vz, *m;
    const double*   temp; // used with cv when u is null
    const double*   u;    // nullable
    const uint32_t* nc;   // nullable
    double          cv;
};

//! doubles of scratch for n particles
size_t conservedScratch(size_t n);
//! out[0..8]: 0.5 sum m v^2, sum u m (or cv T m), linear momentum (3), angular momentum (3), sum nc
hipError_t conservedQuantities(const ConservedArgs& a, double* scratch, double* out, hipStream_t s);

} // namespace sx
