/*! @file sx_gravity.hpp
 * @brief Self-gravity (sx_gravity.hip): arguments and launchers of the upsweep and the Barnes-Hut traversal.
 */
#pragma once

#include "sx_device.hpp"

namespace sx
{

struct GravArgs
{
    uint32_t first, last; // targets
    int      numLeaves, numNodes;
    // linked octree (OctreeData) + geometric node centers/sizes (nodeFpCenters)
    const int32_t*  childOffsets;
    const int32_t*  internalToLeaf;
    const uint32_t* layout;
    const double*   geoCenters;
    const double*   geoSizes;
    int32_t*        leafToNode; // scratch, numLeaves
    // particles
    const double *x, *y, *z;
    const float * m, *h;
    // expansion centers {x, y, z, mac^2} (numNodes x 4) and Cartesian quadrupoles (numNodes x 8, Cqi order)
    double* centers4;
    float*  multipoles;
    float   G, invTheta;
    float * ax, *ay, *az; // gravity is added
    double*   egrav;      // device accumulator (atomic), nullable
    uint32_t* err;        // bit 0: traversal stack exhausted
};

//! expansion centers, MAC radii and multipoles of every node; levelRangeHost: kMaxLevel + 2 node offsets per level
hipError_t gravityUpsweep(const GravArgs& a, const int32_t* levelRangeHost, hipStream_t s);
//! adds G * (M2P + P2P) to ax, ay, az of [first, last) and 0.5 sum G m phi to *egrav
hipError_t gravityTraverse(const GravArgs& a, hipStream_t s);

} // namespace sx
