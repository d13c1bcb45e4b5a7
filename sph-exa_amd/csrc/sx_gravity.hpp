/*! @file sx_gravity.hpp
 * @brief Self-gravity (sx_gravity.hip): arguments and launchers of the upsweep and the Barnes-Hut traversal.
 */
#pragma once

#include <vector>

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
    double*   waveE;      // nullable: per-wavefront potential-energy sums of the traversal ((last-first+63)/64), reduced
                          // into *egrav by one small kernel (one atomic per launch instead of one per wave)
    uint32_t* err;        // bit 0: traversal stack exhausted
    int       fast;       // 1: M2P/P2P in float with rsqrt (displacements formed in double, sums in double)
    const uint8_t* active; // nullable: targets with active[i] == 0 (outside the group view) get no gravity
    unsigned long long* interactions; // nullable: [0] += P2P, [1] += M2P interactions summed over the targets (the
                                      // reference's BhStats sumP2P / sumM2P, nbody/traversal.cuh:346-357, 614-620)
    int    numShells;  // periodic images walked per axis on each side (traversal_cpu.hpp:200-216); 0: the box itself
    double boxL[3];    // box lengths (the image shifts)
};

//! a level-6 SFC cell of one rank's particles (multi-rank gravity): mass center, MAC radius^2, quadrupole (Cqi
//! order, q[0] = mass), cell index (key >> 45) and particle count; box: the MAC geometry relative to the cell's
//! geometric center (center offset, half sizes) -- the cell itself, or, between syncs (particles drifted out of their
//! cells), the box holding the cell and its particles
struct __attribute__((aligned(16))) GCell
{
    double   com[3];
    double   mac2;
    float    q[8];
    uint32_t cell, count;
    float    box[6];
};
static_assert(sizeof(GCell) == 96, "GCell layout");

//! cells [cellBeg[k], cellBeg[k+1]) of key-sorted particles; geometry from the far tree's leaf nodes.  drift: the
//! particles may have left their cells since the sync that formed the cells (skin-list reuse steps): the MAC box
//! holds the cell and its particles (sx_skin.hpp skinRefreshBoxes(withCells) for one rank's tree)
hipError_t cellMoments(const double* x, const double* y, const double* z, const float* m, const uint32_t* cellBeg,
                       const uint32_t* cellIds, int nCells, const int32_t* farLeafToNode, const double* geoC,
                       const double* geoS, float invTheta, GCell* out, hipStream_t s, bool drift = false);
//! near[k] = 1 if cell k violates the vector MAC for any of the target boxes (center[3], half-size[3], stride 8).
//! boxL (nullable): a periodic box's lengths -- the test covers the cell's images shifted by -1, 0, +1 box lengths
//! per axis (the image walk's numShells = 1), with a relative margin on the near side
hipError_t cellNearFlags(const GCell* cells, int nCells, const double* boxes, int nBoxes, uint32_t* near,
                         hipStream_t s, const double* boxL = nullptr);
//! the global root expansion of the two source trees of a rank (near: locals + gravity halos, far: far cells), each
//! source counted once: mass center and M2M of the two roots as upsweepMultipoles combines children, on the host
void combineRoots(const double cN[4], const float mN[8], const double cF[4], const float mF[8], double c[4],
                  float m[8]);
//! a.leafToNode of a tree (leaf index -> node index)
hipError_t farTreeLeafMap(const GravArgs& a, hipStream_t s);
//! far tree (uniform level-6 octree): leaves of the cells with far[k] set carry their moments, all others are
//! massless; then the mass-center / MAC / M2M upsweep
hipError_t farUpsweep(const GravArgs& a, const GCell* cells, const uint32_t* far, int nCells,
                      const int32_t* levelRangeHost, hipStream_t s);
//! the far tree's MAC geometry between syncs: every node's box (a.geoCenters / geoSizes -> outC / outS) with the far
//! cells' leaves replaced by their GCell boxes and every inner node the union of its children's boxes (open box)
hipError_t farRefreshBoxes(const GravArgs& a, const GCell* cells, const uint32_t* far, int nCells,
                           const int32_t* levelRangeHost, double* outC, double* outS, hipStream_t s);

//! expansion centers, MAC radii and multipoles of every node; levelRangeHost: kMaxLevel + 2 node offsets per level
hipError_t gravityUpsweep(const GravArgs& a, const int32_t* levelRangeHost, hipStream_t s);
//! adds G * (M2P + P2P) to ax, ay, az of [first, last) and 0.5 sum G m phi to *egrav
hipError_t gravityTraverse(const GravArgs& a, hipStream_t s);

//! Ewald parameters of one evaluation (ryoanji EwaldParameters<double, float>, nbody/ewald.hpp:58-91): the root's
//! expansion center and quadrupole (Cqi order), the shells, and computeEwaldRealSpace's constants
struct EwaldParams
{
    double cx, cy, cz;
    float  M[8];
    int    numReplicaShells, numEwaldShells, numH;
    double L, lCut2, alpha, alpha2, k1, ka, smallR2;
};

struct EwaldArgs
{
    uint32_t       first, last; // targets
    const double * x, *y, *z;
    const float*   m;
    float *        ax, *ay, *az; // G * correction is added
    float          G;
    const uint8_t* active; // nullable: only targets with active[i] != 0
    const double*  hsum;   // numH x {hr_scaled x, y, z, hfac_cos, hfac_sin} (device)
    double*        usum;   // device accumulator: += uscale * sum m phi (atomic)
    double         uscale;
    EwaldParams    p;
};

//! ewaldInitParameters (ewald.hpp:149-214) on the host: p and the k-space table (numH x 5); -1 if ceil(hCut) > 3
int ewaldInit(EwaldParams& p, std::vector<double>& hsum, const double center[3], const float Mroot[8], double L,
              int numReplicaShells, double lCut, double hCut, double alphaScale, double smallR);
//! computeEwaldRealSpace + computeEwaldKSpace per target (ewald.hpp:380-413): a += G (real + k), *usum += sum m phi
hipError_t ewaldCorrection(const EwaldArgs& a, hipStream_t s);

} // namespace sx
