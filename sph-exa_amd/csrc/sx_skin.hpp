/*! @file sx_skin.hpp
 * @brief Neighbor lists kept behind a skin across steps (sx_skin.hip): the search of a step becomes a filter of the
 *        last build's inflated lists whenever no particle can have entered a target's 2h sphere since that build.
 *
 * A BUILD (the search of sx_neighbors.hip with every radius scaled by skin1 = 1 + s, no h iteration) leaves, per
 * 256-particle cluster, the union U_s of its targets' neighbors within R_i = 2 h_i (1 + s) and per target its SKIN
 * LIST: u16 positions into U_s, ascending (U_s in the upper part of the cluster's union slot, uni[c*ucap + uoff]).
 * The FILTER (skinFilterKernel) then produces the step's exact lists -- the reference criterion d2 < (double)(4 h^2),
 * j != i (cstone/findneighbors.hpp:133-158), h-nc iteration (sph/find_neighbors.hpp:28-33) included -- and the exact
 * union (the U_s entries some target hit, in U_s order) at the slot's start, exactly what the search leaves for the
 * pair kernels.
 *
 * Validity (checked by the filter for every target, every step), Galilean invariant: with u(t) any displacement per
 * step (here the step's displacement of the cluster's first particle), x_i - x_j changes by sum_t (d_i(t) - u(t)) -
 * (d_j(t) - u(t)).  A particle j outside i's skin list at the build (|x_i^b - x_j^b| >= R_i) can now be closer than
 * 2 h_i only if the relative paths add up to R_i - 2 h_i.  From its last step outside the ball of radius R_i around i
 * on, j sits at the end of every step inside the cluster's region (the targets' box grown by max R), so each of its
 * steps is bounded by that step's largest |d - u| in the region (the displacement grid: per cell the component ranges
 * of the end-of-step positions' displacements), and the running sum of those maxima since the build, A_C, bounds its
 * part; i's part is its own relative path d_i = sum_t |d_i(t) - u(t)|.
 * So   2 h_i + d_i + A_C <= R_i (1 - eps)   guarantees the skin list holds every current neighbor of i.  A flow that
 * moves a region as a whole (Noh's infall) does not use up the skin; only relative motion does.  A cluster
 * failing it for some target (or whose build overflowed a capacity) is STALE: it is rebuilt on the spot (a build over
 * the stale clusters only, on node boxes refreshed from the current positions, then the filter); a cluster stale
 * again (its h iteration outgrew the fresh skin) takes the exact search, which writes its lists directly.
 *
 * Between builds the particle order and the tree are kept (no SFC re-sort: that would renumber the union entries);
 * sx_sim does a full sync + build of every cluster when the stale share or the steps since the last full build pass
 * their limits (SkinState).
 *
 * Round 6, what a reuse step may skip (sets, nc and h stay exactly those of the search):
 *  - KEPT: a cluster's exact lists are a function of its targets' kept-hit bits (the skin lists are fixed), so a walk
 *    whose bits equal those recorded with a set of lists (hitMask / hitMaskB) keeps that set: no rank pass, no second
 *    walk, no list writes.  Two sets per cluster (nloc / nlocB): a lattice's h moves between two shells, and the step
 *    after a crossing usually returns to the other set;
 *  - FROZEN: a walk also leaves a lower bound g_i of every skin entry's distance to its target's 2h sphere; while the
 *    growth of d_i + A_C since that walk plus 2|h_i - h_i,ref| stays below it for every target, no hit can have
 *    changed (the same drift bound), and the cluster is not walked at all -- the fused XMass runs over the exact lists.
 */
#pragma once

#include "sx_tree.hpp"

namespace sx
{

using SkinGrid = DispGrid; //!< per-step displacement maxima by cell (sx_device.hpp)

constexpr int kSkinGridN = 64;
constexpr int kSkinCap   = 1920; //!< U_s entries the filter stages (16 B each; a larger skin union takes the exact search)
//! u32 words of kept-hit bits per target (SkinArgs::hitMask): one u16 per 16-entry walk block, up to 256 entries
constexpr uint32_t kSkinMaskWords = 8;

//! filter arguments (one 256-thread workgroup per cluster)
struct SkinArgs
{
    uint32_t first, last, numGroups, ngmax, ng0;
    uint32_t ngmaxS; // skin-list capacity per target
    int      iterateH;
    int      fresh; // 1: the listed clusters were just built: record hb, ob, acc = 0 instead of checking the drift
    float    skin1; // 1 + s
    const double *x, *y, *z;
    float*       h;
    const float* m;
    uint32_t*    nc;
    RecX*        rxOut; // nullable
    // exact lists and unions (output, the pair kernels' nloc / uni[c*ucap ...] / ucount) and the skin unions (input,
    // uni[c*ucap + uoff ...], ucountS[c] entries)
    uint32_t*       nloc;
    uint32_t*       uni;
    uint32_t*       ucount;
    uint32_t        ucap;
    uint32_t        uoff;
    const uint32_t* ucountS;
    // skin state
    const uint32_t* sloc; // skin lists (nlocWords(ngmaxS) words per target, lane-interleaved like nloc)
    const uint32_t* scnt; // skin count + 1 per target (the build's nc)
    float*          hb;    // h at the build
    float*          rel;   // per target: its path relative to its cluster's reference particle since the build
    const float *   dispX, *dispY, *dispZ; // the last step's displacement of every particle
    float*          acc;   // per cluster: sum over the steps since its build of the largest displacement in its region
                           // relative to the reference particle (the first of the cluster)
    const uint32_t* cells; // displacement grid: per cell the component ranges of the last step (kGridWords planes)
    SkinGrid        grid;
    const uint32_t* list;  // nullable: the clusters list[1 .. list[0]], else all
    uint32_t*       stale; // [0] count, [1..] stale clusters (output)
    // nullable (reuse steps): per cluster 1 while its last stale step sent it to a rebuild and it has not been served
    // by a skin since; such a cluster, stale again, is listed in `direct` (the exact search) instead of `stale`
    uint8_t*        streak;
    uint32_t*       direct;
    // nullable: per target the kept-hit bits of the last pass that wrote its cluster's exact lists (kSkinMaskWords u32
    // words, lane-interleaved like nloc; bits 16 (k & 1) .. of word k / 2: walk block k), and per cluster 1 while the
    // exact union and lists at uni / nloc are the ones those bits give (0 once the cluster is stale).  With keepLists
    // (a reuse step after a skin search on the same lists) a cluster whose targets' bits are all unchanged keeps its
    // union and lists: the rank pass and its second walk of the skin lists are skipped
    uint32_t*       hitMask;
    uint8_t*        same;
    int             keepLists;
    // nullable: the second set of exact lists (ListsB, sx_device.hpp; same[c] bits 0 / 1: set A / B holds the lists
    // of its hit masks, bit kListsBSel: B is current).  A pass whose hits match the other set's makes that set current;
    // one that matches neither writes its lists into the other set, so the last two different hit sets stay
    uint32_t*       nlocB;
    uint32_t*       ucountB;
    uint32_t*       hitMaskB;
    uint32_t        uoffB;
    // nullable: per cluster the freeze reference of the last pass that walked its skin lists, the minima over its
    // targets of K_i + 2 h_i and K_i - 2 h_i with K_i = g_i + d_i + A_C, g_i bounding every skin entry's distance to
    // the target's 2h sphere then (-inf: never frozen).  A cluster whose targets have all moved, and whose h have
    // changed, less than that since (keepLists, same) is FROZEN: its exact lists stand, the skin lists are not walked
    float2*         frz;
    DevBox          box;
    const float*    powTab;
    // nullable: the fused XMass (xmassJLoop on the final lists, as sx_hydro_cluster.hip's xmassKernel): xm of every
    // completed target (the std propagator's density seam passes rho), and its RecT {xm, 0, 0, 0}
    float*          xmOut;
    RecT*           rtXm;
    double          K;
    uint32_t*       stats;   // kStatsWords (failures)
    uint4*          clStats; // per cluster {max count, stored, skin entries walked, union}
};

hipError_t skinFilter(const SkinArgs& a, uint32_t numClusters, hipStream_t s);
//! node boxes (center, half size) of the tree refreshed from the current positions: leaf boxes bound their particles,
//! inner boxes their children (for a build between full syncs, when particles have left their cells); withCells:
//! every box also contains the node's cell (the gravity MAC's geometry between syncs: never smaller than the cell's)
hipError_t skinRefreshBoxes(const DevTree& t, const double* x, const double* y, const double* z, const DevBox& box,
                            double* centers, double* sizes, hipStream_t s, bool withCells = false);
//! acc[c] = +inf for the listed clusters (their lists came from the exact search: the next step rebuilds their skin)
hipError_t skinMarkStale(const uint32_t* list, uint32_t numClusters, float* acc, hipStream_t s);
//! per-cluster statistics -> stats (the search's reduction)
hipError_t reduceClusterStats(const uint4* clStats, uint32_t numClusters, uint32_t* stats, hipStream_t s);

} // namespace sx
