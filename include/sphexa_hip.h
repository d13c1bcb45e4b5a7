/*! @file sphexa_hip.h
 * @brief C-ABI of libsphexa_hip.so -- the MI355X (gfx950) hot path of SPH-EXA's VE propagator.
 *
 * Plain C, POD structs and raw device pointers only.  Each entry point replaces one GPU seam of the
 * reference (paths relative to the SPH-EXA tree, lks1248/SPH-EXA @ 2024-10-16):
 *
 *   sx_sfc_keys            cstone::computeSfcKeysGpu            domain/include/cstone/sfc/sfc_gpu.h, sfc_gpu.cu:47
 *   sx_sort_keys           cstone::GpuSfcSorter::setMapFromCodes domain/include/cstone/primitives/primitives_gpu.cu:271-283
 *   sx_gather              cstone::gatherGpu                    primitives/primitives_gpu.cu:86
 *   sx_compute_octree      cstone::computeOctreeGpu / updateOctreeGpu (converged)  tree/csarray_gpu.cu:100-264
 *   sx_build_octree        cstone::buildOctreeGpu               tree/octree_gpu.cu:153-170
 *   sx_node_centers        cstone::computeGeoCentersGpu         focus/source_center_gpu.cu:117-135
 *   sx_compute_groups      cstone::computeFixedGroups (64)      domain/include/cstone/traversal/groups.cuh:13-41
 *   sx_spatial_groups      sph::computeSpatialGroups            sph/include/sph/groups.cu:30-47 (computeGroupSplits<64>,
 *                                                               traversal/groups.cuh:195-310)
 *   sx_find_neighbors      cstone::findNeighbors (+ sph h-nc iteration) findneighbors.hpp:167-188,
 *                                                               sph/include/sph/find_neighbors.hpp:10-44
 *   sx_xmass               sph::cuda::computeXMass              sph/include/sph/sph_gpu.hpp:25, hydro_ve/xmass_gpu.cu:103
 *   sx_ve_def_gradh        sph::cuda::computeVeDefGradh         sph_gpu.hpp:37, hydro_ve/ve_def_gradh_gpu.cu:86
 *   sx_eos                 sph::cuda::computeEOS (VE)           sph_gpu.hpp:40-43, hydro_ve/eos_gpu.cu:74
 *   sx_iad_divv_curlv      sph::cuda::computeIadDivvCurlv       sph_gpu.hpp:45, hydro_ve/iad_divv_curlv_gpu.cu:91
 *   sx_av_switches         sph::cuda::computeAVswitches         sph_gpu.hpp:48, hydro_ve/av_switches_gpu.cu:103
 *   sx_momentum_energy     sph::cuda::computeMomentumEnergy<avClean=false> sph_gpu.hpp:51-53, momentum_energy_gpu.cu:121
 *   sx_momentum_energy_avclean  sph::cuda::computeMomentumEnergy<avClean=true>  (same seam, second instantiation)
 *   sx_density             sph::cuda::computeDensity (std)      sph_gpu.hpp:32, hydro_ve/xmass_gpu.cu:150-164
 *   sx_eos_std             sph::cuda::computeEOS_HydroStd       sph_gpu.hpp:46-47, hydro_std/eos_gpu.cu:54-62
 *   sx_iad                 sph::computeIADGpu (std)             sph_gpu.hpp:19-20, hydro_std/iad_gpu.cu:111-124
 *   sx_momentum_energy_std sph::computeMomentumEnergyStdGpu     sph_gpu.hpp:22-23, hydro_std/momentum_energy_gpu.cu:109
 *   sx_positions           sph::computePositionsGpu             sph_gpu.hpp:64-72, positions_gpu.cu:167-179
 *   sx_mark_ramp           sph::cuda::computeMarkRamp           sph_gpu.hpp:54, hydro_ve/additional_fields.cu:86-98
 *   sx_positions_rungs     sph::computePositionsGpu (rungs)     sph_gpu.hpp:64-72, positions_gpu.cu:110-179
 *   sx_drift_positions     sph::driftPositionsGpu               sph_gpu.hpp:57-62, positions_gpu.cu:45-108
 *   sx_group_divv_timestep sph::groupDivvTimestepGpu            sph_gpu.hpp:80, ts_groups.cu:17-46
 *   sx_group_acc_timestep  sph::groupAccTimestepGpu             sph_gpu.hpp:83, ts_groups.cu:48-81
 *   sx_store_rung          sph::storeRungGpu                    sph_gpu.hpp:86, ts_groups.cu:84-108
 *   sx_rung_timestep       sph::rungTimestep                    sph/include/sph/ts_rungs.hpp:132-145 (sortGroupDt :67-78,
 *                                                               computeMinTimestep :89-105, findRungRanges :116-130)
 *   sx_minimum_group_dt    sph::minimumGroupDt                  ts_rungs.hpp:147-157
 *   sx_extract_groups      sph::extractGroupGpu                 sph/include/sph/groups.hpp:31-48
 *   sx_update_h            sph::updateSmoothingLengthGpu        sph_gpu.hpp:78, update_h_gpu.cu:49-60
 *   sx_max_divv            cstone::MinMaxGpu (rhoTimestep)      sph/ts_global.hpp:72-94
 *   sx_sim_*               one HydroVeProp step (sync + computeForces + integrate), main/src/propagator/ve_hydro.hpp:132-218
 *
 * Conventions (reference semantics preserved):
 *  - Field types follow sph::SphTypes (sph/types.hpp:39-46): x,y,z,temp,u,du double; other hydro fields float.
 *  - Neighbor criterion is the reference CPU one (cstone/findneighbors.hpp:111,133-158):
 *    |r_ij|^2 (double) < float(4 h_i^2), j != i, periodic folding when the particle is within 2h of the box edge.
 *  - nc[i] counts neighbors INCLUDING self (sph/find_neighbors.hpp:26); kernels use min(nc-1, ngmax) of them.
 *  - sx_xmass runs the neighbor search with the coupled h-nc iteration (mutates h, writes nc), exactly like
 *    sph::cuda::computeXMass.  The neighbor list it builds is cached in the context and reused by the later pair
 *    kernels of the same step (the reference GPU re-traverses the tree in each kernel; positions and h do not change
 *    between computeXMass and computeMomentumEnergy in ve_hydro.hpp:132-205).  Call sx_find_neighbors again if x,y,z
 *    or h change.
 *  - Every call is asynchronous on the context stream unless it returns a host scalar (sx_momentum_energy,
 *    sx_max_divv, sx_compute_octree), which synchronises that stream -- like the reference, whose entry points
 *    synchronise (e.g. xmass_gpu.cu:113).
 *  - Return value: SX_OK, or an SX_ERR_* code; sx_last_error() has the message.  The reference turns the same
 *    conditions into std::runtime_error (xmass_gpu.cu:126-127) or exit() (cuda/errorcheck.cuh:30-42).
 */
#ifndef SPHEXA_HIP_H
#define SPHEXA_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SX_OK 0
#define SX_ERR_TRAVERSAL 1   /* neighbor-search candidate buffer exhausted ("GPU traversal stack exhausted") */
#define SX_ERR_NOT_CONVERGED 2 /* coupled h-nc iteration failed to converge (xmass_gpu.cu:127) */
#define SX_ERR_HIP 3         /* HIP runtime error */
#define SX_ERR_ARG 4         /* invalid argument (sizes, missing buffers, no neighbor list) */
#define SX_ERR_NOMEM 5

/*! cstone::Box<double> (sfc/box.hpp:111-191). bnd[k]: 0 open, 1 periodic, 2 fixed (cstone::BoundaryType). */
typedef struct sx_box
{
    double  lim[6]; /* xmin xmax ymin ymax zmin zmax */
    int32_t bnd[3];
} sx_box;

/*! ParticlesData physics members (sph/particles_data.hpp:86-138) used by the VE kernels. */
typedef struct sx_params
{
    double   K;        /* kernel normalisation; sx_kernel_constant() returns the reference value */
    uint32_t ng0;      /* target neighbor count, 100 */
    uint32_t ngmax;    /* max stored neighbors, 150 */
    double   Kcour;    /* 0.2 */
    double   Krho;     /* 0.06 */
    double   gamma;    /* 5/3 */
    float    muiConst; /* 10 */
    float    alphamin, alphamax, decay_constant; /* 0.05, 1.0, 0.2 */
    float    Atmin, Atmax, ramp;                 /* 0.1, 0.2, 10 */
    double   maxDtIncrease;                      /* 1.1 */
    int32_t  avClean; /* sx_sim only: HydroVeProp<avClean=true> (ve_hydro.hpp:50, factory.hpp:56), 0 = off */
    float    theta;   /* gravity opening parameter (sphexa.cpp:127: 0.5 with gravity) */
    double   g;       /* gravitational constant (ParticlesData::g); sx_sim adds self-gravity when != 0 */
    double   eps, etaAcc; /* accelerationTimestep (ts_global.hpp:47-67): 0.005, 0.2 */
    int32_t  propagator;  /* sx_sim only: 0 = ve (HydroVeProp), 1 = std (HydroProp, std_hydro.hpp), 2 = ve-bdt
                             (HydroVeBdtProp, ve_hydro_bdt.hpp: block time-steps, one substep per sx_sim_step);
                             factory.hpp:50-84 */
} sx_params;

/*! Device pointers in sphexa::ParticlesData field order (particles_data.hpp:247-251); NULL where unused.
 *  n = number of particles INCLUDING halos (every array has this length). */
typedef struct sx_fields
{
    size_t    n;
    double *  x, *y, *z;
    float *   x_m1, *y_m1, *z_m1;
    float *   vx, *vy, *vz;
    float*    rho;
    double*   u;
    float *   p, *prho, *tdpdTrho, *h, *m, *c;
    float *   ax, *ay, *az;
    double*   du;
    float*    du_m1;
    float *   c11, *c12, *c13, *c22, *c23, *c33;
    float *   mue, *mui;
    double*   temp;
    float *   cv, *xm, *kx, *divv, *curlv, *alpha, *gradh;
    uint64_t* keys;
    uint32_t* nc;
    float *   dV11, *dV12, *dV13, *dV22, *dV23, *dV33;
    float*    markRamp;
    uint8_t*  rung;
} sx_fields;

/*! cstone::OctreeNsView<double, uint64_t> (tree/octree.hpp:296-316), device pointers. centers/sizes are
 *  Vec3<double> arrays (3 doubles per node). */
typedef struct sx_tree
{
    int32_t         numLeafNodes;
    int32_t         numNodes;
    const uint64_t* prefixes;
    const int32_t*  childOffsets;
    const int32_t*  internalToLeaf;
    const int32_t*  levelRange;
    const uint64_t* leaves;
    const uint32_t* layout; /* leaf -> first particle; numLeafNodes + 1 entries */
    const double*   centers;
    const double*   sizes;
    float           searchExtFactor;
} sx_tree;

/*! sph::GroupView (cstone/traversal/groups.hpp:19-55). The MI355X path partitions [firstBody, lastBody) into
 *  fixed 64-particle SFC blocks (one wavefront each); groupStart/groupEnd are accepted for interface parity. */
typedef struct sx_groups
{
    uint32_t        firstBody, lastBody, numGroups;
    const uint32_t* groupStart;
    const uint32_t* groupEnd;
} sx_groups;

/*! Linked octree arrays (cstone::OctreeData, tree/octree.hpp:318-375), device pointers, caller-owned.
 *  Sizes: numNodes = numLeaves + (numLeaves-1)/7; childOffsets numNodes+1; parents max(1,(numNodes-1)/8);
 *  levelRange 23; internalToLeaf, leafToInternal numNodes. */
typedef struct sx_octree
{
    uint64_t* prefixes;
    int32_t*  childOffsets;
    int32_t*  parents;
    int32_t*  levelRange;
    int32_t*  internalToLeaf;
    int32_t*  leafToInternal;
} sx_octree;

/*! neighbor-search statistics (cstone::NcStats, traversal/find_neighbors.cuh:346-357) */
typedef struct sx_nbstats
{
    uint64_t sumNeighbors;   /* sum over targets of stored neighbors */
    uint32_t maxNeighbors;   /* max true count (excluding self) */
    uint32_t numFailed;      /* h-nc iteration failures */
    uint64_t sumCandidates;  /* candidate particles tested (per target, summed) */
    uint64_t sumUnion;       /* cluster neighbor-union entries, summed over 256-particle clusters */
    uint32_t build;          /* search build used: 0 compact, 1 large, 2 compact overflowed and redone by the large */
    uint32_t maxUnion;       /* largest cluster neighbor union (local lists; 0 otherwise) */
} sx_nbstats;

typedef struct sx_ctx sx_ctx;

/* ---- context --------------------------------------------------------------------------------------------- */
int         sx_create(sx_ctx** ctx, int device);
void        sx_destroy(sx_ctx* ctx);
int         sx_set_stream(sx_ctx* ctx, void* hipStream); /* NULL = the context's own stream */
void*       sx_get_stream(sx_ctx* ctx);
const char* sx_last_error(sx_ctx* ctx);
/*! 1: bit-reproducible arithmetic (no FMA contraction; matches the CPU reference bit-for-bit given the same neighbor
 *  order); 0 (default): FMA-contracted kernels. */
int    sx_set_exact(sx_ctx* ctx, int exact);
double sx_kernel_constant(void); /* K of the sinc^6 kernel, particles_data.hpp:366 */
/*! host evaluation of the register-resident kernel W(v), dW/dv of the fast pair kernels (sx_kernel_poly.hpp), for
 *  checking it against the reference tables */
int    sx_kernel_poly(const float* v, size_t n, float* w, float* dw);
int    sx_copy_tables(sx_ctx* ctx, float* wh_host, float* whd_host); /* 20000-entry f32 tables */
int    sx_synchronize(sx_ctx* ctx);

/* ---- device memory plumbing (for hosts without their own allocator, e.g. ctypes bindings) --------------- */
void* sx_device_alloc(sx_ctx* ctx, size_t bytes);
int   sx_device_free(sx_ctx* ctx, void* ptr);
/*! kind: 1 host->device, 2 device->host, 3 device->device; synchronous w.r.t. the context stream */
int   sx_memcpy(sx_ctx* ctx, void* dst, const void* src, size_t bytes, int kind);
int   sx_memset(sx_ctx* ctx, void* dst, int value, size_t bytes);

/* ---- cstone: SFC keys, sorting, tree -------------------------------------------------------------------- */
int sx_sfc_keys(sx_ctx* ctx, const double* x, const double* y, const double* z, uint64_t* keys, size_t n,
                const sx_box* box);
/*! sort keys ascending in place (stable) and write the permutation: order[i] = old index of sorted element i */
int sx_sort_keys(sx_ctx* ctx, uint64_t* keys, uint32_t* order, size_t n);
/*! dst[i] = src[order[i]] for elements of elemBytes (1,2,4,8,16) */
int sx_gather(sx_ctx* ctx, const uint32_t* order, size_t n, const void* src, void* dst, int elemBytes);
/*! fully converged cornerstone leaves of sorted keys (the unique tree of csarray.hpp:456-467).
 *  leaves: capacity+1 entries, counts: capacity. *numLeaves receives the count; SX_ERR_ARG if capacity is short. */
int sx_compute_octree(sx_ctx* ctx, const uint64_t* sortedKeys, size_t n, uint32_t bucketSize, uint64_t* leaves,
                      uint32_t* counts, int32_t capacity, int32_t* numLeaves);
int sx_build_octree(sx_ctx* ctx, const uint64_t* leaves, int32_t numLeaves, const sx_octree* out);
int sx_node_centers(sx_ctx* ctx, const uint64_t* prefixes, int32_t numNodes, const sx_box* box, double* centers,
                    double* sizes);
/*! layout[i] = exclusive prefix sum of counts (layout has numLeaves+1 entries) */
int sx_leaf_layout(sx_ctx* ctx, const uint32_t* counts, int32_t numLeaves, uint32_t* layout);

/* ---- sph ------------------------------------------------------------------------------------------------- */
/*! fixed groups of 64 SFC-consecutive targets (one wavefront each); groupStart/groupEnd = NULL (implicit) */
int sx_compute_groups(sx_ctx* ctx, uint32_t first, uint32_t last, sx_groups* groups);
/*! computeSpatialGroups: the fixed 64-groups split where consecutive particles are farther apart than
 *  tolFactor * cbrt(smallest leaf volume of the group) in box-scaled coordinates (the reference passes
 *  tolFactor = 2).  Writes groups[0..numGroups] (device array of capacity cap >= last - first + 1) and sets
 *  out->groupStart = groups, out->groupEnd = groups + 1. */
int sx_spatial_groups(sx_ctx* ctx, uint32_t first, uint32_t last, const double* x, const double* y, const double* z,
                      const sx_tree* tree, const sx_box* box, float tolFactor, uint32_t* groups, uint32_t cap,
                      sx_groups* out);
/*! neighbor search for targets [first,last) into the context's list; iterate_h != 0 runs the h-nc iteration
 *  (mutates h). nc has length fields->n (written at [first,last)). stats may be NULL. */
/*! which neighbor-search build sx_find_neighbors runs: 0 automatic (the compact build, four workgroups per CU,
 *  with a device-side fallback to the large build on a capacity overflow; the large one after an overflow or at
 *  > 105 neighbors per target), 1 large only, 2 compact first, 3 compact with a forced overflow of every cluster
 *  (test hook for the fallback).  All give identical h, nc and neighbor lists. */
int sx_set_search_mode(sx_ctx* ctx, int mode);
int sx_find_neighbors(sx_ctx* ctx, const sx_fields* f, const sx_tree* tree, const sx_box* box,
                      const sx_params* p, uint32_t first, uint32_t last, int iterate_h, sx_nbstats* stats);
/*! copy the cached list out / in, CPU layout neighbors[(i-first)*ngmax + k] (device pointers); export zero-fills
 *  slots k >= min(nc[i]-1, ngmax) */
int sx_export_neighbors(sx_ctx* ctx, const uint32_t* nc, uint32_t first, uint32_t last, uint32_t ngmax,
                        uint32_t* neighbors);
int sx_import_neighbors(sx_ctx* ctx, uint32_t first, uint32_t last, uint32_t ngmax, const uint32_t* neighbors);

int sx_xmass(sx_ctx* ctx, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box,
             const sx_tree* tree);
/*! xmass on the cached (or imported) neighbor list, without a new search */
int sx_xmass_only(sx_ctx* ctx, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box);
int sx_ve_def_gradh(sx_ctx* ctx, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box);
int sx_eos(sx_ctx* ctx, uint32_t first, uint32_t last, float mui, double gamma, const double* temp, const float* m,
           const float* kx, const float* xm, const float* gradh, float* prho, float* c, float* rho, float* p);
/*! also writes the velocity gradient dV11..dV33 when f->dV11 != NULL (doGradV: dV11.size() == x.size(),
 *  iad_divv_curlv_gpu.cu:96-97, divv_curlv_kern.hpp:113-121) */
int sx_iad_divv_curlv(sx_ctx* ctx, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box);
int sx_av_switches(sx_ctx* ctx, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box,
                   double minDt);
/*! writes ax,ay,az,du; *minDtCourant receives the min Courant time-step (float, like minDt_ve_device) */
int sx_momentum_energy(sx_ctx* ctx, const sx_groups* g, float* groupDt, const sx_fields* f, const sx_params* p,
                       const sx_box* box, float* minDtCourant);
/*! computeMomentumEnergy<avClean=true> (sph_gpu.hpp:51-53, momentum_energy_gpu.cu:147-152): adds the
 *  avRvCorrection of the AV-cleaning propagator (momentum_energy_kern.hpp:43-63); needs f->dV11..dV33 */
int sx_momentum_energy_avclean(sx_ctx* ctx, const sx_groups* g, float* groupDt, const sx_fields* f,
                               const sx_params* p, const sx_box* box, float* minDtCourant);
/* ---- std propagator (HydroProp, main/src/propagator/std_hydro.hpp:124-184) ----------------------------- */
/*! sph::cuda::computeDensity (sph_gpu.hpp:32, hydro_ve/xmass_gpu.cu:150-164): neighbor search with the h-nc
 *  iteration (like sx_xmass), the XMass loop written to rho, then rho = m / rho.  Needs f->rho. */
int sx_density(sx_ctx* ctx, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box,
               const sx_tree* tree);
/*! density on the cached (or imported) neighbor list, without a new search */
int sx_density_only(sx_ctx* ctx, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box);
/*! sph::cuda::computeEOS_HydroStd (sph_gpu.hpp:46-47, hydro_std/eos_gpu.cu:54-62): p, c from temp and rho */
int sx_eos_std(sx_ctx* ctx, uint32_t first, uint32_t last, float mui, double gamma, const double* temp,
               const float* m, float* rho, float* p, float* c);
/*! sph::computeIADGpu (sph_gpu.hpp:19-20, hydro_std/iad_gpu.cu:111-124): c11..c33 with volumes m/rho */
int sx_iad(sx_ctx* ctx, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box);
/*! sph::computeMomentumEnergyStdGpu (sph_gpu.hpp:22-23, hydro_std/momentum_energy_gpu.cu:109-129): ax,ay,az,du
 *  (alpha = 1, gradh = 1); *minDtCourant receives the min Courant time-step */
int sx_momentum_energy_std(sx_ctx* ctx, const sx_groups* g, const sx_fields* f, const sx_params* p,
                           const sx_box* box, float* minDtCourant);

/*! 2nd-order Press position update + AB2 energy update on temp (positions.hpp:54-139, F2-correct); dt, dt_m1 double
 *  as in the CPU path (the reference GPU path passes them as float). */
int sx_positions(sx_ctx* ctx, uint32_t first, uint32_t last, double dt, double dt_m1, const sx_fields* f,
                 double gamma, float muiConst, const sx_box* box);
int sx_update_h(sx_ctx* ctx, uint32_t first, uint32_t last, uint32_t ng0, const uint32_t* nc, float* h);
/*! updateSmoothingLengthGpu over the targets of a group view (update_h_gpu.cu:49-60; ve_hydro_bdt.hpp:369 passes the
 *  active rungs): explicit groups, or fixed 64-blocks of [firstBody, lastBody) when groupStart is NULL */
int sx_update_h_groups(sx_ctx* ctx, const sx_groups* g, uint32_t ng0, const uint32_t* nc, float* h);

/*! computeMarkRamp (sph_gpu.hpp:54, hydro_ve/additional_fields.cu:47-98): per target the mean over its neighbors of
 *  1 (Atwood > Atmax) or ramp*(Atwood - Atmin) (Atmin <= Atwood <= Atmax), rho = kx m / xm; uses the cached list */
int sx_mark_ramp(sx_ctx* ctx, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box,
                 float* markRamp);

/* ---- block time-steps (HydroVeBdtProp, main/src/propagator/ve_hydro_bdt.hpp) ------------------------------------
 * Groups: explicit [groupStart[g], groupEnd[g]) (sx_spatial_groups, or a slice of a rung-sorted group list) or, with
 * groupStart == NULL, fixed 64-particle blocks of [firstBody, lastBody).  dt_m1[SX_MAX_RUNGS] holds the previous
 * time-step of each rung; rung (nullable) selects dt_m1[rung[i]], else dt_m1[0].  constCv < 0: cv from f->mui
 * (idealGasCv per particle).  f->temp NULL: the update acts on f->u instead. */
#define SX_MAX_RUNGS 4 /* sph::Timestep::maxNumRungs (sph/timestep.h:42) */
/*! computePositionsGpu (sph_gpu.hpp:64-72, positions_gpu.cu:110-179): Press position update + AB2 energy */
int sx_positions_rungs(sx_ctx* ctx, const sx_groups* g, float dt, const float* dt_m1, const uint8_t* rung,
                       const sx_fields* f, double gamma, double constCv, const sx_box* box);
/*! driftPositionsGpu (sph_gpu.hpp:57-62, positions_gpu.cu:45-108): back by dt_back, forward by dt, open box */
int sx_drift_positions(sx_ctx* ctx, const sx_groups* g, float dt, float dt_back, const float* dt_m1,
                       const uint8_t* rung, const sx_fields* f, double gamma, double constCv);
/*! groupDivvTimestepGpu (ts_groups.cu:17-46): groupDt[g] = min(groupDt[g], Krho / |max divv over g|) */
int sx_group_divv_timestep(sx_ctx* ctx, float Krho, const sx_groups* g, const float* divv, float* groupDt);
/*! groupAccTimestepGpu (ts_groups.cu:48-81): groupDt[g] = min(groupDt[g], etaAcc / |a|max^(1/2)) */
int sx_group_acc_timestep(sx_ctx* ctx, float etaAcc, const sx_groups* g, const float* ax, const float* ay,
                          const float* az, float* groupDt);
/*! storeRungGpu (ts_groups.cu:84-108) */
int sx_store_rung(sx_ctx* ctx, const sx_groups* g, uint8_t rung, uint8_t* rungs);
int sx_max_divv(sx_ctx* ctx, uint32_t first, uint32_t last, const float* divv, float* maxDivv);

/* ---- observables ---------------------------------------------------------------------------------------- */
/*! conservedQuantitiesGpu (main/src/observables/conserved_gpu.cu:71-94) and the nc sum of
 *  computeConservedQuantities (conserved_quantities.hpp:118-131) over [first, last) of f, in double:
 *  out = {0.5 sum m v^2, internal energy, linear momentum x y z, angular momentum x y z, sum nc}.  Internal energy
 *  is sum u m when f->u is set, else sum cv T m with cv = idealGasCv(muiConst, gamma).  Synchronises. */
int sx_conserved_quantities(sx_ctx* ctx, const sx_fields* f, uint32_t first, uint32_t last, float muiConst,
                            double gamma, double out[9]);

/* ---- self-gravity: ryoanji MultipoleHolder seam (multipole_holder.cuh:40-66, gravity_wrapper.hpp:104-174) ----- */
/*! expansion centers (mass centers, {x,y,z,mac^2}, numNodes x 4 doubles; mac = 2 max(node size)/theta + |com-geo|,
 *  setMac, source_center.hpp:130-143) and Cartesian quadrupoles (numNodes x 8 floats, Cqi order,
 *  cartesian_qpole.hpp:59-126) of every node of the linked octree over f's particles (single rank: the focus tree
 *  of syncGrav is the local tree).  Bit-identical to the reference CPU upsweep. */
int sx_gravity_upsweep(sx_ctx* ctx, const sx_fields* f, const sx_tree* tree, float theta, double* centers,
                       float* multipoles);
/*! Barnes-Hut traversal for targets [g->firstBody, g->lastBody) (computeGravity, traversal_cpu.hpp:166-230: groups
 *  of 16, vector MAC, quadrupole M2P, P2P softened by h_i + h_j): adds G * acc to f->ax, ay, az and returns the
 *  potential energy 0.5 sum G m phi in *egrav.  With explicit groups (g->groupStart, e.g. the active rungs of
 *  ve-bdt, MultipoleHolder::traverse(gravGroup, ...), ve_hydro_bdt.hpp:279-285) only the targets of those groups are
 *  traversed (the others keep their acceleration) and egrav sums over them.  Open boxes (a periodic box:
 *  sx_gravity_traverse_pbc). */
int sx_gravity_traverse(sx_ctx* ctx, const sx_groups* g, const sx_fields* f, const sx_tree* tree, const sx_box* box,
                        const double* centers, const float* multipoles, float G, double* egrav);
/*! the walk over the periodic images (MultipoleHolder::compute(..., numShells, box, ...), gravity_wrapper.hpp:139-141;
 *  traversal_cpu.hpp:200-216 / traversal.cuh:485-513): as sx_gravity_traverse, the targets shifted by every
 *  (ix Lx, iy Ly, iz Lz), |ix|, |iy|, |iz| <= numShells (0..4); numShells 0 = the box alone.  Periodic self-gravity
 *  is this walk with numShells = EwaldSettings::numReplicaShells followed by sx_gravity_ewald.  No interaction
 *  counting on this path. */
int sx_gravity_traverse_pbc(sx_ctx* ctx, const sx_groups* g, const sx_fields* f, const sx_tree* tree,
                            const sx_box* box, const double* centers, const float* multipoles, float G, int numShells,
                            double* egrav);

/*! ryoanji::EwaldSettings (nbody/ewald.h:15-22); the reference's defaults: 1, 2.6, 2.8, 2.0, 3e-3 */
typedef struct
{
    int    numReplicaShells; /* image shells the tree walk covered (their -erf correction) */
    double lCut;             /* real-space cutoff (box lengths) */
    double hCut;             /* k-space cutoff, ceil(hCut) <= 3 */
    double alphaScale;       /* Ewald splitting alpha = alphaScale / L */
    double smallRScaleFactor;
} sx_ewald_settings;

/*! Ewald correction of periodic self-gravity (computeGravityEwaldGpu, ryoanji/interface/ewald.cu:60-95, i.e.
 *  computeGravityEwald, nbody/ewald.hpp:380-413) for the targets of g: the root's expansion (centers[0..2],
 *  multipoles[0..7], device arrays of sx_gravity_upsweep) summed over the images in real space and in k space; adds
 *  G * correction to f->ax, ay, az and 0.5 G sum m phi to *egrav.  SX_ERR_ARG unless the box is cubic and
 *  ceil(hCut) <= 3.  Only targets of g (explicit groups: their targets) are corrected.  The correction completes a
 *  walk over numReplicaShells image shells (sx_gravity_traverse_pbc). */
int sx_gravity_ewald(sx_ctx* ctx, const sx_groups* g, const sx_fields* f, const sx_box* box, const double* centers,
                     const float* multipoles, float G, const sx_ewald_settings* settings, double* egrav);

/* ---- multi-GPU transport (replaces the reference's MPI calls, see sph-exa_amd/csrc/sx_comm.hpp) ---------- */
typedef struct sx_comm sx_comm;
/*! host-staged collectives supplied by the caller (e.g. torch.distributed gloo): buffers are host memory,
 *  send/recv segments contiguous in rank order; return 0 on success. op: 0 = u32 sum, 1 = f64 min, 2 = f64 sum,
 *  3 = u32 min, 4 = u32 max. */
typedef int (*sx_alltoallv_cb)(void* user, const void* sendHost, const uint64_t* sendBytes, void* recvHost,
                               const uint64_t* recvBytes);
typedef int (*sx_allreduce_cb)(void* user, void* bufHost, uint64_t count, int op);
/*! RCCL unique id (128 bytes) created on rank 0 and broadcast by the caller's control plane */
int  sx_comm_unique_id(void* id128);
/*! RCCL communicator over the node's GPUs (the calling process must have selected its device via sx_create) */
int  sx_comm_create_rccl(sx_comm** comm, int rank, int size, const void* id128);
int  sx_comm_create_host(sx_comm** comm, int rank, int size, sx_alltoallv_cb a2a, sx_allreduce_cb ar, void* user);
void sx_comm_destroy(sx_comm* comm);
/*! the transport's two operations on device buffers, as the domain sync uses them (sx_comm.hpp): every rank sends
 *  sendBytes[q] bytes from send + sendOff[q] to rank q and receives recvBytes[q] at recv + recvOff[q] (MPI_Alltoallv
 *  shape of the reference's Isend/Recv halo and particle exchange, halos/exchange_halos_gpu.cuh:51-143,
 *  domain/domaindecomp_mpi_gpu.cuh:86-171), enqueued on hipStream; and an in-place allreduce of count elements, op 0 =
 *  u32 sum (tree counts, update_mpi_gpu.cuh:75), 1 = f64 min (time-step, ts_global.hpp:106), 2 = f64 sum
 *  (conserved quantities, conserved_quantities.hpp:163-165).  Results are complete when the stream is. */
int  sx_comm_alltoallv(sx_comm* comm, const void* send, const uint64_t* sendBytes, const uint64_t* sendOff, void* recv,
                       const uint64_t* recvBytes, const uint64_t* recvOff, void* hipStream);
int  sx_comm_allreduce(sx_comm* comm, void* dev, uint64_t count, int op, void* hipStream);

/* ---- block time-step host bookkeeping (HydroVeBdtProp::computeRungs, ve_hydro_bdt.hpp:292-331) ---------------- */
/*! sph::Timestep (sph/timestep.h:38-48) */
typedef struct sx_timestep
{
    float    nextDt, elapsedDt, totDt;
    int      numRungs, substep;
    uint32_t rungRanges[SX_MAX_RUNGS + 1];
    float    dt_m1[SX_MAX_RUNGS], dt_drift[SX_MAX_RUNGS];
} sx_timestep;
/*! rungTimestep (ts_rungs.hpp:132-145): sorts groupDt[0, numGroups) ascending in place with groupIndices (the group
 *  of each sorted entry), min-reduces {groupDt[0], groupDt[(uint32_t)(0.4f * numGroups)]} over comm's ranks
 *  (comm NULL: this rank only), numRungs = min(int(log2(dt40 / dtMin)) + 1, SX_MAX_RUNGS), rungRanges by lower bound
 *  of 2^r dtMin, nextDt = min(maxDt, dtMin), totDt = nextDt 2^numRungs; elapsedDt, substep, dt_m1, dt_drift = 0.
 *  numGroups >= 1.  Synchronises the context stream (the results are host values, as in the reference). */
int sx_rung_timestep(sx_ctx* ctx, float* groupDt, uint32_t* groupIndices, uint32_t numGroups, float maxDt,
                     sx_comm* comm, sx_timestep* out);
/*! minimumGroupDt (ts_rungs.hpp:147-157) for the numGroups active groups of substep ts->substep: sorts them as
 *  above, groupIndices[numGroups, ts->rungRanges[SX_MAX_RUNGS]) = the identity; *dt = min(dtMin, (totDt -
 *  elapsedDt) / substeps left), rungRanges over all SX_MAX_RUNGS rungs.  numGroups may be 0 (a rank without active
 *  groups on a substep: it contributes nothing to the min over the ranks).  Synchronises the context stream. */
int sx_minimum_group_dt(sx_ctx* ctx, const sx_timestep* ts, float* groupDt, uint32_t* groupIndices, uint32_t numGroups,
                        sx_comm* comm, float* dt, uint32_t* rungRanges);
/*! extractGroupGpu (groups.hpp:31-48): group k of the output = group indices[first + k] of grp, k < last - first
 *  (device arrays outStart/outEnd; the view they form has firstBody = lastBody = 0) */
int sx_extract_groups(sx_ctx* ctx, const sx_groups* grp, const uint32_t* indices, uint32_t first, uint32_t last,
                      uint32_t* outStart, uint32_t* outEnd);

/* ---- host-side decisions of the SFC domain decomposition (sph-exa_amd/csrc/sx_domain.cpp) -------------- */
/*! equal-count SFC splitters from the all-reduced histogram of 2^histBits key bins (bin = key >> (63-histBits)):
 *  rank q owns keys [split[q], split[q+1]); split has nranks+1 entries.  Replaces cstone::makeSfcAssignment,
 *  domain/include/cstone/domain/domaindecomp.hpp:120. */
int sx_domain_splitters(const uint32_t* hist, uint32_t histBits, int nranks, uint64_t* split);
/*! halo receive layout [lower ranks | numLocal locals | higher ranks] (domain.hpp:196-244): recvOff[q] for each
 *  peer (0 for rank itself), out = {first local, last local, total}. */
int sx_domain_halo_layout(const uint64_t* recvCounts, int nranks, int rank, uint64_t numLocal, uint64_t* recvOff,
                          uint64_t out[3]);

/* ---- device-resident simulation: one HydroVeProp step per call ----------------------------------------- */
typedef struct sx_sim sx_sim;
/*! a simulation of up to capacity particles in box.  Self-gravity (p->g != 0) in a periodic box: the walk over one
 *  image shell + the Ewald correction with the reference's EwaldSettings defaults (gravity_wrapper.hpp:135-157), one
 *  rank, VE or std propagator (SX_ERR_ARG for ve-bdt; several ranks: at sx_sim_set_comm). */
int    sx_sim_create(sx_sim** sim, sx_ctx* ctx, size_t capacity, const sx_params* p, const sx_box* box,
                     uint32_t bucketSize);
void   sx_sim_destroy(sx_sim* sim);
int    sx_sim_init_sedov(sx_sim* sim, uint32_t side);
/*! distribute the step over a communicator: SFC assignment by a global key histogram (all ranks equal counts),
 *  particle exchange, halo discovery and the reference's five halo exchanges per step
 *  (ve_hydro.hpp:150-186), global time-step min.  rank/size come from the communicator. */
int    sx_sim_set_comm(sx_sim* sim, sx_comm* comm);
/*! this rank's share of a Sedov lattice of side^3 particles (contiguous lattice-index slab; the first step's
 *  sync moves particles to their SFC owner) */
int    sx_sim_init_sedov_rank(sx_sim* sim, uint32_t side, int rank, int size);
/*! overlap of the halo exchanges with the pair kernels (default on; several ranks, fast kernels): each exchange of
 *  ve_hydro.hpp:150-186 runs on a communication stream while the clusters whose neighbor union holds no halo are
 *  computed, the rest after it lands.  Results are bitwise identical with it off. */
int    sx_sim_set_overlap(sx_sim* sim, int on);
/*! interior and boundary cluster counts of the last distributed step (0, 0 without overlap) */
int    sx_sim_overlap_stats(sx_sim* sim, uint32_t out[2]);
/*! local particle range [first,last) and total (with halos) of the last step */
int    sx_sim_layout(sx_sim* sim, uint64_t out[4]);
/*! upload a host state (conserved fields, length n) */
int    sx_sim_set_state(sx_sim* sim, size_t n, const double* x, const double* y, const double* z, const float* h,
                        const float* m, const double* temp, const float* vx, const float* vy, const float* vz,
                        const float* x_m1, const float* y_m1, const float* z_m1, const float* du_m1,
                        const float* alpha, const uint64_t* id, double minDt, double minDt_m1);
/*! device field pointers of the current state (valid until the next step).  After a one-rank VE or std step the
 *  keys are those of the updated coordinates (computed by the position update for the next sync), not of the
 *  step's tree; writing x, y or z through these pointers between steps is not supported on that path */
int    sx_sim_fields(sx_sim* sim, sx_fields* f, uint64_t** id);
size_t sx_sim_size(sx_sim* sim);
/*! one VE step; the time-step scalars stay on the device (no host sync unless stats are requested) */
int    sx_sim_step(sx_sim* sim);
/*! minDt, minDt_m1, ttot, minDtCourant, minDtRho (synchronises) */
int    sx_sim_scalars(sx_sim* sim, double out[6]);
/*! per-stage device time of the last step (ms) measured with HIP events, names in stage order */
int    sx_sim_stage_times(sx_sim* sim, float* ms, int cap, const char** names);
int    sx_sim_last_stats(sx_sim* sim, sx_nbstats* stats);
/*! multi-rank self-gravity of the last step: {gravity halos received, remote level-6 cells used as far-field
 *  multipoles, remote cells in total} (zeros on one rank) */
int    sx_sim_gravity_stats(sx_sim* sim, uint64_t out[3]);
/*! count the self-gravity interactions of the following steps (the reference's BhStats, collected only when its
 *  stats are requested, traversal.cuh:346-357): off by default -- the counting traversal is a separate kernel
 *  instantiation, ~8 % slower.  SX_ERR_ARG without gravity. */
int    sx_sim_set_gravity_counting(sx_sim* sim, int enable);
/*! self-gravity interactions of the last VE step on this rank (zeros when counting was off), counted per target as
 *  the reference's BhStats (nbody/traversal.cuh:346-357, 614-620): {sumP2P (source particles), sumM2P (multipole
 *  nodes)}; synchronises.  SX_ERR_ARG without gravity. */
int    sx_sim_gravity_interactions(sx_sim* sim, uint64_t out[2]);
/*! computeConservedQuantities (conserved_quantities.hpp:110-179) of the current state, summed over the ranks of the
 *  communicator: {ecin, eint, egrav, etot, |linmom|, |angmom|, totalNeighbors, linmom x y z, angmom x y z}
 *  (egrav of the last step; synchronises) */
int    sx_sim_conserved(sx_sim* sim, double out[13]);
/*! device time (ms) of each hot kernel alone in the last step (HIP events on the launch stream, bracketing just the
 *  launch): findNeighbors, xmass, veDefGradh, iadDivvCurlv, avSwitches, momentumEnergy */
int    sx_sim_kernel_times(sx_sim* sim, float* ms, int cap, const char** names);
/*! propagator 2 (ve-bdt): the Timestep after the last substep (sph::Timestep, timestep_ of HydroVeBdtProp,
 *  ve_hydro_bdt.hpp:380).  A substep with activeRung(substep, numRungs) == 0 starts a new hierarchy (full sync,
 *  every particle active); the others drift the inactive rungs and compute the active ones (partial sync: halo
 *  x,y,z,h refreshed, order, tree and halo lists kept).  SX_ERR_ARG for the other propagators. */
int    sx_sim_timestep(sx_sim* sim, sx_timestep* ts);
/*! the simulation time d.ttot (a restart's "time" attribute, particles_data.hpp:170-190; set_state starts at 0) */
int    sx_sim_set_time(sx_sim* sim, double ttot);
/*! propagator 2: restart state after sx_sim_set_state (HydroVeBdtProp::load, ve_hydro_bdt.hpp:155-168): the Timestep
 *  saved with the file and the `rung` of each set_state particle (host array, set_state order; NULL keeps rung 0).
 *  SX_ERR_ARG unless activeRung(ts->substep, ts->numRungs) == 0: restart files exist only at hierarchy boundaries
 *  (the reference writes them only when isSynced(), sphexa.cpp:165). */
int    sx_sim_set_timestep(sx_sim* sim, const sx_timestep* ts, const uint8_t* rung);
/*! neighbor lists behind a skin (VE or std propagator, one rank or several, with or without self-gravity -- not with
 *  periodic self-gravity; sph-exa_amd/csrc/sx_skin.hpp):
 *  replaces the per-step Domain::sync + findNeighborsSph of ve_hydro.hpp:140-149 by a filter of the last build's
 *  lists within 2h(1 + factor) while no particle can have entered a target's 2h sphere since that build; stale
 *  clusters are rebuilt at once.  Neighbor sets, h and nc stay those of findNeighbors; between builds the particle
 *  order and tree are kept.  factor 0 restores a sync + search every step; a full sync + build of every cluster
 *  happens at least every maxReuse steps.  Default: factor 0.05, maxReuse 24.  Takes effect at the next step (full
 *  build). */
int    sx_sim_set_skin(sx_sim* sim, float factor, int maxReuse);
/*! the next step does a full sync and builds every cluster's skin (e.g. after writing a restart file, so a run that
 *  continues and one restarted from the file take identical steps) */
int    sx_sim_rebuild_lists(sx_sim* sim);
/*! {full builds, steps served by the filter, clusters rebuilt as stale, clusters sent to the exact search, stale
 *  clusters of the last step, of them exact, skin-list capacity per target, steps searched without the skin while
 *  backing off, the current skin's s and the next build's s (both in millionths), reuse steps redone from a full sync
 *  (clusters stale again after their rebuild), clusters of reuse steps whose targets all kept the hits of the last
 *  step, so the filter kept their exact lists in place, of them frozen: no skin entry could have crossed its target's
 *  2h sphere, so their skin lists were not walked, clusters whose exact search ran concurrently with the rebuild of
 *  the other stale clusters}.  A skin that does not outlast
 *  two steps makes the next build's twice as wide (up to 0.16), then the steps back off to a plain search. */
int    sx_sim_skin_stats(sx_sim* sim, uint64_t out[14]);
/*! the last step's neighbor lists of the local particles as global indices into the state of sx_sim_fields, row-major
 *  out[(i - first) * ngmax + k] for k < min(nc - 1, ngmax) (device buffer of (last - first) * ngmax words; the lists
 *  the step's pair kernels used, cstone::findNeighbors' layout) */
int    sx_sim_export_neighbors(sx_sim* sim, uint32_t* out);

#ifdef __cplusplus
}
#endif

#endif
