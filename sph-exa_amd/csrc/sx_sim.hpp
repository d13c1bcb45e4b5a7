/*! @file sx_sim.hpp
 * @brief the device-resident simulation object behind sx_sim_* (sx_sim.cpp: HydroVeProp / HydroProp steps and the
 *        SFC domain; sx_bdt.cpp: HydroVeBdtProp substeps on the same domain)
 */
#pragma once

#include <hip/hip_runtime.h>

#include <initializer_list>
#include <string>
#include <utility>
#include <vector>

#include "../../include/sphexa_hip.h"
#include "sx_comm.hpp"
#include "sx_hydro.hpp"
#include "sx_tree.hpp"

namespace sx::sim
{

//! device scalars of one rank: ParticlesData time-step members
struct Scalars
{
    double   minDt, minDt_m1, ttot, minDtCourant, minDtRho;
    double   dtCand;   // rank-local candidate, globally min-reduced
    float    courant;  // atomic-min target of the momentum kernel
    unsigned maxDivvU; // order-preserving image of max divv
    double   egrav;    // gravitational potential energy (ParticlesData::egrav)
    unsigned long long maxAccSqBits; // max |a|^2 of the locals (bit image of a non-negative double)
    unsigned gravErr;
};

//! the conserved fields that travel with a particle in the SFC exchange (rung: ve-bdt only, else nullptr)
struct Fields
{
    double *  x, *y, *z, *temp;
    float *   h, *m, *vx, *vy, *vz, *xm1, *ym1, *zm1, *dum1, *alpha;
    uint64_t* id;
    uint8_t*  rung;
};

//! HydroVeBdtProp state (ve_hydro_bdt.hpp:380-400: timestep_, prevTimestep_, groups_, tsGroups_, groupDt_,
//! groupIndices_, activeRungs_, rungs_), host-side like the reference's except for the device group arrays
struct BdtState
{
    sx_timestep ts{}, prev{};
    bool        started{false};
    double      minDt{0}, minDt_m1{0}, ttot{0}; // d.minDt, d.minDt_m1, d.ttot
    float       searchExt{1.f};                 // d.treeView.searchExtFactor
    double      margin{1.05};                   // halo request margin of the last full sync
    double      egrav{0};                       // one rank: egrav of the last substep's traversal
    uint64_t    haloShort{0};                   // substeps whose search spheres left the hierarchy's halo boxes
    uint64_t    hierarchies{0}, warnedAt{~0ull};
    uint32_t*   groupBuf{nullptr};              // groups_ of the last full sync: [start_0 .. start_ng] (one array)
    sx_groups   groups{}, tsGroups{}, active{}, rungs[SX_MAX_RUNGS]{};
    float*      groupDt{nullptr};
    uint32_t*   groupIdx{nullptr};
    uint32_t *  tsStart[2]{}, *tsEnd[2]{}; // extracted (rung-sorted) groups, double-buffered
    uint8_t*    activeMask{nullptr};       // the active view as a target mask (multi-rank gravity)
    uint32_t*   maskRange{nullptr};
    uint64_t    substeps{0};
};

//! skin-list reuse of the neighbor search (sx_skin.hpp), one rank without self-gravity: between full builds the
//! particle order and tree are kept and each step's search is the filter of the last build's skin lists
struct SkinState
{
    float    factor{0.05f};     // s: skin radius 2 h (1 + s); 0 = every step syncs and searches (the reference's flow)
    float    cur{0.05f};        // s of the next build: doubled (up to kMaxSkin) while skins cannot outlast two steps
    float    built{0.05f};      // s of the current skin lists
    int      maxReuse{24};      // steps after a full build before the next one at the latest
    float    staleLimit{0.125f}; // share of stale clusters in a step after which the next step does a full build
    bool     valid{false};      // every cluster's skin lists are current (a full build since the last state change)
    bool     forceBuild{false};
    int      sinceBuild{0};
    uint32_t ngmaxS{0};         // skin-list capacity per target
    // a skin that does not outlast its build by two steps (fast flows: every cluster stale at once) costs more than it
    // saves: the next backoff steps search without it, backoffLen doubling with every such failure (up to 32)
    int      backoff{0}, backoffLen{4};
    int      cleanSinceBuild{0}; // reuse steps since the last full build with a stale share within the limit
    uint64_t plainSteps{0};     // steps searched without the skin while backing off
    // statistics: full builds, steps served by the filter, clusters rebuilt (stale), clusters sent to the exact search
    uint64_t builds{0}, reuseSteps{0}, staleClusters{0}, exactClusters{0};
    // reuse steps whose search was redone from a full sync (clusters stale again after their rebuild on a reuse step:
    // the exact search on the drifted tree's boxes could outgrow its capacities)
    uint64_t resyncs{0};
    uint32_t lastStale{0}, lastExact{0};
    // this step's clusters and stats[13] count (over all ranks with several; the "outlast two steps" test)
    uint64_t stepClusters{0}, stepS13{0};
    // this step: the filter computed XMass of every cluster but the exact-search ones (exactList[1 ..], lastExact)
    bool      xmFused{false};
    uint32_t* exactList{nullptr};
    // the exact lists, hit masks and per-cluster flags the last skin search left (SkinArgs::keepLists), and the
    // clusters whose lists a reuse step kept (statistics)
    bool      listsKept{false};
    const void *keptNloc{nullptr}, *keptUni{nullptr}, *keptMask{nullptr}, *keptSame{nullptr}, *keptFrz{nullptr},
        *keptNlocB{nullptr};
    uint64_t  keptClusters{0}, frozenClusters{0};
    uint64_t  earlyExact{0}; // exact-search clusters searched concurrently with the rebuild of the others
    // the step's second set of exact lists (sel == nullptr unless the step's search was the skin filter)
    sx::ListsB lb{};
};

} // namespace sx::sim

struct sx_sim
{
    using Scalars = sx::sim::Scalars;
    using Fields  = sx::sim::Fields;

    sx_ctx*        ctx;
    sx::NsPolicy   nsPolicy;       // neighbor search: compact or large build (sx_tree.hpp)
    sx::Transport* comm{nullptr};
    sx_comm*       commHandle{nullptr}; // the C-ABI handle of comm (host time-step reductions of ve-bdt)
    sx_params      p;
    sx_box         box;
    sx::DevBox     dbox;
    uint32_t       bucket;
    size_t         cap{0}, n{0}, first{0}, last{0};
    sx::Arena      mem;
    sx::Arena      work;
    sx::DevTree    tree;
    sx::DevTree    localTree;
    // multi-rank gravity: uniform level-6 far tree (built once, own arena) and the per-step near tree over the
    // locals + gravity halos (own arena, so neither clobbers the SPH tree's "dt.*" buffers)
    sx::Arena      farMem;
    sx::Arena      gravWork;
    sx::DevTree    farTree;
    sx::DevTree    nearTree;

    double *  x, *y, *z, *temp;
    float *   h, *m, *vx, *vy, *vz, *xm1, *ym1, *zm1, *dum1, *alpha;
    uint64_t* id;
    uint8_t*  rung{nullptr}; // ve-bdt: the rung of each particle (a conserved field, ve_hydro_bdt.hpp:94)
    uint64_t* keys;
    uint32_t *order, *nc;
    float *   xm, *kx, *gradh, *prho, *c, *divv, *curlv, *c11, *c12, *c13, *c22, *c23, *c33, *ax, *ay, *az;
    double*   du;
    float*    dV[6]{}; // dV11, dV12, dV13, dV22, dV23, dV33 (avClean only)
    float *   rho{nullptr}, *pres{nullptr}; // std propagator only (HydroProp DependentFields rho, p)
    sx::RecX* rx;
    sx::RecV* rv;
    sx::RecT* rt;
    sx::RecS* rs; // std: {rho, p} records, aliasing rt (the std step has no xm/kx/prho/alpha)
    sx::RecC* rc;
    sx::NbLists nb;
    uint32_t* stats;
    uint32_t* statsHost;
    int       sortBits{30};          // key bits the local sort orders first (sortLocals)
    bool      gravCount = false; // count the gravity interactions (sx_sim_set_gravity_counting)
    bool      keysFresh = false; // keys[0, n) hold the current coordinates' SFC keys (set by the position update,
                                 // consumed by the next localSync; cleared by every entry point that sets state)
    uint64_t  sortStats[4]{0, 0, 0, 0}; // sorts requested, done (not the identity), redone on all bits, moved-only
    Scalars*  sc;
    Scalars*  scHost;

    struct Spare
    {
        void** field;
        void*  alt;
        int    elemBytes;
    };
    std::vector<Spare> spares; // double buffers of the conserved fields

    // halo bookkeeping of the current step
    std::vector<uint64_t> haloSend, haloSendOff, haloRecv, haloRecvOff;
    uint32_t*             sendIdx{nullptr};
    uint64_t              numSend{0};
    uint64_t              numHalos{0};
    uint64_t*             cntBuf{nullptr};
    // per rank: its particles' occupied level-6 cells after the last sync (the nonzero global-histogram bins of its
    // SFC range; the splitters are bin boundaries), so the gravity cell all-gather needs no count exchange
    std::vector<uint64_t> cellsOf;
    uint32_t*             syncErr{nullptr}; // the last sync's halo-marking failure flag (device), read with the step's
                                            // statistics instead of a round trip of its own

    // overlap of the halo exchanges with the pair kernels of the interior clusters (no halo in their union):
    // exchanges run on commStream, joined by events; cluster index lists built after each search
    bool        overlap{true};
    hipStream_t commStream{nullptr};
    hipEvent_t  evProd{nullptr}, evComm{nullptr};
    hipEvent_t  evStats{nullptr}; // the search's statistics have reached statsHost
    // the skin search's exact search of the directly stale clusters, concurrent with the rebuild of the others
    hipStream_t auxStream{nullptr};
    hipEvent_t  evAuxIn{nullptr}, evAuxOut{nullptr};
    uint32_t*   clsList{nullptr}; // [interior | boundary] cluster indices (2 x numClusters)
    uint32_t*   clsCount{nullptr};
    uint32_t*   clsHost{nullptr}; // pinned copy of clsCount
    uint32_t    nInterior{0}, nBoundary{0};

    std::vector<hipEvent_t>  ev;
    std::vector<std::string> stageNames;
    std::vector<hipEvent_t>  kev; // begin/end pairs around the hot kernels alone
    std::vector<std::string> kernelNames;
    std::vector<float>       kernelMs;
    std::vector<float>       stageMs;
    sx_nbstats               lastStats{};
    int                      haloRetries{0};
    uint64_t                 gravHalos{0};    // gravity halos of the last multi-rank step
    uint64_t                 gravFarCells{0}; // remote level-6 cells taken as far-field multipoles
    uint64_t                 gravRemoteCells{0};

    sx::sim::BdtState bdt; // propagator 2 only
    sx::sim::SkinState skin;

    Fields fields() const { return Fields{x, y, z, temp, h, m, vx, vy, vz, xm1, ym1, zm1, dum1, alpha, id, rung}; }
};

namespace sx::sim
{

constexpr double kHaloMargin = 1.05; // request radius = 2 * hmax(chunk) * margin (+ quantisation margin)

double quantMargin(const DevBox& b);
//! one rank: keys, local sort (every conserved field follows), converged tree; [first, last) = [0, n)
int localSync(sx_sim* s, hipStream_t st);
//! several ranks: SFC assignment, particle exchange, halo discovery with the request radius 2 hmax margin
int distributedSync(sx_sim* s, hipStream_t st, double margin);
//! halo values of `fields` {device pointer, element bytes} from their owners (send lists of the last sync)
int haloExchange(sx_sim* s, std::initializer_list<std::pair<void*, int>> fields, hipStream_t st);
//! 1 on every rank when some local's search sphere (2h around its current position) leaves its chunk's halo request
//! box (global decision)
int halosOutgrown(sx_sim* s, hipStream_t st, unsigned& flag);
//! multi-rank self-gravity onto ax, ay, az of the locals; active (nullable, indexed like the fields) restricts the
//! targets
//! drift: a skin-list reuse step (particles may have left the cells and request boxes of the last sync): the near/far
//! split takes request boxes of the current positions and every MAC box holds its cell and its particles
//! In a periodic box the near tree and the far tree are both walked over the one image shell, the near/far split
//! takes the cells' images into account, and the Ewald correction uses the two trees' combined root.
int distributedGravity(sx_sim* s, hipStream_t st, const uint8_t* active, bool drift = false);
//! self-gravity with periodic images: the box is periodic (all axes, checked by sx_sim_create) and G != 0
bool periodicGravity(const sx_sim* s);
//! the Ewald correction onto ax, ay, az of the locals from the global root expansion (center c4, quadrupole m8)
int ewaldStep(sx_sim* s, const double c4[4], const float m8[8], const uint8_t* active, hipStream_t st);
//! max |a|^2 of the locals into the device scalars (accelerationTimestep)
void maxAccSq(sx_sim* s, hipStream_t st);

//! HydroVeBdtProp: one substep of the block time-step hierarchy (sx_bdt.cpp)
int stepBdt(sx_sim* s);
//! ve-bdt buffers (called by sx_sim_create for propagator 2)
int allocBdt(sx_sim* s);

} // namespace sx::sim
