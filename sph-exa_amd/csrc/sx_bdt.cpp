/*! @file sx_bdt.cpp
 * @brief HydroVeBdtProp (main/src/propagator/ve_hydro_bdt.hpp:51-378) on the device-resident simulation: one substep
 *        of the block time-step hierarchy per sx_sim_step, on one GPU or SFC-decomposed over several.
 *
 * The host control flow is the reference's; every particle operation is a call through the same seam the reference's
 * propagator calls (sph_gpu.hpp, ts_groups.cu, positions_gpu.cu, MultipoleHolder), i.e. the C-ABI of this library
 * on the context of the simulation, and the domain operations are sx_sim's (sx_sim.cpp):
 *
 *   sync (:171-218)       substep 0 of a hierarchy: Domain::sync (keys, sort, SFC exchange, halos, tree; the halo
 *                         request radius grows by the haloFactor 1 + numRungs/40, :215) + computeSpatialGroups,
 *                         groupDt = FLT_MAX.  Other substeps: exchange x,y,z,h of the halos, keep order, tree and
 *                         halo lists, searchExtFactor *= 1.012, the active view = the rung-sorted groups of rungs
 *                         [0, butterfly(substep)).
 *   computeForces         XMass (search + h iteration on the active view), [xm] halos, VeDefGradh, EOS on all
 *   (:222-290)            locals, [v, prho, c, kx] halos, IAD + divv/curlv (+ velocity gradient with avClean),
 *                         groupDivvTimestep, [c_ij, divv] halos, AV switches, [alpha (+ dV)] halos, momentum + energy
 *                         (Courant dt per group), self-gravity on the active view (all groups on a new hierarchy),
 *                         groupAccTimestep.
 *   computeRungs          rungTimestep on a new hierarchy (min over ranks), else minimumGroupDt; extractGroupGpu.
 *   (:292-331)
 *   integrate (:333-378)  per rung: drift, or drift back + computePositions + storeRung; h update of the active view.
 *
 * Halo sufficiency (several ranks): after every search each local's search sphere (2h around its current position)
 * must lie inside its chunk's halo request box.  On a new hierarchy a failure redoes the sync with a larger radius;
 * inside a hierarchy the reference keeps its halos whatever happens (the halo factor is its only margin) and so does
 * this, with a warning and a count (sx_sim_layout out[3] counts both).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>

#include "sx_sim.hpp"
#include "sx_timestep.hpp"

extern "C" void* sx_ctx_stream_internal(sx_ctx* c);

namespace sx::sim
{
namespace
{

#define BDT_CK(expr)                                                                                                   \
    do                                                                                                                 \
    {                                                                                                                  \
        int rc_ = (expr);                                                                                              \
        if (rc_ != SX_OK) return rc_;                                                                                  \
    } while (0)
#define BDT_HIP(expr)                                                                                                  \
    do                                                                                                                 \
    {                                                                                                                  \
        if ((expr) != hipSuccess) return SX_ERR_HIP;                                                                   \
    } while (0)

//! cstone::butterfly (primitives/math.hpp:27-31)
int butterfly(uint32_t i) { return i == 0 ? 0 : 1 + __builtin_ctz(i); }

//! HydroVeBdtProp::activeRung (ve_hydro_bdt.hpp:108-112)
int activeRung(int substep, int numRungs)
{
    return (substep == 0 || substep >= (1 << (numRungs - 1))) ? 0 : butterfly((uint32_t)substep);
}

//! makeSlicedView (sph/groups.hpp:51-58)
sx_groups sliced(const sx_groups& v, uint32_t first, uint32_t last)
{
    sx_groups g  = v;
    g.numGroups  = last - first;
    g.groupStart = v.groupStart + first;
    g.groupEnd   = v.groupEnd + first;
    return g;
}

//! sphexa::ParticlesData fields of the simulation, halos included (length n)
sx_fields allFields(const sx_sim* s)
{
    sx_fields f{};
    f.n     = s->n;
    f.x     = s->x;
    f.y     = s->y;
    f.z     = s->z;
    f.x_m1  = s->xm1;
    f.y_m1  = s->ym1;
    f.z_m1  = s->zm1;
    f.vx    = s->vx;
    f.vy    = s->vy;
    f.vz    = s->vz;
    f.prho  = s->prho;
    f.h     = s->h;
    f.m     = s->m;
    f.c     = s->c;
    f.ax    = s->ax;
    f.ay    = s->ay;
    f.az    = s->az;
    f.du    = s->du;
    f.du_m1 = s->dum1;
    f.c11   = s->c11;
    f.c12   = s->c12;
    f.c13   = s->c13;
    f.c22   = s->c22;
    f.c23   = s->c23;
    f.c33   = s->c33;
    f.temp  = s->temp;
    f.xm    = s->xm;
    f.kx    = s->kx;
    f.divv  = s->divv;
    f.curlv = s->curlv;
    f.alpha = s->alpha;
    f.gradh = s->gradh;
    f.keys  = s->keys;
    f.nc    = s->nc;
    f.dV11  = s->dV[0];
    f.dV12  = s->dV[1];
    f.dV13  = s->dV[2];
    f.dV22  = s->dV[3];
    f.dV23  = s->dV[4];
    f.dV33  = s->dV[5];
    f.rung  = s->rung;
    return f;
}

//! OctreeNsView of the last full sync with the substep's searchExtFactor
sx_tree treeView(const sx_sim* s)
{
    sx_tree t{};
    t.numLeafNodes    = s->tree.numLeaves;
    t.numNodes        = s->tree.numNodes;
    t.prefixes        = s->tree.prefixes;
    t.childOffsets    = s->tree.childOffsets;
    t.internalToLeaf  = s->tree.internalToLeaf;
    t.levelRange      = s->tree.levelRange;
    t.leaves          = s->tree.leaves;
    t.layout          = s->tree.layout;
    t.centers         = s->tree.centers;
    t.sizes           = s->tree.sizes;
    t.searchExtFactor = s->bdt.searchExt;
    return t;
}

bool distributed(const sx_sim* s) { return s->comm && s->comm->size() > 1; }

//! idealGasCv<float, double>(muiConst, gamma) widened to the double constCv of computePositions (positions.hpp:168)
double constCv(const sx_params& p)
{
    return (double)(float)((double)(8.317e7f / p.muiConst) / (p.gamma - 1.0));
}

//! fullSync (:171-194): Domain::sync, d.treeView with searchExtFactor 1, computeGroups, groupDt_ = FLT_MAX
int fullSync(sx_sim* s, hipStream_t st, double margin)
{
    BdtState& b = s->bdt;
    if (distributed(s)) BDT_CK(distributedSync(s, st, margin));
    else BDT_CK(localSync(s, st));
    b.searchExt = 1.0f;
    b.hierarchies++;
    sx_tree   t = treeView(s);
    sx_groups out{};
    BDT_CK(sx_spatial_groups(s->ctx, (uint32_t)s->first, (uint32_t)s->last, s->x, s->y, s->z, &t, &s->box, 2.0f,
                             b.groupBuf, (uint32_t)(s->cap + 1), &out));
    b.groups = out;
    b.active = out;
    if (out.numGroups) BDT_HIP(hipMemsetD32Async(b.groupDt, 0x7f7fffff, out.numGroups, st)); // FLT_MAX
    return SX_OK;
}

//! partialSync (:196-211): halo coordinates and h, wider tree-cell reach, the active rungs' groups
int partialSync(sx_sim* s, hipStream_t st)
{
    BdtState& b = s->bdt;
    BDT_CK(haloExchange(s, {{s->x, 8}, {s->y, 8}, {s->z, 8}, {s->h, 4}}, st));
    b.searchExt = (float)((double)b.searchExt * 1.012);
    const int hr = butterfly((uint32_t)b.ts.substep);
    b.active     = sliced(b.tsGroups, b.ts.rungRanges[0], b.ts.rungRanges[hr]);
    return SX_OK;
}

//! the active view as a target mask (multi-rank gravity restricts its targets with it)
int viewMask(sx_sim* s, const sx_groups& v, hipStream_t st)
{
    BdtState& b = s->bdt;
    BDT_HIP(hipMemsetAsync(b.activeMask, 0, s->n, st));
    const uint32_t init[2] = {0xffffffffu, 0u};
    BDT_HIP(hipMemcpyAsync(b.maskRange, init, sizeof(init), hipMemcpyHostToDevice, st));
    BDT_HIP(viewRange(GroupArgs{v.firstBody, v.lastBody, v.numGroups, v.groupStart, v.groupEnd}, b.activeMask,
                      b.maskRange, st));
    return SX_OK;
}

//! self-gravity (:272-286): upsweep on the tree of the last full sync, traversal of the gravity group
int gravity(sx_sim* s, hipStream_t st, bool newHierarchy)
{
    BdtState& b = s->bdt;
    // gravGroup: every local target on a new hierarchy (MultipoleHolder::computeSpatialGroups), else activeRungs_
    sx_groups all{};
    all.firstBody    = (uint32_t)s->first;
    all.lastBody     = (uint32_t)s->last;
    const sx_groups& g = newHierarchy ? all : b.active;
    if (distributed(s))
    {
        const uint8_t* mask = nullptr;
        if (!newHierarchy)
        {
            BDT_CK(viewMask(s, g, st));
            mask = b.activeMask;
        }
        BDT_HIP(hipMemsetAsync(&s->sc->egrav, 0, sizeof(double), st));
        BDT_HIP(hipMemsetAsync(&s->sc->gravErr, 0, sizeof(unsigned), st));
        BDT_CK(distributedGravity(s, st, mask));
        unsigned err = 0;
        BDT_HIP(hipMemcpyAsync(&err, &s->sc->gravErr, sizeof(err), hipMemcpyDeviceToHost, st));
        BDT_HIP(hipStreamSynchronize(st));
        if (err) return SX_ERR_TRAVERSAL;
        return SX_OK;
    }
    sx_fields f    = allFields(s);
    sx_tree   t    = treeView(s);
    double*   cent = s->work.get<double>("bdt.gcenters", 4 * (size_t)s->tree.numNodes);
    float*    mp   = s->work.get<float>("bdt.gmultipoles", 8 * (size_t)s->tree.numNodes);
    if (!cent || !mp) return SX_ERR_NOMEM;
    BDT_CK(sx_gravity_upsweep(s->ctx, &f, &t, s->p.theta, cent, mp));
    BDT_CK(sx_gravity_traverse(s->ctx, &g, &f, &t, &s->box, cent, mp, (float)s->p.g, &b.egrav));
    return SX_OK;
}

//! computeForces (:222-290)
int computeForces(sx_sim* s, hipStream_t st, int& ev)
{
    BdtState&   b       = s->bdt;
    const bool  dist    = distributed(s);
    const bool  synced  = activeRung(b.ts.substep, b.ts.numRungs) == 0;
    const auto& p       = s->p;
    sx_ctx*     ctx     = s->ctx;
    double      margin  = kHaloMargin * (1.0 + (double)b.ts.numRungs / 40.0); // setHaloFactor (:215)
    float*      h0      = dist ? s->work.get<float>("bdt.h0", s->cap) : nullptr;
    (void)hipEventRecord(s->ev[ev++], st);
    for (int attempt = 0;; ++attempt)
    {
        if (synced)
        {
            if (attempt > 0)
                BDT_HIP(hipMemcpyAsync(s->h + s->first, h0, (s->last - s->first) * 4, hipMemcpyDeviceToDevice, st));
            BDT_CK(fullSync(s, st, margin));
            if (dist)
                BDT_HIP(hipMemcpyAsync(h0, s->h + s->first, (s->last - s->first) * 4, hipMemcpyDeviceToDevice, st));
            b.margin = margin;
        }
        else if (attempt == 0) BDT_CK(partialSync(s, st));
        if (attempt == 0)
        {
            (void)hipEventRecord(s->ev[ev++], st);
            (void)hipEventRecord(s->ev[ev++], st); // search and XMass share one seam call
        }
        sx_fields f = allFields(s);
        sx_tree   t = treeView(s);
        BDT_CK(sx_xmass(ctx, &b.active, &f, &p, &s->box, &t));
        if (!dist) break;
        unsigned hf = 0;
        BDT_CK(halosOutgrown(s, st, hf));
        if (!hf) break;
        if (!synced)
        {
            // the reference keeps the halos of the hierarchy whatever happens (partialSync, :196-211; the halo
            // factor is its only margin); so does this, but it says so once per hierarchy
            b.haloShort++;
            if (b.warnedAt != b.hierarchies)
                fprintf(stderr, "sx_sim_step (ve-bdt): a search sphere left the halo region of the hierarchy at "
                                "substep %d (halos kept, as the reference does)\n", b.ts.substep);
            b.warnedAt = b.hierarchies;
            break;
        }
        if (attempt >= 3) return SX_ERR_NOT_CONVERGED;
        margin *= 1.5;
        s->haloRetries++;
    }
    sx_fields f = allFields(s);
    (void)hipEventRecord(s->ev[ev++], st);
    BDT_CK(haloExchange(s, {{s->xm, 4}}, st));
    BDT_CK(sx_ve_def_gradh(ctx, &b.active, &f, &p, &s->box));
    (void)hipEventRecord(s->ev[ev++], st);
    BDT_CK(sx_eos(ctx, (uint32_t)s->first, (uint32_t)s->last, p.muiConst, p.gamma, s->temp, s->m, s->kx, s->xm,
                  s->gradh, s->prho, s->c, nullptr, nullptr));
    (void)hipEventRecord(s->ev[ev++], st);
    BDT_CK(haloExchange(s, {{s->vx, 4}, {s->vy, 4}, {s->vz, 4}, {s->prho, 4}, {s->c, 4}, {s->kx, 4}}, st));
    BDT_CK(sx_iad_divv_curlv(ctx, &b.active, &f, &p, &s->box));
    BDT_CK(sx_group_divv_timestep(ctx, (float)p.Krho, &b.active, s->divv, b.groupDt));
    (void)hipEventRecord(s->ev[ev++], st);
    BDT_CK(haloExchange(
        s, {{s->c11, 4}, {s->c12, 4}, {s->c13, 4}, {s->c22, 4}, {s->c23, 4}, {s->c33, 4}, {s->divv, 4}}, st));
    BDT_CK(sx_av_switches(ctx, &b.active, &f, &p, &s->box, b.minDt));
    (void)hipEventRecord(s->ev[ev++], st);
    // with avClean the reference exchanges dV11,dV12,dV22,dV23,dV33 + alpha (:262-266); all six are exchanged here
    if (p.avClean)
    {
        BDT_CK(haloExchange(s,
                            {{s->dV[0], 4}, {s->dV[1], 4}, {s->dV[2], 4}, {s->dV[3], 4}, {s->dV[4], 4}, {s->dV[5], 4},
                             {s->alpha, 4}},
                            st));
        BDT_CK(sx_momentum_energy_avclean(ctx, &b.active, b.groupDt, &f, &p, &s->box, nullptr));
    }
    else
    {
        BDT_CK(haloExchange(s, {{s->alpha, 4}}, st));
        BDT_CK(sx_momentum_energy(ctx, &b.active, b.groupDt, &f, &p, &s->box, nullptr));
    }
    (void)hipEventRecord(s->ev[ev++], st);
    if (p.g != 0.0) BDT_CK(gravity(s, st, synced));
    (void)hipEventRecord(s->ev[ev++], st);
    // groupAccTimestep: groupAccTimestepGpu(d.etaAcc * std::sqrt(d.eps), ...) (ts_rungs.hpp:58-65)
    const float eta = (float)(p.etaAcc * std::sqrt(p.eps));
    BDT_CK(sx_group_acc_timestep(ctx, eta, &b.active, s->ax, s->ay, s->az, b.groupDt));
    return SX_OK;
}

//! computeRungs (:292-331)
int computeRungs(sx_sim* s, hipStream_t st)
{
    BdtState& b    = s->bdt;
    const int high = activeRung(b.ts.substep, b.ts.numRungs);
    if (high == 0)
    {
        b.prev            = b.ts;
        const float maxDt = (float)((double)b.ts.dt_m1[0] * s->p.maxDtIncrease);
        sx_timestep ts{};
        BDT_CK(sx_rung_timestep(s->ctx, b.groupDt, b.groupIdx, b.groups.numGroups, maxDt, s->commHandle, &ts));
        b.ts = ts;
    }
    else
    {
        float    dt = 0;
        uint32_t rr[SX_MAX_RUNGS + 1];
        BDT_CK(sx_minimum_group_dt(s->ctx, &b.ts, b.groupDt, b.groupIdx, b.ts.rungRanges[high], s->commHandle, &dt,
                                   rr));
        b.ts.nextDt = dt;
        for (int r = 0; r < high; ++r)
            b.ts.rungRanges[r] = rr[r];
    }
    if (high == 0 || high > 1)
    {
        if (high > 1) std::swap(b.groups, b.tsGroups);
        // extractGroupGpu(groups_.view(), groupIndices_, 0, rungRanges.back(), tsGroups_) into the spare buffers
        const int      k    = b.groups.groupStart == b.tsStart[0] ? 1 : 0;
        const uint32_t last = b.ts.rungRanges[SX_MAX_RUNGS];
        BDT_CK(sx_extract_groups(s->ctx, &b.groups, b.groupIdx, 0, last, b.tsStart[k], b.tsEnd[k]));
        b.tsGroups = sx_groups{0u, 0u, last, b.tsStart[k], b.tsEnd[k]};
    }
    for (int r = 0; r < b.ts.numRungs; ++r)
        b.rungs[r] = sliced(b.tsGroups, b.ts.rungRanges[r], b.ts.rungRanges[r + 1]);
    (void)st;
    return SX_OK;
}

//! integrate (:333-378)
int integrate(sx_sim* s, hipStream_t st)
{
    BDT_CK(computeRungs(s, st));
    BdtState&      b            = s->bdt;
    sx_timestep&   ts           = b.ts;
    const int      lowestDrift  = butterfly((uint32_t)ts.substep + 1);
    const bool     lastSubstep  = activeRung(ts.substep + 1, ts.numRungs) == 0;
    sx_box         openBox{{0.0, 1.0, 0.0, 1.0, 0.0, 1.0}, {0, 0, 0}}; // cstone::Box<T>(0, 1, open)
    const sx_box&  subBox       = lastSubstep ? s->box : openBox;
    const double   gamma        = s->p.gamma, cv = constCv(s->p);
    const sx_fields f           = allFields(s);
    for (int i = 0; i < ts.numRungs; ++i)
    {
        const bool      useRung = ts.substep == ts.substep % (1 << i); // drift back to the start of the hierarchy
        const bool      advance = i < lowestDrift;
        const float     dt      = ts.nextDt;
        const float*    dt_m1   = useRung ? b.prev.dt_m1 : ts.dt_m1;
        float           m1[SX_MAX_RUNGS];
        std::copy(dt_m1, dt_m1 + SX_MAX_RUNGS, m1);
        const sx_groups& g    = b.rungs[i];
        const bool       live = g.numGroups > 0; // a kernel over zero groups does nothing
        if (advance)
        {
            if (ts.dt_drift[i] > 0 && live)
                BDT_CK(sx_drift_positions(s->ctx, &g, 0.0f, ts.dt_drift[i], m1, s->rung, &f, gamma, cv));
            if (live) BDT_CK(sx_positions_rungs(s->ctx, &g, ts.dt_drift[i] + dt, m1, s->rung, &f, gamma, cv, &subBox));
            ts.dt_m1[i]    = ts.dt_drift[i] + dt;
            ts.dt_drift[i] = 0;
            if (live) BDT_CK(sx_store_rung(s->ctx, &g, (uint8_t)i, s->rung));
        }
        else
        {
            if (live) BDT_CK(sx_drift_positions(s->ctx, &g, ts.dt_drift[i] + dt, ts.dt_drift[i], m1, s->rung, &f, gamma, cv));
            ts.dt_drift[i] += dt;
        }
    }
    BDT_CK(sx_update_h_groups(s->ctx, &b.active, s->p.ng0, s->nc, s->h));
    ts.substep++;
    ts.elapsedDt += ts.nextDt;
    b.ttot += ts.nextDt;
    b.minDt_m1 = b.minDt;
    b.minDt    = ts.nextDt;
    return SX_OK;
}

} // namespace

int allocBdt(sx_sim* s)
{
    BdtState&    b   = s->bdt;
    const size_t cap = std::max<size_t>(1, s->cap);
    b.groupBuf       = s->mem.get<uint32_t>("bdt.groups", cap + 1);
    b.groupDt        = s->mem.get<float>("bdt.groupDt", cap);
    b.groupIdx       = s->mem.get<uint32_t>("bdt.groupIdx", cap);
    for (int k = 0; k < 2; ++k)
    {
        b.tsStart[k] = s->mem.get<uint32_t>(std::string("bdt.tsStart") + char('0' + k), cap);
        b.tsEnd[k]   = s->mem.get<uint32_t>(std::string("bdt.tsEnd") + char('0' + k), cap);
    }
    b.activeMask = s->mem.get<uint8_t>("bdt.mask", cap);
    b.maskRange  = s->mem.get<uint32_t>("bdt.maskRange", 2);
    return s->mem.failed() ? SX_ERR_NOMEM : SX_OK;
}

int stepBdt(sx_sim* s)
{
    hipStream_t st = (hipStream_t)sx_ctx_stream_internal(s->ctx);
    BdtState&   b  = s->bdt;
    if (s->p.avClean && !s->dV[0]) return SX_ERR_ARG;
    if (!b.started)
    {
        // Timestep of a fresh start: one rung, substep 0, dt_m1[0] = the initial minDt (ve_hydro_bdt.hpp:122)
        Scalars sc{};
        BDT_HIP(hipMemcpy(&sc, s->sc, sizeof(Scalars), hipMemcpyDeviceToHost));
        b.ts          = sx_timestep{};
        b.ts.numRungs = 1;
        b.ts.dt_m1[0] = (float)sc.minDt;
        b.prev        = sx_timestep{};
        b.minDt       = sc.minDt;
        b.minDt_m1    = sc.minDt_m1;
        b.ttot        = sc.ttot;
        b.started     = true;
    }
    int ev = 0;
    BDT_CK(computeForces(s, st, ev));
    BDT_CK(integrate(s, st));
    (void)hipEventRecord(s->ev[ev++], st);
    // the time-step scalars of ParticlesData, readable through sx_sim_scalars / sx_sim_conserved
    Scalars* hs = s->scHost;
    BDT_HIP(hipMemcpyAsync(hs, s->sc, sizeof(Scalars), hipMemcpyDeviceToHost, st));
    BDT_HIP(hipStreamSynchronize(st));
    hs->minDt    = b.minDt;
    hs->minDt_m1 = b.minDt_m1;
    hs->ttot     = b.ttot;
    if (s->p.g != 0.0 && !distributed(s)) hs->egrav = b.egrav; // single rank: from the seam's traversal
    BDT_HIP(hipMemcpyAsync(s->sc, hs, sizeof(Scalars), hipMemcpyHostToDevice, st));
    BDT_HIP(hipStreamSynchronize(st));
    for (size_t k = 0; k + 1 < s->ev.size() && (int)k + 1 < ev; ++k)
        (void)hipEventElapsedTime(&s->stageMs[k], s->ev[k], s->ev[k + 1]);
    std::fill(s->kernelMs.begin(), s->kernelMs.end(), 0.f);
    b.substeps++;
    return SX_OK;
}

} // namespace sx::sim

extern "C" int sx_sim_timestep(sx_sim* s, sx_timestep* out)
{
    if (!s || !out || s->p.propagator != 2) return SX_ERR_ARG;
    *out = s->bdt.ts;
    return SX_OK;
}

/*! restart of a ve-bdt run (HydroVeBdtProp::load, ve_hydro_bdt.hpp:155-168): after sx_sim_set_state, the Timestep
 *  the file stored and the conserved field `rung` (ConservedFields, :94) of the set_state particles, in their order.
 *  Only a Timestep at a hierarchy boundary is accepted -- the reference writes restart files only when isSynced()
 *  (sphexa.cpp:165, :220) -- so the next substep is a full sync that starts a new hierarchy from this Timestep, as the
 *  uninterrupted run's next substep does. */
extern "C" int sx_sim_set_timestep(sx_sim* s, const sx_timestep* ts, const uint8_t* rung)
{
    if (!s || !ts || s->p.propagator != 2) return SX_ERR_ARG;
    if (ts->numRungs < 1 || ts->numRungs > SX_MAX_RUNGS) return SX_ERR_ARG;
    if (sx::sim::activeRung(ts->substep, ts->numRungs) != 0) return SX_ERR_ARG;
    const size_t n = s->last - s->first;
    if (rung && n)
    {
        for (size_t i = 0; i < n; ++i)
            if (rung[i] >= SX_MAX_RUNGS) return SX_ERR_ARG;
        if (hipMemcpy(s->rung + s->first, rung, n, hipMemcpyHostToDevice) != hipSuccess) return SX_ERR_HIP;
    }
    sx::sim::Scalars sc{};
    if (hipMemcpy(&sc, s->sc, sizeof(sc), hipMemcpyDeviceToHost) != hipSuccess) return SX_ERR_HIP;
    sx::sim::BdtState& b = s->bdt;
    b.ts                 = *ts;
    b.prev               = sx_timestep{};
    b.minDt              = sc.minDt;
    b.minDt_m1           = sc.minDt_m1;
    b.ttot               = sc.ttot;
    b.started            = true;
    return SX_OK;
}
