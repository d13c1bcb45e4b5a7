/*! @file sx_capi.cpp
 * @brief C-ABI (include/sphexa_hip.h): context, per-call entry points mirroring sph::cuda::compute* and the
 *        cstone GPU tree functions, and the device-resident VE step driver (sx_sim_*).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/sphexa_hip.h"
#include "sx_comm.hpp"
#include "sx_gravity.hpp"
#include "sx_hydro.hpp"
#include "sx_kernel_poly.hpp"
#include "sx_observables.hpp"
#include "sx_tree.hpp"
#include "sx_timestep.hpp"

using namespace sx;

// ---------------------------------------------------------------------------------------------------------------
// kernel tables: sinc^6 kernel, K by Simpson (sph/sph_kernel_tables.hpp:27-101, kernels.hpp:35-57)
// ---------------------------------------------------------------------------------------------------------------
namespace
{

double wharmonic(double v)
{
    if (v == 0.0) return 1.0;
    const double Pv = M_PI_2 * v;
    return std::sin(Pv) / Pv;
}

double wharmonicDerivative(double v)
{
    if (v == 0.0) return 0.0;
    const double Pv    = M_PI_2 * v;
    const double sincv = std::sin(Pv) / Pv;
    return sincv * M_PI_2 * ((std::cos(Pv) / std::sin(Pv)) - 1.0 / Pv);
}

double sinc6(double x) { return std::pow(wharmonic(x), 6.0); }
double sinc6d(double x) { return 6.0 * std::pow(wharmonic(x), 6.0 - 1) * wharmonicDerivative(x); }
double kvol(double x) { return 4.0 * M_PI * x * x * sinc6(x); }

double simpsonK()
{
    const uint64_t n = 2000;
    double a = 0, b = 2.0, h = (b - a) / double(n);
    std::vector<double> odd(n / 2), even(n / 2 - 1);
    for (uint64_t i = 0; i < odd.size(); ++i)
        odd[i] = kvol(a + double(2 * (i + 1) - 1) * h);
    for (uint64_t i = 0; i < even.size(); ++i)
        even[i] = kvol(a + double(2 * (i + 1)) * h);
    std::sort(odd.begin(), odd.end());
    std::sort(even.begin(), even.end());
    double so = 0, se = 0;
    for (double v : odd)
        so += v;
    for (double v : even)
        se += v;
    return 1.0 / (h / 3.0 * (kvol(a) + kvol(b) + 4.0 * so + 2.0 * se));
}

void makeTables(std::vector<float>& wh, std::vector<float>& whd)
{
    wh.resize(kTableSize);
    whd.resize(kTableSize);
    const float dx = (float)((2.0 - 0.0) / (kTableSize - 1));
    for (size_t i = 0; i < (size_t)kTableSize; ++i)
    {
        float nv = (float)(0.0 + (float)i * dx);
        wh[i]    = (float)sinc6((double)nv);
        whd[i]   = (float)sinc6d((double)nv);
    }
}

DevBox toDev(const sx_box* b)
{
    DevBox d{};
    for (int k = 0; k < 6; ++k)
        d.lim[k] = b->lim[k];
    d.anyPbc = 0;
    for (int k = 0; k < 3; ++k)
    {
        d.l[k]   = b->lim[2 * k + 1] - b->lim[2 * k];
        d.il[k]  = 1.0 / (b->lim[2 * k + 1] - b->lim[2 * k]);
        d.pbc[k] = b->bnd[k] == 1;
        d.fbc[k] = b->bnd[k] == 2;
        d.anyPbc |= d.pbc[k];
    }
    return d;
}

double quantMargin(const DevBox& b)
{
    double l = std::max(b.l[0], std::max(b.l[1], b.l[2]));
    return 4.0 * l / double(1u << kMaxLevel);
}

} // namespace

// ---------------------------------------------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------------------------------------------
struct sx_ctx
{
    int         device{0};
    NsPolicy    nsPolicy;       // neighbor search: compact or large build (sx_tree.hpp)
    const uint8_t* viewActive{nullptr}; // active-target mask of the current call's group view (nullptr: all)
    hipStream_t own{nullptr};
    hipStream_t stream{nullptr};
    bool        exact{false};
    Arena       arena;
    float2*     wh{nullptr};
    float2*     whd{nullptr};
    double      K{0};
    std::string err;

    // neighbor-list cache (cluster lists from a search, global lists from an import)
    NbLists   nb;
    uint32_t  nbFirst{0}, nbLast{0}, nbNgmax{0};
    bool      nbValid{false};
    size_t    nbFields{0};

    uint32_t* stats{nullptr}; // device, kStatsWords words
    uint32_t* statsHost{nullptr};
    float*    minDt{nullptr}; // device scalar
    unsigned* maxU{nullptr};  // device scalar
    float*    hostScalar{nullptr};

    float*   powTab{nullptr}; // updateH factor by nc, glibc powf (sx_device.hpp)
    uint32_t powTabNg0{0};

    const HydroLaunch& hydro() const { return exact ? hydro_exact() : hydro_fast(); }
};

//! updateH's pow factor for every nc < kPowTable, computed with the host libm powf the reference calls
static const float* ensurePowTab(sx_ctx* c, uint32_t ng0)
{
    if (c->powTab && c->powTabNg0 == ng0) return c->powTab;
    std::vector<float> t(kPowTable);
    const float        c0 = 1023.0f;
    const float        ex = (float)(1.0 / 10.0);
    t[0]                  = INFINITY;
    for (uint32_t nc = 1; nc < kPowTable; ++nc)
    {
        volatile float base = 1.0f + c0 * ng0 / (float)nc; // volatile: keep the call out of constant folding
        t[nc]               = powf(base, ex);
    }
    c->powTab = c->arena.get<float>("powTab", kPowTable);
    if (hipMemcpy(c->powTab, t.data(), kPowTable * 4, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    c->powTabNg0 = ng0;
    return c->powTab;
}

static int fail(sx_ctx* c, int code, const std::string& msg)
{
    if (c) c->err = msg;
    return code;
}

#define SX_HIP(ctx, call)                                                                                              \
    do {                                                                                                               \
        hipError_t e_ = (call);                                                                                        \
        if (e_ != hipSuccess) return fail(ctx, SX_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_));         \
    } while (0)


extern "C"
{
    void*         sx_ctx_stream_internal(sx_ctx* c) { return c->stream; }
    int           sx_ctx_exact_internal(sx_ctx* c) { return c->exact ? 1 : 0; }
    const float2* sx_ctx_table_internal(sx_ctx* c, int which) { return which ? c->whd : c->wh; }
    const float*  sx_ctx_powtab_internal(sx_ctx* c, uint32_t ng0) { return ensurePowTab(c, ng0); }

    int sx_kernel_poly(const float* v, size_t n, float* w, float* dw)
    {
        for (size_t k = 0; k < n; ++k)
            kernelWdW(v[k], w[k], dw[k]);
        return SX_OK;
    }

    double sx_kernel_constant(void)
    {
        static double K = simpsonK();
        return K;
    }

    int sx_create(sx_ctx** out, int device)
    {
        auto* c   = new sx_ctx;
        c->device = device;
        if (hipSetDevice(device) != hipSuccess) return fail(c, SX_ERR_HIP, "hipSetDevice"), *out = c, SX_ERR_HIP;
        SX_HIP(c, hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking));
        c->stream = c->own;
        c->K      = sx_kernel_constant();
        std::vector<float> wh, whd;
        makeTables(wh, whd);
        float* tmp = c->arena.get<float>("tables.raw", 2 * kTableSize);
        SX_HIP(c, hipMemcpy(tmp, wh.data(), kTableSize * 4, hipMemcpyHostToDevice));
        SX_HIP(c, hipMemcpy(tmp + kTableSize, whd.data(), kTableSize * 4, hipMemcpyHostToDevice));
        c->wh  = c->arena.get<float2>("tables.wh", kTableSize);
        c->whd = c->arena.get<float2>("tables.whd", kTableSize);
        tablePairs(tmp, c->wh, c->stream);
        tablePairs(tmp + kTableSize, c->whd, c->stream);
        c->stats      = c->arena.get<uint32_t>("stats", kStatsWords);
        c->statsHost  = c->arena.pinned<uint32_t>("statsHost", kStatsWords);
        if (c->statsHost) std::fill(c->statsHost, c->statsHost + kStatsWords, 0u);
        c->minDt      = c->arena.get<float>("minDt", 1);
        c->maxU       = c->arena.get<unsigned>("maxU", 1);
        c->hostScalar = c->arena.pinned<float>("hostScalar", 2);
        SX_HIP(c, hipStreamSynchronize(c->stream));
        *out = c;
        return SX_OK;
    }

    void sx_destroy(sx_ctx* c)
    {
        if (!c) return;
        (void)hipDeviceSynchronize();
        c->arena.release();
        if (c->own) (void)hipStreamDestroy(c->own);
        delete c;
    }

    int sx_set_stream(sx_ctx* c, void* s)
    {
        c->stream = s ? (hipStream_t)s : c->own;
        return SX_OK;
    }
    void*       sx_get_stream(sx_ctx* c) { return c->stream; }
    const char* sx_last_error(sx_ctx* c) { return c ? c->err.c_str() : "no context"; }
    int         sx_set_exact(sx_ctx* c, int e)
    {
        c->exact = e != 0;
        return SX_OK;
    }
    int sx_synchronize(sx_ctx* c)
    {
        SX_HIP(c, hipStreamSynchronize(c->stream));
        return SX_OK;
    }

    void* sx_device_alloc(sx_ctx* c, size_t bytes)
    {
        void* p = nullptr;
        if (hipMalloc(&p, std::max<size_t>(bytes, 16)) != hipSuccess)
        {
            fail(c, SX_ERR_NOMEM, "hipMalloc failed");
            return nullptr;
        }
        return p;
    }
    int sx_device_free(sx_ctx* c, void* p)
    {
        SX_HIP(c, hipFree(p));
        return SX_OK;
    }
    int sx_memcpy(sx_ctx* c, void* dst, const void* src, size_t bytes, int kind)
    {
        hipMemcpyKind k = kind == 1 ? hipMemcpyHostToDevice : kind == 2 ? hipMemcpyDeviceToHost
                                                                          : hipMemcpyDeviceToDevice;
        SX_HIP(c, hipMemcpyAsync(dst, src, bytes, k, c->stream));
        SX_HIP(c, hipStreamSynchronize(c->stream));
        return SX_OK;
    }
    int sx_memset(sx_ctx* c, void* dst, int value, size_t bytes)
    {
        SX_HIP(c, hipMemsetAsync(dst, value, bytes, c->stream));
        return SX_OK;
    }

    int sx_copy_tables(sx_ctx* c, float* wh, float* whd)
    {
        std::vector<float> a, b;
        makeTables(a, b);
        std::copy(a.begin(), a.end(), wh);
        std::copy(b.begin(), b.end(), whd);
        return SX_OK;
    }

    // ---- cstone ------------------------------------------------------------------------------------------------

    int sx_sfc_keys(sx_ctx* c, const double* x, const double* y, const double* z, uint64_t* keys, size_t n,
                    const sx_box* box)
    {
        SX_HIP(c, launchSfcKeys(x, y, z, keys, n, toDev(box), c->stream));
        return SX_OK;
    }

    int sx_sort_keys(sx_ctx* c, uint64_t* keys, uint32_t* order, size_t n)
    {
        SX_HIP(c, sortKeys(c->arena, keys, order, n, c->stream));
        return SX_OK;
    }

    int sx_gather(sx_ctx* c, const uint32_t* order, size_t n, const void* src, void* dst, int elemBytes)
    {
        SX_HIP(c, gather(order, n, src, dst, elemBytes, c->stream));
        return SX_OK;
    }

    int sx_compute_octree(sx_ctx* c, const uint64_t* keys, size_t n, uint32_t bucket, uint64_t* leaves,
                          uint32_t* counts, int32_t capacity, int32_t* numLeaves)
    {
        sx_box  ub{{0, 1, 0, 1, 0, 1}, {0, 0, 0}};
        DevTree t;
        SX_HIP(c, buildTree(c->arena, keys, n, bucket, toDev(&ub), t, c->stream));
        *numLeaves = t.numLeaves;
        if (capacity < t.numLeaves) return fail(c, SX_ERR_ARG, "sx_compute_octree: capacity too small");
        SX_HIP(c, hipMemcpyAsync(leaves, t.leaves, (t.numLeaves + 1) * 8, hipMemcpyDeviceToDevice, c->stream));
        SX_HIP(c, hipMemcpyAsync(counts, t.counts, t.numLeaves * 4, hipMemcpyDeviceToDevice, c->stream));
        SX_HIP(c, hipStreamSynchronize(c->stream));
        return SX_OK;
    }

    int sx_build_octree(sx_ctx* c, const uint64_t* leaves, int32_t numLeaves, const sx_octree* out)
    {
        // the cornerstone leaf starts, used as keys with bucket 1, reproduce exactly this tree: a leaf holds one
        // start key (its own), every internal node holds at least two
        DevTree t;
        sx_box  ub{{0, 1, 0, 1, 0, 1}, {0, 0, 0}};
        SX_HIP(c, buildTree(c->arena, leaves, (size_t)numLeaves, 1, toDev(&ub), t, c->stream));
        if (t.numLeaves != numLeaves) return fail(c, SX_ERR_ARG, "sx_build_octree: leaves are not a cornerstone tree");
        int nn = t.numNodes;
        SX_HIP(c, hipMemcpyAsync(out->prefixes, t.prefixes, nn * 8, hipMemcpyDeviceToDevice, c->stream));
        SX_HIP(c, hipMemcpyAsync(out->childOffsets, t.childOffsets, (nn + 1) * 4, hipMemcpyDeviceToDevice, c->stream));
        SX_HIP(c, hipMemcpyAsync(out->parents, t.parents, t.parentsSize() * 4, hipMemcpyDeviceToDevice, c->stream));
        SX_HIP(c, hipMemcpyAsync(out->levelRange, t.levelRange, (kMaxLevel + 2) * 4, hipMemcpyDeviceToDevice,
                                 c->stream));
        SX_HIP(c, hipMemcpyAsync(out->internalToLeaf, t.internalToLeaf, nn * 4, hipMemcpyDeviceToDevice, c->stream));
        SX_HIP(c, hipMemcpyAsync(out->leafToInternal, t.leafToInternal, nn * 4, hipMemcpyDeviceToDevice, c->stream));
        return SX_OK;
    }

    int sx_node_centers(sx_ctx* c, const uint64_t* prefixes, int32_t numNodes, const sx_box* box, double* centers,
                        double* sizes)
    {
        SX_HIP(c, nodeCenters(prefixes, numNodes, toDev(box), centers, sizes, c->stream));
        return SX_OK;
    }

    int sx_leaf_layout(sx_ctx* c, const uint32_t* counts, int32_t numLeaves, uint32_t* layout)
    {
        SX_HIP(c, leafLayout(c->arena, counts, numLeaves, layout, c->stream));
        return SX_OK;
    }

    // ---- sph ---------------------------------------------------------------------------------------------------

    int sx_compute_groups(sx_ctx* c, uint32_t first, uint32_t last, sx_groups* g)
    {
        g->firstBody  = first;
        g->lastBody   = last;
        g->numGroups  = (last - first + kGroupSize - 1) / kGroupSize;
        g->groupStart = nullptr;
        g->groupEnd   = nullptr;
        (void)c;
        return SX_OK;
    }

    int sx_spatial_groups(sx_ctx* c, uint32_t first, uint32_t last, const double* x, const double* y,
                          const double* z, const sx_tree* tree, const sx_box* box, float tolFactor, uint32_t* groups,
                          uint32_t cap, sx_groups* out)
    {
        if (!tree || !box || !groups || !out || last < first || (last > first && (!x || !y || !z)))
            return fail(c, SX_ERR_ARG, "sx_spatial_groups: bad arguments");
        uint32_t ng = 0;
        hipError_t e = spatialGroups(c->arena, first, last, x, y, z, tree->leaves, tree->numLeafNodes, tree->layout,
                                     toDev(box), tolFactor, groups, cap, &ng, c->stream);
        if (e == hipErrorInvalidValue) return fail(c, SX_ERR_ARG, "sx_spatial_groups: group capacity too small");
        SX_HIP(c, e);
        out->firstBody  = first;
        out->lastBody   = last;
        out->numGroups  = ng;
        out->groupStart = groups;
        out->groupEnd   = groups + 1;
        return SX_OK;
    }

    int sx_set_search_mode(sx_ctx* c, int mode)
    {
        if (mode < 0 || mode > 3) return fail(c, SX_ERR_ARG, "sx_set_search_mode: mode must be 0..3");
        c->nsPolicy.mode      = mode;
        c->nsPolicy.largeRuns = 0;
        return SX_OK;
    }

    static int findNeighborsView(sx_ctx* c, const sx_fields* f, const sx_tree* tree, const sx_box* box,
                                 const sx_params* p, uint32_t first, uint32_t last, int iterate_h, sx_nbstats* stats);

    int sx_find_neighbors(sx_ctx* c, const sx_fields* f, const sx_tree* tree, const sx_box* box, const sx_params* p,
                          uint32_t first, uint32_t last, int iterate_h, sx_nbstats* stats)
    {
        c->viewActive = nullptr;
        return findNeighborsView(c, f, tree, box, p, first, last, iterate_h, stats);
    }

    static int findNeighborsView(sx_ctx* c, const sx_fields* f, const sx_tree* tree, const sx_box* box,
                                 const sx_params* p, uint32_t first, uint32_t last, int iterate_h, sx_nbstats* stats)
    {
        if (!f || !tree || !box || !p || last < first || last > f->n)
            return fail(c, SX_ERR_ARG, "sx_find_neighbors: bad arguments");
        NsArgs a{};
        a.first          = first;
        a.last           = last;
        a.numGroups      = (last - first + kGroupSize - 1) / kGroupSize;
        a.ngmax          = p->ngmax;
        a.ng0            = p->ng0;
        a.iterateH       = iterate_h;
        a.x              = f->x;
        a.y              = f->y;
        a.z              = f->z;
        a.h              = f->h;
        a.nc             = f->nc;
        a.childOffsets   = tree->childOffsets;
        a.internalToLeaf = tree->internalToLeaf;
        a.layout         = tree->layout;
        a.centers        = tree->centers;
        a.sizes          = tree->sizes;
        a.box            = toDev(box);
        a.margin         = quantMargin(a.box);
        a.extFactor      = tree->searchExtFactor;
        a.stats          = c->stats;
        a.powTab         = ensurePowTab(c, p->ng0);
        a.prefilter      = 1;
        a.hSave          = c->arena.get<float>("ns.hsave", std::max<uint32_t>(2u * ((last - first) / kCluster + 2u), last - first)); // the two redo lists
        a.policy         = &c->nsPolicy;
        a.clStats        = c->arena.get<uint4>("ns.clstats", (a.numGroups + kClusterWaves - 1) / kClusterWaves);
        a.active         = c->viewActive;
        a.work           = c->arena.get<uint32_t>("ns.work", 16);
        a.hitMasks       = c->arena.get<uint64_t>("ns.masks", searchScratchBytes() / sizeof(uint64_t));
        if (!c->nb.reserve(c->arena, first, last, p->ngmax, true) || !a.powTab || !a.clStats || !a.work || !a.hitMasks)
            return fail(c, SX_ERR_NOMEM, "neighbor list allocation failed");
        a.setLists(c->nb);
        SX_HIP(c, hipMemsetAsync(c->stats, 0, kStatsWords * 4, c->stream));
        SX_HIP(c, findNeighbors(a, c->stream));
        SX_HIP(c, hipMemcpyAsync(c->statsHost, c->stats, kStatsWords * 4, hipMemcpyDeviceToHost, c->stream));
        SX_HIP(c, hipStreamSynchronize(c->stream));
        c->nsPolicy.observe(c->statsHost, last - first);
        c->nbFirst = first;
        c->nbLast  = last;
        c->nbNgmax = p->ngmax;
        c->nbValid = true;
        if (stats)
        {
            stats->numFailed     = c->statsHost[1];
            stats->maxNeighbors  = c->statsHost[2];
            stats->sumNeighbors  = *reinterpret_cast<uint64_t*>(c->statsHost + 4);
            stats->sumCandidates = *reinterpret_cast<uint64_t*>(c->statsHost + 6);
            stats->sumUnion      = *reinterpret_cast<uint64_t*>(c->statsHost + 8);
            stats->build         = c->nsPolicy.lastBuild;
            stats->maxUnion      = c->statsHost[12];
        }
        if (c->statsHost[0] & 1u) return fail(c, SX_ERR_TRAVERSAL, "GPU traversal stack exhausted in neighbor search");
        if (iterate_h && c->statsHost[1]) return fail(c, SX_ERR_NOT_CONVERGED, "coupled nc/h-updated failed to converge");
        return SX_OK;
    }

    int sx_export_neighbors(sx_ctx* c, const uint32_t* nc, uint32_t first, uint32_t last, uint32_t ngmax,
                               uint32_t* out)
    {
        if (!c->nbValid || first != c->nbFirst || last != c->nbLast || ngmax != c->nbNgmax)
            return fail(c, SX_ERR_ARG, "sx_export_neighbors: no matching neighbor list");
        NsArgs a{};
        a.first = first, a.last = last, a.ngmax = ngmax, a.nc = const_cast<uint32_t*>(nc);
        a.setLists(c->nb);
        SX_HIP(c, exportNeighbors(a, out, c->stream));
        return SX_OK;
    }

    int sx_import_neighbors(sx_ctx* c, uint32_t first, uint32_t last, uint32_t ngmax, const uint32_t* in)
    {
        if (!c->nb.reserve(c->arena, first, last, ngmax, false))
            return fail(c, SX_ERR_NOMEM, "neighbor list allocation failed");
        SX_HIP(c, importNeighbors(c->nb.nidx, first, last, ngmax, in, c->stream));
        c->nbFirst = first;
        c->nbLast  = last;
        c->nbNgmax = ngmax;
        c->nbValid = true;
        return SX_OK;
    }
} // extern "C"

// ---- pair-kernel plumbing --------------------------------------------------------------------------------------

namespace
{

struct Records
{
    RecX* rx;
    RecV* rv;
    RecT* rt;
    RecC* rc;
};

Records records(sx_ctx* c, size_t n)
{
    return {c->arena.get<RecX>("rec.x", n), c->arena.get<RecV>("rec.v", n), c->arena.get<RecT>("rec.t", n),
            c->arena.get<RecC>("rec.c", n)};
}

/*! A group view with explicit groups (a GroupView slice, e.g. the active rungs of ve-bdt, whose extracted groups carry
 *  firstBody = lastBody = 0, sph/groups.hpp:33-48) becomes the target range [min start, max end) plus an active-target
 *  mask in c->viewActive: the pair kernels and the search skip every target outside the view's groups, like the
 *  reference kernels that visit only the view's groups.  Without explicit groups: [firstBody, lastBody), all active. */
int resolveView(sx_ctx* c, const sx_groups*& g, sx_groups& tmp, size_t n, bool cachedList = true)
{
    c->viewActive = nullptr;
    if (!g) return fail(c, SX_ERR_ARG, "null group view");
    if (!g->groupStart || g->numGroups == 0) return SX_OK;
    uint8_t*  act = c->arena.get<uint8_t>("view.active", n);
    uint32_t* mm  = c->arena.get<uint32_t>("view.range", 2);
    if (!act || !mm) return fail(c, SX_ERR_NOMEM, "group view scratch");
    const uint32_t init[2] = {0xffffffffu, 0u};
    SX_HIP(c, hipMemsetAsync(act, 0, n, c->stream));
    SX_HIP(c, hipMemcpyAsync(mm, init, sizeof(init), hipMemcpyHostToDevice, c->stream));
    SX_HIP(c, viewRange(GroupArgs{g->firstBody, g->lastBody, g->numGroups, g->groupStart, g->groupEnd}, act, mm,
                        c->stream));
    uint32_t r[2];
    SX_HIP(c, hipMemcpyAsync(r, mm, sizeof(r), hipMemcpyDeviceToHost, c->stream));
    SX_HIP(c, hipStreamSynchronize(c->stream));
    tmp           = *g;
    tmp.firstBody = r[0] < r[1] ? r[0] : 0u;
    tmp.lastBody  = r[0] < r[1] ? r[1] : 0u;
    // a cached neighbor list that covers the view (the step's list over all local targets) is used as it is: its
    // blocks are laid out from its own first target, the mask restricts the targets to the view
    if (cachedList && c->nbValid && c->nbLast <= n && tmp.firstBody < tmp.lastBody && c->nbFirst <= tmp.firstBody &&
        tmp.lastBody <= c->nbLast)
        tmp.firstBody = c->nbFirst, tmp.lastBody = c->nbLast;
    g             = &tmp;
    c->viewActive = act;
    return SX_OK;
}

int checkList(sx_ctx* c, const sx_groups* g, const sx_params* p)
{
    if (g->firstBody >= g->lastBody) return SX_OK; // empty range: zero groups, nothing is launched
    if (!c->nbValid || g->firstBody != c->nbFirst || g->lastBody != c->nbLast || p->ngmax != c->nbNgmax)
        return fail(c, SX_ERR_ARG, "no neighbor list for this range: call sx_xmass or sx_find_neighbors first");
    return SX_OK;
}

PairArgs pairArgs(sx_ctx* c, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box,
                  const Records& r)
{
    PairArgs a{};
    a.first          = g->firstBody;
    a.last           = g->lastBody;
    a.numGroups      = (g->lastBody - g->firstBody + kGroupSize - 1) / kGroupSize;
    a.ngmax          = p->ngmax;
    a.localLists     = c->nb.local;
    a.nidx           = c->nb.nidx;
    a.nloc           = c->nb.nloc;
    a.uni            = c->nb.uni;
    a.ucount         = c->nb.ucount;
    a.ucap           = c->nb.ucap;
    a.nc             = f->nc;
    a.rx             = r.rx;
    a.rv             = r.rv;
    a.rt             = r.rt;
    a.rc             = r.rc;
    a.wh             = c->wh;
    a.whd            = c->whd;
    a.box            = toDev(box);
    a.K              = p->K;
    a.xm             = f->xm;
    a.kx             = f->kx;
    a.gradh          = f->gradh;
    a.c11            = f->c11;
    a.c12            = f->c12;
    a.c13            = f->c13;
    a.c22            = f->c22;
    a.c23            = f->c23;
    a.c33            = f->c33;
    a.divv           = f->divv;
    a.curlv          = f->curlv;
    a.alpha          = f->alpha;
    a.ax             = f->ax;
    a.ay             = f->ay;
    a.az             = f->az;
    a.du             = f->du;
    a.minDt          = c->minDt;
    a.blockDt        = c->arena.get<float>("pair.blockdt", std::max<size_t>(1, (size_t(g->lastBody - g->firstBody) + kCluster - 1) / kCluster));
    a.alphamin       = p->alphamin;
    a.alphamax       = p->alphamax;
    a.decay_constant = p->decay_constant;
    a.Atmin          = p->Atmin;
    a.Atmax          = p->Atmax;
    a.ramp           = p->ramp;
    a.Kcour          = (float)p->Kcour;
    a.dV11           = f->dV11;
    a.dV12           = f->dV12;
    a.dV13           = f->dV13;
    a.dV22           = f->dV22;
    a.dV23           = f->dV23;
    a.dV33           = f->dV33;
    a.avClean        = 0;
    a.active         = c->viewActive;
    return a;
}

int markRamp(sx_ctx* c, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box,
             float* markRampOut)
{
    sx_groups tmpView;
    if (int e = resolveView(c, g, tmpView, f->n)) return e;
    if (!markRampOut || !f->kx || !f->xm || !f->m) return fail(c, SX_ERR_ARG, "sx_mark_ramp: bad arguments");
    if (int e = checkList(c, g, p)) return e;
    if (g->firstBody >= g->lastBody) return SX_OK;
    const size_t n = f->n;
    Records      r = records(c, n);
    if (!r.rx) return fail(c, SX_ERR_NOMEM, "record allocation failed");
    packX(n, f->x, f->y, f->z, f->h, f->m, r.rx, c->stream);
    PairArgs a = pairArgs(c, g, f, p, box, r);
    a.markRamp = markRampOut;
    c->hydro().markRamp(a, c->stream);
    SX_HIP(c, hipGetLastError());
    return SX_OK;
}

int momentumEnergy(sx_ctx* c, const sx_groups* g, float* groupDt, const sx_fields* f, const sx_params* p,
                   const sx_box* box, float* minDtCourant, bool avClean)
{
    const sx_groups* view = g;
    sx_groups        tmp;
    if (int e = resolveView(c, g, tmp, f->n)) return e;
    if (int e = checkList(c, g, p)) return e;
    if (f->tdpdTrho) return fail(c, SX_ERR_ARG, "tdpdTrho != NULL is not supported by the VE momentum kernel");
    if (avClean && !(f->dV11 && f->dV12 && f->dV13 && f->dV22 && f->dV23 && f->dV33))
        return fail(c, SX_ERR_ARG, "avClean momentum needs the velocity gradient dV11..dV33");
    Records r = records(c, f->n);
    packX(f->n, f->x, f->y, f->z, f->h, f->m, r.rx, c->stream);
    packV(f->n, f->vx, f->vy, f->vz, f->c, r.rv, c->stream);
    packT(f->n, f->xm, f->kx, f->prho, f->alpha, r.rt, c->stream);
    packC(f->n, f->c11, f->c12, f->c13, f->c22, f->c23, f->c33, nullptr, r.rc, c->stream);
    float huge = 1e10f; // momentum_energy_gpu.cu:127
    SX_HIP(c, hipMemcpyAsync(c->minDt, &huge, 4, hipMemcpyHostToDevice, c->stream));
    PairArgs a = pairArgs(c, g, f, p, box, r);
    // explicit groups: groupDt[k] of view group k = min over its targets (per-target Courant dt, then one minimum
    // per group); fixed 64-blocks: per block inside the kernel
    const bool viewGroups = groupDt && view->groupStart && view->numGroups;
    a.groupDt             = viewGroups ? nullptr : groupDt;
    a.dtOut               = viewGroups ? c->arena.get<float>("view.dt", f->n) : nullptr;
    a.avClean             = avClean ? 1 : 0;
    c->hydro().momentumEnergy(a, c->stream);
    if (viewGroups)
        SX_HIP(c, groupMin(GroupArgs{view->firstBody, view->lastBody, view->numGroups, view->groupStart,
                                     view->groupEnd},
                           a.dtOut, groupDt, c->stream));
    SX_HIP(c, hipGetLastError());
    SX_HIP(c, hipMemcpyAsync(c->hostScalar, c->minDt, 4, hipMemcpyDeviceToHost, c->stream));
    SX_HIP(c, hipStreamSynchronize(c->stream));
    if (minDtCourant) *minDtCourant = c->hostScalar[0];
    return SX_OK;
}

} // namespace

extern "C"
{

    int sx_mark_ramp(sx_ctx* c, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box,
                     float* markRampOut)
    {
        return markRamp(c, g, f, p, box, markRampOut);
    }

    int sx_xmass(sx_ctx* c, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box,
                 const sx_tree* tree)
    {
        sx_groups tmpView;
        if (int e = resolveView(c, g, tmpView, f->n, false)) return e;
        int rc = findNeighborsView(c, f, tree, box, p, g->firstBody, g->lastBody, 1, nullptr);
        if (rc != SX_OK) return rc;
        Records r = records(c, f->n);
        packX(f->n, f->x, f->y, f->z, f->h, f->m, r.rx, c->stream);
        c->hydro().xmass(pairArgs(c, g, f, p, box, r), c->stream);
        SX_HIP(c, hipGetLastError());
        return SX_OK;
    }

    int sx_xmass_only(sx_ctx* c, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box)
    {
        sx_groups tmpView;
        if (int e = resolveView(c, g, tmpView, f->n)) return e;
        if (int e = checkList(c, g, p)) return e;
        Records r = records(c, f->n);
        packX(f->n, f->x, f->y, f->z, f->h, f->m, r.rx, c->stream);
        c->hydro().xmass(pairArgs(c, g, f, p, box, r), c->stream);
        SX_HIP(c, hipGetLastError());
        return SX_OK;
    }

    int sx_ve_def_gradh(sx_ctx* c, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box)
    {
        sx_groups tmpView;
        if (int e = resolveView(c, g, tmpView, f->n)) return e;
        if (int e = checkList(c, g, p)) return e;
        Records r = records(c, f->n);
        packX(f->n, f->x, f->y, f->z, f->h, f->m, r.rx, c->stream);
        packT(f->n, f->xm, nullptr, nullptr, nullptr, r.rt, c->stream);
        c->hydro().veDefGradh(pairArgs(c, g, f, p, box, r), c->stream);
        SX_HIP(c, hipGetLastError());
        return SX_OK;
    }

    int sx_eos(sx_ctx* c, uint32_t first, uint32_t last, float mui, double gamma, const double* temp, const float* m,
               const float* kx, const float* xm, const float* gradh, float* prho, float* cs, float* rho, float* pr)
    {
        EosArgs a{first, last, mui, gamma, temp, m, kx, xm, gradh, prho, cs, rho, pr};
        c->hydro().eos(a, c->stream);
        SX_HIP(c, hipGetLastError());
        return SX_OK;
    }

    int sx_iad_divv_curlv(sx_ctx* c, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box)
    {
        sx_groups tmpView;
        if (int e = resolveView(c, g, tmpView, f->n)) return e;
        if (int e = checkList(c, g, p)) return e;
        Records r = records(c, f->n);
        packX(f->n, f->x, f->y, f->z, f->h, f->m, r.rx, c->stream);
        packV(f->n, f->vx, f->vy, f->vz, nullptr, r.rv, c->stream);
        packT(f->n, f->xm, f->kx, nullptr, nullptr, r.rt, c->stream);
        c->hydro().iadDivvCurlv(pairArgs(c, g, f, p, box, r), c->stream);
        SX_HIP(c, hipGetLastError());
        return SX_OK;
    }

    int sx_av_switches(sx_ctx* c, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box,
                       double minDt)
    {
        sx_groups tmpView;
        if (int e = resolveView(c, g, tmpView, f->n)) return e;
        if (int e = checkList(c, g, p)) return e;
        Records r = records(c, f->n);
        packX(f->n, f->x, f->y, f->z, f->h, f->m, r.rx, c->stream);
        packV(f->n, f->vx, f->vy, f->vz, f->c, r.rv, c->stream);
        packT(f->n, f->xm, f->kx, nullptr, f->alpha, r.rt, c->stream);
        packC(f->n, f->c11, f->c12, f->c13, f->c22, f->c23, f->c33, f->divv, r.rc, c->stream, f->xm, f->kx);
        PairArgs a = pairArgs(c, g, f, p, box, r);
        a.dt       = minDt;
        c->hydro().avSwitches(a, c->stream);
        SX_HIP(c, hipGetLastError());
        return SX_OK;
    }

    int sx_momentum_energy(sx_ctx* c, const sx_groups* g, float* groupDt, const sx_fields* f, const sx_params* p,
                           const sx_box* box, float* minDtCourant)
    {
        return momentumEnergy(c, g, groupDt, f, p, box, minDtCourant, false);
    }

    int sx_momentum_energy_avclean(sx_ctx* c, const sx_groups* g, float* groupDt, const sx_fields* f,
                                   const sx_params* p, const sx_box* box, float* minDtCourant)
    {
        return momentumEnergy(c, g, groupDt, f, p, box, minDtCourant, true);
    }

    // ---- std propagator (HydroProp, std_hydro.hpp:124-184) --------------------------------------------------

    int sx_density(sx_ctx* c, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box,
                   const sx_tree* tree)
    {
        sx_groups tmpView;
        if (int e = resolveView(c, g, tmpView, f->n, false)) return e;
        if (!f->rho) return fail(c, SX_ERR_ARG, "sx_density needs f->rho");
        int rc = findNeighborsView(c, f, tree, box, p, g->firstBody, g->lastBody, 1, nullptr);
        if (rc != SX_OK) return rc;
        return sx_density_only(c, g, f, p, box);
    }

    int sx_density_only(sx_ctx* c, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box)
    {
        sx_groups tmpView;
        if (int e = resolveView(c, g, tmpView, f->n)) return e;
        if (int e = checkList(c, g, p)) return e;
        if (!f->rho) return fail(c, SX_ERR_ARG, "sx_density needs f->rho");
        Records r = records(c, f->n);
        packX(f->n, f->x, f->y, f->z, f->h, f->m, r.rx, c->stream);
        PairArgs a = pairArgs(c, g, f, p, box, r);
        a.xm       = f->rho; // computeDensity: swap(xm, rho), computeXMass, swap back (xmass_gpu.cu:151-153)
        c->hydro().xmass(a, c->stream);
        c->hydro().xmassToRho(g->firstBody, g->lastBody, f->m, f->rho, c->stream);
        SX_HIP(c, hipGetLastError());
        return SX_OK;
    }

    int sx_eos_std(sx_ctx* c, uint32_t first, uint32_t last, float mui, double gamma, const double* temp,
                   const float* m, float* rho, float* pr, float* cs)
    {
        if (first < last && !(temp && rho && pr && cs)) return fail(c, SX_ERR_ARG, "sx_eos_std: null field");
        EosArgs a{first, last, mui, gamma, temp, m, nullptr, nullptr, nullptr, nullptr, cs, rho, pr};
        c->hydro().eosStd(a, c->stream);
        SX_HIP(c, hipGetLastError());
        return SX_OK;
    }

    int sx_iad(sx_ctx* c, const sx_groups* g, const sx_fields* f, const sx_params* p, const sx_box* box)
    {
        sx_groups tmpView;
        if (int e = resolveView(c, g, tmpView, f->n)) return e;
        if (int e = checkList(c, g, p)) return e;
        if (!f->rho) return fail(c, SX_ERR_ARG, "sx_iad needs f->rho");
        Records r = records(c, f->n);
        RecS*   rs = c->arena.get<RecS>("rec.s", f->n);
        packX(f->n, f->x, f->y, f->z, f->h, f->m, r.rx, c->stream);
        packS(f->n, f->rho, nullptr, rs, c->stream);
        PairArgs a = pairArgs(c, g, f, p, box, r);
        a.rs       = rs;
        c->hydro().iadStd(a, c->stream);
        SX_HIP(c, hipGetLastError());
        return SX_OK;
    }

    int sx_momentum_energy_std(sx_ctx* c, const sx_groups* g, const sx_fields* f, const sx_params* p,
                               const sx_box* box, float* minDtCourant)
    {
        sx_groups tmpView;
        if (int e = resolveView(c, g, tmpView, f->n)) return e;
        if (int e = checkList(c, g, p)) return e;
        if (!(f->rho && f->p)) return fail(c, SX_ERR_ARG, "sx_momentum_energy_std needs f->rho and f->p");
        Records r = records(c, f->n);
        RecS*   rs = c->arena.get<RecS>("rec.s", f->n);
        packX(f->n, f->x, f->y, f->z, f->h, f->m, r.rx, c->stream);
        packV(f->n, f->vx, f->vy, f->vz, f->c, r.rv, c->stream);
        packS(f->n, f->rho, f->p, rs, c->stream);
        packC(f->n, f->c11, f->c12, f->c13, f->c22, f->c23, f->c33, nullptr, r.rc, c->stream);
        float huge = 1e10f; // hydro_std/momentum_energy_gpu.cu:115
        SX_HIP(c, hipMemcpyAsync(c->minDt, &huge, 4, hipMemcpyHostToDevice, c->stream));
        PairArgs a = pairArgs(c, g, f, p, box, r);
        a.rs       = rs;
        c->hydro().momentumStd(a, c->stream);
        SX_HIP(c, hipGetLastError());
        SX_HIP(c, hipMemcpyAsync(c->hostScalar, c->minDt, 4, hipMemcpyDeviceToHost, c->stream));
        SX_HIP(c, hipStreamSynchronize(c->stream));
        if (minDtCourant) *minDtCourant = c->hostScalar[0];
        return SX_OK;
    }

    int sx_positions(sx_ctx* c, uint32_t first, uint32_t last, double dt, double dt_m1, const sx_fields* f,
                     double gamma, float muiConst, const sx_box* box)
    {
        PosArgs a{};
        a.first   = first;
        a.last    = last;
        a.dt      = dt;
        a.dt_m1   = dt_m1;
        a.dtPtr   = nullptr;
        a.box     = toDev(box);
        a.x       = f->x;
        a.y       = f->y;
        a.z       = f->z;
        a.x_m1    = f->x_m1;
        a.y_m1    = f->y_m1;
        a.z_m1    = f->z_m1;
        a.vx      = f->vx;
        a.vy      = f->vy;
        a.vz      = f->vz;
        a.ax      = f->ax;
        a.ay      = f->ay;
        a.az      = f->az;
        a.temp    = f->temp;
        a.du      = f->du;
        a.du_m1   = f->du_m1;
        a.h       = f->h;
        a.constCv = idealGasCv(muiConst, gamma);
        c->hydro().positions(a, c->stream);
        SX_HIP(c, hipGetLastError());
        return SX_OK;
    }

    // ---- block time-steps (ve-bdt seam: ts_groups.cu, positions_gpu.cu) ---------------------------------------

    static GroupArgs toGroups(const sx_groups* g)
    {
        return GroupArgs{g->firstBody, g->lastBody, g->numGroups, g->groupStart, g->groupEnd};
    }

    static RungPosArgs rungArgs(const sx_groups* g, float dt, const float* dt_m1, const uint8_t* rung,
                                const sx_fields* f, double gamma, double constCv)
    {
        RungPosArgs a{};
        a.grp  = toGroups(g);
        a.dt   = dt;
        for (int k = 0; k < kMaxNumRungs; ++k)
            a.dt_m1[k] = dt_m1[k];
        a.rung  = rung;
        a.x = f->x, a.y = f->y, a.z = f->z;
        a.x_m1 = f->x_m1, a.y_m1 = f->y_m1, a.z_m1 = f->z_m1;
        a.vx = f->vx, a.vy = f->vy, a.vz = f->vz;
        a.ax = f->ax, a.ay = f->ay, a.az = f->az;
        a.temp = f->temp, a.u = f->temp ? nullptr : f->u;
        a.du = f->du, a.du_m1 = f->du_m1, a.h = f->h, a.mui = f->mui;
        a.gamma = gamma, a.constCv = constCv;
        return a;
    }

    static bool groupsOk(const sx_groups* g) { return g && (g->numGroups == 0 || !g->groupStart == !g->groupEnd); }

    int sx_positions_rungs(sx_ctx* c, const sx_groups* g, float dt, const float* dt_m1, const uint8_t* rung,
                           const sx_fields* f, double gamma, double constCv, const sx_box* box)
    {
        if (!groupsOk(g) || !dt_m1 || !f || !box || (constCv < 0 && !f->mui))
            return fail(c, SX_ERR_ARG, "sx_positions_rungs: bad arguments");
        RungPosArgs a = rungArgs(g, dt, dt_m1, rung, f, gamma, constCv);
        a.box         = toDev(box);
        SX_HIP(c, rungPositions(a, c->stream));
        return SX_OK;
    }

    int sx_drift_positions(sx_ctx* c, const sx_groups* g, float dt, float dt_back, const float* dt_m1,
                           const uint8_t* rung, const sx_fields* f, double gamma, double constCv)
    {
        if (!groupsOk(g) || !dt_m1 || !f || (constCv < 0 && !f->mui))
            return fail(c, SX_ERR_ARG, "sx_drift_positions: bad arguments");
        RungPosArgs a = rungArgs(g, dt, dt_m1, rung, f, gamma, constCv);
        a.dtBack      = dt_back;
        SX_HIP(c, driftPositions(a, c->stream));
        return SX_OK;
    }

    int sx_group_divv_timestep(sx_ctx* c, float Krho, const sx_groups* g, const float* divv, float* groupDt)
    {
        if (!groupsOk(g) || (g->numGroups && (!divv || !groupDt)))
            return fail(c, SX_ERR_ARG, "sx_group_divv_timestep: bad arguments");
        SX_HIP(c, groupDivvTimestep(Krho, toGroups(g), divv, groupDt, c->stream));
        return SX_OK;
    }

    int sx_group_acc_timestep(sx_ctx* c, float etaAcc, const sx_groups* g, const float* ax, const float* ay,
                              const float* az, float* groupDt)
    {
        if (!groupsOk(g) || (g->numGroups && (!ax || !ay || !az || !groupDt)))
            return fail(c, SX_ERR_ARG, "sx_group_acc_timestep: bad arguments");
        SX_HIP(c, groupAccTimestep(etaAcc, toGroups(g), ax, ay, az, groupDt, c->stream));
        return SX_OK;
    }

    int sx_store_rung(sx_ctx* c, const sx_groups* g, uint8_t rung, uint8_t* rungs)
    {
        if (!groupsOk(g) || (g->numGroups && !rungs)) return fail(c, SX_ERR_ARG, "sx_store_rung: bad arguments");
        SX_HIP(c, storeRung(toGroups(g), rung, rungs, c->stream));
        return SX_OK;
    }

    // ---- rung bookkeeping (ts_rungs.hpp:67-157): device sort and lower bounds, host decisions -------------------

    sx::Transport* sx_comm_transport_internal(sx_comm* c);

    //! computeMinTimestep (ts_rungs.hpp:89-105): sortGroupDt, the index sequence up to numGroupsTot, the minimum and
    //! the fast-fraction time-step {groupDt[0], groupDt[LocalIndex(0.4f * numGroups)]}, min-reduced over the ranks
    static int computeMinTimestep(sx_ctx* c, float* groupDt, uint32_t* groupIndices, uint32_t numGroups,
                                  uint32_t numGroupsTot, sx_comm* comm, float out[2])
    {
        RungScratch sc{};
        sc.keys     = c->arena.get<float>("rung.keys", numGroups);
        sc.vals     = c->arena.get<uint32_t>("rung.vals", numGroups);
        sc.tmpBytes = sortGroupDtTmpBytes(numGroups);
        sc.tmp      = c->arena.get<char>("rung.tmp", std::max<size_t>(1, sc.tmpBytes));
        double* d   = c->arena.get<double>("rung.mins", 2);
        if (!sc.keys || !sc.vals || !sc.tmp || !d) return fail(c, SX_ERR_NOMEM, "rung scratch");
        SX_HIP(c, sortGroupDt(groupDt, groupIndices, numGroups, numGroupsTot, sc, c->stream));
        const float    fastFraction = 0.4f;
        const uint32_t kFast        = (uint32_t)(fastFraction * (float)numGroups);
        if (numGroups) SX_HIP(c, pickDt(groupDt, kFast, d, c->stream));
        else
        {
            // a rank without active groups (possible on a substep of a multi-rank hierarchy) still joins the
            // reduction, with nothing to contribute
            const double inf[2] = {INFINITY, INFINITY};
            SX_HIP(c, hipMemcpyAsync(d, inf, sizeof(inf), hipMemcpyHostToDevice, c->stream));
        }
        if (sx::Transport* t = sx_comm_transport_internal(comm); t && t->size() > 1)
            if (!t->allreduceMinF64(d, 2, c->stream)) return fail(c, SX_ERR_HIP, "rung time-step: allreduce failed");
        double h[2];
        SX_HIP(c, hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, c->stream));
        SX_HIP(c, hipStreamSynchronize(c->stream));
        out[0] = (float)h[0], out[1] = (float)h[1];
        return SX_OK;
    }

    //! findRungRanges (ts_rungs.hpp:116-130) on the sorted groupDt
    static int findRungRanges(sx_ctx* c, float minDt, const float* groupDt, uint32_t numGroups, int numRungs,
                              uint32_t* out)
    {
        uint32_t* d = c->arena.get<uint32_t>("rung.ranges", kMaxNumRungs + 1);
        if (!d) return fail(c, SX_ERR_NOMEM, "rung ranges");
        SX_HIP(c, rungRanges(groupDt, numGroups, minDt, numRungs, d, c->stream));
        SX_HIP(c, hipMemcpyAsync(out, d, 4 * (kMaxNumRungs + 1), hipMemcpyDeviceToHost, c->stream));
        SX_HIP(c, hipStreamSynchronize(c->stream));
        return SX_OK;
    }

    int sx_rung_timestep(sx_ctx* c, float* groupDt, uint32_t* groupIndices, uint32_t numGroups, float maxDt,
                         sx_comm* comm, sx_timestep* out)
    {
        if (!groupDt || !groupIndices || !out || numGroups == 0)
            return fail(c, SX_ERR_ARG, "sx_rung_timestep: bad arguments");
        float mins[2];
        if (int e = computeMinTimestep(c, groupDt, groupIndices, numGroups, numGroups, comm, mins)) return e;
        // the reference's unqualified log2 on a float quotient inside namespace sph is ::log2(double)
        const int numRungs = std::min(int(::log2(mins[1] / mins[0])) + 1, kMaxNumRungs);
        sx_timestep ts{};
        if (int e = findRungRanges(c, mins[0], groupDt, numGroups, numRungs, ts.rungRanges)) return e;
        mins[0]      = std::min(maxDt, mins[0]);
        ts.nextDt    = mins[0];
        ts.totDt     = mins[0] * (float)(1 << numRungs);
        ts.numRungs  = numRungs;
        ts.elapsedDt = 0.0f;
        ts.substep   = 0;
        *out         = ts;
        return SX_OK;
    }

    int sx_minimum_group_dt(sx_ctx* c, const sx_timestep* ts, float* groupDt, uint32_t* groupIndices,
                            uint32_t numGroups, sx_comm* comm, float* dt, uint32_t* ranges)
    {
        if (!ts || !groupDt || !groupIndices || !dt || !ranges || numGroups > ts->rungRanges[kMaxNumRungs])
            return fail(c, SX_ERR_ARG, "sx_minimum_group_dt: bad arguments");
        float mins[2];
        if (int e = computeMinTimestep(c, groupDt, groupIndices, numGroups, ts->rungRanges[kMaxNumRungs], comm, mins))
            return e;
        if (int e = findRungRanges(c, mins[0], groupDt, numGroups, kMaxNumRungs, ranges)) return e;
        const float timeLeft     = ts->totDt - ts->elapsedDt;
        const int   substepsLeft = (1 << ts->numRungs) - ts->substep;
        *dt                      = std::min(mins[0], timeLeft / (float)substepsLeft);
        return SX_OK;
    }

    int sx_extract_groups(sx_ctx* c, const sx_groups* g, const uint32_t* indices, uint32_t first, uint32_t last,
                          uint32_t* outStart, uint32_t* outEnd)
    {
        if (!groupsOk(g) || last < first || (last > first && (!indices || !outStart || !outEnd)))
            return fail(c, SX_ERR_ARG, "sx_extract_groups: bad arguments");
        SX_HIP(c, extractGroups(toGroups(g), indices, first, last, outStart, outEnd, c->stream));
        return SX_OK;
    }

    int sx_update_h(sx_ctx* c, uint32_t first, uint32_t last, uint32_t ng0, const uint32_t* nc, float* h)
    {
        const float* tab = ensurePowTab(c, ng0);
        if (!tab) return fail(c, SX_ERR_NOMEM, "powTab");
        c->hydro().updateH(first, last, ng0, nc, h, tab, c->stream);
        SX_HIP(c, hipGetLastError());
        return SX_OK;
    }

    int sx_update_h_groups(sx_ctx* c, const sx_groups* g, uint32_t ng0, const uint32_t* nc, float* h)
    {
        if (!g || !nc || !h || (g->numGroups && !g->groupStart != !g->groupEnd))
            return fail(c, SX_ERR_ARG, "sx_update_h_groups: bad arguments");
        const float* tab = ensurePowTab(c, ng0);
        if (!tab) return fail(c, SX_ERR_NOMEM, "powTab");
        const uint32_t ng = g->groupStart ? g->numGroups
                                          : (g->lastBody > g->firstBody ? (g->lastBody - g->firstBody + 63) / 64 : 0);
        SX_HIP(c, updateHGroups(GroupArgs{g->firstBody, g->lastBody, ng, g->groupStart, g->groupEnd}, ng0, nc, h, tab,
                                c->stream));
        return SX_OK;
    }

    int sx_max_divv(sx_ctx* c, uint32_t first, uint32_t last, const float* divv, float* out)
    {
        SX_HIP(c, maxFloat(divv, first, last, c->maxU, c->stream));
        unsigned u;
        SX_HIP(c, hipMemcpyAsync(c->hostScalar, c->maxU, 4, hipMemcpyDeviceToHost, c->stream));
        SX_HIP(c, hipStreamSynchronize(c->stream));
        std::memcpy(&u, c->hostScalar, 4);
        u = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
        std::memcpy(out, &u, 4);
        return SX_OK;
    }

} // extern "C"

// ---- self-gravity (MultipoleHolder seam, ryoanji/interface/multipole_holder.cuh:40-66) -------------------------

namespace
{

GravArgs gravArgs(sx_ctx* c, const sx_fields* f, const sx_tree* t)
{
    GravArgs a{};
    a.numLeaves      = t->numLeafNodes;
    a.numNodes       = t->numNodes;
    a.childOffsets   = t->childOffsets;
    a.internalToLeaf = t->internalToLeaf;
    a.layout         = t->layout;
    a.geoCenters     = t->centers;
    a.geoSizes       = t->sizes;
    a.x = f->x, a.y = f->y, a.z = f->z, a.m = f->m, a.h = f->h;
    a.ax = f->ax, a.ay = f->ay, a.az = f->az;
    return a;
}

} // namespace

extern "C"
{
    int sx_conserved_quantities(sx_ctx* c, const sx_fields* f, uint32_t first, uint32_t last, float muiConst,
                                double gamma, double out[9])
    {
        if (last > first && !(f->x && f->y && f->z && f->vx && f->vy && f->vz && f->m && (f->u || f->temp)))
            return fail(c, SX_ERR_ARG, "sx_conserved_quantities: null field");
        ConservedArgs a{first, last, f->x, f->y, f->z, f->vx, f->vy, f->vz, f->m, f->temp, f->u, f->nc,
                        (double)idealGasCv(muiConst, gamma)};
        double* scratch = c->arena.get<double>("obs.scratch", conservedScratch(last > first ? last - first : 0));
        double* dout    = c->arena.get<double>("obs.out", 10);
        double* hout    = c->arena.pinned<double>("obs.host", 10);
        SX_HIP(c, conservedQuantities(a, scratch, dout, c->stream));
        SX_HIP(c, hipMemcpyAsync(hout, dout, 9 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
        SX_HIP(c, hipStreamSynchronize(c->stream));
        for (int k = 0; k < 9; ++k)
            out[k] = hout[k];
        return SX_OK;
    }

    int sx_gravity_upsweep(sx_ctx* c, const sx_fields* f, const sx_tree* tree, float theta, double* centers,
                           float* multipoles)
    {
        if (!f || !tree || !centers || !multipoles || !(theta > 0.0f) || tree->numNodes < 1)
            return fail(c, SX_ERR_ARG, "sx_gravity_upsweep: bad arguments");
        GravArgs a   = gravArgs(c, f, tree);
        a.leafToNode = c->arena.get<int32_t>("grav.leafToNode", (size_t)tree->numLeafNodes);
        a.centers4   = centers;
        a.multipoles = multipoles;
        a.invTheta   = 1.0f / theta;
        a.fast       = c->exact ? 0 : 1; // exact: the reference's sequential leaf sums (bit-identical); fast: per wave
        int32_t lr[kMaxLevel + 2];
        SX_HIP(c, hipMemcpyAsync(lr, tree->levelRange, sizeof(lr), hipMemcpyDeviceToHost, c->stream));
        SX_HIP(c, hipStreamSynchronize(c->stream));
        SX_HIP(c, gravityUpsweep(a, lr, c->stream));
        return SX_OK;
    }

    static int gravityTraverseShells(sx_ctx* c, const sx_groups* g, const sx_fields* f, const sx_tree* tree,
                                     const sx_box* box, const double* centers, const float* multipoles, float G,
                                     int numShells, double* egrav)
    {
        // explicit groups (mHolder_.traverse(gravGroup, ...), ve_hydro_bdt.hpp:279-285): only their targets
        sx_groups tmp;
        if (int rc = resolveView(c, g, tmp, f->n, false)) return rc;
        GravArgs a   = gravArgs(c, f, tree);
        a.numShells  = numShells;
        a.boxL[0] = box->lim[1] - box->lim[0], a.boxL[1] = box->lim[3] - box->lim[2];
        a.boxL[2] = box->lim[5] - box->lim[4];
        a.first      = g->firstBody;
        a.last       = g->lastBody;
        a.active     = c->viewActive;
        a.centers4   = const_cast<double*>(centers);
        a.multipoles = const_cast<float*>(multipoles);
        a.G          = G;
        double* acc  = c->arena.get<double>("grav.egrav", 1);
        uint32_t* er = c->arena.get<uint32_t>("grav.err", 1);
        a.egrav      = acc;
        a.err        = er;
        a.fast       = c->exact ? 0 : 1; // exact: the reference's double M2P/P2P; fast: float expansions
        SX_HIP(c, hipMemsetAsync(acc, 0, sizeof(double), c->stream));
        SX_HIP(c, hipMemsetAsync(er, 0, sizeof(uint32_t), c->stream));
        a.waveE      = c->arena.get<double>("grav.waveE", (a.last - a.first + kWave - 1) / kWave + 1);
        SX_HIP(c, gravityTraverse(a, c->stream));
        double   eh = 0;
        uint32_t eb = 0;
        SX_HIP(c, hipMemcpyAsync(&eh, acc, sizeof(double), hipMemcpyDeviceToHost, c->stream));
        SX_HIP(c, hipMemcpyAsync(&eb, er, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
        SX_HIP(c, hipStreamSynchronize(c->stream));
        if (eb) return fail(c, SX_ERR_TRAVERSAL, "GPU traversal stack exhausted in Barnes-Hut");
        if (egrav) *egrav = eh;
        return SX_OK;
    }

    int sx_gravity_traverse(sx_ctx* c, const sx_groups* g, const sx_fields* f, const sx_tree* tree, const sx_box* box,
                            const double* centers, const float* multipoles, float G, double* egrav)
    {
        if (!g || !f || !tree || !box || !centers || !multipoles || g->lastBody > f->n)
            return fail(c, SX_ERR_ARG, "sx_gravity_traverse: bad arguments");
        // a periodic box needs the walk's image shells (sx_gravity_traverse_pbc) and the Ewald correction
        if (box->bnd[0] == 1 || box->bnd[1] == 1 || box->bnd[2] == 1)
            return fail(c, SX_ERR_ARG, "sx_gravity_traverse: periodic box (use sx_gravity_traverse_pbc)");
        return gravityTraverseShells(c, g, f, tree, box, centers, multipoles, G, 0, egrav);
    }

    int sx_gravity_traverse_pbc(sx_ctx* c, const sx_groups* g, const sx_fields* f, const sx_tree* tree,
                                const sx_box* box, const double* centers, const float* multipoles, float G,
                                int numShells, double* egrav)
    {
        if (!g || !f || !tree || !box || !centers || !multipoles || g->lastBody > f->n || numShells < 0 ||
            numShells > 4)
            return fail(c, SX_ERR_ARG, "sx_gravity_traverse_pbc: bad arguments");
        return gravityTraverseShells(c, g, f, tree, box, centers, multipoles, G, numShells, egrav);
    }

    int sx_gravity_ewald(sx_ctx* c, const sx_groups* g, const sx_fields* f, const sx_box* box, const double* centers,
                         const float* multipoles, float G, const sx_ewald_settings* st, double* egrav)
    {
        if (!g || !f || !box || !centers || !multipoles || !st || g->lastBody > f->n)
            return fail(c, SX_ERR_ARG, "sx_gravity_ewald: bad arguments");
        const double lx = box->lim[1] - box->lim[0], ly = box->lim[3] - box->lim[2], lz = box->lim[5] - box->lim[4];
        if (std::min(lx, std::min(ly, lz)) != std::max(lx, std::max(ly, lz)))
            return fail(c, SX_ERR_ARG, "Ewald gravity requires cubic bounding boxes");
        sx_groups tmp;
        if (int rc = resolveView(c, g, tmp, f->n, false)) return rc;
        // the root's expansion, as the reference reads it (gravity_wrapper.hpp:149-152: two D2H copies)
        double center4[4];
        float  Mroot[8];
        SX_HIP(c, hipMemcpyAsync(center4, centers, sizeof(center4), hipMemcpyDeviceToHost, c->stream));
        SX_HIP(c, hipMemcpyAsync(Mroot, multipoles, sizeof(Mroot), hipMemcpyDeviceToHost, c->stream));
        SX_HIP(c, hipStreamSynchronize(c->stream));
        EwaldArgs a{};
        std::vector<double> hs;
        if (ewaldInit(a.p, hs, center4, Mroot, lx, st->numReplicaShells, st->lCut, st->hCut, st->alphaScale,
                      st->smallRScaleFactor))
            return fail(c, SX_ERR_ARG, "sx_gravity_ewald: ceil(hCut) > 3");
        if (a.p.numEwaldShells == 0) return SX_OK;
        double* hd = c->arena.get<double>("ewald.hsum", std::max<size_t>(hs.size(), 5));
        double* us = c->arena.get<double>("ewald.usum", 1);
        if (!hd || !us) return fail(c, SX_ERR_NOMEM, "sx_gravity_ewald: out of memory");
        if (!hs.empty())
            SX_HIP(c, hipMemcpyAsync(hd, hs.data(), hs.size() * sizeof(double), hipMemcpyHostToDevice, c->stream));
        SX_HIP(c, hipMemsetAsync(us, 0, sizeof(double), c->stream));
        a.first = g->firstBody, a.last = g->lastBody;
        a.x = f->x, a.y = f->y, a.z = f->z, a.m = f->m;
        a.ax = f->ax, a.ay = f->ay, a.az = f->az;
        a.G = G, a.active = c->viewActive, a.hsum = hd, a.usum = us, a.uscale = 1.0;
        SX_HIP(c, ewaldCorrection(a, c->stream));
        double u = 0;
        SX_HIP(c, hipMemcpyAsync(&u, us, sizeof(double), hipMemcpyDeviceToHost, c->stream));
        SX_HIP(c, hipStreamSynchronize(c->stream));
        if (egrav) *egrav += 0.5 * G * u;
        return SX_OK;
    }
} // extern "C"

