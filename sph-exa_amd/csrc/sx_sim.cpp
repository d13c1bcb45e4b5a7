/*! @file sx_sim.cpp
 * @brief Device-resident VE time step (sx_sim_*): HydroVeProp::computeForces + integrate
 *        (main/src/propagator/ve_hydro.hpp:132-218) for one GPU, all state kept in HBM.
 *
 * Step = sync (Hilbert keys, radix sort, reorder of every conserved field, converged tree) -> neighbor search with
 * h-nc iteration -> XMass -> VeDefGradh -> EOS -> IAD+divv/curlv -> max divv -> AV switches -> momentum/energy ->
 * time-step (device scalar, no host round trip) -> positions/energy -> h update.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <type_traits>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/sphexa_hip.h"
#include "sx_hydro.hpp"
#include "sx_tree.hpp"

using namespace sx;

namespace
{

DevBox toDevBox(const sx_box* b)
{
    DevBox d{};
    for (int k = 0; k < 6; ++k)
        d.lim[k] = b->lim[k];
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

//! device scalars of one rank: ParticlesData time-step members
struct Scalars
{
    double   minDt, minDt_m1, ttot, minDtCourant, minDtRho;
    float    courant;  // atomic-min target of the momentum kernel
    unsigned maxDivvU; // order-preserving image of max divv
};

//! computeTimestep (ts_global.hpp:97-112, single rank) and rhoTimestep (:72-94) on the device
__global__ void timestepKernel(Scalars* s, double Krho, double maxDtIncrease)
{
    unsigned u = s->maxDivvU;
    u          = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
    float maxDivv   = __uint_as_float(u);
    s->minDtRho     = Krho / (double)fabsf(maxDivv);
    s->minDtCourant = (double)s->courant;
    double m        = INFINITY;
    double cand[3]  = {s->minDtCourant, s->minDtRho, maxDtIncrease * s->minDt};
    for (int k = 0; k < 3; ++k)
        m = cand[k] < m ? cand[k] : m;
    s->ttot += m;
    s->minDt_m1 = s->minDt;
    s->minDt    = m;
}

__global__ void resetScalarsKernel(Scalars* s)
{
    s->courant  = 1e10f;
    s->maxDivvU = 0;
}

//! Sedov lattice (grid.hpp:102-132, sedov_init.hpp:48-96), particle index = z-major lattice index
__global__ void sedovInitKernel(uint32_t side, size_t n, double* x, double* y, double* z, float* h, float* m,
                                double* temp, float* vx, float* vy, float* vz, float* xm1, float* ym1, float* zm1,
                                float* dum1, float* alpha, uint64_t* id, float hInit, float mPart, double ener0,
                                double width2, double u0, float cv)
{
    size_t li = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (li >= n) return;
    const double r = 0.5, step = (2. * r) / side, r_ini = -r + 0.5 * step;
    size_t       i = li / ((size_t)side * side), j = (li / side) % side, k = li % side;
    double       lz = r_ini + (i * step), ly = r_ini + (j * step), lx = r_ini + (k * step);
    x[li] = lx;
    y[li] = ly;
    z[li] = lz;
    h[li] = hInit;
    m[li] = mPart;
    double r2 = lx * lx + ly * ly + lz * lz;
    double ui = ener0 * exp(-(r2 / width2)) + u0;
    temp[li]  = ui / (double)cv;
    vx[li] = vy[li] = vz[li] = 0.f;
    xm1[li] = ym1[li] = zm1[li] = 0.f;
    dum1[li]  = 0.f;
    alpha[li] = 0.05f;
    id[li]    = li;
}

} // namespace

struct sx_sim
{
    sx_ctx*   ctx;
    sx_params p;
    sx_box    box;
    DevBox    dbox;
    uint32_t  bucket;
    size_t    cap{0}, n{0};
    Arena     mem; // persistent particle fields (double-buffered conserved set)
    Arena     work;
    DevTree   tree;

    // conserved (A/B for the reorder)
    double *  x, *y, *z, *temp;
    float *   h, *m, *vx, *vy, *vz, *xm1, *ym1, *zm1, *dum1, *alpha;
    uint64_t* id;
    // dependent
    uint64_t* keys;
    uint32_t *order, *nc;
    float *   xm, *kx, *gradh, *prho, *c, *divv, *curlv, *c11, *c12, *c13, *c22, *c23, *c33, *ax, *ay, *az;
    double*   du;
    RecX*     rx;
    RecV*     rv;
    RecT*     rt;
    RecC*     rc;
    uint32_t* nidx;
    uint32_t* stats;
    uint32_t* statsHost;
    Scalars*  sc;
    Scalars*  scHost;

    struct Spare
    {
        void** field;
        void*  alt;
        int    elemBytes;
    };
    std::vector<Spare> spares; // double buffers of the conserved fields for the SFC reorder

    std::vector<hipEvent_t>  ev;
    std::vector<std::string> stageNames;
    std::vector<float>       stageMs;
    sx_nbstats               lastStats{};
};

// internal: accessors implemented in sx_capi.cpp
extern "C" void* sx_ctx_stream_internal(sx_ctx* c);
extern "C" int   sx_ctx_exact_internal(sx_ctx* c);
extern "C" const float2* sx_ctx_table_internal(sx_ctx* c, int which);
extern "C" const float*  sx_ctx_powtab_internal(sx_ctx* c, uint32_t ng0);

namespace
{

void allocFields(sx_sim* s, size_t cap)
{
    auto& a = s->mem;
    s->x    = a.get<double>("x", cap);
    s->y    = a.get<double>("y", cap);
    s->z    = a.get<double>("z", cap);
    s->temp = a.get<double>("temp", cap);
    s->h    = a.get<float>("h", cap);
    s->m    = a.get<float>("m", cap);
    s->vx   = a.get<float>("vx", cap);
    s->vy   = a.get<float>("vy", cap);
    s->vz   = a.get<float>("vz", cap);
    s->xm1  = a.get<float>("x_m1", cap);
    s->ym1  = a.get<float>("y_m1", cap);
    s->zm1  = a.get<float>("z_m1", cap);
    s->dum1 = a.get<float>("du_m1", cap);
    s->alpha = a.get<float>("alpha", cap);
    s->id    = a.get<uint64_t>("id", cap);
    s->keys  = a.get<uint64_t>("keys", cap);
    s->order = a.get<uint32_t>("order", cap);
    s->nc    = a.get<uint32_t>("nc", cap);
    s->xm    = a.get<float>("xm", cap);
    s->kx    = a.get<float>("kx", cap);
    s->gradh = a.get<float>("gradh", cap);
    s->prho  = a.get<float>("prho", cap);
    s->c     = a.get<float>("c", cap);
    s->divv  = a.get<float>("divv", cap);
    s->curlv = a.get<float>("curlv", cap);
    s->c11   = a.get<float>("c11", cap);
    s->c12   = a.get<float>("c12", cap);
    s->c13   = a.get<float>("c13", cap);
    s->c22   = a.get<float>("c22", cap);
    s->c23   = a.get<float>("c23", cap);
    s->c33   = a.get<float>("c33", cap);
    s->ax    = a.get<float>("ax", cap);
    s->ay    = a.get<float>("ay", cap);
    s->az    = a.get<float>("az", cap);
    s->du    = a.get<double>("du", cap);
    s->rx    = a.get<RecX>("rx", cap);
    s->rv    = a.get<RecV>("rv", cap);
    s->rt    = a.get<RecT>("rt", cap);
    s->rc    = a.get<RecC>("rc", cap);
    auto spare = [&](auto*& field, const char* tag) {
        using T = std::remove_reference_t<decltype(*field)>;
        s->spares.push_back({reinterpret_cast<void**>(&field), a.get<T>(std::string(tag) + ".alt", cap), (int)sizeof(T)});
    };
    spare(s->x, "x");
    spare(s->y, "y");
    spare(s->z, "z");
    spare(s->h, "h");
    spare(s->m, "m");
    spare(s->temp, "temp");
    spare(s->vx, "vx");
    spare(s->vy, "vy");
    spare(s->vz, "vz");
    spare(s->xm1, "x_m1");
    spare(s->ym1, "y_m1");
    spare(s->zm1, "z_m1");
    spare(s->dum1, "du_m1");
    spare(s->alpha, "alpha");
    spare(s->id, "id");
    size_t groups = (cap + kGroupSize - 1) / kGroupSize;
    s->nidx      = a.get<uint32_t>("nidx", groups * s->p.ngmax * kWave);
    s->stats     = a.get<uint32_t>("stats", 8);
    s->statsHost = a.pinned<uint32_t>("statsHost", 8);
    s->sc        = a.get<Scalars>("scalars", 1);
    s->scHost    = a.pinned<Scalars>("scalarsHost", 1);
}

PairArgs simPairArgs(sx_sim* s)
{
    PairArgs a{};
    a.first          = 0;
    a.last           = (uint32_t)s->n;
    a.numGroups      = (uint32_t)((s->n + kGroupSize - 1) / kGroupSize);
    a.ngmax          = s->p.ngmax;
    a.nidx           = s->nidx;
    a.nc             = s->nc;
    a.rx             = s->rx;
    a.rv             = s->rv;
    a.rt             = s->rt;
    a.rc             = s->rc;
    a.wh             = sx_ctx_table_internal(s->ctx, 0);
    a.whd            = sx_ctx_table_internal(s->ctx, 1);
    a.box            = s->dbox;
    a.K              = s->p.K;
    a.xm             = s->xm;
    a.kx             = s->kx;
    a.gradh          = s->gradh;
    a.c11            = s->c11;
    a.c12            = s->c12;
    a.c13            = s->c13;
    a.c22            = s->c22;
    a.c23            = s->c23;
    a.c33            = s->c33;
    a.divv           = s->divv;
    a.curlv          = s->curlv;
    a.alpha          = s->alpha;
    a.ax             = s->ax;
    a.ay             = s->ay;
    a.az             = s->az;
    a.du             = s->du;
    a.minDt          = &s->sc->courant;
    a.alphamin       = s->p.alphamin;
    a.alphamax       = s->p.alphamax;
    a.decay_constant = s->p.decay_constant;
    a.dtPtr          = &s->sc->minDt;
    a.Atmin          = s->p.Atmin;
    a.Atmax          = s->p.Atmax;
    a.ramp           = s->p.ramp;
    a.Kcour          = (float)s->p.Kcour;
    return a;
}

} // namespace

#define SIM_HIP(call)                                                                                                  \
    do {                                                                                                               \
        if ((call) != hipSuccess) return SX_ERR_HIP;                                                                   \
    } while (0)

extern "C"
{

    int sx_sim_create(sx_sim** out, sx_ctx* ctx, size_t capacity, const sx_params* p, const sx_box* box,
                      uint32_t bucketSize)
    {
        auto* s   = new sx_sim;
        s->ctx    = ctx;
        s->p      = *p;
        s->box    = *box;
        s->dbox   = toDevBox(box);
        s->bucket = bucketSize;
        s->cap    = capacity;
        allocFields(s, capacity);
        if (s->mem.failed())
        {
            delete s;
            return SX_ERR_NOMEM;
        }
        const char* names[] = {"sync", "FindNeighbors", "XMass", "VeDefGradh", "EOS", "IadDivvCurlv",
                               "AVswitches", "MomentumEnergy", "UpdateQuantities"};
        s->stageNames.assign(std::begin(names), std::end(names));
        s->ev.resize(s->stageNames.size() + 1);
        for (auto& e : s->ev)
            hipEventCreate(&e);
        s->stageMs.assign(s->stageNames.size(), 0.f);
        Scalars init{1e-6, 1e-6, 0.0, INFINITY, INFINITY, 1e10f, 0};
        hipMemcpy(s->sc, &init, sizeof(Scalars), hipMemcpyHostToDevice);
        *out = s;
        return SX_OK;
    }

    void sx_sim_destroy(sx_sim* s)
    {
        if (!s) return;
        (void)hipDeviceSynchronize();
        for (auto& e : s->ev)
            (void)hipEventDestroy(e);
        delete s;
    }

    size_t sx_sim_size(sx_sim* s) { return s->n; }

    int sx_sim_init_sedov(sx_sim* s, uint32_t side)
    {
        size_t n = (size_t)side * side * side;
        if (n > s->cap) return SX_ERR_ARG;
        s->n           = n;
        double r       = 0.5;
        double hInit   = std::cbrt(3.0 / (4 * M_PI) * s->p.ng0 * std::pow(2 * r, 3) / n) * 0.5;
        double width   = 0.1;
        double ener0   = 1.0 / std::pow(M_PI, 1.5) / 1. / std::pow(width, 3.0);
        float  cv      = idealGasCv(s->p.muiConst, s->p.gamma);
        auto   st      = (hipStream_t)sx_ctx_stream_internal(s->ctx);
        sedovInitKernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(
            side, n, s->x, s->y, s->z, s->h, s->m, s->temp, s->vx, s->vy, s->vz, s->xm1, s->ym1, s->zm1, s->dum1,
            s->alpha, s->id, (float)hInit, (float)(1.0 / n), ener0, width * width, 1e-8, cv);
        Scalars init{1e-6, 1e-6, 0.0, INFINITY, INFINITY, 1e10f, 0};
        SIM_HIP(hipMemcpyAsync(s->sc, &init, sizeof(Scalars), hipMemcpyHostToDevice, st));
        SIM_HIP(hipStreamSynchronize(st));
        return SX_OK;
    }

    int sx_sim_set_state(sx_sim* s, size_t n, const double* x, const double* y, const double* z, const float* h,
                         const float* m, const double* temp, const float* vx, const float* vy, const float* vz,
                         const float* x_m1, const float* y_m1, const float* z_m1, const float* du_m1,
                         const float* alpha, const uint64_t* id, double minDt, double minDt_m1)
    {
        if (n > s->cap) return SX_ERR_ARG;
        s->n    = n;
        auto cp = [n](void* d, const void* h, size_t es) { return hipMemcpy(d, h, n * es, hipMemcpyHostToDevice); };
        SIM_HIP(cp(s->x, x, 8));
        SIM_HIP(cp(s->y, y, 8));
        SIM_HIP(cp(s->z, z, 8));
        SIM_HIP(cp(s->h, h, 4));
        SIM_HIP(cp(s->m, m, 4));
        SIM_HIP(cp(s->temp, temp, 8));
        SIM_HIP(cp(s->vx, vx, 4));
        SIM_HIP(cp(s->vy, vy, 4));
        SIM_HIP(cp(s->vz, vz, 4));
        SIM_HIP(cp(s->xm1, x_m1, 4));
        SIM_HIP(cp(s->ym1, y_m1, 4));
        SIM_HIP(cp(s->zm1, z_m1, 4));
        SIM_HIP(cp(s->dum1, du_m1, 4));
        SIM_HIP(cp(s->alpha, alpha, 4));
        SIM_HIP(cp(s->id, id, 8));
        Scalars init{minDt, minDt_m1, 0.0, INFINITY, INFINITY, 1e10f, 0};
        SIM_HIP(hipMemcpy(s->sc, &init, sizeof(Scalars), hipMemcpyHostToDevice));
        return SX_OK;
    }

    int sx_sim_fields(sx_sim* s, sx_fields* f, uint64_t** id)
    {
        std::memset(f, 0, sizeof(*f));
        f->n     = s->n;
        f->x     = s->x;
        f->y     = s->y;
        f->z     = s->z;
        f->x_m1  = s->xm1;
        f->y_m1  = s->ym1;
        f->z_m1  = s->zm1;
        f->vx    = s->vx;
        f->vy    = s->vy;
        f->vz    = s->vz;
        f->prho  = s->prho;
        f->h     = s->h;
        f->m     = s->m;
        f->c     = s->c;
        f->ax    = s->ax;
        f->ay    = s->ay;
        f->az    = s->az;
        f->du    = s->du;
        f->du_m1 = s->dum1;
        f->c11   = s->c11;
        f->c12   = s->c12;
        f->c13   = s->c13;
        f->c22   = s->c22;
        f->c23   = s->c23;
        f->c33   = s->c33;
        f->temp  = s->temp;
        f->xm    = s->xm;
        f->kx    = s->kx;
        f->divv  = s->divv;
        f->curlv = s->curlv;
        f->alpha = s->alpha;
        f->gradh = s->gradh;
        f->keys  = s->keys;
        f->nc    = s->nc;
        if (id) *id = s->id;
        return SX_OK;
    }

    int sx_sim_step(sx_sim* s)
    {
        hipStream_t       st = (hipStream_t)sx_ctx_stream_internal(s->ctx);
        const HydroLaunch& H = sx_ctx_exact_internal(s->ctx) ? hydro_exact() : hydro_fast();
        const size_t      n  = s->n;
        int               ev = 0;
        SIM_HIP(hipEventRecord(s->ev[ev++], st));

        // ---- sync: keys, sort, reorder, tree -------------------------------------------------------------
        SIM_HIP(launchSfcKeys(s->x, s->y, s->z, s->keys, n, s->dbox, st));
        SIM_HIP(sortKeys(s->work, s->keys, s->order, n, st));
        for (auto& sp : s->spares)
        {
            SIM_HIP(gather(s->order, n, *sp.field, sp.alt, sp.elemBytes, st));
            std::swap(*sp.field, sp.alt);
        }
        SIM_HIP(buildTree(s->work, s->keys, n, s->bucket, s->dbox, s->tree, st));
        SIM_HIP(hipEventRecord(s->ev[ev++], st));

        // ---- neighbors + h iteration ---------------------------------------------------------------------
        NsArgs na{};
        na.first          = 0;
        na.last           = (uint32_t)n;
        na.numGroups      = (uint32_t)((n + kGroupSize - 1) / kGroupSize);
        na.ngmax          = s->p.ngmax;
        na.ng0            = s->p.ng0;
        na.iterateH       = 1;
        na.x              = s->x;
        na.y              = s->y;
        na.z              = s->z;
        na.h              = s->h;
        na.nc             = s->nc;
        na.nidx           = s->nidx;
        na.childOffsets   = s->tree.childOffsets;
        na.internalToLeaf = s->tree.internalToLeaf;
        na.layout         = s->tree.layout;
        na.centers        = s->tree.centers;
        na.sizes          = s->tree.sizes;
        na.box            = s->dbox;
        na.margin         = 4.0 * std::max(s->dbox.l[0], std::max(s->dbox.l[1], s->dbox.l[2])) / double(1u << kMaxLevel);
        na.stats          = s->stats;
        na.powTab         = sx_ctx_powtab_internal(s->ctx, s->p.ng0);
        SIM_HIP(hipMemsetAsync(s->stats, 0, 32, st));
        resetScalarsKernel<<<1, 1, 0, st>>>(s->sc);
        SIM_HIP(findNeighbors(na, st));
        SIM_HIP(hipMemcpyAsync(s->statsHost, s->stats, 32, hipMemcpyDeviceToHost, st));
        SIM_HIP(hipEventRecord(s->ev[ev++], st));

        PairArgs pa = simPairArgs(s);
        // ---- XMass
        packX(n, s->x, s->y, s->z, s->h, s->m, s->rx, st);
        H.xmass(pa, st);
        SIM_HIP(hipEventRecord(s->ev[ev++], st));
        // ---- VeDefGradh
        packT(n, s->xm, nullptr, nullptr, nullptr, s->rt, st);
        H.veDefGradh(pa, st);
        SIM_HIP(hipEventRecord(s->ev[ev++], st));
        // ---- EOS
        EosArgs ea{0, (uint32_t)n, s->p.muiConst, s->p.gamma, s->temp, s->m, s->kx, s->xm, s->gradh, s->prho, s->c,
                   nullptr, nullptr};
        H.eos(ea, st);
        SIM_HIP(hipEventRecord(s->ev[ev++], st));
        // ---- IAD + divv/curlv, rho time-step
        packV(n, s->vx, s->vy, s->vz, s->c, s->rv, st);
        packT(n, s->xm, s->kx, s->prho, s->alpha, s->rt, st);
        H.iadDivvCurlv(pa, st);
        SIM_HIP(maxFloat(s->divv, 0, (uint32_t)n, &s->sc->maxDivvU, st));
        SIM_HIP(hipEventRecord(s->ev[ev++], st));
        // ---- AV switches
        packC(n, s->c11, s->c12, s->c13, s->c22, s->c23, s->c33, s->divv, s->rc, st);
        H.avSwitches(pa, st);
        SIM_HIP(hipEventRecord(s->ev[ev++], st));
        // ---- momentum + energy
        packT(n, s->xm, s->kx, s->prho, s->alpha, s->rt, st);
        H.momentumEnergy(pa, st);
        SIM_HIP(hipEventRecord(s->ev[ev++], st));
        // ---- integrate
        timestepKernel<<<1, 1, 0, st>>>(s->sc, s->p.Krho, s->p.maxDtIncrease);
        PosArgs qa{};
        qa.first   = 0;
        qa.last    = (uint32_t)n;
        qa.dtPtr   = &s->sc->minDt;
        qa.box     = s->dbox;
        qa.x       = s->x;
        qa.y       = s->y;
        qa.z       = s->z;
        qa.x_m1    = s->xm1;
        qa.y_m1    = s->ym1;
        qa.z_m1    = s->zm1;
        qa.vx      = s->vx;
        qa.vy      = s->vy;
        qa.vz      = s->vz;
        qa.ax      = s->ax;
        qa.ay      = s->ay;
        qa.az      = s->az;
        qa.temp    = s->temp;
        qa.du      = s->du;
        qa.du_m1   = s->dum1;
        qa.h       = s->h;
        qa.constCv = idealGasCv(s->p.muiConst, s->p.gamma);
        H.positions(qa, st);
        H.updateH(0, (uint32_t)n, s->p.ng0, s->nc, s->h, na.powTab, st);
        SIM_HIP(hipEventRecord(s->ev[ev++], st));
        SIM_HIP(hipGetLastError());
        SIM_HIP(hipStreamSynchronize(st));

        for (size_t k = 0; k < s->stageMs.size(); ++k)
            hipEventElapsedTime(&s->stageMs[k], s->ev[k], s->ev[k + 1]);
        s->lastStats.numFailed     = s->statsHost[1];
        s->lastStats.maxNeighbors  = s->statsHost[2];
        s->lastStats.sumNeighbors  = *reinterpret_cast<uint64_t*>(s->statsHost + 4);
        s->lastStats.sumCandidates = *reinterpret_cast<uint64_t*>(s->statsHost + 6);
        if (s->statsHost[0] & 1u) return SX_ERR_TRAVERSAL;
        return SX_OK;
    }

    int sx_sim_scalars(sx_sim* s, double out[5])
    {
        hipStream_t st = (hipStream_t)sx_ctx_stream_internal(s->ctx);
        SIM_HIP(hipMemcpyAsync(s->scHost, s->sc, sizeof(Scalars), hipMemcpyDeviceToHost, st));
        SIM_HIP(hipStreamSynchronize(st));
        out[0] = s->scHost->minDt;
        out[1] = s->scHost->minDt_m1;
        out[2] = s->scHost->ttot;
        out[3] = s->scHost->minDtCourant;
        out[4] = s->scHost->minDtRho;
        return SX_OK;
    }

    int sx_sim_stage_times(sx_sim* s, float* ms, int cap, const char** names)
    {
        int k = 0;
        for (; k < cap && k < (int)s->stageMs.size(); ++k)
        {
            ms[k] = s->stageMs[k];
            if (names) names[k] = s->stageNames[k].c_str();
        }
        return k;
    }

    int sx_sim_last_stats(sx_sim* s, sx_nbstats* st)
    {
        *st = s->lastStats;
        return SX_OK;
    }

} // extern "C"
