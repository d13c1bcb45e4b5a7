/*! @file ref_harness.cpp
 *
 * TEST INFRASTRUCTURE ONLY -- builds oracle/_ref/libsphexa_ref.so, the reference's own CPU path
 * compiled from its header-only sources where they lie under /root/reference (see oracle/Makefile).
 * Nothing here is copied from the reference: this file only *calls* the reference templates through
 * a plain C ABI so that tests/ can pin oracle/sph_oracle.c (the CPU restatement) against the real
 * thing, and bench.py can time the reference CPU path as `cpu_baseline.kind = "reference"`.
 *
 * Reference entry points exercised (paths relative to /root/reference):
 *   - kernel tables / K             sph/include/sph/sph_kernel_tables.hpp:78-172
 *   - Hilbert keys                  domain/include/cstone/sfc/sfc.hpp:284-291
 *   - cornerstone leaves            domain/include/cstone/tree/csarray.hpp:456-467 (computeOctree)
 *   - linked octree                 domain/include/cstone/tree/octree.hpp:185-213 (buildOctreeCpu)
 *   - node centers / sizes          domain/include/cstone/focus/source_center.hpp:146-157
 *   - neighbor search (+h iter)     sph/include/sph/find_neighbors.hpp:10-44, cstone/findneighbors.hpp:95-188
 *   - VE kernels (the *Impl loops)  sph/include/sph/hydro_ve/{xmass,ve_def_gradh,eos,iad_divv_curlv,
 *                                   av_switches,momentum_energy}.hpp
 *   - integrator                    sph/include/sph/positions.hpp:90-139, update_h.hpp:12-22
 *
 * Two documented deviations from "call the reference verbatim":
 *   F2: updateTempHost's `using Tdu = decltype(d.du[0])` is `double&`, which reinterprets the
 *       float du_m1 storage as a double.  The mock dataset below gives `du` a by-value element access, so
 *       `Tdu` becomes `double` and the reference loop runs unmodified but correct (GPU semantics,
 *       positions_gpu.cu:160-163).
 *   MPI: computeTimestep (ts_global.hpp:97-112) and rhoTimestep (:72-94) live in a header that includes <mpi.h>.
 *       The parity build (SX_REF_MPI, oracle/Makefile) compiles that header against the image's MPICH
 *       (/opt/conda/include, single-rank MPI_Init) and ref_step calls both as they are; the timing build
 *       (libsphexa_ref_fast.so, bench.py's cpu_baseline on the GPU box) restates their single-rank arithmetic, so
 *       it loads without an MPI runtime.  ref_rho_timestep / ref_compute_timestep expose them to the tests.
 *   Domain::sync (single rank) is restated as: Hilbert keys -> sort_by_key -> reorder -> fully converged
 *       cornerstone tree (bucket 64) -> buildOctreeCpu -> nodeFpCenters -> layout. The reference's focus tree
 *       converges incrementally over steps; neighbor *sets* do not depend on the tree, only their order.
 */

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <vector>

#include "cstone/findneighbors.hpp"
#include "cstone/focus/source_center.hpp"
#include "cstone/primitives/gather.hpp"
#include "cstone/tree/csarray.hpp"
#include "cstone/tree/octree.hpp"

#include "sph/kernels.hpp" // must precede find_neighbors.hpp (uses updateH unqualified)
#include "sph/find_neighbors.hpp"
#include "sph/hydro_ve/av_switches.hpp"
#include "sph/hydro_ve/eos.hpp"
#include "sph/hydro_ve/iad_divv_curlv.hpp"
#include "sph/hydro_ve/momentum_energy.hpp"
#include "sph/hydro_ve/ve_def_gradh.hpp"
#include "sph/hydro_ve/xmass.hpp"
#include "sph/hydro_std/density.hpp"
#include "sph/hydro_std/eos.hpp"
#include "sph/hydro_std/iad.hpp"
#include "sph/hydro_std/momentum_energy.hpp"
#include "sph/positions.hpp"
#include "sph/sph_kernel_tables.hpp"
#include "sph/update_h.hpp"
#ifdef SX_REF_MPI
#include "cstone/primitives/mpi_wrappers.hpp" // MpiType, used unqualified by ts_global.hpp
#include "sph/ts_global.hpp"
#include "sph/ts_rungs.hpp" // findRungRanges<false> is host code; the rest of the file needs GPU primitives
#endif

#include "ryoanji/nbody/traversal_cpu.hpp"
#include "ryoanji/nbody/upsweep_cpu.hpp"

#include "sx_host_types.h"

using KeyType = uint64_t;
using Tc      = double;
using Th      = float;

namespace
{

//! @brief non-owning vector view with the subset of std::vector used by the reference *Impl loops
template<class T>
struct PtrVec
{
    T*     p{nullptr};
    size_t n{0};
    T*     data() const { return p; }
    size_t size() const { return n; }
    bool   empty() const { return n == 0; }
    T&     operator[](size_t i) const { return p[i]; }
};

//! found by ADL for computeDensityImpl's unqualified swap(d.xm, d.rho) (hydro_std/density.hpp:44-46)
template<class T>
void swap(PtrVec<T>& a, PtrVec<T>& b)
{
    std::swap(a.p, b.p);
    std::swap(a.n, b.n);
}

//! @brief by-value element access: makes updateTempHost's `decltype(d.du[0])` a value type (F2 fix)
template<class T>
struct ValVec
{
    T*     p{nullptr};
    size_t n{0};
    T*     data() const { return p; }
    size_t size() const { return n; }
    bool   empty() const { return n == 0; }
    T      operator[](size_t i) const { return p[i]; }
};

//! @brief mock of sphexa::ParticlesData<CpuTag>: members named as in particles_data.hpp:62-375
template<class T>
struct MockData
{
    using RealType        = double;
    using HydroType       = T;
    using Tm              = T;
    using AcceleratorType = cstone::CpuTag; // computeDensityImpl dispatches computeXMass on it (density.hpp:45)

    unsigned ng0{100}, ngmax{150};
    double   K{0};
    double   minDt{1e-6}, minDt_m1{1e-6}, minDtCourant{INFINITY}, minDtRho{INFINITY};
    double   Kcour{0.2}, Krho{0.06}, gamma{5.0 / 3.0}, sincIndex{6.0};
    double   ttot{0}, g{0}, maxDtIncrease{1.1}, etaAcc{0.2}, eps{0.005}; // computeTimestep (ts_global.hpp:97-112)
    float    muiConst{10.0};
    T        alphamin{0.05}, alphamax{1.0}, decay_constant{0.2};
    T        Atmin{0.1}, Atmax{0.2}, ramp{1.0 / (0.2 - 0.1)};

    PtrVec<double>             x, y, z;
    PtrVec<T>                  x_m1, y_m1, z_m1, vx, vy, vz, h, m, alpha, du_m1;
    PtrVec<double>             temp, u;
    ValVec<double>             du;
    PtrVec<T>                  ax, ay, az, prho, tdpdTrho, c, xm, kx, gradh, divv, curlv, rho, p, mui;
    PtrVec<T>                  c11, c12, c13, c22, c23, c33, dV11, dV12, dV13, dV22, dV23, dV33;
    PtrVec<unsigned>           nc;
    PtrVec<cstone::LocalIndex> neighbors;
    PtrVec<T>                  wh, whd;
};

cstone::Box<double> makeBox(const ox_box* b)
{
    auto bt = [](int v) { return static_cast<cstone::BoundaryType>(v); };
    return cstone::Box<double>(b->lim[0], b->lim[1], b->lim[2], b->lim[3], b->lim[4], b->lim[5], bt(b->bnd[0]),
                               bt(b->bnd[1]), bt(b->bnd[2]));
}

std::vector<float> g_wh, g_whd;

#ifdef SX_REF_MPI
//! single-rank MPI for the reference's global time-step (MPICH singleton init)
void refMpiInit()
{
    int on = 0;
    MPI_Initialized(&on);
    if (!on) MPI_Init(nullptr, nullptr);
}
#endif
double             g_K = 0;

void ensureTables()
{
    if (!g_wh.empty()) return;
    auto k = sph::getSphKernel(sph::SphKernelType::sinc_n, 6.0);
    auto d = sph::getSphKernelDerivative(sph::SphKernelType::sinc_n, 6.0);
    g_K    = sph::kernel_3D_k(k, 2.0);
    auto a = sph::tabulateFunction<float, sph::lt::kTableSize>(k, 0, 2);
    auto b = sph::tabulateFunction<float, sph::lt::kTableSize>(d, 0, 2);
    g_wh.assign(a.begin(), a.end());
    g_whd.assign(b.begin(), b.end());
}

struct TreeArrays
{
    std::vector<KeyType>              leaves, prefixes;
    std::vector<unsigned>             counts;
    std::vector<cstone::TreeNodeIndex> childOffsets, parents, levelRange, internalToLeaf, leafToInternal;
    std::vector<cstone::Vec3<double>> centers, sizes;
    std::vector<cstone::LocalIndex>   layout;

    void build(const KeyType* keys, size_t n, unsigned bucket, const cstone::Box<double>& box)
    {
        auto [tree, cnt] = cstone::computeOctree(keys, keys + n, bucket);
        leaves           = std::move(tree);
        counts           = std::move(cnt);
        cstone::TreeNodeIndex nLeaf = cstone::nNodes(leaves);
        cstone::TreeNodeIndex nInt  = (nLeaf - 1) / 7;
        cstone::TreeNodeIndex nTot  = nLeaf + nInt;
        prefixes.assign(nTot, 0);
        childOffsets.assign(nTot + 1, 0);
        parents.assign(std::max(1, (nTot - 1) / 8), 0);
        levelRange.assign(cstone::maxTreeLevel<KeyType>{} + 2, 0);
        internalToLeaf.assign(nTot, 0);
        leafToInternal.assign(nTot, 0);
        cstone::buildOctreeCpu(leaves.data(), nLeaf, nInt, prefixes.data(), childOffsets.data(), parents.data(),
                               levelRange.data(), internalToLeaf.data(), leafToInternal.data());
        centers.resize(nTot);
        sizes.resize(nTot);
        cstone::nodeFpCenters<KeyType>(gsl::span<const KeyType>(prefixes.data(), nTot), centers.data(), sizes.data(),
                                       box);
        layout.assign(nLeaf + 1, 0);
        std::copy(counts.begin(), counts.end(), layout.begin());
        std::exclusive_scan(layout.begin(), layout.end(), layout.begin(), cstone::LocalIndex(0));
    }

    cstone::OctreeNsView<double, KeyType> view() const
    {
        cstone::OctreeNsView<double, KeyType> v;
        v.numLeafNodes   = cstone::nNodes(leaves);
        v.prefixes       = prefixes.data();
        v.childOffsets   = childOffsets.data();
        v.internalToLeaf = internalToLeaf.data();
        v.levelRange     = levelRange.data();
        v.leaves         = leaves.data();
        v.layout         = layout.data();
        v.centers        = centers.data();
        v.sizes          = sizes.data();
        return v;
    }
};

template<class T>
void bindState(MockData<T>& d, ox_state* s, const ox_params* p)
{
    size_t n = s->n;
    d.x      = {s->x, n};
    d.y      = {s->y, n};
    d.z      = {s->z, n};
    d.x_m1   = {s->x_m1, n};
    d.y_m1   = {s->y_m1, n};
    d.z_m1   = {s->z_m1, n};
    d.vx     = {s->vx, n};
    d.vy     = {s->vy, n};
    d.vz     = {s->vz, n};
    d.h      = {s->h, n};
    d.m      = {s->m, n};
    d.alpha  = {s->alpha, n};
    d.du_m1  = {s->du_m1, n};
    d.temp   = {s->temp, n};
    d.du     = {s->du, n};
    d.ax     = {s->ax, n};
    d.ay     = {s->ay, n};
    d.az     = {s->az, n};
    d.prho   = {s->prho, n};
    d.c      = {s->c, n};
    d.xm     = {s->xm, n};
    d.kx     = {s->kx, n};
    d.gradh  = {s->gradh, n};
    d.divv   = {s->divv, n};
    d.curlv  = {s->curlv, n};
    d.c11    = {s->c11, n};
    d.c12    = {s->c12, n};
    d.c13    = {s->c13, n};
    d.c22    = {s->c22, n};
    d.c23    = {s->c23, n};
    d.c33    = {s->c33, n};
    d.nc     = {s->nc, n};
    if (p && p->prop == 1)
    {
        // rho, p are HydroProp DependentFields (std_hydro.hpp:78-79); HydroVeProp leaves them unallocated, which
        // keeps computeEOS_Impl from writing them (hydro_ve/eos.hpp)
        d.rho = {s->rho, n};
        d.p   = {s->p, n};
    }
    if (p && p->avClean)
    {
        // GradVFields acquired (ve_hydro.hpp:80-85): dV11.size() == x.size() turns on doGradV
        d.dV11 = {s->dV11, n};
        d.dV12 = {s->dV12, n};
        d.dV13 = {s->dV13, n};
        d.dV22 = {s->dV22, n};
        d.dV23 = {s->dV23, n};
        d.dV33 = {s->dV33, n};
    }
    d.minDt    = s->minDt;
    d.minDt_m1 = s->minDt_m1;
    if (p)
    {
        d.ng0            = p->ng0;
        d.ngmax          = p->ngmax;
        d.K              = p->K;
        d.Kcour          = p->Kcour;
        d.Krho           = p->Krho;
        d.gamma          = p->gamma;
        d.muiConst       = p->muiConst;
        d.alphamin       = p->alphamin;
        d.alphamax       = p->alphamax;
        d.decay_constant = p->decay_constant;
    }
}

template<class V>
void permute(V* a, const std::vector<uint64_t>& ord, std::vector<char>& scratch)
{
    size_t n = ord.size();
    scratch.resize(n * sizeof(V));
    V* tmp = reinterpret_cast<V*>(scratch.data());
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n; ++i)
        tmp[i] = a[ord[i]];
    std::memcpy(a, tmp, n * sizeof(V));
}

} // namespace

extern "C"
{

    //! @brief K (Simpson, 2000 intervals) and the 20000-entry f32 tables of sinc^6 (particles_data.hpp:364-371)
    void ref_kernel_tables(float* wh, float* whd, double* K)
    {
        ensureTables();
        std::copy(g_wh.begin(), g_wh.end(), wh);
        std::copy(g_whd.begin(), g_whd.end(), whd);
        *K = g_K;
    }

    void ref_kernel_tables_f64(double* wh, double* whd, double* K)
    {
        auto k = sph::getSphKernel(sph::SphKernelType::sinc_n, 6.0);
        auto d = sph::getSphKernelDerivative(sph::SphKernelType::sinc_n, 6.0);
        auto a = sph::tabulateFunction<double, sph::lt::kTableSize>(k, 0, 2);
        auto b = sph::tabulateFunction<double, sph::lt::kTableSize>(d, 0, 2);
        std::copy(a.begin(), a.end(), wh);
        std::copy(b.begin(), b.end(), whd);
        *K = sph::kernel_3D_k(k, 2.0);
    }

    double ref_sphynx_3d_k(double n) { return sph::sphynx_3D_k(n); }

    float ref_update_h(unsigned ng0, unsigned nc, float h) { return sph::updateH(ng0, nc, h); }

    float ref_lookup(const float* table, float v) { return sph::lt::lookup(table, v); }

    void ref_sfc_keys(const double* x, const double* y, const double* z, size_t n, const ox_box* b, uint64_t* keys)
    {
        cstone::computeSfcKeys(x, y, z, cstone::sfcKindPointer(keys), n, makeBox(b));
    }

    /*! @brief fully converged cornerstone leaf array for sorted keys (csarray.hpp:456-467)
     *  @return number of leaves; leaves/counts written only if cap >= numLeaves (+1 for leaves)
     */
    int ref_compute_octree(const uint64_t* keys, size_t n, unsigned bucket, uint64_t* leaves, unsigned* counts,
                           int cap)
    {
        auto [tree, cnt] = cstone::computeOctree(keys, keys + n, bucket);
        int nLeaf        = cstone::nNodes(tree);
        if (cap >= nLeaf)
        {
            std::copy(tree.begin(), tree.end(), leaves);
            std::copy(cnt.begin(), cnt.end(), counts);
        }
        return nLeaf;
    }

    //! @brief buildOctreeCpu (octree.hpp:185-213); arrays sized numNodes = numLeaves + (numLeaves-1)/7
    void ref_build_octree(const uint64_t* leaves, int numLeaves, uint64_t* prefixes, int* childOffsets, int* parents,
                          int* levelRange, int* internalToLeaf, int* leafToInternal)
    {
        int nInt = (numLeaves - 1) / 7;
        int nTot = numLeaves + nInt;
        std::fill(childOffsets, childOffsets + nTot, 0);
        cstone::buildOctreeCpu(leaves, numLeaves, nInt, prefixes, childOffsets, parents, levelRange, internalToLeaf,
                               leafToInternal);
    }

    void ref_node_centers(const uint64_t* prefixes, int numNodes, const ox_box* b, double* centers, double* sizes)
    {
        cstone::nodeFpCenters<KeyType>(gsl::span<const KeyType>(prefixes, numNodes),
                                       reinterpret_cast<cstone::Vec3<double>*>(centers),
                                       reinterpret_cast<cstone::Vec3<double>*>(sizes), makeBox(b));
    }

    /*! @brief neighbor search over [first,last) with the reference's own tree built from sorted keys.
     *  iterate_h != 0: sph::findNeighborsSph (h-nc iteration, nc includes self)
     *  iterate_h == 0: cstone::findNeighbors batch (count excludes self)
     *  neighbors: (last-first) * ngmax, CPU layout neighbors[(i-first)*ngmax + k]
     */
    void ref_find_neighbors(const double* x, const double* y, const double* z, float* h, const uint64_t* keys,
                            size_t n, unsigned first, unsigned last, const ox_box* b, unsigned bucket, unsigned ng0,
                            unsigned ngmax, int iterate_h, uint32_t* neighbors, uint32_t* nc)
    {
        auto       box = makeBox(b);
        TreeArrays t;
        t.build(keys, n, bucket, box);
        auto view = t.view();
        if (iterate_h)
        {
            sph::findNeighborsSph(x, y, z, h, first, last, box, view, ng0, ngmax, neighbors, nc);
        }
        else
        {
            std::vector<double> hd(h, h + n); // cstone::findNeighbors batch overload takes T=double h
            (void)hd;
            cstone::LocalIndex numWork = last - first;
#pragma omp parallel for
            for (cstone::LocalIndex i = 0; i < numWork; ++i)
            {
                nc[i] = cstone::findNeighbors(i + first, x, y, z, h, view, box, ngmax, neighbors + size_t(i) * ngmax);
            }
        }
    }

    // ---------------------------------------------------------------------------------------------------
    // VE kernels: run the reference compute*Impl loops over [first,last) with explicit neighbor lists
    // ---------------------------------------------------------------------------------------------------

    static MockData<float> kernelData(ox_state* s, const ox_params* p, const uint32_t* neighbors)
    {
        ensureTables();
        MockData<float> d;
        bindState(d, s, p);
        d.neighbors = {const_cast<uint32_t*>(neighbors), size_t(-1)};
        d.wh        = {g_wh.data(), g_wh.size()};
        d.whd       = {g_whd.data(), g_whd.size()};
        return d;
    }

    void ref_xmass(ox_state* s, const ox_params* p, const ox_box* b, const uint32_t* neighbors, unsigned first,
                   unsigned last)
    {
        auto d = kernelData(s, p, neighbors);
        sph::computeXMassImpl(first, last, d, makeBox(b));
    }

    void ref_ve_def_gradh(ox_state* s, const ox_params* p, const ox_box* b, const uint32_t* neighbors,
                          unsigned first, unsigned last)
    {
        auto d = kernelData(s, p, neighbors);
        sph::computeVeDefGradhImpl(first, last, d, makeBox(b));
    }

    void ref_eos(ox_state* s, const ox_params* p, unsigned first, unsigned last)
    {
        auto d = kernelData(s, p, nullptr);
        sph::computeEOS_Impl(first, last, d);
    }

    void ref_iad_divv_curlv(ox_state* s, const ox_params* p, const ox_box* b, const uint32_t* neighbors,
                            unsigned first, unsigned last)
    {
        auto d = kernelData(s, p, neighbors);
        sph::computeIadDivvCurlvImpl(first, last, d, makeBox(b));
    }

    void ref_av_switches(ox_state* s, const ox_params* p, const ox_box* b, const uint32_t* neighbors,
                         unsigned first, unsigned last)
    {
        auto d = kernelData(s, p, neighbors);
        sph::computeAVswitchesImpl(first, last, d, makeBox(b));
    }

    double ref_momentum_energy(ox_state* s, const ox_params* p, const ox_box* b, const uint32_t* neighbors,
                               unsigned first, unsigned last)
    {
        auto d = kernelData(s, p, neighbors);
        if (p->avClean) sph::computeMomentumEnergyImpl<true>(first, last, d, makeBox(b));
        else sph::computeMomentumEnergyImpl<false>(first, last, d, makeBox(b));
        s->minDtCourant = d.minDtCourant;
        return d.minDtCourant;
    }

    // ---- std propagator kernels (HydroProp, std_hydro.hpp:124-166) --------------------------------------

    void ref_density(ox_state* s, const ox_params* p, const ox_box* b, const uint32_t* neighbors, unsigned first,
                     unsigned last)
    {
        auto            d = kernelData(s, p, neighbors);
        sph::GroupView  g{first, last, 0, nullptr, nullptr};
        sph::computeDensityImpl(g, d, makeBox(b));
    }

    void ref_eos_std(ox_state* s, const ox_params* p, unsigned first, unsigned last)
    {
        auto d = kernelData(s, p, nullptr);
        sph::computeEOS_HydroStdImpl(first, last, d);
    }

    void ref_iad_std(ox_state* s, const ox_params* p, const ox_box* b, const uint32_t* neighbors, unsigned first,
                     unsigned last)
    {
        auto d = kernelData(s, p, neighbors);
        sph::computeIADImpl(first, last, d, makeBox(b));
    }

    double ref_momentum_energy_std(ox_state* s, const ox_params* p, const ox_box* b, const uint32_t* neighbors,
                                   unsigned first, unsigned last)
    {
        auto d = kernelData(s, p, neighbors);
        sph::computeMomentumEnergyStdImpl(first, last, d, makeBox(b));
        s->minDtCourant = d.minDtCourant;
        return d.minDtCourant;
    }

    void ref_positions(ox_state* s, const ox_params* p, const ox_box* b, unsigned first, unsigned last)
    {
        auto d = kernelData(s, p, nullptr);
        sph::updatePositionsHost(first, last, d, makeBox(b));
        sph::updateTempHost(first, last, d);
    }

    //! periodic images of the walk (computeGravity's numShells, traversal_cpu.hpp:180); ref_set_gravity_shells
    static int g_numShells = 0;

    /*! @brief self-gravity with the reference's own functions on the tree of the key-sorted state (single rank):
     *  expansion centers as FocusedOctree::updateCenters + setMacRadius(1/theta) (octree_focus_mpi.hpp:325-459),
     *  ryoanji::computeLeafMultipoles + upsweepMultipoles (global_multipole.hpp:44-71 without the MPI exchanges),
     *  ryoanji::computeGravity (traversal_cpu.hpp:166-230, numShells: g_numShells).  cap < 0: return the node count. */
    static double gravityOnTree(ox_state* s, const ox_params* p, const cstone::Box<double>& box, TreeArrays& t,
                                unsigned first, unsigned last, double* centersOut, float* multipolesOut, int cap)
    {
        using namespace cstone;
        TreeNodeIndex nLeaf = nNodes(t.leaves), nTot = TreeNodeIndex(t.prefixes.size()), nInt = nTot - nLeaf;
        std::vector<SourceCenterType<double>> centers(nTot);
        computeLeafMassCenter<double, float, double>(gsl::span<const double>(s->x, s->n),
                                                     gsl::span<const double>(s->y, s->n),
                                                     gsl::span<const double>(s->z, s->n),
                                                     gsl::span<const float>(s->m, s->n),
                                                     {t.leafToInternal.data() + nInt, size_t(nLeaf)}, t.layout.data(),
                                                     centers.data());
        upsweep({t.levelRange.data(), t.levelRange.size()}, {t.childOffsets.data(), t.childOffsets.size()},
                centers.data(), CombineSourceCenter<double>{});
        setMac<double, KeyType>({t.prefixes.data(), t.prefixes.size()}, {centers.data(), centers.size()},
                                1.0f / p->theta, box);
        std::vector<ryoanji::CartesianQuadrupole<float>> mp(nTot);
        ryoanji::computeLeafMultipoles(s->x, s->y, s->z, s->m, {t.leafToInternal.data() + nInt, size_t(nLeaf)},
                                       t.layout.data(), centers.data(), mp.data());
        ryoanji::upsweepMultipoles({t.levelRange.data(), t.levelRange.size()}, t.childOffsets.data(), centers.data(),
                                   mp.data());
        // computeGravity works on leaf-index ranges: targets [layout[l0], layout[l1])
        TreeNodeIndex l0 = TreeNodeIndex(std::upper_bound(t.layout.begin(), t.layout.end(), first) - t.layout.begin()) - 1;
        TreeNodeIndex l1 = TreeNodeIndex(std::lower_bound(t.layout.begin(), t.layout.end(), last) - t.layout.begin());
        double egrav = 0;
        ryoanji::computeGravity(t.childOffsets.data(), t.internalToLeaf.data(), centers.data(), mp.data(),
                                t.layout.data(), l0, l1, s->x, s->y, s->z, s->h, s->m, box, float(p->g),
                                (double*)nullptr, s->ax, s->ay, s->az, &egrav, g_numShells);
        if (centersOut && cap >= nTot) std::memcpy(centersOut, centers.data(), sizeof(double) * 4 * nTot);
        if (multipolesOut && cap >= nTot) std::memcpy(multipolesOut, mp.data(), sizeof(float) * 8 * nTot);
        return egrav;
    }

    void ref_set_gravity_shells(int numShells) { g_numShells = numShells; }

    double ref_gravity(ox_state* s, const ox_params* p, const ox_box* b, unsigned bucket, unsigned first,
                       unsigned last, double* centersOut, float* multipolesOut, int cap)
    {
        auto       box = makeBox(b);
        TreeArrays t;
        t.build(s->keys, s->n, bucket, box);
        if (cap < 0) return double(t.prefixes.size());
        return gravityOnTree(s, p, box, t, first, last, centersOut, multipolesOut, cap);
    }

    void ref_update_h_range(ox_state* s, unsigned ng0, unsigned first, unsigned last)
    {
        sph::updateSmoothingLengthCpu(first, last, ng0, s->nc, s->h);
    }

    /*! @brief one full VE time step on a single rank (ve_hydro.hpp:132-218 + sphexa.cpp loop body)
     *
     * Sync (restated, see file header) reorders every conserved field, id, and keys by the Hilbert key.
     * Returns 0, or the number of particles whose h-nc iteration failed to converge.
     */
    int ref_step(ox_state* s, const ox_params* p, const ox_box* b, unsigned bucket)
    {
        auto   box = makeBox(b);
        size_t n   = s->n;

        // --- domain::sync (single rank): keys, sort, reorder, tree
        cstone::computeSfcKeys(s->x, s->y, s->z, cstone::sfcKindPointer(s->keys), n, box);
        std::vector<uint64_t> ord(n);
        std::iota(ord.begin(), ord.end(), uint64_t(0));
        cstone::sort_by_key(s->keys, s->keys + n, ord.begin());
        std::vector<char> scratch;
        permute(s->x, ord, scratch);
        permute(s->y, ord, scratch);
        permute(s->z, ord, scratch);
        permute(s->h, ord, scratch);
        permute(s->m, ord, scratch);
        permute(s->temp, ord, scratch);
        permute(s->vx, ord, scratch);
        permute(s->vy, ord, scratch);
        permute(s->vz, ord, scratch);
        permute(s->x_m1, ord, scratch);
        permute(s->y_m1, ord, scratch);
        permute(s->z_m1, ord, scratch);
        permute(s->du_m1, ord, scratch);
        permute(s->alpha, ord, scratch);
        permute(s->id, ord, scratch);

        TreeArrays t;
        t.build(s->keys, n, bucket, box);
        auto view = t.view();

        auto d = kernelData(s, p, nullptr);
        std::vector<uint32_t> nbr(n * size_t(d.ngmax));
        d.neighbors = {nbr.data(), nbr.size()};

        // --- computeForces
        // findNeighborsSph addresses a target's list as neighbors + i * ngmax with i a 32-bit LocalIndex
        // (find_neighbors.hpp:26): past 2^32 / ngmax targets (28.6M at ngmax 150) the offset wraps.  A reference run
        // holds that many particles only on several ranks, each calling it over its own range with its own list
        // (findNeighborsSfc, :54-55); the harness does the same per chunk of 2^24 targets on one rank (Sedov -n 400,
        // 64M particles).  Every target's search is independent of the others, so the lists, nc and h are those of
        // one call wherever it does not wrap.
        for (size_t f = 0; f < n; f += size_t(1) << 24)
        {
            const size_t l = std::min(n, f + (size_t(1) << 24));
            sph::findNeighborsSph(s->x, s->y, s->z, s->h, cstone::LocalIndex(f), cstone::LocalIndex(l), box, view,
                                  d.ng0, d.ngmax, nbr.data() + f * size_t(d.ngmax), s->nc + f);
        }
        if (p->prop == 1)
        {
            // HydroProp::computeForces (std_hydro.hpp:124-166): minDtRho is never set there
            sph::GroupView g{0, cstone::LocalIndex(n), 0, nullptr, nullptr};
            sph::computeDensityImpl(g, d, box);
            sph::computeEOS_HydroStdImpl(0, n, d);
            sph::computeIADImpl(0, n, d, box);
            sph::computeMomentumEnergyStdImpl(0, n, d, box);
        }
        else
        {
            sph::computeXMassImpl(0, n, d, box);
            sph::computeVeDefGradhImpl(0, n, d, box);
            sph::computeEOS_Impl(0, n, d);
            sph::computeIadDivvCurlvImpl(0, n, d, box);
#ifdef SX_REF_MPI
            d.minDtRho = sph::rhoTimestep(0, n, d);
#else
            {   // rhoTimestep (ts_global.hpp:72-94), single rank
                float maxDivv = -INFINITY;
#pragma omp parallel for reduction(max : maxDivv)
                for (size_t i = 0; i < n; ++i)
                    maxDivv = std::max(s->divv[i], maxDivv);
                d.minDtRho = d.Krho / std::abs(maxDivv);
            }
#endif
            sph::computeAVswitchesImpl(0, n, d, box);
            if (p->avClean) sph::computeMomentumEnergyImpl<true>(0, n, d, box);
            else sph::computeMomentumEnergyImpl<false>(0, n, d, box);
        }
        double minDtAcc = INFINITY;
        if (p->g != 0.0)
        {
            // mHolder_.upsweep + traverse (ve_hydro.hpp:193-202), accelerationTimestep (ts_global.hpp:47-67)
            s->egrav = gravityOnTree(s, p, box, t, 0, unsigned(n), nullptr, nullptr, 0);
        }
#ifdef SX_REF_MPI
        refMpiInit();
        d.g      = p->g;
        d.etaAcc = p->etaAcc;
        d.eps    = p->eps;
        d.ttot   = s->ttot;
        sph::computeTimestep(0, n, d);
        s->ttot = d.ttot;
#else
        if (p->g != 0.0)
        {
            double maxAccSq = 0.0;
            for (size_t i = 0; i < n; ++i)
            {
                cstone::Vec3<double> X{s->ax[i], s->ay[i], s->az[i]};
                maxAccSq = std::max(norm2(X), maxAccSq);
            }
            minDtAcc = p->etaAcc * std::sqrt(p->eps / std::sqrt(maxAccSq));
        }

        // --- integrate: computeTimestep (ts_global.hpp:97-112 without MPI_Allreduce)
        double minDtLoc = std::min({minDtAcc, d.minDtCourant, d.minDtRho, 1.1 * d.minDt});
        s->ttot += minDtLoc;
        d.minDt_m1 = d.minDt;
        d.minDt    = minDtLoc;
#endif
        sph::updatePositionsHost(0, n, d, box);
        sph::updateTempHost(0, n, d);
        sph::updateSmoothingLengthCpu(0, n, d.ng0, s->nc, s->h);

        s->minDt        = d.minDt;
        s->minDt_m1     = d.minDt_m1;
        s->minDtCourant = d.minDtCourant;
        s->minDtRho     = d.minDtRho;
        return 0;
    }

    /*! @brief std KATs in double precision (sph/test/std.cpp:98-127): particle 0 vs neighbors 1..4 in the open box
     *  [0,6]^3.  cols: 5 x 19 doubles, column order x y z h m rho vx vy vz c p c11 c12 c13 c22 c23 c33 (xm kx unused).
     *  out: c11 c12 c13 c22 c23 c33, grad_Px grad_Py grad_Pz du maxvsignal */
    void ref_kat_std_f64(const double* cols, double* out)
    {
        constexpr int       np = 5, nc = 17;
        std::vector<double> c[nc];
        for (int k = 0; k < nc; ++k)
            for (int i = 0; i < np; ++i)
                c[k].push_back(cols[i * 19 + k]);
        auto wh  = sph::tabulateFunction<double, sph::lt::kTableSize>(sph::getSphKernel(sph::sinc_n, 6.0), 0, 2);
        auto whd = sph::tabulateFunction<double, sph::lt::kTableSize>(sph::getSphKernelDerivative(sph::sinc_n, 6.0),
                                                                      0, 2);
        double                          K = sph::sphynx_3D_k(6.0);
        cstone::Box<double>             box(0, 6, cstone::BoundaryType::open);
        std::vector<cstone::LocalIndex> nb{1, 2, 3, 4};
        sph::IADJLoopSTD(0, K, box, nb.data(), 4u, c[0].data(), c[1].data(), c[2].data(), c[3].data(), c[4].data(),
                         c[5].data(), wh.data(), whd.data(), &out[0], &out[1], &out[2], &out[3], &out[4], &out[5]);
        sph::momentumAndEnergyJLoop(0, K, box, nb.data(), 4u, c[0].data(), c[1].data(), c[2].data(), c[6].data(),
                                    c[7].data(), c[8].data(), c[3].data(), c[4].data(), c[5].data(), c[10].data(),
                                    c[9].data(), c[11].data(), c[12].data(), c[13].data(), c[14].data(), c[15].data(),
                                    c[16].data(), wh.data(), whd.data(), &out[6], &out[7], &out[8], &out[9],
                                    &out[10]);
    }

    //! @brief KAT helpers in double precision (sph/test/ve.cpp:52-233), particle 0 vs neighbors 1..98
    void ref_kat_f64(const double* cols, int npart, double mpart, double* out)
    {
        // cols: npart x 31, column order of ve.cpp:75-76
        std::vector<std::vector<double>> c(31, std::vector<double>(npart));
        for (int i = 0; i < npart; ++i)
            for (int k = 0; k < 31; ++k)
                c[k][i] = cols[i * 31 + k];
        auto& x = c[0];  auto& y = c[1];  auto& z = c[2];  auto& vx = c[3]; auto& vy = c[4]; auto& vz = c[5];
        auto& h = c[6];  auto& cc = c[7]; auto& c11 = c[8]; auto& c12 = c[9]; auto& c13 = c[10];
        auto& c22 = c[11]; auto& c23 = c[12]; auto& c33 = c[13]; auto& p = c[14]; auto& gradh = c[15];
        auto& rho0 = c[16]; auto& alpha = c[28]; auto& divv = c[30];
        std::vector<double> m(npart, mpart), xm(npart), kx(npart), prho(npart);
        double K = sph::sphynx_3D_k(6.0);
        for (int i = 0; i < npart; ++i)
        {
            xm[i]   = mpart / rho0[i];
            kx[i]   = K * xm[i] / std::pow(h[i], 3);
            prho[i] = p[i] / (kx[i] * m[i] * m[i] * gradh[i]);
        }
        std::vector<double> dvxdx = c[19], dvxdy = c[20], dvxdz = c[21], dvydx = c[22], dvydy = c[23],
                            dvydz = c[24], dvzdx = c[25], dvzdy = c[26], dvzdz = c[27];
        std::vector<double> dV11(npart), dV12(npart), dV13(npart), dV22(npart), dV23(npart), dV33(npart);
        for (int i = 0; i < npart; ++i)
        {
            dV11[i] = dvxdx[i];
            dV12[i] = dvxdy[i] + dvydx[i];
            dV13[i] = dvxdz[i] + dvzdx[i];
            dV22[i] = dvydy[i];
            dV23[i] = dvydz[i] + dvzdy[i];
            dV33[i] = dvzdz[i];
        }
        auto wh  = sph::tabulateFunction<double, sph::lt::kTableSize>(sph::getSphKernel(sph::sinc_n, 6.0), 0, 2);
        auto whd = sph::tabulateFunction<double, sph::lt::kTableSize>(sph::getSphKernelDerivative(sph::sinc_n, 6.0),
                                                                      0, 2);
        cstone::Box<double>             box(-1e9, 1e9, cstone::BoundaryType::open);
        std::vector<cstone::LocalIndex> nb(npart - 1);
        std::iota(nb.begin(), nb.end(), 1);
        unsigned nn = npart - 1;

        out[0] = sph::AVswitchesJLoop(0, K, box, nb.data(), nn, x.data(), y.data(), z.data(), vx.data(), vy.data(),
                                      vz.data(), h.data(), cc.data(), c11.data(), c12.data(), c13.data(), c22.data(),
                                      c23.data(), c33.data(), wh.data(), whd.data(), kx.data(), xm.data(),
                                      divv.data(), 0.3, 0.05, 1.0, 0.2, alpha[0]);
        double dv[8];
        sph::divV_curlVJLoop(0, K, box, nb.data(), nn, x.data(), y.data(), z.data(), vx.data(), vy.data(), vz.data(),
                             h.data(), c11.data(), c12.data(), c13.data(), c22.data(), c23.data(), c33.data(),
                             wh.data(), whd.data(), kx.data(), xm.data(), &dv[0], &dv[1], &dv[2], &dv[3], &dv[4],
                             &dv[5], &dv[6], &dv[7], true);
        for (int k = 0; k < 8; ++k)
            out[1 + k] = dv[k];
        double iad[6];
        sph::IADJLoop(0, K, box, nb.data(), nn, x.data(), y.data(), z.data(), h.data(), wh.data(), whd.data(),
                      xm.data(), kx.data(), &iad[0], &iad[1], &iad[2], &iad[3], &iad[4], &iad[5]);
        for (int k = 0; k < 6; ++k)
            out[9 + k] = iad[k];
        double r[5];
        sph::momentumAndEnergyJLoop<false>(0, K, box, nb.data(), nn, x.data(), y.data(), z.data(), vx.data(),
                                           vy.data(), vz.data(), h.data(), m.data(), prho.data(), (const double*)nullptr,
                                           cc.data(), c11.data(), c12.data(), c13.data(), c22.data(), c23.data(),
                                           c33.data(), 0.1, 0.2, 10.0, wh.data(), kx.data(), xm.data(), alpha.data(),
                                           dV11.data(), dV12.data(), dV13.data(), dV22.data(), dV23.data(),
                                           dV33.data(), &r[1], &r[2], &r[3], &r[0], &r[4]);
        for (int k = 0; k < 5; ++k)
            out[15 + k] = r[k]; // du, ax, ay, az, maxvsignal
        auto [kxi, gradhi] = sph::veDefGradhJLoop(0, K, box, nb.data(), nn, x.data(), y.data(), z.data(), h.data(),
                                                  m.data(), wh.data(), whd.data(), xm.data());
        out[20] = kxi;
        out[21] = gradhi;
        out[22] = sph::xmassJLoop(0, K, box, nb.data(), nn, x.data(), y.data(), z.data(), h.data(), m.data(),
                                  wh.data(), whd.data());
    }

#ifdef SX_REF_MPI
    /*! sph::rhoTimestep (ts_global.hpp:72-94) on n divv values: Krho / |max divv| */
    double ref_rho_timestep(const float* divv, size_t n, double Krho)
    {
        MockData<float> d;
        d.divv = PtrVec<float>{const_cast<float*>(divv), n};
        d.Krho = Krho;
        return sph::rhoTimestep(0, n, d);
    }

    /*! sph::computeTimestep (ts_global.hpp:97-112, MPI_Allreduce over one rank) with accelerationTimestep
     *  (:47-67) when g != 0.  io[0..6] = minDt, minDt_m1, ttot, minDtCourant, minDtRho, g, maxDtIncrease (in),
     *  minDt, minDt_m1, ttot updated in place */
    void ref_compute_timestep(double* io, const float* ax, const float* ay, const float* az, size_t n, double etaAcc,
                              double eps)
    {
        refMpiInit();
        MockData<float> d;
        d.ax = PtrVec<float>{const_cast<float*>(ax), n};
        d.ay = PtrVec<float>{const_cast<float*>(ay), n};
        d.az = PtrVec<float>{const_cast<float*>(az), n};
        d.minDt = io[0], d.minDt_m1 = io[1], d.ttot = io[2], d.minDtCourant = io[3], d.minDtRho = io[4];
        d.g = io[5], d.maxDtIncrease = io[6], d.etaAcc = etaAcc, d.eps = eps;
        sph::computeTimestep(0, n, d);
        io[0] = d.minDt, io[1] = d.minDt_m1, io[2] = d.ttot;
    }
    /*! sph::findRungRanges<false> (ts_rungs.hpp:116-130) on ascending groupDt: out[0..maxNumRungs] */
    void ref_find_rung_ranges(float minDt, const float* groupDt, uint32_t numGroups, int numRungs, uint32_t* out)
    {
        auto r = sph::findRungRanges<false>(minDt, groupDt, numGroups, numRungs);
        for (size_t k = 0; k < r.size(); ++k)
            out[k] = r[k];
    }
#endif
} // extern "C"
