/*! @file sph_gpu.hpp
 * @brief C++20 mirror of SPH-EXA's GPU seam (sph/include/sph/sph_gpu.hpp:15-80) on top of libsphexa_hip.so.
 *
 * Drop-in for the `sph::cuda::compute*` functions that ve_hydro.hpp calls through the HaveGpu<Acc> dispatch
 * (e.g. hydro_ve/xmass.hpp:69-74): same names, same argument meaning, same error behaviour (std::runtime_error with
 * the reference messages of xmass_gpu.cu:126-127).  Header-only, no HIP or thrust dependency: the dataset is
 * accessed duck-typed through `d.devData.<field>` (thrust::device_vector or anything with data()), `d.treeView`
 * (cstone::OctreeNsView), and the ParticlesData scalar members (K, ng0, ngmax, Kcour, Krho, gamma, muiConst,
 * alphamin, alphamax, decay_constant, Atmin, Atmax, ramp, minDt, minDtCourant).
 *
 * Replacing the reference's GPU kernels therefore means compiling this header instead of the hydro_ve
 * `*_gpu.cu` translation units.
 */
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>

#include "sphexa_hip.h"

namespace sphexa_amd
{

namespace detail
{
// raw device pointer of a thrust::device_vector (data().get()), a std::vector-like (data()) or a raw pointer
template<class V>
auto raw(V& v, int) -> decltype(v.data().get())
{
    return v.data().get();
}
template<class V>
auto raw(V& v, long) -> decltype(v.data())
{
    return v.data();
}
template<class T>
T* raw(T* p, int)
{
    return p;
}
template<class V>
auto rawPtr(V& v)
{
    return (v.size() == 0) ? decltype(raw(v, 0)){nullptr} : raw(v, 0);
}
} // namespace detail

//! one context per process (the reference uses the device exposed by the launcher, gpu_config.cuh:62-67)
inline sx_ctx* context(int device = 0)
{
    static sx_ctx* ctx = [device] {
        sx_ctx* c = nullptr;
        if (sx_create(&c, device) != SX_OK) throw std::runtime_error("sphexa_amd: sx_create failed");
        return c;
    }();
    return ctx;
}

inline void check(int rc, const char* what)
{
    if (rc == SX_OK) return;
    if (rc == SX_ERR_TRAVERSAL) throw std::runtime_error("GPU traversal stack exhausted in neighbor search\n");
    if (rc == SX_ERR_NOT_CONVERGED) throw std::runtime_error("coupled nc/h-updated failed to converge");
    throw std::runtime_error(std::string(what) + ": " + sx_last_error(context()));
}

template<class Box>
sx_box toBox(const Box& b)
{
    sx_box r{};
    r.lim[0] = b.xmin(), r.lim[1] = b.xmax(), r.lim[2] = b.ymin(), r.lim[3] = b.ymax(), r.lim[4] = b.zmin(),
    r.lim[5] = b.zmax();
    r.bnd[0] = (int32_t)b.boundaryX(), r.bnd[1] = (int32_t)b.boundaryY(), r.bnd[2] = (int32_t)b.boundaryZ();
    return r;
}

template<class Dataset>
sx_params toParams(const Dataset& d)
{
    sx_params p{};
    p.K              = d.K;
    p.ng0            = d.ng0;
    p.ngmax          = d.ngmax;
    p.Kcour          = d.Kcour;
    p.Krho           = d.Krho;
    p.gamma          = d.gamma;
    p.muiConst       = d.muiConst;
    p.alphamin       = d.alphamin;
    p.alphamax       = d.alphamax;
    p.decay_constant = d.decay_constant;
    p.Atmin          = d.Atmin;
    p.Atmax          = d.Atmax;
    p.ramp           = d.ramp;
    p.maxDtIncrease  = 1.1;
    return p;
}

//! DeviceParticlesData (particles_data_gpu.cuh:51-211) -> sx_fields, in the reference field order
template<class Dataset>
sx_fields toFields(Dataset& d)
{
    using detail::rawPtr;
    auto&     dv = d.devData;
    sx_fields f{};
    f.n        = dv.x.size();
    f.x        = rawPtr(dv.x);
    f.y        = rawPtr(dv.y);
    f.z        = rawPtr(dv.z);
    f.x_m1     = rawPtr(dv.x_m1);
    f.y_m1     = rawPtr(dv.y_m1);
    f.z_m1     = rawPtr(dv.z_m1);
    f.vx       = rawPtr(dv.vx);
    f.vy       = rawPtr(dv.vy);
    f.vz       = rawPtr(dv.vz);
    f.rho      = rawPtr(dv.rho);
    f.p        = rawPtr(dv.p);
    f.prho     = rawPtr(dv.prho);
    f.tdpdTrho = rawPtr(dv.tdpdTrho);
    f.h        = rawPtr(dv.h);
    f.m        = rawPtr(dv.m);
    f.c        = rawPtr(dv.c);
    f.ax       = rawPtr(dv.ax);
    f.ay       = rawPtr(dv.ay);
    f.az       = rawPtr(dv.az);
    f.du       = rawPtr(dv.du);
    f.du_m1    = rawPtr(dv.du_m1);
    f.c11      = rawPtr(dv.c11);
    f.c12      = rawPtr(dv.c12);
    f.c13      = rawPtr(dv.c13);
    f.c22      = rawPtr(dv.c22);
    f.c23      = rawPtr(dv.c23);
    f.c33      = rawPtr(dv.c33);
    f.temp     = rawPtr(dv.temp);
    f.xm       = rawPtr(dv.xm);
    f.kx       = rawPtr(dv.kx);
    f.divv     = rawPtr(dv.divv);
    f.curlv    = (dv.curlv.size() == dv.x.size()) ? rawPtr(dv.curlv) : nullptr; // iad_divv_curlv.hpp:77
    f.alpha    = rawPtr(dv.alpha);
    f.gradh    = rawPtr(dv.gradh);
    f.keys     = rawPtr(dv.keys);
    f.nc       = rawPtr(dv.nc);
    if constexpr (requires { dv.dV11; })
    {
        // GradVFields: non-empty only with avClean (ve_hydro.hpp:80-85); doGradV = dV11.size() == x.size()
        if (dv.dV11.size() == dv.x.size())
        {
            f.dV11 = rawPtr(dv.dV11), f.dV12 = rawPtr(dv.dV12), f.dV13 = rawPtr(dv.dV13);
            f.dV22 = rawPtr(dv.dV22), f.dV23 = rawPtr(dv.dV23), f.dV33 = rawPtr(dv.dV33);
        }
    }
    return f;
}

//! cstone::OctreeNsView<double, uint64_t> -> sx_tree (centers/sizes are Vec3<double> arrays)
template<class TreeView>
sx_tree toTree(const TreeView& t)
{
    sx_tree r{};
    r.numLeafNodes    = t.numLeafNodes;
    r.prefixes        = reinterpret_cast<const uint64_t*>(t.prefixes);
    r.childOffsets    = t.childOffsets;
    r.internalToLeaf  = t.internalToLeaf;
    r.levelRange      = t.levelRange;
    r.leaves          = reinterpret_cast<const uint64_t*>(t.leaves);
    r.layout          = t.layout;
    r.centers         = reinterpret_cast<const double*>(t.centers);
    r.sizes           = reinterpret_cast<const double*>(t.sizes);
    r.searchExtFactor = t.searchExtFactor;
    return r;
}

template<class GroupView>
sx_groups toGroups(const GroupView& g)
{
    return sx_groups{(uint32_t)g.firstBody, (uint32_t)g.lastBody, (uint32_t)g.numGroups, g.groupStart, g.groupEnd};
}

} // namespace sphexa_amd

namespace sph::cuda
{

//! sph_gpu.hpp:25 -- neighbor search + h-nc iteration + xm (xmass_gpu.cu:103-128)
template<class GroupView, class Dataset, class Box>
void computeXMass(const GroupView& grp, Dataset& d, const Box& box)
{
    namespace sa = sphexa_amd;
    auto g = sa::toGroups(grp);
    auto f = sa::toFields(d);
    auto p = sa::toParams(d);
    auto b = sa::toBox(box);
    auto t = sa::toTree(d.treeView);
    sa::check(sx_xmass(sa::context(), &g, &f, &p, &b, &t), "computeXMass");
}

//! sph_gpu.hpp:37 (ve_def_gradh_gpu.cu:86)
template<class GroupView, class Dataset, class Box>
void computeVeDefGradh(const GroupView& grp, Dataset& d, const Box& box)
{
    namespace sa = sphexa_amd;
    auto g = sa::toGroups(grp);
    auto f = sa::toFields(d);
    auto p = sa::toParams(d);
    auto b = sa::toBox(box);
    sa::check(sx_ve_def_gradh(sa::context(), &g, &f, &p, &b), "computeVeDefGradh");
}

//! sph_gpu.hpp:40-43 (hydro_ve/eos_gpu.cu:74)
template<class Tt, class Tm, class Thydro>
void computeEOS(size_t firstParticle, size_t lastParticle, Tm mui, double gamma, const Tt* temp, const Tm* m,
                const Thydro* kx, const Thydro* xm, const Thydro* gradh, Thydro* prho, Thydro* c, Thydro* rho,
                Thydro* p)
{
    namespace sa = sphexa_amd;
    sa::check(sx_eos(sa::context(), (uint32_t)firstParticle, (uint32_t)lastParticle, (float)mui, gamma, temp, m, kx,
                     xm, gradh, prho, c, rho, p),
              "computeEOS");
}

//! sph_gpu.hpp:45 (iad_divv_curlv_gpu.cu:91)
template<class GroupView, class Dataset, class Box>
void computeIadDivvCurlv(const GroupView& grp, Dataset& d, const Box& box)
{
    namespace sa = sphexa_amd;
    auto g = sa::toGroups(grp);
    auto f = sa::toFields(d);
    auto p = sa::toParams(d);
    auto b = sa::toBox(box);
    sa::check(sx_iad_divv_curlv(sa::context(), &g, &f, &p, &b), "computeIadDivvCurlv");
}

//! sph_gpu.hpp:48 (av_switches_gpu.cu:103); uses d.minDt like the reference
template<class GroupView, class Dataset, class Box>
void computeAVswitches(const GroupView& grp, Dataset& d, const Box& box)
{
    namespace sa = sphexa_amd;
    auto g = sa::toGroups(grp);
    auto f = sa::toFields(d);
    auto p = sa::toParams(d);
    auto b = sa::toBox(box);
    sa::check(sx_av_switches(sa::context(), &g, &f, &p, &b, d.minDt), "computeAVswitches");
}

//! sph_gpu.hpp:51-53 (momentum_energy_gpu.cu:121-145): writes ax,ay,az,du and d.minDtCourant
template<bool avClean, class GroupView, class Dataset, class Box>
void computeMomentumEnergy(const GroupView& grp, float* groupDt, Dataset& d, const Box& box)
{
    namespace sa = sphexa_amd;
    auto  g = sa::toGroups(grp);
    auto  f = sa::toFields(d);
    auto  p = sa::toParams(d);
    auto  b = sa::toBox(box);
    float minDt;
    // both instantiations of the reference seam (momentum_energy_gpu.cu:147-152)
    if constexpr (avClean)
        sa::check(sx_momentum_energy_avclean(sa::context(), &g, groupDt, &f, &p, &b, &minDt), "computeMomentumEnergy");
    else sa::check(sx_momentum_energy(sa::context(), &g, groupDt, &f, &p, &b, &minDt), "computeMomentumEnergy");
    d.minDtCourant = minDt;
}

//! sph_gpu.hpp:31-32 (hydro_ve/xmass_gpu.cu:150-164): std density -- search + h iteration, XMass into rho,
//! rho = m / rho
template<class GroupView, class Dataset, class Box>
void computeDensity(const GroupView& grp, Dataset& d, const Box& box)
{
    namespace sa = sphexa_amd;
    auto g = sa::toGroups(grp);
    auto f = sa::toFields(d);
    auto p = sa::toParams(d);
    auto b = sa::toBox(box);
    auto t = sa::toTree(d.treeView);
    sa::check(sx_density(sa::context(), &g, &f, &p, &b, &t), "computeDensity");
}

//! sph_gpu.hpp:46-47 (hydro_std/eos_gpu.cu:54-62)
template<class Tu, class Trho, class Tp, class Tc>
void computeEOS_HydroStd(size_t firstParticle, size_t lastParticle, Trho mui, Tu gamma, const Tu* temp, const Trho* m,
                         Trho* rho, Tp* p, Tc* c)
{
    namespace sa = sphexa_amd;
    sa::check(sx_eos_std(sa::context(), (uint32_t)firstParticle, (uint32_t)lastParticle, (float)mui, (double)gamma,
                         temp, m, rho, p, c),
              "computeEOS_HydroStd");
}

//! sph_gpu.hpp:53-54 (hydro_ve/additional_fields.cu:86-98): the markRamp diagnostic field over [first, last) on the
//! step's cached neighbor list
template<class Dataset, class Box>
void computeMarkRamp(size_t first, size_t last, Dataset& d, const Box& box)
{
    namespace sa = sphexa_amd;
    sx_groups g{(uint32_t)first, (uint32_t)last, (uint32_t)((last - first + 63) / 64), nullptr, nullptr};
    auto      f = sa::toFields(d);
    auto      p = sa::toParams(d);
    auto      b = sa::toBox(box);
    sa::check(sx_mark_ramp(sa::context(), &g, &f, &p, &b, sa::detail::rawPtr(d.devData.markRamp)), "computeMarkRamp");
    sa::check(sx_synchronize(sa::context()), "computeMarkRamp");
}

} // namespace sph::cuda

namespace sph
{

//! sph_gpu.hpp:19-20 (hydro_std/iad_gpu.cu:111-124)
template<class GroupView, class Dataset, class Box>
void computeIADGpu(const GroupView& grp, Dataset& d, const Box& box)
{
    namespace sa = sphexa_amd;
    auto g = sa::toGroups(grp);
    auto f = sa::toFields(d);
    auto p = sa::toParams(d);
    auto b = sa::toBox(box);
    sa::check(sx_iad(sa::context(), &g, &f, &p, &b), "computeIADGpu");
}

//! sph_gpu.hpp:22-23 (hydro_std/momentum_energy_gpu.cu:109-129): writes ax,ay,az,du and d.minDtCourant
template<class GroupView, class Dataset, class Box>
void computeMomentumEnergyStdGpu(const GroupView& grp, Dataset& d, const Box& box)
{
    namespace sa = sphexa_amd;
    auto  g = sa::toGroups(grp);
    auto  f = sa::toFields(d);
    auto  p = sa::toParams(d);
    auto  b = sa::toBox(box);
    float minDt;
    sa::check(sx_momentum_energy_std(sa::context(), &g, &f, &p, &b, &minDt), "computeMomentumEnergyStdGpu");
    d.minDtCourant = minDt;
}

//! sph_gpu.hpp:15-17 (sph/groups.cu:30-47): computeGroupSplits<64> with tolFactor 2 into groups.data
template<class Dataset, class Box, class GroupData>
void computeSpatialGroups(size_t first, size_t last, Dataset& d, const Box& box, GroupData& groups)
{
    namespace sa = sphexa_amd;
    groups.data.resize(last - first + 2);
    auto      b = sa::toBox(box);
    auto      t = sa::toTree(d.treeView);
    auto&     dv = d.devData;
    sx_groups out{};
    sa::check(sx_spatial_groups(sa::context(), (uint32_t)first, (uint32_t)last, sa::detail::rawPtr(dv.x),
                                sa::detail::rawPtr(dv.y), sa::detail::rawPtr(dv.z), &t, &b, 2.0f,
                                sa::detail::rawPtr(groups.data), (uint32_t)(last - first + 2), &out),
              "computeSpatialGroups");
    groups.data.resize(out.numGroups + 1);
    groups.firstBody  = first;
    groups.lastBody   = last;
    groups.numGroups  = out.numGroups;
    groups.groupStart = sa::detail::rawPtr(groups.data);
    groups.groupEnd   = sa::detail::rawPtr(groups.data) + 1;
}

namespace detail_bdt
{
template<class A>
void dtArray(const A& dt_m1, float (&out)[SX_MAX_RUNGS])
{
    for (int k = 0; k < SX_MAX_RUNGS; ++k)
        out[k] = dt_m1[k];
}
template<class T>
constexpr bool isF32 = std::is_same_v<std::remove_cv_t<T>, float>;
template<class T>
constexpr bool isF64 = std::is_same_v<std::remove_cv_t<T>, double>;
} // namespace detail_bdt

/*! sph_gpu.hpp:64-72 (positions_gpu.cu:110-179): rung-aware Press position update + AB2 energy update.
 *  The MI355X library stores the reference's SphTypes: coordinates, temp/u and du in double, the rest in float */
template<class GroupView, class Tc, class Tv, class Ta, class Tdu, class Tm1, class Tu, class Thydro, class DtM1,
         class Box>
void computePositionsGpu(const GroupView& grp, float dt, DtM1 dt_m1, Tc* x, Tc* y, Tc* z, Tv* vx, Tv* vy, Tv* vz,
                         Tm1* x_m1, Tm1* y_m1, Tm1* z_m1, Ta* ax, Ta* ay, Ta* az, const uint8_t* rung, Tu* temp, Tu* u,
                         Tdu* du, Tm1* du_m1, Thydro* h, Thydro* mui, Tc gamma, Tc constCv, const Box& box)
{
    namespace sa = sphexa_amd;
    using namespace detail_bdt;
    static_assert(isF64<Tc> && isF32<Tv> && isF32<Ta> && isF64<Tdu> && isF32<Tm1> && isF64<Tu> && isF32<Thydro>,
                  "computePositionsGpu: the MI355X library implements the SphTypes precision (sph/types.hpp:39-46)");
    sx_fields f{};
    f.x = x, f.y = y, f.z = z, f.vx = vx, f.vy = vy, f.vz = vz, f.x_m1 = x_m1, f.y_m1 = y_m1, f.z_m1 = z_m1;
    f.ax = ax, f.ay = ay, f.az = az, f.temp = temp, f.u = u, f.du = du, f.du_m1 = du_m1, f.h = h, f.mui = mui;
    float d[SX_MAX_RUNGS];
    dtArray(dt_m1, d);
    auto g = sa::toGroups(grp);
    auto b = sa::toBox(box);
    sa::check(sx_positions_rungs(sa::context(), &g, dt, d, rung, &f, (double)gamma, (double)constCv, &b),
              "computePositionsGpu");
}

//! sph_gpu.hpp:57-62 (positions_gpu.cu:45-108): drift back by dt_back, forward by dt (open box)
template<class GroupView, class Tc, class Thydro, class Tm1, class Tdu, class DtM1>
void driftPositionsGpu(const GroupView& grp, float dt, float dt_back, DtM1 dt_m1, Tc* x, Tc* y, Tc* z, Thydro* vx,
                       Thydro* vy, Thydro* vz, const Tm1* x_m1, const Tm1* y_m1, const Tm1* z_m1, const Thydro* ax,
                       const Thydro* ay, const Thydro* az, const uint8_t* rung, Tc* temp, Tc* u, Tdu* du, Tm1* du_m1,
                       Thydro* mui, Tc gamma, Tc constCv)
{
    namespace sa = sphexa_amd;
    using namespace detail_bdt;
    static_assert(isF64<Tc> && isF32<Thydro> && isF32<Tm1> && isF64<Tdu>,
                  "driftPositionsGpu: the MI355X library implements the SphTypes precision (sph/types.hpp:39-46)");
    sx_fields f{};
    f.x = x, f.y = y, f.z = z, f.vx = vx, f.vy = vy, f.vz = vz;
    f.x_m1 = const_cast<Tm1*>(x_m1), f.y_m1 = const_cast<Tm1*>(y_m1), f.z_m1 = const_cast<Tm1*>(z_m1);
    f.ax = const_cast<Thydro*>(ax), f.ay = const_cast<Thydro*>(ay), f.az = const_cast<Thydro*>(az);
    f.temp = temp, f.u = u, f.du = du, f.du_m1 = du_m1, f.mui = mui;
    float d[SX_MAX_RUNGS];
    dtArray(dt_m1, d);
    auto g = sa::toGroups(grp);
    sa::check(sx_drift_positions(sa::context(), &g, dt, dt_back, d, rung, &f, (double)gamma, (double)constCv),
              "driftPositionsGpu");
}

//! sph_gpu.hpp:80-81 (ts_groups.cu:17-46)
template<class GroupView, class T>
void groupDivvTimestepGpu(float Krho, const GroupView& grp, const T* divv, float* groupDt)
{
    static_assert(detail_bdt::isF32<T>, "groupDivvTimestepGpu: float hydro fields (SphTypes)");
    namespace sa = sphexa_amd;
    auto g = sa::toGroups(grp);
    sa::check(sx_group_divv_timestep(sa::context(), Krho, &g, divv, groupDt), "groupDivvTimestepGpu");
}

//! sph_gpu.hpp:83-84 (ts_groups.cu:48-81)
template<class GroupView, class T>
void groupAccTimestepGpu(float etaAcc, const GroupView& grp, const T* ax, const T* ay, const T* az, float* groupDt)
{
    static_assert(detail_bdt::isF32<T>, "groupAccTimestepGpu: float hydro fields (SphTypes)");
    namespace sa = sphexa_amd;
    auto g = sa::toGroups(grp);
    sa::check(sx_group_acc_timestep(sa::context(), etaAcc, &g, ax, ay, az, groupDt), "groupAccTimestepGpu");
}

//! sph_gpu.hpp:86 (ts_groups.cu:84-108)
template<class GroupView>
void storeRungGpu(const GroupView& grp, uint8_t rung, uint8_t* particleRungs)
{
    namespace sa = sphexa_amd;
    auto g = sa::toGroups(grp);
    sa::check(sx_store_rung(sa::context(), &g, rung, particleRungs), "storeRungGpu");
}

//! sph_gpu.hpp:71-72 (update_h_gpu.cu:49-60)
template<class GroupView, class Th>
void updateSmoothingLengthGpu(const GroupView& grp, unsigned ng0, const unsigned* nc, Th* h)
{
    namespace sa = sphexa_amd;
    const sx_groups g = sa::toGroups(grp);
    sa::check(sx_update_h_groups(sa::context(), &g, ng0, nc, h), "updateSmoothingLengthGpu");
}

} // namespace sph
