/*! Compile (and link) check of the C++ mirror (sph-exa_amd/host/sphexa_amd/sph_gpu.hpp) against the REFERENCE's own
 *  types: cstone::Box<double> (sfc/box.hpp), cstone::GroupView / GroupData (traversal/groups.hpp),
 *  cstone::OctreeNsView<double, uint64_t> (tree/octree.hpp), util::array<float, Timestep::maxNumRungs>
 *  (sph/timestep.h), and a dataset whose devData has the members and element types of DeviceParticlesData
 *  (sph/particles_data_gpu.cuh:78-105: thrust::device_vector, the image's rocThrust when built with hipcc
 *  -DSX_REAL_THRUST, else a minimal stand-in).
 *  Every function the reference's sph/include/sph/sph_gpu.hpp:15-89 declares is instantiated with the argument types
 *  the reference's propagators pass (ve_hydro.hpp, ve_hydro_bdt.hpp, std_hydro.hpp).  Built by
 *  tests/test_mirror_compile.py with g++ -I<reference include dirs>; never run (no GPU is touched). */
#include <cstdint>
#include <memory>
#include <vector>

// GroupData<GpuTag>::data and every DeviceParticlesData field are thrust::device_vectors (traversal/groups.hpp:31-39,
// sph/particles_data_gpu.cuh:78-105).  With SX_REAL_THRUST (hipcc) the image's rocThrust is used, so the mirror's
// thrust branch of rawPtr (data().get()) is compiled against the real device_vector / device_ptr.  Without it (g++,
// no HIP headers) a TEST-ONLY stand-in with the members the mirror touches takes its place; defining
// THRUST_MAJOR_VERSION keeps cuda_stubs.h:59-66 from forward-declaring the real one.
#ifdef SX_REAL_THRUST
#include <thrust/device_vector.h>
#else
#define THRUST_MAJOR_VERSION 0
namespace thrust
{
template<class T>
struct device_ptr
{
    T* p;
    T* get() const { return p; }
};
template<class T, class Alloc = std::allocator<T>>
class device_vector
{
public:
    device_ptr<T> data() { return {v_.data()}; }
    size_t        size() const { return v_.size(); }
    void          resize(size_t n) { v_.resize(n); }

private:
    std::vector<T, Alloc> v_;
};
} // namespace thrust
#endif

#ifdef SX_REAL_THRUST
// hipcc defines __HIPCC__, which switches the reference's headers to their CUDA-source configuration: cuda_utils.hpp
// then includes <cuda_runtime.h> (cuda_utils.cuh:5; the reference's HIP build hipifies its sources first, README
// 109-113) and util/tuple.hpp:67-81 re-specialises std::tuple_element for thrust::tuple, which rocThrust already does.
// The reference headers are therefore read in their host configuration (cuda_stubs.h, as its CPU build does), with
// CUDART_VERSION >= 12.4 skipping the tuple traits (the path tuple.hpp takes on current CUDA), while thrust is rocThrust.
#pragma push_macro("__HIPCC__")
#undef __HIPCC__
#define CUDART_VERSION 12040
#endif
#include "cstone/sfc/box.hpp"
#include "cstone/traversal/groups.hpp"
#include "cstone/tree/octree.hpp"
#include "sph/timestep.h"
#ifdef SX_REAL_THRUST
#pragma pop_macro("__HIPCC__")
#endif

#include "sphexa_amd/sph_gpu.hpp"

struct DevData
{
    // DeviceParticlesData's field type: thrust::device_vector (the real one with SX_REAL_THRUST)
    template<class T>
    using V = thrust::device_vector<T>;
    V<double>   x, y, z, temp, u, du;
    V<float>    x_m1, y_m1, z_m1, du_m1;
    V<float>    vx, vy, vz, rho, p, prho, tdpdTrho, h, m, c, cv, mue, mui, divv, curlv, ax, ay, az;
    V<float>    c11, c12, c13, c22, c23, c33, alpha, xm, kx, gradh, dV11, dV12, dV13, dV22, dV23, dV33, markRamp;
    V<uint64_t> keys;
    V<unsigned> nc;
    V<uint8_t>  rung;
};

struct Dataset
{
    using RealType = double;
    using KeyType  = uint64_t;
    DevData                                 devData;
    cstone::OctreeNsView<double, uint64_t> treeView{};
    double K{1}, Kcour{0.2}, Krho{0.06}, gamma{5.0 / 3.0}, minDt{1e-6}, minDtCourant{0};
    unsigned ng0{100}, ngmax{150};
    float    muiConst{10}, alphamin{0.05}, alphamax{1}, decay_constant{0.2}, Atmin{0.1}, Atmax{0.2}, ramp{10};
};

//! raw device pointer of a field, as the reference's rawPtr (cstone/cuda/cuda_utils.hpp)
template<class T>
T* P(thrust::device_vector<T>& v)
{
    return v.data().get();
}

void instantiate(Dataset& d, const cstone::Box<double>& box, const cstone::GroupView& grp,
                 cstone::GroupData<cstone::CpuTag>& groups, cstone::GroupData<cstone::GpuTag>& groupsGpu,
                 float* groupDt)
{
    auto& dv = d.devData;
    sph::computeSpatialGroups(0, 100, d, box, groups);
    sph::computeSpatialGroups(0, 100, d, box, groupsGpu); // the seam's own type (sph_gpu.hpp:17)
    sph::cuda::computeXMass(grp, d, box);
    sph::cuda::computeDensity(grp, d, box);
    sph::cuda::computeVeDefGradh(grp, d, box);
    sph::cuda::computeEOS(0, 100, d.muiConst, d.gamma, P(dv.temp), P(dv.m), P(dv.kx), P(dv.xm),
                          P(dv.gradh), P(dv.prho), P(dv.c), P(dv.rho), P(dv.p));
    sph::cuda::computeIadDivvCurlv(grp, d, box);
    sph::cuda::computeAVswitches(grp, d, box);
    sph::cuda::computeMomentumEnergy<false>(grp, groupDt, d, box);
    sph::cuda::computeMomentumEnergy<true>(grp, groupDt, d, box);
    sph::cuda::computeEOS_HydroStd(0, 100, d.muiConst, d.gamma, P(dv.temp), P(dv.m), P(dv.rho),
                                   P(dv.p), P(dv.c));
    sph::cuda::computeMarkRamp(0, 100, d, box);
    sph::computeIADGpu(grp, d, box);
    sph::computeMomentumEnergyStdGpu(grp, d, box);
    util::array<float, sph::Timestep::maxNumRungs> dt_m1{1e-6f, 2e-6f, 4e-6f, 8e-6f};
    sph::computePositionsGpu(grp, 1e-6f, dt_m1, P(dv.x), P(dv.y), P(dv.z), P(dv.vx), P(dv.vy),
                             P(dv.vz), P(dv.x_m1), P(dv.y_m1), P(dv.z_m1), P(dv.ax), P(dv.ay),
                             P(dv.az), P(dv.rung), P(dv.temp), P(dv.u), P(dv.du), P(dv.du_m1),
                             P(dv.h), P(dv.mui), d.gamma, -1.0, box);
    sph::driftPositionsGpu(grp, 1e-6f, 5e-7f, dt_m1, P(dv.x), P(dv.y), P(dv.z), P(dv.vx), P(dv.vy),
                           P(dv.vz), P(dv.x_m1), P(dv.y_m1), P(dv.z_m1), P(dv.ax), P(dv.ay),
                           P(dv.az), P(dv.rung), P(dv.temp), P(dv.u), P(dv.du), P(dv.du_m1),
                           P(dv.mui), d.gamma, -1.0);
    sph::updateSmoothingLengthGpu(grp, d.ng0, P(dv.nc), P(dv.h));
    sph::groupDivvTimestepGpu(float(d.Krho), grp, P(dv.divv), groupDt);
    sph::groupAccTimestepGpu(0.2f, grp, P(dv.ax), P(dv.ay), P(dv.az), groupDt);
    sph::storeRungGpu(grp, uint8_t(1), P(dv.rung));
}

int main(int argc, char**)
{
    if (argc > 100) // never executed: the check is that this links against libsphexa_hip.so
    {
        Dataset                           d;
        cstone::Box<double>               box(0, 1, cstone::BoundaryType::periodic);
        cstone::GroupView                 grp{0, 100, 2, nullptr, nullptr};
        cstone::GroupData<cstone::CpuTag> groups;
        cstone::GroupData<cstone::GpuTag> groupsGpu;
        float                             groupDt[2];
        instantiate(d, box, grp, groups, groupsGpu, groupDt);
    }
    return 0;
}
