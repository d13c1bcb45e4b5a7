/*! @file mock_dataset.hpp
 * @brief Reference-shaped stand-ins for the host examples: a ParticlesData-like dataset whose devData fields are
 *        device vectors (DeviceParticlesData, particles_data_gpu.cuh:51-211), and cstone-like Box / GroupView /
 *        OctreeNsView (sfc/box.hpp:111-191, traversal/groups.hpp:19-55, tree/octree.hpp:296-316) -- what a reference
 *        propagator hands to the seam (host/sphexa_amd/sph_gpu.hpp).
 */
#pragma once

#include <vector>

#include "sphexa_amd/sph_gpu.hpp"

namespace mock
{

//! stands in for thrust::device_vector<T> in DeviceParticlesData
template<class T>
struct DevVec
{
    T*     p{nullptr};
    size_t n{0};
    void   resize(size_t k)
    {
        p = static_cast<T*>(sx_device_alloc(sphexa_amd::context(), k * sizeof(T)));
        n = k;
        sx_memset(sphexa_amd::context(), p, 0, k * sizeof(T));
    }
    T*     data() { return p; }
    size_t size() const { return n; }
    void   upload(const std::vector<T>& h) { sx_memcpy(sphexa_amd::context(), p, h.data(), n * sizeof(T), 1); }
    std::vector<T> download()
    {
        std::vector<T> h(n);
        sx_memcpy(sphexa_amd::context(), h.data(), p, n * sizeof(T), 2);
        return h;
    }
};

enum class BoundaryType : char { open = 0, periodic = 1, fixed = 2 };

struct Box // cstone::Box<double> accessors used by the adapter
{
    double       lim[6];
    BoundaryType b;
    double       xmin() const { return lim[0]; }
    double       xmax() const { return lim[1]; }
    double       ymin() const { return lim[2]; }
    double       ymax() const { return lim[3]; }
    double       zmin() const { return lim[4]; }
    double       zmax() const { return lim[5]; }
    BoundaryType boundaryX() const { return b; }
    BoundaryType boundaryY() const { return b; }
    BoundaryType boundaryZ() const { return b; }
};

struct GroupView // cstone GroupView
{
    unsigned        firstBody, lastBody, numGroups;
    const unsigned* groupStart;
    const unsigned* groupEnd;
};

struct OctreeNsView // cstone::OctreeNsView<double, uint64_t>
{
    int             numLeafNodes;
    const uint64_t* prefixes;
    const int*      childOffsets;
    const int*      internalToLeaf;
    const int*      levelRange;
    const uint64_t* leaves;
    const unsigned* layout;
    const double*   centers;
    const double*   sizes;
    float           searchExtFactor{1.0f};
};

struct DeviceData // DeviceParticlesData fields touched by the VE path
{
    DevVec<double>   x, y, z, temp, du;
    DevVec<float>    x_m1, y_m1, z_m1, vx, vy, vz, rho, p, prho, tdpdTrho, h, m, c, ax, ay, az, du_m1;
    DevVec<float>    c11, c12, c13, c22, c23, c33, xm, kx, divv, curlv, alpha, gradh;
    DevVec<uint64_t> keys;
    DevVec<unsigned> nc;
};

struct Dataset // ParticlesData<GpuTag> members used by the VE path
{
    unsigned     ng0{100}, ngmax{150};
    double       K{sx_kernel_constant()};
    double       Kcour{0.2}, Krho{0.06}, gamma{5.0 / 3.0};
    float        muiConst{10.0f};
    float        alphamin{0.05f}, alphamax{1.0f}, decay_constant{0.2f};
    float        Atmin{0.1f}, Atmax{0.2f}, ramp{1.0f / (0.2f - 0.1f)};
    double       minDt{1e-6}, minDtCourant{0};
    DeviceData   devData;
    OctreeNsView treeView;
};

} // namespace mock
