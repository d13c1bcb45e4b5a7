/*! @file ve_forces.cpp
 * @brief Drives HydroVeProp::computeForces (ve_hydro.hpp:132-205, single rank) through the C++ mirror of the
 *        reference GPU seam (host/sphexa_amd/sph_gpu.hpp) with reference-shaped types: a ParticlesData-like
 *        dataset whose devData fields are device vectors, cstone-like Box / GroupView / OctreeNsView.
 *
 * Usage: ve_forces <in.bin> <out.bin> [std]
 *   in.bin : u64 n, then x,y,z (f64), h,m (f32), temp (f64), vx,vy,vz,alpha (f32) -- particles already SFC-sorted
 *   out.bin: nc (u32), h, xm, kx, gradh, prho, c, c11..c33, divv, curlv, alpha, ax, ay, az (f32), du (f64),
 *            minDtCourant (f64)
 *   with "std": HydroProp::computeForces (std_hydro.hpp:124-166) instead; out.bin: nc (u32), h, rho, p, c,
 *            c11..c33, ax, ay, az (f32), du (f64), minDtCourant (f64)
 * The tree is built with the C-ABI cstone entry points (what Domain::sync + octreeProperties provide).
 */
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "mock_dataset.hpp"


template<class T>
static void rd(FILE* f, std::vector<T>& v, size_t n)
{
    v.resize(n);
    if (fread(v.data(), sizeof(T), n, f) != n) throw std::runtime_error("short read");
}

template<class T>
static void wr(FILE* f, const std::vector<T>& v)
{
    fwrite(v.data(), sizeof(T), v.size(), f);
}

int main(int argc, char** argv)
{
    if (argc < 3) return 2;
    FILE*    in = fopen(argv[1], "rb");
    uint64_t n  = 0;
    if (!in || fread(&n, 8, 1, in) != 1) return 3;
    std::vector<double> x, y, z, temp;
    std::vector<float>  h, m, vx, vy, vz, alpha;
    rd(in, x, n), rd(in, y, n), rd(in, z, n), rd(in, h, n), rd(in, m, n), rd(in, temp, n);
    rd(in, vx, n), rd(in, vy, n), rd(in, vz, n), rd(in, alpha, n);
    fclose(in);

    using namespace mock;
    Dataset d;
    auto&   dv = d.devData;
    for (auto* v : {&dv.x, &dv.y, &dv.z, &dv.temp, &dv.du})
        v->resize(n);
    for (auto* v : {&dv.x_m1, &dv.y_m1, &dv.z_m1, &dv.vx, &dv.vy, &dv.vz, &dv.prho, &dv.h, &dv.m, &dv.c, &dv.ax, &dv.ay,
                    &dv.az, &dv.du_m1, &dv.c11, &dv.c12, &dv.c13, &dv.c22, &dv.c23, &dv.c33, &dv.xm, &dv.kx, &dv.divv,
                    &dv.curlv, &dv.alpha, &dv.gradh})
        v->resize(n);
    dv.keys.resize(n);
    dv.nc.resize(n);
    dv.x.upload(x), dv.y.upload(y), dv.z.upload(z), dv.h.upload(h), dv.m.upload(m), dv.temp.upload(temp);
    dv.vx.upload(vx), dv.vy.upload(vy), dv.vz.upload(vz), dv.alpha.upload(alpha);

    Box     box{{-0.5, 0.5, -0.5, 0.5, -0.5, 0.5}, BoundaryType::periodic};
    sx_ctx* ctx = sphexa_amd::context();
    sx_box  sb  = sphexa_amd::toBox(box);

    // Domain::sync (already sorted input) + octreeProperties via the cstone C-ABI
    using sphexa_amd::check;
    check(sx_sfc_keys(ctx, dv.x.data(), dv.y.data(), dv.z.data(), dv.keys.data(), n, &sb), "keys");
    int            cap = (int)(2 * n / 64 * 8 + 64), nLeaf = 0;
    DevVec<uint64_t> leaves;
    DevVec<unsigned> counts, layout;
    leaves.resize(cap + 1);
    counts.resize(cap + 1);
    check(sx_compute_octree(ctx, dv.keys.data(), n, 64, leaves.data(), counts.data(), cap, &nLeaf), "octree");
    int              nNodes = nLeaf + (nLeaf - 1) / 7;
    DevVec<uint64_t> prefixes;
    DevVec<int>      childOffsets, parents, levelRange, i2l, l2i;
    prefixes.resize(nNodes), childOffsets.resize(nNodes + 1), parents.resize(std::max(1, (nNodes - 1) / 8));
    levelRange.resize(23), i2l.resize(nNodes), l2i.resize(nNodes);
    sx_octree oc{prefixes.data(), childOffsets.data(), parents.data(), levelRange.data(), i2l.data(), l2i.data()};
    check(sx_build_octree(ctx, leaves.data(), nLeaf, &oc), "build_octree");
    DevVec<double> centers, sizes;
    centers.resize(3 * nNodes), sizes.resize(3 * nNodes);
    check(sx_node_centers(ctx, prefixes.data(), nNodes, &sb, centers.data(), sizes.data()), "centers");
    layout.resize(nLeaf + 1);
    check(sx_leaf_layout(ctx, counts.data(), nLeaf, layout.data()), "layout");
    d.treeView = OctreeNsView{nLeaf, prefixes.data(), childOffsets.data(), i2l.data(), levelRange.data(),
                              leaves.data(), layout.data(), centers.data(), sizes.data(), 1.0f};

    GroupView grp{0, (unsigned)n, (unsigned)((n + 63) / 64), nullptr, nullptr};
    if (argc > 3 && std::strcmp(argv[3], "std") == 0)
    {
        // std_hydro.hpp:124-166 (single rank: no halo exchanges)
        dv.rho.resize(n), dv.p.resize(n);
        sph::cuda::computeDensity(grp, d, box);
        sph::cuda::computeEOS_HydroStd(0, n, d.muiConst, d.gamma, dv.temp.data(), dv.m.data(), dv.rho.data(),
                                       dv.p.data(), dv.c.data());
        sph::computeIADGpu(grp, d, box);
        sph::computeMomentumEnergyStdGpu(grp, d, box);
        FILE* out = fopen(argv[2], "wb");
        wr(out, dv.nc.download());
        for (auto* v : {&dv.h, &dv.rho, &dv.p, &dv.c, &dv.c11, &dv.c12, &dv.c13, &dv.c22, &dv.c23, &dv.c33, &dv.ax,
                        &dv.ay, &dv.az})
            wr(out, v->download());
        wr(out, dv.du.download());
        wr(out, std::vector<double>{d.minDtCourant});
        fclose(out);
        printf("std_forces: %llu particles, minDtCourant %.9e\n", (unsigned long long)n, d.minDtCourant);
        return 0;
    }
    // ve_hydro.hpp:132-205 (single rank: no halo exchanges)
    sph::cuda::computeXMass(grp, d, box);
    sph::cuda::computeVeDefGradh(grp, d, box);
    sph::cuda::computeEOS(0, n, d.muiConst, d.gamma, dv.temp.data(), dv.m.data(), dv.kx.data(), dv.xm.data(),
                          dv.gradh.data(), dv.prho.data(), dv.c.data(), (float*)nullptr, (float*)nullptr);
    sph::cuda::computeIadDivvCurlv(grp, d, box);
    sph::cuda::computeAVswitches(grp, d, box);
    sph::cuda::computeMomentumEnergy<false>(grp, nullptr, d, box);

    FILE* out = fopen(argv[2], "wb");
    wr(out, dv.nc.download());
    for (auto* v : {&dv.h, &dv.xm, &dv.kx, &dv.gradh, &dv.prho, &dv.c, &dv.c11, &dv.c12, &dv.c13, &dv.c22, &dv.c23,
                    &dv.c33, &dv.divv, &dv.curlv, &dv.alpha, &dv.ax, &dv.ay, &dv.az})
        wr(out, v->download());
    wr(out, dv.du.download());
    wr(out, std::vector<double>{d.minDtCourant});
    fclose(out);
    printf("ve_forces: %llu particles, minDtCourant %.9e\n", (unsigned long long)n, d.minDtCourant);
    return 0;
}
