/*! @file ve_seam_bench.cpp
 * @brief Throughput of the drop-in path: whole HydroVeProp steps (ve_hydro.hpp:132-218, one rank) driven the way a
 *        reference propagator drives the GPU seam -- every particle operation a call of the C++ mirror of
 *        sph/include/sph/sph_gpu.hpp:15-80 (host/sphexa_amd/sph_gpu.hpp) or of the cstone C-ABI, each call complete
 *        before the next, with reference-shaped types (mock_dataset.hpp).
 *
 * Usage: ve_seam_bench <side> <steps> <warmup>     (Sedov lattice, sedov_init.hpp:48-96 values)
 * One step:
 *   sync          Domain::sync on one rank: SFC keys, stable key sort, every conserved field gathered in key order,
 *                 converged cornerstone tree + linked octree + node geometry + leaf layout (sx_sfc_keys, sx_sort_keys,
 *                 sx_gather, sx_compute_octree, sx_build_octree, sx_node_centers, sx_leaf_layout)
 *   forces        computeXMass (search + h iteration), computeVeDefGradh, computeEOS, computeIadDivvCurlv,
 *                 computeAVswitches, computeMomentumEnergy<false> (sph::cuda::*)
 *   timestep      rhoTimestep (sx_max_divv) and computeTimestep's minimum (ts_global.hpp:72-112) on the host
 *   integrate     computePositions (sx_positions) + updateSmoothingLength (sx_update_h)
 * Prints one JSON line: ms per step (host clock around each whole step), the stage split, particle-updates/s.
 * The neighbor list of computeXMass is cached and reused by the later kernels of the step; there is no
 * skin reuse on this path: every step syncs and searches, as the reference's propagator does.
 */
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

#include "mock_dataset.hpp"

namespace
{

using Clock = std::chrono::steady_clock;

double ms(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); }

//! idealGasCv<float, double> (sph/eos.hpp:13-18)
float idealGasCv(float mui, double gamma) { return (float)((double)(8.317e7f / mui) / (gamma - 1.0f)); }

} // namespace

int main(int argc, char** argv)
{
    if (argc < 4)
    {
        fprintf(stderr, "usage: ve_seam_bench <side> <steps> <warmup>\n");
        return 2;
    }
    const size_t side = std::strtoul(argv[1], nullptr, 10);
    const int    steps = std::atoi(argv[2]), warmup = std::atoi(argv[3]);
    const size_t n = side * side * side;

    using namespace mock;
    using sphexa_amd::check;
    Dataset d;
    auto&   dv  = d.devData;
    sx_ctx* ctx = sphexa_amd::context();

    // ---- Sedov lattice (grid.hpp:102-132, sedov_init.hpp:48-96), generated on the host and uploaded
    {
        std::vector<double> x(n), y(n), z(n), temp(n);
        const double        r = 0.5, step = 2 * r / side, rIni = -r + 0.5 * step, width = 0.1;
        const double        ener0 = 1.0 / std::pow(M_PI, 1.5) / 1.0 / std::pow(width, 3.0);
        const float         cv    = idealGasCv(d.muiConst, d.gamma);
        for (size_t i = 0; i < side; ++i)
            for (size_t j = 0; j < side; ++j)
                for (size_t k = 0; k < side; ++k)
                {
                    const size_t q = (i * side + j) * side + k;
                    x[q] = rIni + k * step, y[q] = rIni + j * step, z[q] = rIni + i * step;
                    const double r2 = x[q] * x[q] + y[q] * y[q] + z[q] * z[q];
                    temp[q]         = (ener0 * std::exp(-(r2 / (width * width))) + 1e-8) / (double)cv;
                }
        for (auto* v : {&dv.x, &dv.y, &dv.z, &dv.temp, &dv.du})
            v->resize(n);
        for (auto* v : {&dv.x_m1, &dv.y_m1, &dv.z_m1, &dv.vx, &dv.vy, &dv.vz, &dv.prho, &dv.h, &dv.m, &dv.c, &dv.ax,
                        &dv.ay, &dv.az, &dv.du_m1, &dv.c11, &dv.c12, &dv.c13, &dv.c22, &dv.c23, &dv.c33, &dv.xm, &dv.kx,
                        &dv.divv, &dv.curlv, &dv.alpha, &dv.gradh})
            v->resize(n);
        dv.keys.resize(n);
        dv.nc.resize(n);
        dv.x.upload(x), dv.y.upload(y), dv.z.upload(z), dv.temp.upload(temp);
        const float hInit = (float)(std::cbrt(3.0 / (4 * M_PI) * d.ng0 * std::pow(2 * r, 3) / n) * 0.5);
        dv.h.upload(std::vector<float>(n, hInit));
        dv.m.upload(std::vector<float>(n, (float)(1.0 / n)));
        dv.alpha.upload(std::vector<float>(n, 0.05f));
    }
    // the spare of every conserved field (the sync's gather target) and the tree buffers
    DevVec<double>   sx_, sy_, sz_, stemp_;
    DevVec<float>    sh_, sm_, svx_, svy_, svz_, sxm1_, sym1_, szm1_, sdum1_, salpha_;
    DevVec<unsigned> order;
    for (auto* v : {&sx_, &sy_, &sz_, &stemp_})
        v->resize(n);
    for (auto* v : {&sh_, &sm_, &svx_, &svy_, &svz_, &sxm1_, &sym1_, &szm1_, &sdum1_, &salpha_})
        v->resize(n);
    order.resize(n);
    const int        cap = (int)(2 * n / 64 * 8 + 64);
    DevVec<uint64_t> leaves, prefixes;
    DevVec<unsigned> counts, layout;
    DevVec<int>      childOffsets, parents, levelRange, i2l, l2i;
    DevVec<double>   centers, sizes;
    leaves.resize(cap + 1), counts.resize(cap + 1), layout.resize(cap + 1);
    const int nodeCap = cap + cap / 7 + 8;
    prefixes.resize(nodeCap), childOffsets.resize(nodeCap + 1), parents.resize(nodeCap / 8 + 1);
    levelRange.resize(23), i2l.resize(nodeCap), l2i.resize(nodeCap), centers.resize(3 * nodeCap);
    sizes.resize(3 * nodeCap);

    Box          box{{-0.5, 0.5, -0.5, 0.5, -0.5, 0.5}, BoundaryType::periodic};
    const sx_box sb = sphexa_amd::toBox(box);
    GroupView    grp{0, (unsigned)n, (unsigned)((n + 63) / 64), nullptr, nullptr};
    double       minDt = 1e-6, minDt_m1 = 1e-6, ttot = 0;
    const double Krho = d.Krho, maxDtIncrease = 1.1;

    auto sync = [&] {
        check(sx_sfc_keys(ctx, dv.x.data(), dv.y.data(), dv.z.data(), dv.keys.data(), n, &sb), "keys");
        check(sx_sort_keys(ctx, dv.keys.data(), order.data(), n), "sort");
        auto gather = [&](auto& field, auto& spare) {
            check(sx_gather(ctx, order.data(), n, field.data(), spare.data(), (int)sizeof(*field.data())), "gather");
            std::swap(field.p, spare.p);
        };
        gather(dv.x, sx_), gather(dv.y, sy_), gather(dv.z, sz_), gather(dv.temp, stemp_), gather(dv.h, sh_);
        gather(dv.m, sm_), gather(dv.vx, svx_), gather(dv.vy, svy_), gather(dv.vz, svz_), gather(dv.x_m1, sxm1_);
        gather(dv.y_m1, sym1_), gather(dv.z_m1, szm1_), gather(dv.du_m1, sdum1_), gather(dv.alpha, salpha_);
        int nLeaf = 0;
        check(sx_compute_octree(ctx, dv.keys.data(), n, 64, leaves.data(), counts.data(), cap, &nLeaf), "octree");
        const int nNodes = nLeaf + (nLeaf - 1) / 7;
        sx_octree oc{prefixes.data(), childOffsets.data(), parents.data(), levelRange.data(), i2l.data(), l2i.data()};
        check(sx_build_octree(ctx, leaves.data(), nLeaf, &oc), "build_octree");
        check(sx_node_centers(ctx, prefixes.data(), nNodes, &sb, centers.data(), sizes.data()), "centers");
        check(sx_leaf_layout(ctx, counts.data(), nLeaf, layout.data()), "layout");
        check(sx_synchronize(ctx), "sync");
        d.treeView = OctreeNsView{nLeaf, prefixes.data(), childOffsets.data(), i2l.data(), levelRange.data(),
                                  leaves.data(), layout.data(), centers.data(), sizes.data(), 1.0f};
    };

    const char* names[] = {"sync", "XMass", "VeDefGradh", "EOS", "IadDivvCurlv", "AVswitches", "MomentumEnergy",
                           "Timestep", "Positions", "UpdateH"};
    constexpr int kStages = 10;
    double        stage[kStages] = {0}, total = 0;
    for (int s = 0; s < warmup + steps; ++s)
    {
        Clock::time_point t[kStages + 1];
        t[0] = Clock::now();
        sync();
        t[1] = Clock::now();
        d.minDt = minDt;
        sph::cuda::computeXMass(grp, d, box);
        check(sx_synchronize(ctx), "xmass");
        t[2] = Clock::now();
        sph::cuda::computeVeDefGradh(grp, d, box);
        check(sx_synchronize(ctx), "vedefgradh");
        t[3] = Clock::now();
        sph::cuda::computeEOS(0, n, d.muiConst, d.gamma, dv.temp.data(), dv.m.data(), dv.kx.data(), dv.xm.data(),
                              dv.gradh.data(), dv.prho.data(), dv.c.data(), (float*)nullptr, (float*)nullptr);
        check(sx_synchronize(ctx), "eos");
        t[4] = Clock::now();
        sph::cuda::computeIadDivvCurlv(grp, d, box);
        check(sx_synchronize(ctx), "iad");
        t[5] = Clock::now();
        sph::cuda::computeAVswitches(grp, d, box);
        check(sx_synchronize(ctx), "av");
        t[6] = Clock::now();
        sph::cuda::computeMomentumEnergy<false>(grp, nullptr, d, box);
        check(sx_synchronize(ctx), "momentum");
        t[7] = Clock::now();
        // rhoTimestep + computeTimestep (ts_global.hpp:72-112, one rank, no gravity)
        float maxDivv = 0;
        check(sx_max_divv(ctx, 0, (uint32_t)n, dv.divv.data(), &maxDivv), "maxDivv");
        const double minDtRho = Krho / std::fabs((double)maxDivv);
        const double dt = std::min({(double)d.minDtCourant, minDtRho, maxDtIncrease * minDt});
        minDt_m1 = minDt, minDt = dt, ttot += dt;
        t[8] = Clock::now();
        sx_fields f = sphexa_amd::toFields(d);
        check(sx_positions(ctx, 0, (uint32_t)n, minDt, minDt_m1, &f, d.gamma, d.muiConst, &sb), "positions");
        check(sx_synchronize(ctx), "positions");
        t[9] = Clock::now();
        check(sx_update_h(ctx, 0, (uint32_t)n, d.ng0, dv.nc.data(), dv.h.data()), "updateH");
        check(sx_synchronize(ctx), "updateH");
        t[10] = Clock::now();
        if (s < warmup) continue;
        for (int k = 0; k < kStages; ++k)
            stage[k] += ms(t[k], t[k + 1]);
        total += ms(t[0], t[kStages]);
    }
    const double msStep = total / steps;
    printf("{\"path\": \"C-ABI seam (sph_gpu.hpp mirror), reference VE propagator order, one rank, every call "
           "synchronous, sync + search every step\", \"workload\": \"Sedov -n %zu (%zu particles)\", \"steps\": %d, "
           "\"warmup\": %d, \"ms_per_step\": %.4f, \"value\": %.6e, \"unit\": \"particle-updates/s\", \"ttot\": %.9e, "
           "\"minDt\": %.9e, \"stages_ms\": {",
           side, n, steps, warmup, msStep, n / (msStep * 1e-3), ttot, minDt);
    for (int k = 0; k < kStages; ++k)
        printf("%s\"%s\": %.4f", k ? ", " : "", names[k], stage[k] / steps);
    printf("}}\n");
    return 0;
}
