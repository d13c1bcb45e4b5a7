// TEST INFRASTRUCTURE ONLY -- the reference's multi-rank self-gravity on the CPU, compiled from /root/reference by
// oracle/Makefile into oracle/_ref/grav_mpi_ref and run under the image's MPICH (mpiexec -n P) by
// oracle/gen_grav_mpi.py.  Per rank, exactly what HydroVeProp's gravity does with MultipoleHolderCpu
// (main/src/propagator/gravity_wrapper.hpp:45-94) after Domain::syncGrav (cstone/domain/domain.hpp:246-300):
//   domain.syncGrav(keys, x, y, z, h, m, {id}, scratch)            -- SFC decomposition + focus tree + halos
//   ryoanji::computeGlobalMultipoles(...)                           -- global_multipole.hpp:44-77
//   ryoanji::computeGravity(..., startCell, endCell, ..., G, ...)   -- traversal_cpu.hpp:166-230
// on the particles of an input file (each rank an index slab, as the tests hand them out), with the types of
// sphexa's ParticlesData (x, y, z double; h, m, ax, ay, az float).  No reference source is copied here: this file
// only calls the reference's templates, as ryoanji/test/interface/global_upsweep_cpu.cpp does.
//
//   grav_mpi_ref <in.bin> <out-prefix> <bucketSize> <theta> <G>
//   in.bin: u64 n, then n x {f64 x, f64 y, f64 z, f32 h, f32 m, u64 id}; box: 6 f64 limits + 3 i32 boundary types
//   out-prefix<rank>.bin: u64 nLocal, f64 egrav (all ranks, reduced), then nLocal x {u64 id, f32 ax, f32 ay, f32 az}
#include <mpi.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <string>
#include <tuple>
#include <vector>

#include "cstone/domain/domain.hpp"
#include "ryoanji/interface/global_multipole.hpp"
#include "ryoanji/nbody/traversal_cpu.hpp"

int main(int argc, char** argv)
{
    MPI_Init(&argc, &argv);
    int rank = 0, numRanks = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &numRanks);
    if (argc < 6)
    {
        if (rank == 0) std::fprintf(stderr, "usage: grav_mpi_ref in.bin out-prefix bucketSize theta G\n");
        MPI_Abort(MPI_COMM_WORLD, 2);
    }
    const unsigned bucketSize = (unsigned)std::atoi(argv[3]);
    const float    theta      = (float)std::atof(argv[4]);
    const float    G          = (float)std::atof(argv[5]);

    FILE*    in = std::fopen(argv[1], "rb");
    uint64_t n  = 0;
    double   lim[6];
    int32_t  bnd[3];
    if (!in || std::fread(&n, 8, 1, in) != 1 || std::fread(lim, 8, 6, in) != 6 || std::fread(bnd, 4, 3, in) != 3)
        MPI_Abort(MPI_COMM_WORLD, 3);
    const uint64_t first = n * rank / numRanks, last = n * (rank + 1) / numRanks;
    std::vector<double>   x, y, z;
    std::vector<float>    h, m;
    std::vector<uint64_t> id;
    for (uint64_t i = 0; i < n; ++i)
    {
        double   p[3];
        float    hm[2];
        uint64_t k;
        if (std::fread(p, 8, 3, in) != 3 || std::fread(hm, 4, 2, in) != 2 || std::fread(&k, 8, 1, in) != 1)
            MPI_Abort(MPI_COMM_WORLD, 3);
        if (i < first || i >= last) continue;
        x.push_back(p[0]), y.push_back(p[1]), z.push_back(p[2]);
        h.push_back(hm[0]), m.push_back(hm[1]), id.push_back(k);
    }
    std::fclose(in);

    using KeyType = uint64_t;
    using T       = double;
    auto bt       = [](int32_t b) { return static_cast<cstone::BoundaryType>(b); };
    cstone::Box<T> box(lim[0], lim[1], lim[2], lim[3], lim[4], lim[5], bt(bnd[0]), bt(bnd[1]), bt(bnd[2]));

    // the global tree bucket of sphexa.cpp:134-135 and the focus bucket 64 (:133)
    cstone::Domain<KeyType, T> domain(rank, numRanks, bucketSize, 64, theta, box);
    std::vector<KeyType>       keys(x.size());
    // scratch buffers: one of each exchanged element type (f32 h, m; u64 id; f64 coordinates), the last one is the
    // SFC order (sphexa passes its dependent fields, ve_hydro.hpp:118-126)
    std::vector<T>        s1, s2, s3;
    std::vector<float>    sf;
    std::vector<uint64_t> su;
    domain.syncGrav(keys, x, y, z, h, m, std::tie(id), std::tie(s1, s2, sf, su, s3));
    // halo masses: the propagator fills them with m[first] (equal masses, ve_hydro.hpp:145-147); syncGrav moves
    // only x, y, z, h of the halos
    std::fill(m.begin(), m.begin() + domain.startIndex(), m[domain.startIndex()]);
    std::fill(m.begin() + domain.endIndex(), m.end(), m[domain.startIndex()]);

    const auto& focusTree = domain.focusTree();
    const auto  octree    = focusTree.octreeViewAcc();
    std::vector<ryoanji::CartesianQuadrupole<float>> multipoles(octree.numNodes);
    ryoanji::computeGlobalMultipoles(x.data(), y.data(), z.data(), m.data(), x.size(), domain.globalTree(), focusTree,
                                     domain.layout().data(), multipoles.data());

    std::vector<float> ax(x.size(), 0.f), ay(x.size(), 0.f), az(x.size(), 0.f);
    double             egrav = 0;
    ryoanji::computeGravity(octree.childOffsets, octree.internalToLeaf, focusTree.expansionCentersAcc().data(),
                            multipoles.data(), domain.layout().data(), domain.startCell(), domain.endCell(), x.data(),
                            y.data(), z.data(), h.data(), m.data(), domain.box(), G, (double*)nullptr, ax.data(),
                            ay.data(), az.data(), &egrav, 0);
    MPI_Allreduce(MPI_IN_PLACE, &egrav, 1, MPI_DOUBLE, MPI_SUM, MPI_COMM_WORLD);

    const uint64_t nl  = domain.endIndex() - domain.startIndex();
    std::string    out = std::string(argv[2]) + std::to_string(rank) + ".bin";
    FILE*          f   = std::fopen(out.c_str(), "wb");
    std::fwrite(&nl, 8, 1, f);
    std::fwrite(&egrav, 8, 1, f);
    for (uint64_t i = domain.startIndex(); i < domain.endIndex(); ++i)
    {
        std::fwrite(&id[i], 8, 1, f);
        std::fwrite(&ax[i], 4, 1, f);
        std::fwrite(&ay[i], 4, 1, f);
        std::fwrite(&az[i], 4, 1, f);
    }
    std::fclose(f);
    MPI_Finalize();
    return 0;
}
