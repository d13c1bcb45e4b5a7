/*! @file ewald_ref.cpp
 * @brief TEST INFRASTRUCTURE ONLY (never linked into sph-exa_amd/): the reference's own Ewald periodic-gravity
 *        correction on the CPU, compiled from its header where it lies under $(REF) by oracle/Makefile.
 *
 * ref_gravity_ewald calls ryoanji::computeGravityEwald (ryoanji/src/ryoanji/nbody/ewald.hpp:380-413) with the types
 * of the GPU seam's instantiation (interface/ewald.cu:104: CartesianQuadrupole<float> multipoles, double coordinates,
 * float accelerations and masses, double energy).  It adds G * (real-space + k-space correction) to ax, ay, az and
 * returns 0.5 G sum m_i phi_i.  tests/test_ewald_oracle.py pins the numpy restatement (oracle/ewald.py) to it.
 */
#include "ryoanji/nbody/ewald.hpp"

extern "C" double ref_gravity_ewald(const double* rootCenter, const float* Mroot, unsigned n, const double* x,
                                    const double* y, const double* z, const float* m, double lo, double hi, float G,
                                    int numReplicaShells, double lCut, double hCut, double alphaScale, double smallR,
                                    float* ax, float* ay, float* az)
{
    ryoanji::CartesianQuadrupole<float> M;
    for (int k = 0; k < 8; ++k)
        M[k] = Mroot[k];
    cstone::Box<double> box(lo, hi, cstone::BoundaryType::periodic);
    ryoanji::EwaldSettings s;
    s.numReplicaShells     = numReplicaShells;
    s.lCut                 = lCut;
    s.hCut                 = hCut;
    s.alpha_scale          = alphaScale;
    s.small_R_scale_factor = smallR;
    double utot = 0;
    ryoanji::computeGravityEwald(cstone::Vec3<double>{rootCenter[0], rootCenter[1], rootCenter[2]}, M, 0u, n, x, y, z,
                                 m, box, G, (double*)nullptr, ax, ay, az, &utot, s);
    return utot;
}
