/* Host-side plain-C types shared by the CPU oracle (oracle/sph_oracle.c) and the
 * reference harness (oracle/ref_harness.cpp).
 *
 * TEST INFRASTRUCTURE ONLY: nothing under oracle/ is linked into or called by the
 * product library (sph-exa_amd/).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load these symbols, and only as the checker.
 *
 * Field types follow sph::SphTypes (reference sph/include/sph/types.hpp:39-46):
 * coordinates, temp and du are double; every other hydro field is float.
 */
#ifndef SX_HOST_TYPES_H
#define SX_HOST_TYPES_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Mirrors cstone::Box<double> (reference domain/include/cstone/sfc/box.hpp:111-191).
 * bnd: 0 = open, 1 = periodic, 2 = fixed (cstone::BoundaryType). */
typedef struct ox_box
{
    double  lim[6]; /* xmin xmax ymin ymax zmin zmax */
    int32_t bnd[3];
} ox_box;

/* Physics constants held in ParticlesData (reference particles_data.hpp:86-138). */
typedef struct ox_params
{
    double   K;        /* kernel normalisation (kernel_3D_k, sph_kernel_tables.hpp:78-85) */
    uint32_t ng0;      /* 100 */
    uint32_t ngmax;    /* 150 */
    double   Kcour;    /* 0.2  */
    double   Krho;     /* 0.06 */
    double   gamma;    /* 5/3  */
    float    muiConst; /* 10   */
    float    alphamin, alphamax, decay_constant; /* 0.05, 1.0, 0.2 */
    float    Atmin, Atmax, ramp;                 /* 0.1, 0.2, 1/(Atmax-Atmin) */
    double   maxDtIncrease;                      /* 1.1 */
    int32_t  avClean; /* HydroVeProp<avClean> (ve_hydro.hpp:50): IAD writes dV11..dV33, momentum adds avRvCorrection */
    float    theta;   /* gravity opening parameter (--theta, sphexa.cpp:127: 0.5 with gravity) */
    double   g;       /* gravitational constant (ParticlesData::g, 0 = no self-gravity) */
    double   eps;     /* 0.005 (accelerationTimestep, ts_global.hpp:47-67) */
    double   etaAcc;  /* 0.2 */
    int32_t  prop;    /* ox_step: 0 = VE (HydroVeProp, ve_hydro.hpp), 1 = std (HydroProp, std_hydro.hpp:124-184) */
} ox_params;

/* Host particle state of the VE propagator (ve_hydro.hpp:70-85 conserved + dependent fields). */
typedef struct ox_state
{
    size_t n;
    /* conserved */
    double *x, *y, *z;
    float  *x_m1, *y_m1, *z_m1;
    float  *vx, *vy, *vz;
    double *temp;
    float  *h, *m, *alpha;
    float  *du_m1;
    uint64_t* id; /* particle identity, carried through the SFC reorder (not a reference field) */
    /* dependent */
    double*   du;
    float    *ax, *ay, *az, *prho, *c, *xm, *kx, *gradh, *divv, *curlv;
    float    *c11, *c12, *c13, *c22, *c23, *c33;
    uint32_t* nc;
    uint64_t* keys;
    float    *dV11, *dV12, *dV13, *dV22, *dV23, *dV33; /* velocity gradient (GradVFields), avClean only */
    float    *rho, *p; /* density and pressure of the std propagator (HydroProp DependentFields) */
    /* scalars (ParticlesData members) */
    double minDt, minDt_m1, ttot, minDtCourant, minDtRho;
    double egrav; /* gravitational potential energy of the last step (ParticlesData::egrav) */
} ox_state;

#ifdef __cplusplus
}
#endif

#endif
