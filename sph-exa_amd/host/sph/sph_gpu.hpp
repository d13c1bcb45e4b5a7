/*! @file sph_gpu.hpp
 * @brief Drop-in replacement of the reference's GPU seam header sph/include/sph/sph_gpu.hpp.
 *
 * Put sph-exa_amd/host ahead of the reference's sph/include on the include path and every `#include "sph/sph_gpu.hpp"`
 * of the reference (hydro_ve/*.hpp, hydro_std/*.hpp, positions.hpp, groups.hpp, update_h.hpp, ts_rungs.hpp, the
 * propagators) reaches this file: the same cstone includes and using-declarations as the original
 * (sph_gpu.hpp:1-12), then the MI355X definitions of every seam function (sphexa_amd/sph_gpu.hpp) over
 * libsphexa_hip.so instead of the reference's extern templates instantiated in its .cu files.
 * tests/test_mirror_compile.py compiles the reference's HydroVeProp (main/src/propagator/ve_hydro.hpp) with it.
 */
#pragma once

#include "cstone/sfc/box.hpp"
#include "cstone/traversal/groups.hpp"
#include "cstone/tree/octree.hpp"
#include "cstone/tree/definitions.h"
#include "sph/timestep.h"

namespace sph
{
using cstone::GroupData;
using cstone::GroupView;
} // namespace sph

#include "sphexa_amd/sph_gpu.hpp"
