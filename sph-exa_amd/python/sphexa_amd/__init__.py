"""ctypes binding of libsphexa_hip.so (include/sphexa_hip.h) -- the host-side mirror used by tests and bench.

The product is the C-ABI library; this module only marshals plain pointers.  It never falls back to a CPU
path: if the library is missing, importing `lib()` raises.
"""
import ctypes as C
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(os.path.dirname(HERE))          # .../sph-exa_amd
ROOT = os.path.dirname(PKG)
# SPHEXA_AMD_LIB selects another in-tree build of the same library (A/B timing of kernel variants)
LIB_PATH = os.environ.get("SPHEXA_AMD_LIB") or os.path.join(PKG, "lib", "libsphexa_hip.so")
HEADER = os.path.join(ROOT, "include", "sphexa_hip.h")

SX_OK, SX_ERR_TRAVERSAL, SX_ERR_NOT_CONVERGED, SX_ERR_HIP, SX_ERR_ARG, SX_ERR_NOMEM = range(6)
KTABLE = 20000
GROUP = 64


class SxBox(C.Structure):
    _fields_ = [("lim", C.c_double * 6), ("bnd", C.c_int32 * 3)]


class SxParams(C.Structure):
    _fields_ = [("K", C.c_double), ("ng0", C.c_uint32), ("ngmax", C.c_uint32), ("Kcour", C.c_double),
                ("Krho", C.c_double), ("gamma", C.c_double), ("muiConst", C.c_float), ("alphamin", C.c_float),
                ("alphamax", C.c_float), ("decay_constant", C.c_float), ("Atmin", C.c_float),
                ("Atmax", C.c_float), ("ramp", C.c_float), ("maxDtIncrease", C.c_double), ("avClean", C.c_int32),
                ("theta", C.c_float), ("g", C.c_double), ("eps", C.c_double), ("etaAcc", C.c_double),
                ("propagator", C.c_int32)]


_P = C.c_void_p
FIELD_ORDER = [  # sx_fields, ParticlesData order
    ("x", _P), ("y", _P), ("z", _P), ("x_m1", _P), ("y_m1", _P), ("z_m1", _P), ("vx", _P), ("vy", _P), ("vz", _P),
    ("rho", _P), ("u", _P), ("p", _P), ("prho", _P), ("tdpdTrho", _P), ("h", _P), ("m", _P), ("c", _P),
    ("ax", _P), ("ay", _P), ("az", _P), ("du", _P), ("du_m1", _P), ("c11", _P), ("c12", _P), ("c13", _P),
    ("c22", _P), ("c23", _P), ("c33", _P), ("mue", _P), ("mui", _P), ("temp", _P), ("cv", _P), ("xm", _P),
    ("kx", _P), ("divv", _P), ("curlv", _P), ("alpha", _P), ("gradh", _P), ("keys", _P), ("nc", _P),
    ("dV11", _P), ("dV12", _P), ("dV13", _P), ("dV22", _P), ("dV23", _P), ("dV33", _P), ("markRamp", _P),
    ("rung", _P)]


class SxFields(C.Structure):
    _fields_ = [("n", C.c_size_t)] + FIELD_ORDER


class SxTree(C.Structure):
    _fields_ = [("numLeafNodes", C.c_int32), ("numNodes", C.c_int32), ("prefixes", _P), ("childOffsets", _P),
                ("internalToLeaf", _P), ("levelRange", _P), ("leaves", _P), ("layout", _P), ("centers", _P),
                ("sizes", _P), ("searchExtFactor", C.c_float)]


class SxEwaldSettings(C.Structure):
    """sx_ewald_settings (ryoanji::EwaldSettings, nbody/ewald.h:15-22); the reference's defaults"""
    _fields_ = [("numReplicaShells", C.c_int), ("lCut", C.c_double), ("hCut", C.c_double), ("alphaScale", C.c_double),
                ("smallRScaleFactor", C.c_double)]

    def __init__(self, numReplicaShells=1, lCut=2.6, hCut=2.8, alphaScale=2.0, smallRScaleFactor=3.0e-3):
        super().__init__(numReplicaShells, lCut, hCut, alphaScale, smallRScaleFactor)


class SxGroups(C.Structure):
    _fields_ = [("firstBody", C.c_uint32), ("lastBody", C.c_uint32), ("numGroups", C.c_uint32),
                ("groupStart", _P), ("groupEnd", _P)]


class SxTimestep(C.Structure):
    """sph::Timestep (sph/timestep.h:38-48)"""
    _fields_ = [("nextDt", C.c_float), ("elapsedDt", C.c_float), ("totDt", C.c_float), ("numRungs", C.c_int),
                ("substep", C.c_int), ("rungRanges", C.c_uint32 * 5), ("dt_m1", C.c_float * 4),
                ("dt_drift", C.c_float * 4)]


class SxOctree(C.Structure):
    _fields_ = [("prefixes", _P), ("childOffsets", _P), ("parents", _P), ("levelRange", _P),
                ("internalToLeaf", _P), ("leafToInternal", _P)]


class SxNbStats(C.Structure):
    _fields_ = [("sumNeighbors", C.c_uint64), ("maxNeighbors", C.c_uint32), ("numFailed", C.c_uint32),
                ("sumCandidates", C.c_uint64), ("sumUnion", C.c_uint64), ("build", C.c_uint32),
                ("maxUnion", C.c_uint32)]


# field dtypes (sph::SphTypes, sph/types.hpp:39-46)
DTYPES = {k: np.float32 for k, _ in FIELD_ORDER}
DTYPES.update(x=np.float64, y=np.float64, z=np.float64, u=np.float64, du=np.float64, temp=np.float64,
              keys=np.uint64, nc=np.uint32, rung=np.uint8)

_lib = None

# host-staged transport callbacks (sx_alltoallv_cb / sx_allreduce_cb)
ALLTOALLV_CB = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p,
                           C.POINTER(C.c_uint64))
ALLREDUCE_CB = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int)


def header_symbols():
    """every sx_* function declared in include/sphexa_hip.h"""
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sx_[a-z0-9_]+)\s*\(", txt)))


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(f"{LIB_PATH} not built (run __graft_entry__.build() or make -C sph-exa_amd)")
    L = C.CDLL(LIB_PATH)
    vp, i32, u32, sz = C.c_void_p, C.c_int32, C.c_uint32, C.c_size_t
    sig = {
        "sx_create": (C.c_int, [C.POINTER(vp), C.c_int]),
        "sx_destroy": (None, [vp]),
        "sx_set_stream": (C.c_int, [vp, vp]),
        "sx_get_stream": (vp, [vp]),
        "sx_last_error": (C.c_char_p, [vp]),
        "sx_set_exact": (C.c_int, [vp, C.c_int]),
        "sx_kernel_constant": (C.c_double, []),
        "sx_copy_tables": (C.c_int, [vp, vp, vp]),
        "sx_kernel_poly": (C.c_int, [vp, C.c_size_t, vp, vp]),
        "sx_synchronize": (C.c_int, [vp]),
        "sx_device_alloc": (vp, [vp, sz]),
        "sx_device_free": (C.c_int, [vp, vp]),
        "sx_memcpy": (C.c_int, [vp, vp, vp, sz, C.c_int]),
        "sx_memset": (C.c_int, [vp, vp, C.c_int, sz]),
        "sx_sfc_keys": (C.c_int, [vp, vp, vp, vp, vp, sz, C.POINTER(SxBox)]),
        "sx_sort_keys": (C.c_int, [vp, vp, vp, sz]),
        "sx_gather": (C.c_int, [vp, vp, sz, vp, vp, C.c_int]),
        "sx_compute_octree": (C.c_int, [vp, vp, sz, u32, vp, vp, i32, C.POINTER(i32)]),
        "sx_build_octree": (C.c_int, [vp, vp, i32, C.POINTER(SxOctree)]),
        "sx_node_centers": (C.c_int, [vp, vp, i32, C.POINTER(SxBox), vp, vp]),
        "sx_leaf_layout": (C.c_int, [vp, vp, i32, vp]),
        "sx_compute_groups": (C.c_int, [vp, u32, u32, C.POINTER(SxGroups)]),
        "sx_set_search_mode": (C.c_int, [vp, C.c_int]),
        "sx_mark_ramp": (C.c_int, [vp, C.POINTER(SxGroups), C.POINTER(SxFields), C.POINTER(SxParams),
                                   C.POINTER(SxBox), vp]),
        "sx_positions_rungs": (C.c_int, [vp, C.POINTER(SxGroups), C.c_float, vp, vp, C.POINTER(SxFields), C.c_double,
                                         C.c_double, C.POINTER(SxBox)]),
        "sx_drift_positions": (C.c_int, [vp, C.POINTER(SxGroups), C.c_float, C.c_float, vp, vp, C.POINTER(SxFields),
                                         C.c_double, C.c_double]),
        "sx_group_divv_timestep": (C.c_int, [vp, C.c_float, C.POINTER(SxGroups), vp, vp]),
        "sx_group_acc_timestep": (C.c_int, [vp, C.c_float, C.POINTER(SxGroups), vp, vp, vp, vp]),
        "sx_store_rung": (C.c_int, [vp, C.POINTER(SxGroups), C.c_uint8, vp]),
        "sx_rung_timestep": (C.c_int, [vp, vp, vp, u32, C.c_float, vp, C.POINTER(SxTimestep)]),
        "sx_minimum_group_dt": (C.c_int, [vp, C.POINTER(SxTimestep), vp, vp, u32, vp, C.POINTER(C.c_float), vp]),
        "sx_extract_groups": (C.c_int, [vp, C.POINTER(SxGroups), vp, u32, u32, vp, vp]),
        "sx_spatial_groups": (C.c_int, [vp, u32, u32, vp, vp, vp, C.POINTER(SxTree), C.POINTER(SxBox), C.c_float,
                                        vp, u32, C.POINTER(SxGroups)]),
        "sx_find_neighbors": (C.c_int, [vp, C.POINTER(SxFields), C.POINTER(SxTree), C.POINTER(SxBox),
                                        C.POINTER(SxParams), u32, u32, C.c_int, C.POINTER(SxNbStats)]),
        "sx_export_neighbors": (C.c_int, [vp, vp, u32, u32, u32, vp]),
        "sx_import_neighbors": (C.c_int, [vp, u32, u32, u32, vp]),
        "sx_xmass": (C.c_int, [vp, C.POINTER(SxGroups), C.POINTER(SxFields), C.POINTER(SxParams), C.POINTER(SxBox),
                               C.POINTER(SxTree)]),
        "sx_xmass_only": (C.c_int, [vp, C.POINTER(SxGroups), C.POINTER(SxFields), C.POINTER(SxParams),
                                    C.POINTER(SxBox)]),
        "sx_ve_def_gradh": (C.c_int, [vp, C.POINTER(SxGroups), C.POINTER(SxFields), C.POINTER(SxParams),
                                      C.POINTER(SxBox)]),
        "sx_eos": (C.c_int, [vp, u32, u32, C.c_float, C.c_double, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "sx_iad_divv_curlv": (C.c_int, [vp, C.POINTER(SxGroups), C.POINTER(SxFields), C.POINTER(SxParams),
                                        C.POINTER(SxBox)]),
        "sx_av_switches": (C.c_int, [vp, C.POINTER(SxGroups), C.POINTER(SxFields), C.POINTER(SxParams),
                                     C.POINTER(SxBox), C.c_double]),
        "sx_momentum_energy": (C.c_int, [vp, C.POINTER(SxGroups), vp, C.POINTER(SxFields), C.POINTER(SxParams),
                                         C.POINTER(SxBox), C.POINTER(C.c_float)]),
        "sx_momentum_energy_avclean": (C.c_int, [vp, C.POINTER(SxGroups), vp, C.POINTER(SxFields),
                                                 C.POINTER(SxParams), C.POINTER(SxBox), C.POINTER(C.c_float)]),
        "sx_density": (C.c_int, [vp, C.POINTER(SxGroups), C.POINTER(SxFields), C.POINTER(SxParams),
                                 C.POINTER(SxBox), C.POINTER(SxTree)]),
        "sx_density_only": (C.c_int, [vp, C.POINTER(SxGroups), C.POINTER(SxFields), C.POINTER(SxParams),
                                      C.POINTER(SxBox)]),
        "sx_eos_std": (C.c_int, [vp, u32, u32, C.c_float, C.c_double, vp, vp, vp, vp, vp]),
        "sx_iad": (C.c_int, [vp, C.POINTER(SxGroups), C.POINTER(SxFields), C.POINTER(SxParams), C.POINTER(SxBox)]),
        "sx_momentum_energy_std": (C.c_int, [vp, C.POINTER(SxGroups), C.POINTER(SxFields), C.POINTER(SxParams),
                                             C.POINTER(SxBox), C.POINTER(C.c_float)]),
        "sx_positions": (C.c_int, [vp, u32, u32, C.c_double, C.c_double, C.POINTER(SxFields), C.c_double,
                                   C.c_float, C.POINTER(SxBox)]),
        "sx_update_h": (C.c_int, [vp, u32, u32, u32, vp, vp]),
        "sx_update_h_groups": (C.c_int, [vp, vp, u32, vp, vp]),
        "sx_max_divv": (C.c_int, [vp, u32, u32, vp, C.POINTER(C.c_float)]),
        "sx_sim_create": (C.c_int, [C.POINTER(vp), vp, sz, C.POINTER(SxParams), C.POINTER(SxBox), u32]),
        "sx_sim_destroy": (None, [vp]),
        "sx_sim_init_sedov": (C.c_int, [vp, u32]),
        "sx_sim_set_state": (C.c_int, [vp, sz] + [vp] * 15 + [C.c_double, C.c_double]),
        "sx_sim_fields": (C.c_int, [vp, C.POINTER(SxFields), C.POINTER(vp)]),
        "sx_sim_size": (sz, [vp]),
        "sx_sim_step": (C.c_int, [vp]),
        "sx_sim_scalars": (C.c_int, [vp, C.POINTER(C.c_double)]),
        "sx_sim_stage_times": (C.c_int, [vp, C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_char_p)]),
        "sx_sim_last_stats": (C.c_int, [vp, C.POINTER(SxNbStats)]),
        "sx_sim_kernel_times": (C.c_int, [vp, C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_char_p)]),
        "sx_sim_set_comm": (C.c_int, [vp, vp]),
        "sx_sim_gravity_stats": (C.c_int, [vp, C.POINTER(C.c_uint64)]),
        "sx_sim_gravity_interactions": (C.c_int, [vp, C.POINTER(C.c_uint64)]),
        "sx_sim_set_gravity_counting": (C.c_int, [vp, C.c_int]),
        "sx_sim_conserved": (C.c_int, [vp, C.POINTER(C.c_double)]),
        "sx_conserved_quantities": (C.c_int, [vp, C.POINTER(SxFields), u32, u32, C.c_float, C.c_double,
                                              C.POINTER(C.c_double)]),
        "sx_sim_init_sedov_rank": (C.c_int, [vp, u32, C.c_int, C.c_int]),
        "sx_sim_layout": (C.c_int, [vp, C.POINTER(C.c_uint64)]),
        "sx_sim_set_overlap": (C.c_int, [vp, C.c_int]),
        "sx_sim_overlap_stats": (C.c_int, [vp, C.POINTER(C.c_uint32)]),
        "sx_sim_timestep": (C.c_int, [vp, C.POINTER(SxTimestep)]),
        "sx_sim_set_timestep": (C.c_int, [vp, C.POINTER(SxTimestep), vp]),
        "sx_sim_set_time": (C.c_int, [vp, C.c_double]),
        "sx_sim_set_skin": (C.c_int, [vp, C.c_float, C.c_int]),
        "sx_sim_rebuild_lists": (C.c_int, [vp]),
        "sx_sim_skin_stats": (C.c_int, [vp, C.POINTER(C.c_uint64)]),
        "sx_sim_export_neighbors": (C.c_int, [vp, vp]),
        "sx_comm_unique_id": (C.c_int, [vp]),
        "sx_comm_create_rccl": (C.c_int, [C.POINTER(vp), C.c_int, C.c_int, vp]),
        "sx_comm_create_host": (C.c_int, [C.POINTER(vp), C.c_int, C.c_int, ALLTOALLV_CB, ALLREDUCE_CB, vp]),
        "sx_comm_destroy": (None, [vp]),
        "sx_comm_alltoallv": (C.c_int, [vp, vp, vp, vp, vp, vp, vp, vp]),
        "sx_comm_allreduce": (C.c_int, [vp, vp, C.c_uint64, C.c_int, vp]),
        "sx_domain_splitters": (C.c_int, [vp, u32, C.c_int, vp]),
        "sx_gravity_upsweep": (C.c_int, [vp, C.POINTER(SxFields), C.POINTER(SxTree), C.c_float, vp, vp]),
        "sx_gravity_traverse": (C.c_int, [vp, C.POINTER(SxGroups), C.POINTER(SxFields), C.POINTER(SxTree),
                                          C.POINTER(SxBox), vp, vp, C.c_float, C.POINTER(C.c_double)]),
        "sx_gravity_traverse_pbc": (C.c_int, [vp, C.POINTER(SxGroups), C.POINTER(SxFields), C.POINTER(SxTree),
                                              C.POINTER(SxBox), vp, vp, C.c_float, C.c_int, C.POINTER(C.c_double)]),
        "sx_gravity_ewald": (C.c_int, [vp, C.POINTER(SxGroups), C.POINTER(SxFields), C.POINTER(SxBox), vp, vp,
                                       C.c_float, C.POINTER(SxEwaldSettings), C.POINTER(C.c_double)]),
        "sx_domain_halo_layout": (C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, vp, vp]),
    }
    for name, (res, args) in sig.items():
        # a measurement build named by SPHEXA_AMD_LIB (an A/B against an older library) may predate an entry
        if os.environ.get("SPHEXA_AMD_LIB") and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def domain_splitters(hist, hist_bits, nranks):
    """equal-count SFC splitters (nranks+1 keys) from an all-reduced key histogram (sx_domain_splitters)"""
    h = np.ascontiguousarray(hist, dtype=np.uint32)
    if h.size != 1 << hist_bits:
        raise ValueError("histogram size must be 2^hist_bits")
    out = np.zeros(nranks + 1, np.uint64)
    rc = lib().sx_domain_splitters(h.ctypes.data, hist_bits, nranks, out.ctypes.data)
    if rc != SX_OK:
        raise SxError(f"sx_domain_splitters failed: {rc}")
    return out


def halo_layout(recv_counts, rank, num_local):
    """halo receive offsets [lower ranks | locals | higher ranks] and (first, last, total) (sx_domain_halo_layout)"""
    rc_ = np.ascontiguousarray(recv_counts, dtype=np.uint64)
    off = np.zeros(rc_.size, np.uint64)
    out = np.zeros(3, np.uint64)
    rc = lib().sx_domain_halo_layout(rc_.ctypes.data, rc_.size, rank, num_local, off.ctypes.data, out.ctypes.data)
    if rc != SX_OK:
        raise SxError(f"sx_domain_halo_layout failed: {rc}")
    return off, tuple(int(v) for v in out)


def default_params(K=None, ngmax=150, ng0=100, av_clean=False, g=0.0, theta=0.5, std=False, bdt=False):
    """ParticlesData defaults (particles_data.hpp:86-138); av_clean selects HydroVeProp<true> (with bdt:
    HydroVeBdtProp<true>), std the std propagator (HydroProp) and bdt the block time-step VE propagator
    (HydroVeBdtProp, one substep per step) in sx_sim."""
    if std and bdt:
        raise ValueError("std and bdt are different propagators")
    if K is None:
        K = lib().sx_kernel_constant()
    return SxParams(K=K, ng0=ng0, ngmax=ngmax, Kcour=0.2, Krho=0.06, gamma=5.0 / 3.0, muiConst=10.0, alphamin=0.05,
                    alphamax=1.0, decay_constant=0.2, Atmin=0.1, Atmax=0.2,
                    ramp=float(np.float32(1.0) / (np.float32(0.2) - np.float32(0.1))), maxDtIncrease=1.1,
                    avClean=1 if av_clean else 0, theta=theta, g=g, eps=0.005, etaAcc=0.2,
                    propagator=1 if std else (2 if bdt else 0))


def make_box(lim, bnd):
    b = SxBox()
    for k in range(6):
        b.lim[k] = float(lim[k])
    for k in range(3):
        b.bnd[k] = int(bnd[k])
    return b


# the step attributes of a restart file, in the order ParticlesData::loadOrStoreAttributes writes them
# (particles_data.hpp:170-190) followed by Box::loadOrStore (box.hpp:170-171)
ATTRIBUTE_NAMES = ["iteration", "numParticlesGlobal", "ng0", "ngmax", "time", "minDt", "minDt_m1", "Kcour", "Krho",
                   "gravConstant", "gamma", "eps", "etaAcc", "muiConst", "alphamin", "alphamax", "decay_constant",
                   "sincIndex", "kernelChoice", "box", "boundaryType"]


def reference_attributes(params, box, scalars, iteration, num_particles_global):
    """the reference's restart attributes with the reference's types (size_t/uint64 counters, double scalars, float
    muiConst/alpha parameters, int kernel choice, 6 box limits, 3 boundary-type chars)"""
    p = params
    return {
        "iteration": np.uint64(iteration), "numParticlesGlobal": np.uint64(num_particles_global),
        "ng0": np.uint32(p.ng0), "ngmax": np.uint32(p.ngmax), "time": np.float64(scalars["ttot"]),
        "minDt": np.float64(scalars["minDt"]), "minDt_m1": np.float64(scalars["minDt_m1"]),
        "Kcour": np.float64(p.Kcour), "Krho": np.float64(p.Krho), "gravConstant": np.float64(p.g),
        "gamma": np.float64(p.gamma), "eps": np.float64(p.eps), "etaAcc": np.float64(p.etaAcc),
        "muiConst": np.float32(p.muiConst), "alphamin": np.float32(p.alphamin), "alphamax": np.float32(p.alphamax),
        "decay_constant": np.float32(p.decay_constant), "sincIndex": np.float64(6.0),  # sinc_6, the kernel tabulated
        "kernelChoice": np.int32(0),  # SphKernelType::sinc_n
        "box": np.array([box.lim[k] for k in range(6)], dtype=np.float64),
        "boundaryType": np.array([box.bnd[k] for k in range(3)], dtype=np.int8),
    }


class SxError(RuntimeError):
    pass


class Context:
    def __init__(self, device=0, exact=False):
        self.L = lib()
        self.h = C.c_void_p()
        rc = self.L.sx_create(C.byref(self.h), device)
        self.check(rc, "sx_create")
        self.L.sx_set_exact(self.h, 1 if exact else 0)
        self.allocs = []

    def check(self, rc, what=""):
        if rc != SX_OK:
            msg = self.L.sx_last_error(self.h) if self.h else b"?"
            raise SxError(f"{what}: code {rc}: {msg.decode() if msg else ''}")

    def set_exact(self, exact):
        self.L.sx_set_exact(self.h, 1 if exact else 0)

    # ---- device arrays --------------------------------------------------------------------------------------
    def alloc(self, n, dtype):
        nbytes = int(n) * np.dtype(dtype).itemsize
        p = self.L.sx_device_alloc(self.h, nbytes)
        if not p:
            raise SxError("device alloc failed")
        self.allocs.append(p)
        return DeviceArray(self, p, int(n), dtype)

    def upload(self, arr):
        arr = np.ascontiguousarray(arr)
        d = self.alloc(arr.size, arr.dtype)
        self.check(self.L.sx_memcpy(self.h, d.ptr, arr.ctypes.data, arr.nbytes, 1), "upload")
        return d

    def free(self, arr):
        """release one DeviceArray of alloc/upload"""
        if arr.ptr in self.allocs:
            self.allocs.remove(arr.ptr)
            self.L.sx_device_free(self.h, arr.ptr)

    def free_all(self):
        for p in self.allocs:
            self.L.sx_device_free(self.h, p)
        self.allocs = []

    def close(self):
        self.free_all()
        if self.h:
            self.L.sx_destroy(self.h)
            self.h = None

    def sync(self):
        self.check(self.L.sx_synchronize(self.h), "sync")


class DeviceArray:
    def __init__(self, ctx, ptr, n, dtype):
        self.ctx, self.ptr, self.n, self.dtype = ctx, ptr, n, np.dtype(dtype)

    def get(self):
        out = np.empty(self.n, self.dtype)
        self.ctx.check(self.ctx.L.sx_memcpy(self.ctx.h, out.ctypes.data, self.ptr, out.nbytes, 2), "download")
        return out

    def set(self, arr):
        arr = np.ascontiguousarray(arr, dtype=self.dtype)
        assert arr.size == self.n
        self.ctx.check(self.ctx.L.sx_memcpy(self.ctx.h, self.ptr, arr.ctypes.data, arr.nbytes, 1), "upload")


class DeviceState:
    """A full ParticlesData-like device field set built from a host dict of numpy arrays."""

    def __init__(self, ctx, host, grad_v=False, std=False):
        """grad_v: also allocate the velocity gradient dV11..dV33 (GradVFields of the avClean propagator);
        std: also allocate rho and p (DependentFields of the std propagator, std_hydro.hpp:78-79)"""
        self.ctx = ctx
        n = len(host["x"])
        self.n = n
        self.dev = {}
        self.fields = SxFields()
        self.fields.n = n
        grad = ("dV11", "dV12", "dV13", "dV22", "dV23", "dV33")
        for name, _ in FIELD_ORDER:
            if name in ("tdpdTrho", "u", "mue", "mui", "cv", "markRamp", "rung") or \
                    (name in grad and not grad_v) or (name in ("rho", "p") and not std):
                continue
            dt = DTYPES[name]
            if name in host:
                d = ctx.upload(np.asarray(host[name], dtype=dt))
            else:
                d = ctx.alloc(n, dt)
                ctx.L.sx_memset(ctx.h, d.ptr, 0, n * np.dtype(dt).itemsize)
            self.dev[name] = d
            setattr(self.fields, name, d.ptr)

    def get(self, name):
        return self.dev[name].get()

    def set(self, name, arr):
        self.dev[name].set(arr)


class Comm:
    """Inter-GPU transport. backend 'rccl' (RCCL over xGMI, production) or 'host' (staged through host memory and
    torch.distributed -- used to run several ranks on one GPU in tests). torch.distributed must be initialised
    (gloo) by the caller; it is only the control plane (unique-id broadcast) for 'rccl'."""

    def __init__(self, backend="rccl"):
        import torch
        import torch.distributed as dist

        self.L = lib()
        self.rank, self.size = dist.get_rank(), dist.get_world_size()
        self.h = C.c_void_p()
        if backend == "rccl":
            uid = (C.c_uint8 * 128)()
            if self.rank == 0:
                rc = self.L.sx_comm_unique_id(uid)
                if rc != SX_OK:
                    raise SxError("ncclGetUniqueId failed")
            t = torch.tensor(list(uid), dtype=torch.uint8)
            dist.broadcast(t, 0)
            for k in range(128):
                uid[k] = int(t[k])
            rc = self.L.sx_comm_create_rccl(C.byref(self.h), self.rank, self.size, uid)
        else:
            def a2a(user, send, sendBytes, recv, recvBytes):
                try:
                    sb = [int(sendBytes[q]) for q in range(self.size)]
                    rb = [int(recvBytes[q]) for q in range(self.size)]
                    src = np.ctypeslib.as_array((C.c_uint8 * max(1, sum(sb))).from_address(send)) if sum(sb) else \
                        np.zeros(1, np.uint8)
                    out = torch.empty(sum(rb), dtype=torch.uint8)
                    dist.all_to_all_single(out, torch.from_numpy(src[:sum(sb)].copy()), rb, sb)
                    if sum(rb):
                        C.memmove(recv, out.numpy().ctypes.data, sum(rb))
                    return 0
                except Exception as e:  # noqa: BLE001 -- report through the return code
                    print("alltoallv callback failed:", e)
                    return 1

            def allreduce(user, buf, count, op):
                try:
                    if op in (0, 3, 4):  # u32 sum, min, max
                        a = np.ctypeslib.as_array((C.c_uint32 * count).from_address(buf))
                        t = torch.from_numpy(a.astype(np.int64))
                        dist.all_reduce(t, op={0: dist.ReduceOp.SUM, 3: dist.ReduceOp.MIN, 4: dist.ReduceOp.MAX}[op])
                        a[:] = t.numpy().astype(np.uint32)
                    else:
                        a = np.ctypeslib.as_array((C.c_double * count).from_address(buf))
                        t = torch.from_numpy(a.copy())
                        dist.all_reduce(t, op=dist.ReduceOp.MIN if op == 1 else dist.ReduceOp.SUM)
                        a[:] = t.numpy()
                    return 0
                except Exception as e:  # noqa: BLE001
                    print("allreduce callback failed:", e)
                    return 1

            self._cbs = (ALLTOALLV_CB(a2a), ALLREDUCE_CB(allreduce))
            rc = self.L.sx_comm_create_host(C.byref(self.h), self.rank, self.size, self._cbs[0], self._cbs[1], None)
        if rc != SX_OK:
            raise SxError(f"communicator creation failed ({backend}): {rc}")

    def alltoallv(self, send, send_bytes, send_off, recv, recv_bytes, recv_off, stream=None):
        """sx_comm_alltoallv on device pointers (byte counts / offsets per rank); enqueued on `stream`"""
        arr = [np.ascontiguousarray(a, dtype=np.uint64) for a in (send_bytes, send_off, recv_bytes, recv_off)]
        if any(a.size != self.size for a in arr):
            raise ValueError("alltoallv: one count and one offset per rank")
        rc = self.L.sx_comm_alltoallv(self.h, send, arr[0].ctypes.data, arr[1].ctypes.data, recv, arr[2].ctypes.data,
                                      arr[3].ctypes.data, stream)
        if rc != SX_OK:
            raise SxError(f"sx_comm_alltoallv failed: {rc}")

    ALLREDUCE_OPS = {"sum_u32": 0, "min_f64": 1, "sum_f64": 2, "min_u32": 3, "max_u32": 4}

    def allreduce(self, dev, count, op, stream=None):
        """sx_comm_allreduce in place on a device buffer: op 'sum_u32', 'min_f64' or 'sum_f64'"""
        rc = self.L.sx_comm_allreduce(self.h, dev, int(count), self.ALLREDUCE_OPS[op], stream)
        if rc != SX_OK:
            raise SxError(f"sx_comm_allreduce failed: {rc}")

    def close(self):
        if self.h:
            self.L.sx_comm_destroy(self.h)
            self.h = None


class Sim:
    """device-resident VE propagator on one GPU (sx_sim_*)"""

    def __init__(self, ctx, capacity, box, params=None, bucket=64):
        self.ctx = ctx
        self.L = ctx.L
        self.params = params or default_params()
        self.box = box
        self.iteration = 0  # completed steps (the reference's "iteration" attribute)
        self.h = C.c_void_p()
        ctx.check(self.L.sx_sim_create(C.byref(self.h), ctx.h, int(capacity), C.byref(self.params), C.byref(box),
                                       bucket), "sx_sim_create")

    def init_sedov(self, side, rank=0, size=1):
        self.ctx.check(self.L.sx_sim_init_sedov_rank(self.h, side, rank, size), "init_sedov")

    def set_comm(self, comm):
        self.comm = comm
        self.ctx.check(self.L.sx_sim_set_comm(self.h, comm.h), "set_comm")

    def set_overlap(self, on):
        self.ctx.check(self.L.sx_sim_set_overlap(self.h, int(bool(on))), "set_overlap")

    def overlap_stats(self):
        out = (C.c_uint32 * 2)()
        self.L.sx_sim_overlap_stats(self.h, out)
        return dict(interior=out[0], boundary=out[1])

    def layout(self):
        out = (C.c_uint64 * 4)()
        self.L.sx_sim_layout(self.h, out)
        return dict(first=out[0], last=out[1], n=out[2], haloRetries=out[3])

    def set_state(self, st, minDt=1e-6, minDt_m1=1e-6):
        arrs = [np.ascontiguousarray(st[k], dtype=t) for k, t in [
            ("x", np.float64), ("y", np.float64), ("z", np.float64), ("h", np.float32), ("m", np.float32),
            ("temp", np.float64), ("vx", np.float32), ("vy", np.float32), ("vz", np.float32), ("x_m1", np.float32),
            ("y_m1", np.float32), ("z_m1", np.float32), ("du_m1", np.float32), ("alpha", np.float32),
            ("id", np.uint64)]]
        self._keep = arrs
        self.ctx.check(self.L.sx_sim_set_state(self.h, arrs[0].size, *[a.ctypes.data for a in arrs],
                                               float(minDt), float(minDt_m1)), "set_state")

    CONSERVED = ["x", "y", "z", "h", "m", "temp", "vx", "vy", "vz", "x_m1", "y_m1", "z_m1", "du_m1", "alpha", "id"]

    def save_checkpoint(self, path, num_particles_global=None):
        """restart file of this rank: the conserved fields under the reference's field names
        (ParticlesData::fieldNames, particles_data.hpp:247-251; the set HydroVeProp restarts from,
        ve_hydro.hpp:74 + x,y,z,h,m) and the step attributes under the reference's names
        (reference_attributes: ParticlesData::loadOrStoreAttributes, particles_data.hpp:142-193, and
        Box::loadOrStore, box.hpp:168-175).  A path ending in ".h5" appends a step to an H5Part-layout file (the
        reference's format, sphexa_amd.h5part over the image's serial HDF5); any other path writes an .npz."""
        bdt = self.params.propagator == 2
        if bdt:
            ts = self.timestep()
            if not self._hierarchy_boundary(ts):
                # the reference writes files only when isSynced() (sphexa.cpp:165): inside a block time-step hierarchy
                # the state is not restartable (drifted inactive rungs, halo lists of the hierarchy's sync)
                raise ValueError(f"ve-bdt checkpoint inside a time-step hierarchy (substep {ts['substep']} of "
                                 f"{1 << (ts['numRungs'] - 1)}): save after the hierarchy's last substep")
        st = self.get(self.CONSERVED + (["rung"] if bdt else []))
        # a run restarted from this file begins with a full sync + neighbor build; so does this one's next step, so
        # the two take identical steps (skin lists, sx_sim_rebuild_lists)
        self.rebuild_lists()
        if num_particles_global is None:
            num_particles_global = self.size()
            comm = getattr(self, "comm", None)
            if comm is not None and comm.size > 1:  # numParticlesGlobal is the sum over the ranks
                import torch
                import torch.distributed as dist

                t = torch.tensor([num_particles_global], dtype=torch.int64)
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
                num_particles_global = int(t.item())
        attrs = reference_attributes(self.params, self.box, self.scalars(), self.iteration, num_particles_global)
        if bdt:  # Timestep::loadOrStore(writer, "ts::") (sph/timestep.h:29-33, HydroVeBdtProp::save)
            attrs["ts::numRungs"] = np.int32(ts["numRungs"])
            attrs["ts::dt_m1"] = np.array(ts["dt_m1"], dtype=np.float32)
        if str(path).endswith(".h5"):
            from . import h5part

            h5part.write_step(path, st, attrs, mode="a")
        else:
            np.savez(path, **st, **attrs)

    @staticmethod
    def _hierarchy_boundary(ts):
        """HydroVeBdtProp::isSynced (ve_hydro_bdt.hpp:108-112, :220) for the NEXT substep"""
        return ts["substep"] == 0 or ts["substep"] >= (1 << (ts["numRungs"] - 1))

    # attributes ParticlesData::loadOrStoreAttributes restores (particles_data.hpp:170-190) that are parameters of
    # this Sim (fixed at sx_sim_create): a restart must run with the stored values
    PARAM_ATTRIBUTES = ["ng0", "ngmax", "Kcour", "Krho", "gravConstant", "gamma", "eps", "etaAcc", "muiConst",
                        "alphamin", "alphamax", "decay_constant"]

    def _read_checkpoint(self, path, step):
        """{name: array or scalar} of a restart file: the conserved fields (+ rung), and the attributes present"""
        mine = reference_attributes(self.params, self.box, {"ttot": 0.0, "minDt": 0.0, "minDt_m1": 0.0}, 0, 0)
        if str(path).endswith(".h5"):
            from . import h5part

            names = self.CONSERVED + (["rung"] if self.params.propagator == 2 else [])
            with h5part.H5PartFile(path, "r") as f:
                f.set_step(step)
                present = set(f.attrib_names())
                fields = {k: f.read_field(k, DTYPES.get(k, np.uint64)) for k in names if f.field_info(k) is not None}
            types = {k: np.asarray(v).dtype for k, v in mine.items()}
            types.update({"ts::numRungs": np.int32, "ts::dt_m1": np.float32, "ttot": np.float64})
            _, attrs = h5part.read_step(path, {}, {k: t for k, t in types.items() if k in present}, step)
            return {**fields, **attrs}
        with np.load(path, allow_pickle=False) as d:
            return {k: d[k] for k in d.files}

    def load_checkpoint(self, path, step=-1):
        """continue from save_checkpoint's file (.h5: its step `step`, negative = the last, as the reference's
        --init file.h5:step; .npz: the one state): set_state with the saved fields and time-steps; returns the time.
        The stored parameters must equal this Sim's (ValueError otherwise: the reference would load them, a Sim's
        parameters are fixed at creation).  Files of the earlier format (time under 'ttot', no 'iteration') load
        with iteration 0."""
        d = self._read_checkpoint(path, step)
        mine = reference_attributes(self.params, self.box, {"ttot": 0.0, "minDt": 0.0, "minDt_m1": 0.0}, 0, 0)
        bad = [k for k in self.PARAM_ATTRIBUTES if k in d and d[k] != mine[k]]
        if bad:
            raise ValueError("restart file parameters differ from this Sim's: " +
                             ", ".join(f"{k}={d[k]!r} (Sim: {mine[k]!r})" for k in bad))
        st = {k: d[k] for k in self.CONSERVED}
        self.set_state(st, float(d["minDt"]), float(d["minDt_m1"]))
        if self.params.propagator == 2 and "ts::numRungs" in d:
            # HydroVeBdtProp::load (ve_hydro_bdt.hpp:155-168): Timestep numRungs + dt_m1, substep 0, and the rungs
            if "rung" not in d:
                raise ValueError("restart file has ts::numRungs but no 'rung' field")
            rung = np.ascontiguousarray(d["rung"], dtype=np.uint8)
            if rung.shape != (len(st["x"]),):
                raise ValueError(f"restart file's 'rung' has {rung.size} entries for {len(st['x'])} particles")
            ts = SxTimestep()
            ts.numRungs = int(d["ts::numRungs"])
            for k, v in enumerate(np.asarray(d["ts::dt_m1"], np.float32)):
                ts.dt_m1[k] = float(v)
            self._keep_rung = rung
            self.ctx.check(self.L.sx_sim_set_timestep(self.h, C.byref(ts), rung.ctypes.data), "set_timestep")
        self.iteration = int(d["iteration"]) if "iteration" in d else 0
        t = float(d["time"] if "time" in d else d["ttot"])
        self.ctx.check(self.L.sx_sim_set_time(self.h, t), "set_time")
        return t

    def set_skin(self, factor=0.05, max_reuse=24):
        """neighbor lists behind a skin of relative width `factor` (sx_sim_set_skin; 0: sync + search every step)"""
        self.ctx.check(self.L.sx_sim_set_skin(self.h, float(factor), int(max_reuse)), "set_skin")

    def rebuild_lists(self):
        """the next step does a full sync + build of every skin (sx_sim_rebuild_lists)"""
        self.ctx.check(self.L.sx_sim_rebuild_lists(self.h), "rebuild_lists")

    def skin_stats(self):
        out = (C.c_uint64 * 14)()
        self.ctx.check(self.L.sx_sim_skin_stats(self.h, out), "skin_stats")
        d = dict(zip(["builds", "reuse_steps", "stale_clusters", "exact_clusters", "last_stale", "last_exact",
                      "capacity", "plain_steps"], list(out)[:8]))
        d["factor"], d["next_factor"] = out[8] * 1e-6, out[9] * 1e-6
        d["resyncs"] = out[10]
        d["kept_clusters"] = out[11]
        d["frozen_clusters"] = out[12]
        d["early_exact"] = out[13]
        return d

    def neighbor_sets(self):
        """the last step's neighbor lists as {particle id: sorted array of neighbor ids} (sx_sim_export_neighbors)"""
        n = self.size()
        ngmax = int(self.params.ngmax)
        buf = self.ctx.alloc(max(1, n * ngmax), np.uint32)
        try:
            self.ctx.check(self.L.sx_sim_export_neighbors(self.h, buf.ptr), "export_neighbors")
            rows = buf.get()[: n * ngmax].reshape(n, ngmax)
        finally:
            self.ctx.free(buf)
        g = self.get(["id", "nc"])
        ids, nc = g["id"], g["nc"].astype(np.int64)
        return {int(ids[i]): np.sort(ids[rows[i, : min(nc[i] - 1, ngmax)]]) for i in range(n)}

    def step(self):
        rc = self.L.sx_sim_step(self.h)
        if rc != SX_OK:
            raise SxError(f"sx_sim_step failed with code {rc}")
        self.iteration += 1

    def size(self):
        return self.L.sx_sim_size(self.h)

    def scalars(self):
        out = (C.c_double * 6)()
        self.ctx.check(self.L.sx_sim_scalars(self.h, out), "scalars")
        return dict(zip(["minDt", "minDt_m1", "ttot", "minDtCourant", "minDtRho", "egrav"], list(out)))

    def fields(self):
        f = SxFields()
        idp = C.c_void_p()
        self.L.sx_sim_fields(self.h, C.byref(f), C.byref(idp))
        return f, idp.value

    def get(self, names):
        f, idp = self.fields()
        n = self.size()
        out = {}
        for name in names:
            ptr = idp if name == "id" else getattr(f, name)
            dt = np.uint64 if name == "id" else DTYPES[name]
            out[name] = DeviceArray(self.ctx, ptr, n, dt).get()
        return out

    def stage_times(self):
        ms = (C.c_float * 16)()
        names = (C.c_char_p * 16)()
        k = self.L.sx_sim_stage_times(self.h, ms, 16, names)
        return {names[i].decode(): ms[i] for i in range(k)}

    def kernel_times(self):
        ms = (C.c_float * 16)()
        names = (C.c_char_p * 16)()
        k = self.L.sx_sim_kernel_times(self.h, ms, 16, names)
        return {names[i].decode(): ms[i] for i in range(k)}

    def stats(self):
        s = SxNbStats()
        self.L.sx_sim_last_stats(self.h, C.byref(s))
        return dict(sumNeighbors=s.sumNeighbors, maxNeighbors=s.maxNeighbors, numFailed=s.numFailed,
                    sumCandidates=s.sumCandidates, sumUnion=s.sumUnion, build=s.build, maxUnion=s.maxUnion)

    def conserved(self):
        """computeConservedQuantities over all ranks (sx_sim_conserved)"""
        out = (C.c_double * 13)()
        self.ctx.check(self.L.sx_sim_conserved(self.h, out), "conserved")
        names = ["ecin", "eint", "egrav", "etot", "linmom", "angmom", "totalNeighbors", "px", "py", "pz", "Lx", "Ly",
                 "Lz"]
        return dict(zip(names, list(out)))

    def timestep(self):
        """ve-bdt: the Timestep after the last substep (sx_sim_timestep)"""
        ts = SxTimestep()
        self.ctx.check(self.L.sx_sim_timestep(self.h, C.byref(ts)), "timestep")
        return dict(nextDt=ts.nextDt, elapsedDt=ts.elapsedDt, totDt=ts.totDt, numRungs=ts.numRungs,
                    substep=ts.substep, rungRanges=list(ts.rungRanges), dt_m1=list(ts.dt_m1),
                    dt_drift=list(ts.dt_drift))

    def gravity_stats(self):
        out = (C.c_uint64 * 3)()
        self.L.sx_sim_gravity_stats(self.h, out)
        return dict(halos=out[0], far_cells=out[1], remote_cells=out[2])

    def set_gravity_counting(self, enable=True):
        """count the gravity interactions of the following steps (sx_sim_set_gravity_counting; off by default)"""
        self.ctx.check(self.L.sx_sim_set_gravity_counting(self.h, 1 if enable else 0), "set_gravity_counting")

    def gravity_interactions(self):
        """P2P and M2P interactions of the last step (sx_sim_gravity_interactions; the reference's BhStats)"""
        out = (C.c_uint64 * 2)()
        self.ctx.check(self.L.sx_sim_gravity_interactions(self.h, out), "gravity_interactions")
        return dict(p2p=out[0], m2p=out[1])

    def close(self):
        if self.h:
            self.L.sx_sim_destroy(self.h)
            self.h = None
