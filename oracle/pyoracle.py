"""Python side of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Loads oracle/libsphexa_oracle.so (the plain-C restatement, oracle/sph_oracle.c) and, when it was built
in this container, oracle/_ref/libsphexa_ref.so (the reference's own CPU path compiled from
/root/reference by oracle/Makefile).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg import this module, and only as the checker; the product library never links or calls it.

Also holds the numpy restatement of the Sedov / Noh initial conditions used to feed both sides:
  Sedov: main/src/init/sedov_init.hpp:48-96, sedov_constants.hpp:11-21, grid.hpp:102-132
  Noh:   main/src/init/noh_init.hpp:46-100 (lattice-cut-sphere substitute)
"""

import ctypes as C
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "libsphexa_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "libsphexa_ref.so")

KTABLE = 20000


class OxBox(C.Structure):
    _fields_ = [("lim", C.c_double * 6), ("bnd", C.c_int32 * 3)]


class OxParams(C.Structure):
    _fields_ = [("K", C.c_double), ("ng0", C.c_uint32), ("ngmax", C.c_uint32), ("Kcour", C.c_double),
                ("Krho", C.c_double), ("gamma", C.c_double), ("muiConst", C.c_float), ("alphamin", C.c_float),
                ("alphamax", C.c_float), ("decay_constant", C.c_float), ("Atmin", C.c_float),
                ("Atmax", C.c_float), ("ramp", C.c_float), ("maxDtIncrease", C.c_double), ("avClean", C.c_int32),
                ("theta", C.c_float), ("g", C.c_double), ("eps", C.c_double), ("etaAcc", C.c_double), ("prop", C.c_int32)]


STATE_FIELDS = [
    ("x", np.float64), ("y", np.float64), ("z", np.float64),
    ("x_m1", np.float32), ("y_m1", np.float32), ("z_m1", np.float32),
    ("vx", np.float32), ("vy", np.float32), ("vz", np.float32),
    ("temp", np.float64), ("h", np.float32), ("m", np.float32), ("alpha", np.float32),
    ("du_m1", np.float32), ("id", np.uint64),
    ("du", np.float64),
    ("ax", np.float32), ("ay", np.float32), ("az", np.float32), ("prho", np.float32), ("c", np.float32),
    ("xm", np.float32), ("kx", np.float32), ("gradh", np.float32), ("divv", np.float32), ("curlv", np.float32),
    ("c11", np.float32), ("c12", np.float32), ("c13", np.float32), ("c22", np.float32), ("c23", np.float32),
    ("c33", np.float32), ("nc", np.uint32), ("keys", np.uint64),
    ("dV11", np.float32), ("dV12", np.float32), ("dV13", np.float32), ("dV22", np.float32), ("dV23", np.float32),
    ("dV33", np.float32), ("rho", np.float32), ("p", np.float32),
]
CONSERVED = ["x", "y", "z", "x_m1", "y_m1", "z_m1", "vx", "vy", "vz", "temp", "h", "m", "alpha", "du_m1", "id"]

_CT = {np.float64: C.c_double, np.float32: C.c_float, np.uint64: C.c_uint64, np.uint32: C.c_uint32}


class OxState(C.Structure):
    _fields_ = [("n", C.c_size_t)] + [(name, C.POINTER(_CT[t])) for name, t in STATE_FIELDS] + [
        ("minDt", C.c_double), ("minDt_m1", C.c_double), ("ttot", C.c_double), ("minDtCourant", C.c_double),
        ("minDtRho", C.c_double), ("egrav", C.c_double)]


def default_params(K, av_clean=False, g=0.0, theta=0.5, std=False):
    """ParticlesData defaults (particles_data.hpp:86-138); av_clean selects HydroVeProp<true>; g != 0 turns on
    self-gravity with opening parameter theta (sphexa.cpp:127); std selects the std propagator (HydroProp)."""
    return OxParams(K=K, ng0=100, ngmax=150, Kcour=0.2, Krho=0.06, gamma=5.0 / 3.0, muiConst=10.0,
                    alphamin=0.05, alphamax=1.0, decay_constant=0.2, Atmin=0.1, Atmax=0.2,
                    ramp=float(np.float32(1.0) / (np.float32(0.2) - np.float32(0.1))), maxDtIncrease=1.1,
                    avClean=1 if av_clean else 0, theta=theta, g=g, eps=0.005, etaAcc=0.2,
                    prop=1 if std else 0)


def make_box(lo=-0.5, hi=0.5, periodic=True):
    b = OxBox()
    for k, v in enumerate([lo, hi, lo, hi, lo, hi]):
        b.lim[k] = v
    for k in range(3):
        b.bnd[k] = 1 if periodic else 0
    return b


class HostState:
    """numpy-owned particle state with an OxState view."""

    def __init__(self, n):
        self.n = n
        self.arrays = {name: np.zeros(n, dtype=t) for name, t in STATE_FIELDS}
        self.minDt = 1e-6
        self.minDt_m1 = 1e-6
        self.ttot = 0.0
        self.minDtCourant = math.inf
        self.minDtRho = math.inf
        self.egrav = 0.0

    def __getattr__(self, item):
        arrays = self.__dict__.get("arrays")
        if arrays is not None and item in arrays:
            return arrays[item]
        raise AttributeError(item)

    def struct(self):
        s = OxState()
        s.n = self.n
        for name, t in STATE_FIELDS:
            a = self.arrays[name]
            assert a.flags["C_CONTIGUOUS"] and a.dtype == t
            setattr(s, name, a.ctypes.data_as(C.POINTER(_CT[t])))
        s.minDt, s.minDt_m1, s.ttot = self.minDt, self.minDt_m1, self.ttot
        s.minDtCourant, s.minDtRho = self.minDtCourant, self.minDtRho
        s.egrav = self.egrav
        self._s = s
        return s

    def pull(self, s):
        self.minDt, self.minDt_m1, self.ttot = s.minDt, s.minDt_m1, s.ttot
        self.minDtCourant, self.minDtRho = s.minDtCourant, s.minDtRho
        self.egrav = s.egrav

    def copy(self):
        o = HostState(self.n)
        for k, v in self.arrays.items():
            o.arrays[k][:] = v
        o.minDt, o.minDt_m1, o.ttot = self.minDt, self.minDt_m1, self.ttot
        o.minDtCourant, o.minDtRho = self.minDtCourant, self.minDtRho
        return o


def ideal_gas_cv(mui=np.float32(10.0), gamma=5.0 / 3.0):
    """idealGasCv<float,double> (sph/eos.hpp:13-18): R is a float constant, result float."""
    R = np.float32(8.317e7)
    return np.float32(np.float64(R / np.float32(mui)) / (gamma - 1.0))


def sedov_state(side):
    """Sedov lattice IC (sedov_init.hpp:48-96, 106-130; grid.hpp:102-132); box [-0.5,0.5]^3 periodic."""
    r = 0.5
    n = side ** 3
    st = HostState(n)
    step = (2.0 * r) / side
    r_ini = -r + 0.5 * step
    idx = np.arange(side, dtype=np.float64)
    coord = r_ini + idx * step
    zz, yy, xx = np.meshgrid(coord, coord, coord, indexing="ij")
    st.x[:] = xx.ravel()
    st.y[:] = yy.ravel()
    st.z[:] = zz.ravel()
    ng0 = 100
    total_volume = (2 * r) ** 3
    h_init = np.cbrt(3.0 / (4 * math.pi) * ng0 * total_volume / n) * 0.5
    st.m[:] = np.float32(1.0 / n)
    st.h[:] = np.float32(h_init)
    st.alpha[:] = np.float32(0.05)
    width = 0.1
    ener0 = 1.0 / math.pi ** 1.5 / 1.0 / width ** 3.0
    u0 = 1e-8
    cv = ideal_gas_cv()
    r2 = st.x * st.x + st.y * st.y + st.z * st.z
    ui = ener0 * np.exp(-(r2 / (width * width))) + u0
    st.temp[:] = ui / np.float64(cv)
    st.id[:] = np.arange(n, dtype=np.uint64)
    st.minDt = 1e-6
    st.minDt_m1 = 1e-6
    return st, make_box(-r, r, True)


def pbc_wave_state(side, eps=0.3):
    """periodic self-gravity test IC: the Sedov lattice (periodic box [-0.5, 0.5]^3, total mass 1) at its ambient
    temperature, the particle masses modulated by 1 + eps sin(2 pi x): a density wave whose periodic field is
    g_x = (4 pi G eps / k) cos(k x), k = 2 pi (Poisson's equation with the mean density removed, as the Ewald sum does)"""
    st, box = sedov_state(side)
    st.temp[:] = np.float64(st.temp.min())
    st.m[:] = (st.m.astype(np.float64) * (1.0 + eps * np.sin(2.0 * math.pi * st.x))).astype(np.float32)
    return st, box


def noh_state(side):
    """Noh substitute: side^3 lattice in [-0.5,0.5]^3 cut to r<=0.5, open box,
    v = -r_hat, x_m1 = v dt0, T = 1e-20/cv, dt0 = 1e-4 (noh_init.hpp:46-100 field values)."""
    r = 0.5
    step = (2.0 * r) / side
    r_ini = -r + 0.5 * step
    idx = np.arange(side, dtype=np.float64)
    coord = r_ini + idx * step
    zz, yy, xx = np.meshgrid(coord, coord, coord, indexing="ij")
    x, y, z = xx.ravel(), yy.ravel(), zz.ravel()
    rad = np.sqrt(x * x + y * y + z * z)
    keep = rad <= r
    x, y, z, rad = x[keep], y[keep], z[keep], rad[keep]
    n = x.size
    st = HostState(n)
    st.x[:], st.y[:], st.z[:] = x, y, z
    vol = 4.0 / 3.0 * math.pi * r ** 3
    ng0 = 100
    h_init = np.cbrt(3.0 / (4 * math.pi) * ng0 * vol / n) * 0.5
    st.m[:] = np.float32(1.0 / n)
    st.h[:] = np.float32(h_init)
    st.alpha[:] = np.float32(0.05)
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = np.where(rad > 0, 1.0 / rad, 0.0)
    st.vx[:] = (-x * inv).astype(np.float32)
    st.vy[:] = (-y * inv).astype(np.float32)
    st.vz[:] = (-z * inv).astype(np.float32)
    st.temp[:] = 1e-20 / np.float64(ideal_gas_cv())
    # the integrator's previous displacement: x_m1 = v * minDt (noh_init.hpp:96-98, float storage of a double product)
    for d in ("x", "y", "z"):
        st.arrays[d + "_m1"][:] = (st.arrays["v" + d].astype(np.float64) * 1e-4).astype(np.float32)
    st.id[:] = np.arange(n, dtype=np.uint64)
    st.minDt = 1e-4
    st.minDt_m1 = 1e-4
    lo, hi = -0.5 - 1e-3, 0.5 + 1e-3
    return st, make_box(lo, hi, False)


def evrard_state(side):
    """Evrard collapse substitute (the glass block is unavailable): side^3 lattice in [-1,1]^3 cut to
    r <= 1, contracted by sqrt(r) to a 1/r density profile (evrard_init.hpp:90-108 contractRhoProfile), field values of
    initEvrardFields (:50-88): m = 1/N, u0 = 0.05, v = 0, h from the 1/r concentration; G = 1, dt0 = 1e-4.
    Open box [-1.25,1.25]^3: the reference re-fits open boxes to the particles every sync (makeGlobalBox), this
    fixed box leaves room for the outer shell to expand."""
    r = 1.0
    step = (2.0 * r) / side
    coord = -r + 0.5 * step + np.arange(side, dtype=np.float64) * step
    zz, yy, xx = np.meshgrid(coord, coord, coord, indexing="ij")
    x, y, z = xx.ravel(), yy.ravel(), zz.ravel()
    rad0 = np.sqrt(x * x + y * y + z * z)
    keep = (rad0 <= r) & (rad0 > 1e-9 * r)  # odd sides: no particle at the singular center (h -> 0)
    x, y, z, rad0 = x[keep], y[keep], z[keep], rad0[keep]
    con = np.sqrt(rad0)
    x, y, z = x * con, y * con, z * con
    n = x.size
    st = HostState(n)
    st.x[:], st.y[:], st.z[:] = x, y, z
    st.m[:] = np.float32(1.0 / n)
    st.alpha[:] = np.float32(0.05)
    cv = ideal_gas_cv()
    st.temp[:] = 0.05 / np.float64(cv)
    total_volume = 4.0 * math.pi / 3.0 * r ** 3
    c0 = 2.0 / 3.0 * n / total_volume
    radius = np.sqrt(x * x + y * y + z * z)
    conc = c0 / np.maximum(radius, 1e-12)
    st.h[:] = (np.cbrt(3.0 / (4.0 * math.pi) * 100 / conc) * 0.5).astype(np.float32)
    st.id[:] = np.arange(n, dtype=np.uint64)
    st.minDt = 1e-4
    st.minDt_m1 = 1e-4
    return st, make_box(-1.25 * r, 1.25 * r, False)


def _bind(lib):
    P = C.c_void_p
    u32p = C.POINTER(C.c_uint32)
    for name, res, args in [
        ("kernel_tables", None, [C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_double)]),
        ("sfc_keys", None, [P, P, P, C.c_size_t, C.POINTER(OxBox), P]),
        ("compute_octree", C.c_int, [P, C.c_size_t, C.c_uint, P, P, C.c_int]),
        ("build_octree", None, [P, C.c_int, P, P, P, P, P, P]),
        ("node_centers", None, [P, C.c_int, C.POINTER(OxBox), P, P]),
        ("find_neighbors", None, [P, P, P, P, P, C.c_size_t, C.c_uint, C.c_uint, C.POINTER(OxBox), C.c_uint,
                                  C.c_uint, C.c_uint, C.c_int, u32p, u32p]),
        ("xmass", None, [C.POINTER(OxState), C.POINTER(OxParams), C.POINTER(OxBox), u32p, C.c_uint, C.c_uint]),
        ("ve_def_gradh", None, [C.POINTER(OxState), C.POINTER(OxParams), C.POINTER(OxBox), u32p, C.c_uint,
                                C.c_uint]),
        ("eos", None, [C.POINTER(OxState), C.POINTER(OxParams), C.c_uint, C.c_uint]),
        ("iad_divv_curlv", None, [C.POINTER(OxState), C.POINTER(OxParams), C.POINTER(OxBox), u32p, C.c_uint,
                                  C.c_uint]),
        ("av_switches", None, [C.POINTER(OxState), C.POINTER(OxParams), C.POINTER(OxBox), u32p, C.c_uint,
                               C.c_uint]),
        ("momentum_energy", C.c_double, [C.POINTER(OxState), C.POINTER(OxParams), C.POINTER(OxBox), u32p,
                                          C.c_uint, C.c_uint]),
        ("density", None, [C.POINTER(OxState), C.POINTER(OxParams), C.POINTER(OxBox), u32p, C.c_uint, C.c_uint]),
        ("eos_std", None, [C.POINTER(OxState), C.POINTER(OxParams), C.c_uint, C.c_uint]),
        ("iad_std", None, [C.POINTER(OxState), C.POINTER(OxParams), C.POINTER(OxBox), u32p, C.c_uint, C.c_uint]),
        ("momentum_energy_std", C.c_double, [C.POINTER(OxState), C.POINTER(OxParams), C.POINTER(OxBox), u32p,
                                              C.c_uint, C.c_uint]),
        ("positions", None, [C.POINTER(OxState), C.POINTER(OxParams), C.POINTER(OxBox), C.c_uint, C.c_uint]),
        ("update_h_range", None, [C.POINTER(OxState), C.c_uint, C.c_uint, C.c_uint]),
        ("step", C.c_int, [C.POINTER(OxState), C.POINTER(OxParams), C.POINTER(OxBox), C.c_uint]),
        ("update_h", C.c_float, [C.c_uint, C.c_uint, C.c_float]),
        ("gravity", C.c_double, [C.POINTER(OxState), C.POINTER(OxParams), C.POINTER(OxBox), C.c_uint, C.c_uint,
                                 C.c_uint, P, P, C.c_int]),
        ("set_scales", None, [P, P, P, P, P]),
        ("make_splits", C.c_int, [C.c_uint64, P]),
        ("group_splits", C.c_int, [C.c_uint32, C.c_uint32, P, P, P, P, C.c_int, P, C.POINTER(OxBox), C.c_float,
                                   P]),
    ]:
        for prefix in ("ref_", "ox_"):
            if hasattr(lib, prefix + name):
                f = getattr(lib, prefix + name)
                f.restype = res
                f.argtypes = args
                setattr(lib, name, f)
    return lib


class Lib:
    """Thin wrapper that offers the same python API for both the reference and the restatement."""

    def __init__(self, path):
        self.path = path
        self.lib = _bind(C.CDLL(path))
        wh = np.zeros(KTABLE, np.float32)
        whd = np.zeros(KTABLE, np.float32)
        K = C.c_double()
        self.lib.kernel_tables(wh.ctypes.data_as(C.POINTER(C.c_float)), whd.ctypes.data_as(C.POINTER(C.c_float)),
                               C.byref(K))
        self.wh, self.whd, self.K = wh, whd, K.value

    def params(self, av_clean=False, g=0.0, theta=0.5, std=False):
        return default_params(self.K, av_clean, g, theta, std)

    SCALES = ("du", "a", "dv", "gradh", "alpha")

    def scales_on(self, n):
        """make the oracle's J-loops export per-particle error scales (sums of |term|, ox_set_scales) into fresh
        float64 arrays of length n, indexed like the state the kernels run on; returns the dict of arrays"""
        self._scales = {k: np.zeros(n, np.float64) for k in self.SCALES}
        self.lib.set_scales(*[self._scales[k].ctypes.data for k in self.SCALES])
        return self._scales

    def make_splits(self, mask):
        out = np.zeros(65, np.uint32)
        k = self.lib.make_splits(int(mask), out.ctypes.data)
        return out[:k].tolist()

    def group_splits(self, first, last, x, y, z, leaves, layout, box, tol_factor=2.0):
        """computeGroupSplits<64> restated (sph_oracle.c ox_group_splits): group boundaries, length numGroups+1"""
        x, y, z = (np.ascontiguousarray(a, np.float64) for a in (x, y, z))
        leaves = np.ascontiguousarray(leaves, np.uint64)
        layout = np.ascontiguousarray(layout, np.uint32)
        nl = leaves.size - 1
        ng = self.lib.group_splits(first, last, x.ctypes.data, y.ctypes.data, z.ctypes.data, leaves.ctypes.data, nl,
                                   layout.ctypes.data, C.byref(box), tol_factor, None)
        out = np.zeros(ng + 1, np.uint32)
        self.lib.group_splits(first, last, x.ctypes.data, y.ctypes.data, z.ctypes.data, leaves.ctypes.data, nl,
                              layout.ctypes.data, C.byref(box), tol_factor, out.ctypes.data)
        return out

    def scales_off(self):
        self.lib.set_scales(None, None, None, None, None)
        self._scales = None

    def sfc_keys(self, st, box):
        self.lib.sfc_keys(st.x.ctypes.data, st.y.ctypes.data, st.z.ctypes.data, st.n, C.byref(box),
                          st.keys.ctypes.data)
        return st.keys

    def octree(self, keys, bucket):
        n = keys.size
        nleaf = self.lib.compute_octree(keys.ctypes.data, n, bucket, None, None, 0)
        leaves = np.zeros(nleaf + 1, np.uint64)
        counts = np.zeros(nleaf, np.uint32)
        self.lib.compute_octree(keys.ctypes.data, n, bucket, leaves.ctypes.data, counts.ctypes.data, nleaf)
        nint = (nleaf - 1) // 7
        ntot = nleaf + nint
        out = dict(leaves=leaves, counts=counts, prefixes=np.zeros(ntot, np.uint64),
                   childOffsets=np.zeros(ntot + 1, np.int32), parents=np.zeros(max(1, (ntot - 1) // 8), np.int32),
                   levelRange=np.zeros(23, np.int32), internalToLeaf=np.zeros(ntot, np.int32),
                   leafToInternal=np.zeros(ntot, np.int32))
        self.lib.build_octree(leaves.ctypes.data, nleaf, out["prefixes"].ctypes.data, out["childOffsets"].ctypes.data,
                              out["parents"].ctypes.data, out["levelRange"].ctypes.data,
                              out["internalToLeaf"].ctypes.data, out["leafToInternal"].ctypes.data)
        return out

    def node_centers(self, prefixes, box):
        nn = prefixes.size
        c = np.zeros((nn, 3), np.float64)
        s = np.zeros((nn, 3), np.float64)
        self.lib.node_centers(prefixes.ctypes.data, nn, C.byref(box), c.ctypes.data, s.ctypes.data)
        return c, s

    def find_neighbors(self, st, box, first=0, last=None, bucket=64, iterate_h=True, ngmax=150, ng0=100):
        last = st.n if last is None else last
        nbr = np.zeros((last - first) * ngmax, np.uint32)
        nc = np.zeros(last - first, np.uint32)
        self.lib.find_neighbors(st.x.ctypes.data, st.y.ctypes.data, st.z.ctypes.data, st.h.ctypes.data,
                                st.keys.ctypes.data, st.n, first, last, C.byref(box), bucket, ng0, ngmax,
                                int(iterate_h), nbr.ctypes.data_as(C.POINTER(C.c_uint32)),
                                nc.ctypes.data_as(C.POINTER(C.c_uint32)))
        return nbr, nc

    def _kern(self, name, st, box, nbr, first, last, params=None):
        p = params or self.params()
        s = st.struct()
        f = getattr(self.lib, name)
        ptr = nbr.ctypes.data_as(C.POINTER(C.c_uint32))
        errs = getattr(self.lib, "ox_list_errors", None)
        if errs is not None:
            errs.restype = C.c_ulonglong
            self.lib.ox_clear_list_errors()
        r = f(C.byref(s), C.byref(p), C.byref(box), ptr, first, last)
        if errs is not None and errs():
            raise AssertionError(f"{name}: {errs()} neighbor-list entries outside [0, {st.n}) (list under test is bad)")
        st.pull(s)
        return r

    def xmass(self, st, box, nbr, first=0, last=None, params=None):
        return self._kern("xmass", st, box, nbr, first, st.n if last is None else last, params)

    def ve_def_gradh(self, st, box, nbr, first=0, last=None, params=None):
        return self._kern("ve_def_gradh", st, box, nbr, first, st.n if last is None else last, params)

    def iad_divv_curlv(self, st, box, nbr, first=0, last=None, params=None):
        return self._kern("iad_divv_curlv", st, box, nbr, first, st.n if last is None else last, params)

    def av_switches(self, st, box, nbr, first=0, last=None, params=None):
        return self._kern("av_switches", st, box, nbr, first, st.n if last is None else last, params)

    def momentum_energy(self, st, box, nbr, first=0, last=None, params=None):
        return self._kern("momentum_energy", st, box, nbr, first, st.n if last is None else last, params)

    def density(self, st, box, nbr, first=0, last=None, params=None):
        return self._kern("density", st, box, nbr, first, st.n if last is None else last, params)

    def iad_std(self, st, box, nbr, first=0, last=None, params=None):
        return self._kern("iad_std", st, box, nbr, first, st.n if last is None else last, params)

    def momentum_energy_std(self, st, box, nbr, first=0, last=None, params=None):
        return self._kern("momentum_energy_std", st, box, nbr, first, st.n if last is None else last, params)

    def eos_std(self, st, first=0, last=None, params=None):
        p = params or self.params()
        s = st.struct()
        self.lib.eos_std(C.byref(s), C.byref(p), first, st.n if last is None else last)

    def eos(self, st, first=0, last=None, params=None):
        p = params or self.params()
        s = st.struct()
        self.lib.eos(C.byref(s), C.byref(p), first, st.n if last is None else last)

    def update_h_range(self, st, ng0, first=0, last=None):
        """updateSmoothingLength over [first, last) (ox_update_h_range)"""
        s = st.struct()
        self.lib.update_h_range(C.byref(s), ng0, first, st.n if last is None else last)
        st.pull(s)

    def positions(self, st, box, first=0, last=None, params=None):
        p = params or self.params()
        s = st.struct()
        self.lib.positions(C.byref(s), C.byref(p), C.byref(box), first, st.n if last is None else last)

    def gravity(self, st, box, params, first=0, last=None, bucket=64):
        """self-gravity of a key-sorted state: adds G*acc to ax, ay, az of [first, last); returns
        (egrav, centers (numNodes x 4: mass center, mac^2), multipoles (numNodes x 8 float))"""
        last = st.n if last is None else last
        s = st.struct()
        nn = int(self.lib.gravity(C.byref(s), C.byref(params), C.byref(box), bucket, first, last, None, None, -1))
        cen = np.zeros((nn, 4), np.float64)
        mp = np.zeros((nn, 8), np.float32)
        s = st.struct()
        eg = self.lib.gravity(C.byref(s), C.byref(params), C.byref(box), bucket, first, last, cen.ctypes.data,
                              mp.ctypes.data, nn)
        return eg, cen, mp

    def step(self, st, box, bucket=64, params=None):
        p = params or self.params()
        s = st.struct()
        r = self.lib.step(C.byref(s), C.byref(p), C.byref(box), bucket)
        st.pull(s)
        return r


def ref_available():
    """oracle/_ref was built here (checked without mapping the library into the process)"""
    return os.path.exists(REF_SO)


def load_ref():
    """The reference's own CPU path, or None when it was not built (e.g. on the GPU box without the .so)."""
    if not os.path.exists(REF_SO):
        return None
    return Lib(REF_SO)


def load_oracle():
    if not os.path.exists(ORACLE_SO):
        raise FileNotFoundError(ORACLE_SO + " not built: run `make -C oracle`")
    return Lib(ORACLE_SO)


def total_energy(st):
    """kinetic + internal energy (conserved_quantities.hpp:49-93 restated; u = cv*T)."""
    cv = np.float64(ideal_gas_cv())
    v2 = st.vx.astype(np.float64) ** 2 + st.vy.astype(np.float64) ** 2 + st.vz.astype(np.float64) ** 2
    m = st.m.astype(np.float64)
    return float(np.sum(0.5 * m * v2) + np.sum(m * cv * st.temp))


def converge_h(lib, st, box, bucket=64):
    """set st.h to the smoothing lengths after the h-nc iteration of the first search (findNeighborsSph) on this
    state, in the state's own order: the following steps then start from converged h, so a decomposed run (whose
    halos keep the pre-iteration h, as in the reference) sees the same h as a single domain"""
    tmp = st.copy()
    keys = lib.sfc_keys(tmp, box).copy()
    srt = np.argsort(keys, kind="stable")
    for name in ("x", "y", "z", "h"):
        tmp.arrays[name][:] = tmp.arrays[name][srt]
    tmp.keys[:] = keys[srt]
    lib.find_neighbors(tmp, box, bucket=bucket, iterate_h=True)
    st.h[srt] = tmp.h
    return st


def conserved_quantities(st, first=0, last=None, mui=np.float32(10.0), gamma=5.0 / 3.0):
    """localConservedQuantities (main/src/observables/conserved_quantities.hpp:49-101) restated in numpy, float64:
    (0.5 sum m |v|^2, sum cv T m, linear momentum, angular momentum, sum nc)"""
    last = st.n if last is None else last
    s = slice(first, last)
    m = st.m[s].astype(np.float64)
    X = np.stack([st.x[s], st.y[s], st.z[s]], 1).astype(np.float64)
    V = np.stack([st.vx[s], st.vy[s], st.vz[s]], 1).astype(np.float64)
    ekin = 0.5 * float(np.sum(m * np.sum(V * V, 1)))
    eint = float(np.sum(np.float64(ideal_gas_cv(mui, gamma)) * st.temp[s] * m))
    lin = np.sum(m[:, None] * V, 0)
    ang = np.sum(m[:, None] * np.cross(X, V), 0)
    return ekin, eint, lin, ang, int(np.sum(st.nc[s].astype(np.int64)))


# ---- block time-step rung bookkeeping (numpy restatement of sph/include/sph/ts_rungs.hpp) -----------------------
# Only findRungRanges<false> of ts_rungs.hpp is host code: oracle/_ref compiles it (with the image's MPICH for the
# header's <mpi.h>) and tests/test_rungs_oracle.py pins find_rung_ranges to it.  sortGroupDt / computeMinTimestep /
# rungTimestep / minimumGroupDt call GPU-only primitives (cstone::sortByKeyGpu, sequenceGpu, memcpyD2H from the
# reference's CUDA sources): their restatement is pinned by the reference text (cited per line) and hand cases.
MAX_NUM_RUNGS = 4  # sph::Timestep::maxNumRungs (sph/timestep.h:42)


def sort_group_dt(group_dt, num_groups, num_groups_tot):
    """sortGroupDt (ts_rungs.hpp:67-78) + the index sequence of computeMinTimestep (:97-98): a stable sort of
    groupDt[0, numGroups) by value (thrust sort_by_key on the identity), indices numGroups.. past it"""
    dt = np.asarray(group_dt, np.float32).copy()
    order = np.argsort(dt[:num_groups], kind="stable").astype(np.uint32)
    dt[:num_groups] = dt[:num_groups][order]
    idx = np.concatenate([order, np.arange(num_groups, num_groups_tot, dtype=np.uint32)])
    return dt, idx


def min_timestep(group_dt, num_groups, num_groups_tot):
    """computeMinTimestep (ts_rungs.hpp:89-105), one rank: sorted dt, indices, {dt[0], dt[LocalIndex(0.4f n)]}"""
    dt, idx = sort_group_dt(group_dt, num_groups, num_groups_tot)
    k = int(np.float32(0.4) * np.float32(num_groups))  # float fastFraction * LocalIndex, truncated (:85)
    return dt, idx, (dt[0], dt[k])


def find_rung_ranges(min_dt, dt_sorted, num_groups, num_rungs):
    """findRungRanges (ts_rungs.hpp:116-130): [0, lower_bound(2^r minDt) for 0 < r < numRungs, numGroups ...]"""
    rr = [0] + [num_groups] * MAX_NUM_RUNGS
    for r in range(1, num_rungs):
        max_dt_rung = np.float32(np.float32(1 << r) * np.float32(min_dt))  # (1 << rung) * minDt in float
        rr[r] = int(np.searchsorted(dt_sorted[:num_groups], max_dt_rung, side="left"))
    return rr


def rung_timestep(group_dt, num_groups, max_dt):
    """rungTimestep (ts_rungs.hpp:132-145) -> (sorted dt, indices, Timestep as a dict)"""
    dt, idx, (d0, d1) = min_timestep(group_dt, num_groups, num_groups)
    # unqualified log2 of a float quotient in namespace sph: ::log2(double)
    num_rungs = min(int(math.log2(float(np.float32(d1 / d0)))) + 1, MAX_NUM_RUNGS)
    rr = find_rung_ranges(d0, dt, num_groups, num_rungs)
    d0 = min(np.float32(max_dt), d0)
    ts = dict(nextDt=np.float32(d0), elapsedDt=np.float32(0), totDt=np.float32(d0 * np.float32(1 << num_rungs)),
              numRungs=num_rungs, substep=0, rungRanges=rr)
    return dt, idx, ts


def minimum_group_dt(ts, group_dt, num_groups):
    """minimumGroupDt (ts_rungs.hpp:147-157) -> (sorted dt, indices, dt, rungRanges)"""
    dt, idx, (d0, _) = min_timestep(group_dt, num_groups, ts["rungRanges"][MAX_NUM_RUNGS])
    rr = find_rung_ranges(d0, dt, num_groups, MAX_NUM_RUNGS)
    time_left = np.float32(np.float32(ts["totDt"]) - np.float32(ts["elapsedDt"]))
    substeps_left = (1 << ts["numRungs"]) - ts["substep"]
    return dt, idx, min(d0, np.float32(time_left / np.float32(substeps_left))), rr


def extract_groups(group_start, group_end, indices, first, last):
    """extractGroupGpu (sph/groups.hpp:31-48)"""
    sel = np.asarray(indices[first:last], np.int64)
    return np.asarray(group_start)[sel].astype(np.uint32), np.asarray(group_end)[sel].astype(np.uint32)
