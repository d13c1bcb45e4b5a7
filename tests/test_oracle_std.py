"""std propagator (HydroProp, main/src/propagator/std_hydro.hpp:124-184) in the oracle: pinned bit-exact to the
reference's own std templates (oracle/_ref) and checked against the std KATs (sph/test/std.cpp:98-127).

The reference tests run only where oracle/_ref exists (this container); the KATs run everywhere.
"""
import ctypes as C

import numpy as np
import pytest

import golden_util as gu
import pyoracle as po

needs_ref = pytest.mark.skipif(not po.ref_available(), reason="oracle/_ref not built")


@pytest.fixture(scope="module")
def ref():
    return po.load_ref()  # loaded only by the tests that need it (never on the GPU box, where it is absent)

# sph/test/std.cpp:57-87 -- five particles in the open box [0,6]^3, particle 0 against neighbors 1..4 (data)
KAT = {
    "x": [1.0, 1.1, 3.2, 1.3, 2.4], "y": [1.1, 1.2, 1.3, 4.4, 5.5], "z": [1.2, 2.3, 1.4, 1.5, 1.6],
    "h": [5.0, 5.1, 5.2, 5.3, 5.4], "m": [1.1, 1.2, 1.3, 1.4, 1.5], "rho": [0.014, 0.015, 0.016, 0.017, 0.018],
    "vx": [0.010, -0.020, 0.030, -0.040, 0.050], "vy": [-0.011, 0.021, -0.031, 0.041, -0.051],
    "vz": [0.091, -0.081, 0.071, -0.061, 0.055], "c": [0.4, 0.5, 0.6, 0.7, 0.8], "p": [0.2, 0.3, 0.4, 0.5, 0.6],
    "c11": [0.21, 0.27, 0.10, 0.45, 0.46], "c12": [-0.22, -0.29, -0.11, -0.44, -0.47],
    "c13": [-0.23, -0.31, -0.12, -0.43, -0.48], "c22": [0.24, 0.32, 0.13, 0.42, 0.49],
    "c23": [-0.25, -0.33, -0.14, -0.41, -0.50], "c33": [0.26, 0.34, 0.15, 0.40, 0.51],
}
# (expected, abs tolerance) asserted by std.cpp:104-109 (IAD) and :120-126 (momentum/energy), T=double
KAT_IAD = [(0.68826690779384281, 1e-8), (-0.12963692768970825, 1e-8), (-0.20435302538490346, 1e-8),
           (0.39616100688793993, 1e-8), (-0.16797800827029263, 1e-8), (1.9055087813473524, 1e-8)]
KAT_ME = {"ax": (14.407211846688075, 1.3e-7), "ay": (-1.2396802157028355, 1.4e-7),
          "az": (15.596554152643426, 2.15e-7), "du": (-0.40541191600274296, 1e-8),
          "maxvsignal": (1.4112466828564341, 1e-10)}
COLS = ["x", "y", "z", "h", "m", "rho", "vx", "vy", "vz", "c", "p", "c11", "c12", "c13", "c22", "c23", "c33"]


def kat_state():
    st = po.HostState(5)
    for k, v in KAT.items():
        st.arrays[k][:] = np.asarray(v, dtype=st.arrays[k].dtype)
    st.nc[:] = 5  # particle 0: four neighbors + self
    nbr = np.zeros(150 * 5, np.uint32)
    nbr[:4] = [1, 2, 3, 4]
    box = po.OxBox()
    for k, v in enumerate([0, 6, 0, 6, 0, 6]):
        box.lim[k] = v
    return st, box, nbr


def sphynx_3d_k(n):
    """sph_kernel_tables.hpp:62-75 (std.cpp:62 uses this K)"""
    b0, b1, b2, b3 = 2.7012593e-2, 2.0410827e-2, 3.7451957e-3, 4.7013839e-2
    return b0 + b1 * np.sqrt(n) + b2 * n + b3 * np.sqrt(n * n * n)


def test_oracle_std_kat():
    """the float restatement against the double-precision KAT values: relative 2e-6 (float rounding + table)"""
    ora = po.load_oracle()
    st, box, nbr = kat_state()
    p = ora.params(std=True)
    p.K = sphynx_3d_k(6.0)
    ora.iad_std(st, box, nbr, 0, 1, p)
    got = [float(st.arrays[k][0]) for k in ("c11", "c12", "c13", "c22", "c23", "c33")]
    for g, (e, tol) in zip(got, KAT_IAD):
        assert abs(g - e) <= max(tol, 2e-6 * abs(e)), (g, e)
    st, box, nbr = kat_state()
    ora.momentum_energy_std(st, box, nbr, 0, 1, p)
    # maxvsignal through the Courant step: dt = Kcour * h / maxvsignal (tsKCourant, kernels.hpp:12-18)
    mvs = np.float32(p.Kcour) * np.float32(KAT["h"][0]) / np.float32(st.minDtCourant)
    got = {"ax": st.ax[0], "ay": st.ay[0], "az": st.az[0], "du": st.du[0], "maxvsignal": mvs}
    for k, (e, tol) in KAT_ME.items():
        assert abs(float(got[k]) - e) <= max(tol, 2e-6 * abs(e)), (k, got[k], e)


@pytest.mark.parametrize("name", ["std_sedov10.npz", "std_noh12.npz"])
def test_std_steps_golden(name):
    """oracle std steps against the reference's std steps frozen in tests/golden (oracle/gen_golden.py)"""
    ora = po.load_oracle()
    d = gu.load(name)
    box = gu.box_from(d["box"])
    st = gu.state_from(d, "s0_")
    p = ora.params(std=True)
    for s in range(1, 4):
        ora.step(st, box, params=p)
        ref_st = gu.state_from(d, f"s{s}_")
        for k in st.arrays:
            assert np.array_equal(st.arrays[k], ref_st.arrays[k]), (name, s, k)
        assert (st.minDt, st.minDt_m1, st.ttot) == (ref_st.minDt, ref_st.minDt_m1, ref_st.ttot)


def test_std_kernels_golden():
    ora = po.load_oracle()
    d = gu.load("std_kernels.npz")
    box = gu.box_from(d["box"])
    st = gu.state_from(d, "in_")
    p = ora.params(std=True)
    nbr, nc = ora.find_neighbors(st, box, iterate_h=True)
    assert np.array_equal(nc, d["nc"]) and np.array_equal(nbr, d["nbr"])
    st.nc[:] = nc
    ora.density(st, box, nbr, params=p)
    assert np.array_equal(st.rho, d["rho"])
    ora.eos_std(st, params=p)
    assert np.array_equal(st.p, d["p"]) and np.array_equal(st.c, d["c"])
    ora.iad_std(st, box, nbr, params=p)
    for k in ["c11", "c12", "c13", "c22", "c23", "c33"]:
        assert np.array_equal(st.arrays[k], d[k]), k
    assert ora.momentum_energy_std(st, box, nbr, params=p) == d["minDtCourant"][0]
    for k in ["du", "ax", "ay", "az"]:
        assert np.array_equal(st.arrays[k], d[k]), k


@needs_ref
def test_reference_std_kat_double(ref):
    """the reference's own std loops (T=double) reproduce the std.cpp assertions with their tolerances"""
    cols = np.array([[KAT[c][i] for c in COLS] + [0.0, 0.0] for i in range(5)], np.float64)
    out = np.zeros(11)
    f = ref.lib.ref_kat_std_f64
    f.argtypes = [C.c_void_p, C.c_void_p]
    f(cols.ctypes.data, out.ctypes.data)
    for g, (e, tol) in zip(out[:6], KAT_IAD):
        assert abs(g - e) <= tol, (g, e)
    for g, k in zip(out[6:], ["ax", "ay", "az", "du", "maxvsignal"]):
        e, tol = KAT_ME[k]
        assert abs(g - e) <= tol, (k, g, e)


@needs_ref
@pytest.mark.parametrize("ic,side,steps", [("sedov", 12, 4), ("noh", 14, 4)])
def test_full_steps_std(ref, ic, side, steps):
    """HydroProp steps: density, EOS_HydroStd, IAD, momentumEnergySTD, time-step without the rho limit"""
    ora = po.load_oracle()
    st, box = (po.sedov_state if ic == "sedov" else po.noh_state)(side)
    a, b = st.copy(), st.copy()
    pr, px = ref.params(std=True), ora.params(std=True)
    for _ in range(steps):
        ref.step(a, box, params=pr)
        ora.step(b, box, params=px)
        for k in a.arrays:
            assert np.array_equal(a.arrays[k], b.arrays[k]), k
        assert a.minDt == b.minDt and a.minDtCourant == b.minDtCourant
    assert np.all(b.rho > 0) and np.any(b.ax != 0)


def random_sorted_state(lib, n, seed):
    rng = np.random.default_rng(seed)
    st = po.HostState(n)
    st.x[:] = rng.uniform(-0.5, 0.5, n)
    st.y[:] = rng.uniform(-0.5, 0.5, n)
    st.z[:] = np.clip(rng.normal(0, 0.12, n), -0.5, 0.4999)
    box = po.make_box(-0.5, 0.5, True)
    keys = lib.sfc_keys(st, box).copy()
    o = np.argsort(keys, kind="stable")
    for k in ("x", "y", "z"):
        st.arrays[k][:] = st.arrays[k][o]
    st.keys[:] = keys[o]
    st.h[:] = np.float32(0.03)
    st.m[:] = (rng.uniform(0.5, 1.5, n) / n).astype(np.float32)
    st.temp[:] = rng.uniform(1e-3, 2e-3, n)
    for k in ("vx", "vy", "vz"):
        st.arrays[k][:] = rng.normal(0, 0.3, n).astype(np.float32)
    return st, box


@needs_ref
def test_std_kernels_random(ref):
    """each std kernel alone on a clustered periodic state with random masses and velocities"""
    ora = po.load_oracle()
    st, box = random_sorted_state(ora, 3000, 11)
    nbr, nc = ora.find_neighbors(st, box)
    st.nc[:] = nc
    p = ora.params(std=True)
    a, b = st.copy(), st.copy()
    for name in ("density", "eos_std", "iad_std", "momentum_energy_std"):
        if name == "eos_std":
            ref.eos_std(a, params=p)
            ora.eos_std(b, params=p)
        else:
            getattr(ref, name)(a, box, nbr, params=p)
            getattr(ora, name)(b, box, nbr, params=p)
        for k in a.arrays:
            assert np.array_equal(a.arrays[k], b.arrays[k]), (name, k)
    assert a.minDtCourant == b.minDtCourant
