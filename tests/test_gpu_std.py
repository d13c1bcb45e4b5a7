"""GPU parity of the std propagator (HydroProp, main/src/propagator/std_hydro.hpp:124-184) through the C-ABI:
sx_density, sx_eos_std, sx_iad, sx_momentum_energy_std and sx_sim with propagator = 1.

  * exact variant (no FMA) on the reference's own neighbor list -> bit-identical to the reference's std loops
    (fixture std_kernels.npz, made by oracle/gen_golden.py from oracle/_ref);
  * fast variant (LDS-staged cluster kernels, FMA, polynomial W) -> |a - b| <= 2e-5 * scale + 1e-6 * max|b|;
  * full std steps (own search order) -> nc/h exact after step 1, floats within rtol 1e-4 + 1e-5 * max.
"""
import ctypes as C

import numpy as np
import pytest

import golden_util as gu
import gpu_util as gutil
import pyoracle as po
import sphexa_amd as sx

pytestmark = pytest.mark.gpu

OUT = ["rho", "p", "c", "c11", "c12", "c13", "c22", "c23", "c33", "du", "ax", "ay", "az", "minDtCourant"]


@pytest.fixture(scope="module")
def ctx():
    c = sx.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def ora():
    return po.load_oracle()


def std_chain(ctx, d, exact):
    ctx.set_exact(exact)
    box = gutil.box_to_sx(gu.box_from(d["box"]))
    st = gu.state_from(d, "in_")
    n = st.n
    host = gutil.host_dict(st)
    host["nc"] = d["nc"]
    ds = sx.DeviceState(ctx, host, std=True)
    p = sx.default_params(std=True)
    nb = ctx.upload(d["nbr"])
    ctx.check(ctx.L.sx_import_neighbors(ctx.h, 0, n, 150, nb.ptr), "import")
    g = sx.SxGroups(firstBody=0, lastBody=n, numGroups=(n + 63) // 64)
    L, h, f = ctx.L, ctx.h, ds.fields
    out = {}
    ctx.check(L.sx_density_only(h, C.byref(g), C.byref(f), C.byref(p), C.byref(box)), "density")
    out["rho"] = ds.get("rho")
    ctx.check(L.sx_eos_std(h, 0, n, 10.0, 5.0 / 3.0, f.temp, f.m, f.rho, f.p, f.c), "eos_std")
    out["p"], out["c"] = ds.get("p"), ds.get("c")
    ctx.check(L.sx_iad(h, C.byref(g), C.byref(f), C.byref(p), C.byref(box)), "iad")
    for k in ["c11", "c12", "c13", "c22", "c23", "c33"]:
        out[k] = ds.get(k)
    mdt = C.c_float()
    ctx.check(L.sx_momentum_energy_std(h, C.byref(g), C.byref(f), C.byref(p), C.byref(box), C.byref(mdt)), "me")
    out["minDtCourant"] = np.array([mdt.value])
    for k in ["du", "ax", "ay", "az"]:
        out[k] = ds.get(k)
    ctx.set_exact(False)
    return out


def test_std_kernels_exact_variant_bitwise(ctx):
    d = gu.load("std_kernels.npz")
    out = std_chain(ctx, d, exact=True)
    for k in OUT:
        ref = d[k].astype(out[k].dtype)
        assert np.array_equal(out[k], ref), (k, np.max(np.abs(out[k].astype(float) - ref)))
    ctx.free_all()


def scale_of(k, d):
    if k in ("c12", "c13", "c23"):
        return np.maximum(np.maximum(np.abs(d["c11"]), np.abs(d["c22"])), np.abs(d["c33"])).astype(np.float64)
    if k in ("ax", "ay", "az"):
        return np.sqrt(d["ax"].astype(np.float64) ** 2 + d["ay"] ** 2 + d["az"] ** 2)
    return np.abs(d[k].astype(np.float64))


def test_std_kernels_fast_variant_tolerance(ctx):
    d = gu.load("std_kernels.npz")
    out = std_chain(ctx, d, exact=False)
    for k in OUT:
        a = out[k].astype(np.float64)
        b = d[k].astype(np.float64)
        err = np.abs(a - b)
        tol = 2e-5 * scale_of(k, d) + 1e-6 * np.max(np.abs(b))
        assert np.all(err <= tol), (k, float(np.max(err / (scale_of(k, d) + 1e-300))))
    ctx.free_all()


def test_density_with_own_search(ctx):
    """sx_density = search + h iteration + xmass into rho + m/rho (computeDensity): nc and h exact"""
    d = gu.load("std_kernels.npz")
    box = gutil.box_to_sx(gu.box_from(d["box"]))
    st = gu.state_from(d, "in_")
    n = st.n
    ds = sx.DeviceState(ctx, gutil.host_dict(st), std=True)
    tree, _ = gutil.device_tree(ctx, ds.dev["keys"], n, 64, box)
    p = sx.default_params(std=True)
    g = sx.SxGroups(firstBody=0, lastBody=n, numGroups=(n + 63) // 64)
    ctx.check(ctx.L.sx_density(ctx.h, C.byref(g), C.byref(ds.fields), C.byref(p), C.byref(box), C.byref(tree)),
              "density")
    assert np.array_equal(ds.get("nc"), d["nc"])
    ok, info = gutil.close(ds.get("rho"), d["rho"], rtol=2e-6)
    assert ok, info
    ctx.free_all()


STD_FLOATS = ["x", "y", "z", "vx", "vy", "vz", "temp", "x_m1", "y_m1", "z_m1", "du_m1", "rho", "p", "c", "c11",
              "c22", "c33", "du", "ax", "ay", "az"]


def run_std_steps(ctx, ora, st, obox, steps):
    """std steps of sx_sim, each checked per particle against an oracle step from the same state
    (gpu_util.shadow_steps; the oracle exports the magnitude of the momentumEnergySTD terms for du and a)"""
    sim = sx.Sim(ctx, st.n, gutil.box_to_sx(obox), params=sx.default_params(std=True))
    sim.set_state(st.arrays, st.minDt, st.minDt_m1)

    def rho_limit(s, sim, ref):
        assert sim.scalars()["minDtRho"] == float("inf")  # HydroProp never sets the rho limit

    gutil.shadow_steps(ctx, ora, sim, obox, steps, ora.params(std=True), STD_FLOATS, on_step=rho_limit)
    sim.close()


@pytest.mark.parametrize("ic,side,steps", [("sedov", 16, 3), ("noh", 16, 3)])
def test_std_sim_steps_vs_oracle(ctx, ora, ic, side, steps):
    st, obox = (po.sedov_state if ic == "sedov" else po.noh_state)(side)
    run_std_steps(ctx, ora, st, obox, steps)


def test_std_golden_fixture_steps(ctx, ora):
    """the oracle reproduces the reference's std steps (std_sedov10.npz) bit for bit; the GPU steps from the
    fixture state are checked per particle against it"""
    d = gu.load("std_sedov10.npz")
    obox = gu.box_from(d["box"])
    ref = gu.state_from(d, "s0_")
    for s in (1, 2, 3):
        ora.step(ref, obox, params=ora.params(std=True))
        fx = gu.state_from(d, f"s{s}_")
        for k in STD_FLOATS + ["nc", "h", "id"]:
            assert np.array_equal(ref.arrays[k], fx.arrays[k]), (s, k)
    run_std_steps(ctx, ora, gu.state_from(d, "s0_"), obox, 3)
