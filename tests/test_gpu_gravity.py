"""Self-gravity on the GPU (sx_gravity_upsweep / sx_gravity_traverse) against the CPU oracle, whose gravity is pinned
bit-exact to the reference's ryoanji CPU functions (tests/test_oracle_gravity.py).

* expansion centers + MAC radii and quadrupoles: bit-identical (same sequential order per node) with the exact
  variant; the fast variant sums each leaf over a wave (check_upsweep_fast: to double / float rounding);
* accelerations: each target sees the reference's M2P/P2P set (16-target groups, per-quarter MAC), only the double
  summation order differs: |a - a_ref| <= 1e-6 |a_ref| + 1e-7 max|a|; egrav to 1e-10;
* golden fixture evrard14 (the reference's own outputs) the same way;
* the production (fast) traversal evaluates M2P/P2P in float with rsqrt (displacements formed in double, sums in
  double): |a - a_ref| <= 1e-5 |a_ref| + 1e-6 max|a|, egrav to 1e-6.
The exact traversal runs with sx_set_exact(1), like the exact hydro kernels.
"""
import ctypes as C

import numpy as np
import pytest

import golden_util as gu
import gpu_util as gutil
import pyoracle as po
import sphexa_amd as sx

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = sx.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def ora():
    return po.load_oracle()


def gpu_gravity(ctx, st, obox, theta=0.5, G=1.0, first=0, last=None, exact=True):
    last = st.n if last is None else last
    ctx.set_exact(exact)
    box = gutil.box_to_sx(obox)
    ds = sx.DeviceState(ctx, gutil.host_dict(st))
    tree, host = gutil.device_tree(ctx, ds.dev["keys"], st.n, 64, box)
    nn = tree.numNodes
    cen = ctx.alloc(4 * nn, np.float64)
    mp = ctx.alloc(8 * nn, np.float32)
    ctx.check(ctx.L.sx_gravity_upsweep(ctx.h, C.byref(ds.fields), C.byref(tree), theta, cen.ptr, mp.ptr), "upsweep")
    g = sx.SxGroups(firstBody=first, lastBody=last, numGroups=(last - first + 63) // 64)
    eg = C.c_double()
    ctx.check(ctx.L.sx_gravity_traverse(ctx.h, C.byref(g), C.byref(ds.fields), C.byref(tree), C.byref(box), cen.ptr,
                                        mp.ptr, G, C.byref(eg)), "traverse")
    out = {k: ds.get(k) for k in ("ax", "ay", "az")}
    out["centers"] = cen.get().reshape(-1, 4)
    out["multipoles"] = mp.get().reshape(-1, 8)
    out["egrav"] = eg.value
    ctx.set_exact(False)
    return out


def check_upsweep_fast(cen, mp, cen_ref, mp_ref):
    """the fast upsweep (one wave per leaf, sums in double over the wave, the quadrupole rounded to float once) against
    the reference's sequential leaf sums: centers to double rounding, each node's moments within 1e-5 of its largest"""
    assert np.allclose(cen[:, :3], cen_ref[:, :3], rtol=0, atol=1e-12 * np.abs(cen_ref[:, :3]).max())
    assert np.allclose(cen[:, 3], cen_ref[:, 3], rtol=1e-12, atol=0)  # MAC radius squared (setMac)
    scale = np.abs(mp_ref).max(axis=1, keepdims=True)
    assert np.all(np.abs(mp.astype(np.float64) - mp_ref) <= 1e-5 * scale), np.max(np.abs(mp - mp_ref) / (scale + 1e-300))


def check_acc(out, ref_arrays, rtol=1e-6, atol_frac=1e-7):
    amax = max(np.max(np.abs(ref_arrays[k])) for k in ("ax", "ay", "az"))
    for k in ("ax", "ay", "az"):
        a, b = out[k].astype(np.float64), ref_arrays[k].astype(np.float64)
        assert np.all(np.abs(a - b) <= rtol * np.abs(b) + atol_frac * amax), (k, np.max(np.abs(a - b)))


@pytest.mark.parametrize("side,theta", [(21, 0.5), (24, 0.9)])
def test_gravity_fast_variant(ctx, ora, side, theta):
    st, box = po.evrard_state(side)
    gutil.sorted_state(st, box, ora)
    out = gpu_gravity(ctx, st, box, theta=theta, exact=False)
    ref = st.copy()
    eg, cen, mp = ora.gravity(ref, box, ora.params(g=1.0, theta=theta))
    check_upsweep_fast(out["centers"], out["multipoles"], cen, mp)
    check_acc(out, ref.arrays, rtol=1e-5, atol_frac=1e-6)
    assert out["egrav"] == pytest.approx(eg, rel=1e-6)
    ctx.free_all()


@pytest.mark.parametrize("side,theta", [(14, 0.5), (21, 0.5), (24, 0.3), (24, 0.9)])
def test_gravity_vs_oracle(ctx, ora, side, theta):
    st, box = po.evrard_state(side)
    gutil.sorted_state(st, box, ora)
    out = gpu_gravity(ctx, st, box, theta=theta)
    ref = st.copy()
    eg, cen, mp = ora.gravity(ref, box, ora.params(g=1.0, theta=theta))
    assert np.array_equal(out["centers"], cen)
    assert np.array_equal(out["multipoles"], mp)
    check_acc(out, ref.arrays)
    assert out["egrav"] == pytest.approx(eg, rel=1e-10)
    ctx.free_all()


def test_gravity_sub_range(ctx, ora):
    """targets [first, last) only (a rank's locals among halos): the others keep their acceleration"""
    st, box = po.evrard_state(18)
    gutil.sorted_state(st, box, ora)
    st.ax[:] = 0.25
    f, l = 100, st.n - 77
    out = gpu_gravity(ctx, st, box, first=f, last=l)
    ref = st.copy()
    ora.gravity(ref, box, ora.params(g=1.0), first=f, last=l)
    check_acc(out, ref.arrays)
    assert np.all(out["ax"][:f] == 0.25) and np.all(out["ax"][l:] == 0.25)
    ctx.free_all()


def test_gravity_golden(ctx):
    d = gu.load("evrard14.npz")
    box = gu.box_from(d["box"])
    st = gu.state_from(d, "s0_")
    out = gpu_gravity(ctx, st, box)
    assert np.array_equal(out["centers"], d["grav_centers"])
    assert np.array_equal(out["multipoles"], d["grav_multipoles"])
    check_acc(out, {k: d["grav_" + k] for k in ("ax", "ay", "az")})
    assert out["egrav"] == pytest.approx(float(d["grav_egrav"][0]), rel=1e-10)
    ctx.free_all()


@pytest.mark.parametrize("side,steps", [(16, 3), (22, 2)])
def test_sim_steps_with_gravity(ctx, ora, side, steps):
    """VE + self-gravity steps of sx_sim (own search, cluster kernels, gravity, acceleration time-step) vs the
    oracle's ox_step with g = 1 (Evrard substitute), per particle (gpu_util.StepChecker; the oracle's scale of a
    includes the magnitude of the gravity terms, so the float M2P/P2P rounding is covered)"""
    from test_gpu_parity import FLOATS

    st, obox = po.evrard_state(side)
    sim = sx.Sim(ctx, st.n, gutil.box_to_sx(obox), params=sx.default_params(g=1.0, theta=0.5))
    sim.set_state(st.arrays, st.minDt, st.minDt_m1)

    def egrav(s, sim, ref):
        assert sim.scalars()["egrav"] == pytest.approx(ref.egrav, rel=1e-5)

    gutil.shadow_steps(ctx, ora, sim, obox, steps, ora.params(g=1.0, theta=0.5), FLOATS, on_step=egrav)
    sim.close()


def test_traverse_group_view(ctx):
    """explicit groups (the ve-bdt active rungs: mHolder_.traverse(gravGroup, ...), ve_hydro_bdt.hpp:279-285): the
    targets of the view's groups get the full traversal's accelerations bitwise (the same wave, the same lists), every
    other target keeps its acceleration, egrav sums over the view"""
    st, obox = po.evrard_state(14)
    keys = po.load_oracle().sfc_keys(st, obox).copy()
    o = np.argsort(keys, kind="stable")
    for k in st.arrays:
        st.arrays[k][:] = st.arrays[k][o]
    st.keys[:] = keys[o]
    full = gpu_gravity(ctx, st, obox, exact=False)
    # a view of every third 64-particle group (the reference extracts such group slices, sph/groups.hpp:31-48)
    n = st.n
    starts = np.arange(0, n, 64, dtype=np.uint32)
    sel = starts[::3]
    gs = ctx.alloc(len(sel), np.uint32)
    ge = ctx.alloc(len(sel), np.uint32)
    gs.set(sel)
    ge.set(np.minimum(sel + 64, n).astype(np.uint32))
    box = gutil.box_to_sx(obox)
    ds = sx.DeviceState(ctx, gutil.host_dict(st))
    inview = np.zeros(n, bool)
    for s0 in sel:
        inview[s0:min(s0 + 64, n)] = True
    marker = np.float32(123.5)
    for k in ("ax", "ay", "az"):
        ds.set(k, np.where(inview, np.float32(0), marker).astype(np.float32))
    tree, host = gutil.device_tree(ctx, ds.dev["keys"], n, 64, box)
    nn = tree.numNodes
    cen = ctx.alloc(4 * nn, np.float64)
    mp = ctx.alloc(8 * nn, np.float32)
    ctx.check(ctx.L.sx_gravity_upsweep(ctx.h, C.byref(ds.fields), C.byref(tree), 0.5, cen.ptr, mp.ptr), "upsweep")
    g = sx.SxGroups(firstBody=0, lastBody=0, numGroups=len(sel), groupStart=gs.ptr, groupEnd=ge.ptr)
    eg = C.c_double()
    ctx.check(ctx.L.sx_gravity_traverse(ctx.h, C.byref(g), C.byref(ds.fields), C.byref(tree), C.byref(box), cen.ptr,
                                        mp.ptr, 1.0, C.byref(eg)), "traverse view")
    for k in ("ax", "ay", "az"):
        got = ds.get(k)
        assert np.all(got[~inview] == marker), k
        assert np.array_equal(got[inview], full[k][inview]), k
    assert 0 > eg.value > full["egrav"]  # part of the sum, same sign


@pytest.mark.parametrize("exact", [False, True])
def test_interaction_counts(ctx, exact):
    """sx_sim_gravity_interactions counts per target like the reference's BhStats (traversal.cuh:346-357): with an
    opening angle so small that every node violates the MAC (mac = 2 size / theta + |com - center| beyond the box even for level-21 nodes), every target interacts by P2P with every particle
    (sumP2P = N^2, sumM2P = 0); at theta = 0.5 both kinds occur (at least one M2P node per target on average) and fewer sources than
    N^2 are visited by P2P"""
    from sphexa_amd import ic

    arrays, lim, bnd, dt0 = ic.evrard(24)  # ~7k particles: at theta 0.5 most sources are then far enough for M2P
    n = arrays["x"].size
    counts = {}
    for theta in (1e-20, 0.5):
        ctx.set_exact(exact)
        sim = sx.Sim(ctx, n, sx.make_box(lim, bnd), params=sx.default_params(g=1.0, theta=theta))
        try:
            sim.set_state(arrays, dt0, dt0)
            sim.step()
            assert sim.gravity_interactions() == {"p2p": 0, "m2p": 0}  # counting is off by default
            sim.set_gravity_counting(True)
            sim.step()
            counts[theta] = sim.gravity_interactions()
        finally:
            sim.close()
            ctx.set_exact(False)
    assert counts[1e-20] == {"p2p": n * n, "m2p": 0}, (n, counts)
    c = counts[0.5]
    assert c["m2p"] >= n and 0 < c["p2p"] < 0.8 * n * n, (n, c)
