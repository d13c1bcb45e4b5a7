"""The Ewald correction of periodic self-gravity on the GPU (sx_gravity_ewald, the reference's computeGravityEwaldGpu)
against the reference's own outputs and the restatement pinned to it bit for bit (tests/test_ewald_oracle.py):
* tests/golden/ewald_ref.npz (ryoanji::computeGravityEwald compiled from the reference, oracle/gen_ewald.py), three
  settings: |a - a_ref| <= 2e-6 max|a_ref| (float accelerations; the device's double exp/erf/erfc/sin/cos may differ
  from the C library's by a few ulp; measured on MI355X: bit-identical on all three), energy to 1e-10;
* a larger periodic cube against the restatement, with a target sub-range (the others untouched);
* physics: a uniform lattice in its periodic box feels no net force -- the 27 images summed directly (numpy, softened
  like P2P) plus the GPU correction with numReplicaShells = 1 leave < 2e-3 of the direct sum's largest |a| (the
  restatement: 7.9e-4);
* a non-cubic box is refused (the reference throws, ewald.hpp:386);
* the walk over the periodic images (sx_gravity_traverse_pbc, numShells 1) against the reference's computeGravity with
  numShells = 1 (tests/golden/grav_pbc_ref.npz, oracle/gen_grav_pbc.py): upsweep bit-identical, accelerations as the
  open walk's test (exact variant: 1e-6 |a| + 1e-7 max|a|; fast: 1e-5, 1e-6), egrav 1e-10 / 1e-6;
* the whole step in a periodic box with self-gravity (walk + Ewald): a uniform medium at rest feels no force (< 1e-2
  of the open box's largest gravity); ve-bdt with periodic self-gravity is refused."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

import golden_util as gu
import sphexa_amd as sx

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import ewald as ew  # noqa: E402
import gen_ewald as ge  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = sx.Context(0)
    yield c
    c.close()


def gpu_ewald(ctx, x, y, z, m, M, center, lo, hi, G, settings, first=0, last=None, acc0=None, lims=None):
    n = len(x)
    last = n if last is None else last
    host = {"x": x, "y": y, "z": z, "m": m}
    if acc0 is not None:
        host.update(ax=acc0[0], ay=acc0[1], az=acc0[2])
    ds = sx.DeviceState(ctx, host)
    cen = ctx.upload(np.array([center[0], center[1], center[2], 0.0], np.float64))
    mp = ctx.upload(np.asarray(M, np.float32))
    box = sx.make_box(lims or [lo, hi, lo, hi, lo, hi], [1, 1, 1])
    g = sx.SxGroups(firstBody=first, lastBody=last, numGroups=(last - first + 63) // 64)
    s = sx.SxEwaldSettings(**settings)
    eg = C.c_double(0.0)
    rc = ctx.L.sx_gravity_ewald(ctx.h, C.byref(g), C.byref(ds.fields), C.byref(box), cen.ptr, mp.ptr, G, C.byref(s),
                                C.byref(eg))
    return rc, np.stack([ds.get("ax"), ds.get("ay"), ds.get("az")]), eg.value


def _settings(s):
    t = {**ew.SETTINGS, **s}
    return dict(numReplicaShells=t["numReplicaShells"], lCut=t["lCut"], hCut=t["hCut"], alphaScale=t["alpha_scale"],
                smallRScaleFactor=t["small_R_scale_factor"])


@pytest.mark.parametrize("case", list(ge.CASES))
def test_ewald_vs_reference_golden(ctx, case):
    d = gu.load("ewald_ref.npz")
    lo, hi = d["box"]
    rc, acc, eg = gpu_ewald(ctx, d["x"], d["y"], d["z"], d["m"], d["M"], d["center"], lo, hi, float(d["G"][0]),
                            _settings(ge.CASES[case]))
    assert rc == 0
    ref = d[f"{case}_acc"].astype(np.float64)
    err = np.abs(acc - ref).max() / np.abs(ref).max()
    print(case, "max |a - a_ref| / max|a_ref|", f"{err:.2g}", "exact fraction", float(np.mean(acc == d[f"{case}_acc"])))
    assert err <= 2e-6, err
    assert eg == pytest.approx(float(d[f"{case}_egrav"][0]), rel=1e-10)
    ctx.free_all()


def test_ewald_vs_restatement_subrange(ctx):
    lo, hi = -1.0, 1.5
    x, y, z, m = ge.cube(n=5000, seed=21, lo=lo, hi=hi)
    M, c = ge.root_moments(x, y, z, m)
    acc0 = np.full((3, len(x)), 0.25, np.float32)
    f, l = 123, len(x) - 77
    rc, acc, eg = gpu_ewald(ctx, x, y, z, m, M, c, lo, hi, 0.5, _settings({}), first=f, last=l, acc0=acc0)
    assert rc == 0
    ref = acc0.copy()
    e_ref = ew.gravity_ewald(x[f:l], y[f:l], z[f:l], m[f:l], M, c, hi - lo, 0.5, ref[0, f:l], ref[1, f:l],
                             ref[2, f:l])
    assert np.all(acc[:, :f] == 0.25) and np.all(acc[:, l:] == 0.25)
    scale = np.abs(ref[:, f:l] - 0.25).max()
    assert np.abs(acc - ref).max() <= 2e-6 * scale + 1e-7, np.abs(acc - ref).max()
    assert eg == pytest.approx(e_ref, rel=1e-10)
    ctx.free_all()


def test_lattice_periodic_force_vanishes(ctx):
    side = 10
    L, lo = 1.0, -0.5
    g1 = (np.arange(side) + 0.5) / side * L + lo
    X, Y, Z = np.meshgrid(g1, g1, g1, indexing="ij")
    x, y, z = X.ravel(), Y.ravel(), Z.ravel()
    n = x.size
    m = np.full(n, 1.0 / n, np.float32)
    h = np.full(n, 0.6 / side)
    M, c = ge.root_moments(x, y, z, m)
    # the walk's part: the central box and its 26 neighbors summed directly, softened with h_i + h_j like P2P
    A = np.zeros((3, n))
    for ix in (-1, 0, 1):
        for iy in (-1, 0, 1):
            for iz in (-1, 0, 1):
                dx = x[None, :] + ix * L - x[:, None]
                dy = y[None, :] + iy * L - y[:, None]
                dz = z[None, :] + iz * L - z[:, None]
                R2e = np.maximum(dx * dx + dy * dy + dz * dz, (h[:, None] + h[None, :]) ** 2)
                w = m[None, :] / R2e ** 1.5
                if ix == iy == iz == 0:
                    np.fill_diagonal(w, 0.0)
                A += np.stack([(dx * w).sum(1), (dy * w).sum(1), (dz * w).sum(1)])
    amax = np.sqrt((A ** 2).sum(0)).max()
    rc, acc, _ = gpu_ewald(ctx, x, y, z, m, M, c, lo, lo + L, 1.0, _settings({"numReplicaShells": 1}),
                           acc0=A.astype(np.float32))
    assert rc == 0
    rest = np.sqrt((acc.astype(np.float64) ** 2).sum(0)).max()
    print("lattice: direct 27-image max |a|", f"{amax:.3g}", "after the Ewald correction", f"{rest:.3g}")
    assert rest < 2e-3 * amax, (rest, amax)
    ctx.free_all()


def test_ewald_refuses_non_cubic_box(ctx):
    x, y, z, m = ge.cube(n=100, seed=3)
    M, c = ge.root_moments(x, y, z, m)
    rc, _, _ = gpu_ewald(ctx, x, y, z, m, M, c, -0.5, 0.5, 1.0, _settings({}),
                         lims=[-0.5, 0.5, -0.5, 0.5, -0.5, 0.6])
    assert rc == sx.SX_ERR_ARG
    ctx.free_all()


@pytest.mark.parametrize("exact", [True, False])
def test_periodic_walk_vs_reference(ctx, exact):
    import gen_grav_pbc as gp
    import gpu_util as gutil
    import pyoracle as po
    d = gu.load("grav_pbc_ref.npz")
    ora = po.load_oracle()
    st, obox = gp.state()
    keys = ora.sfc_keys(st, obox).copy()
    o = np.argsort(keys, kind="stable")
    for k in po.CONSERVED:
        st.arrays[k][:] = st.arrays[k][o]
    st.keys[:] = keys[o]
    assert np.array_equal(st.x, d["x"]) and np.array_equal(st.m, d["m"])
    ctx.set_exact(exact)
    try:
        box = gutil.box_to_sx(obox)
        ds = sx.DeviceState(ctx, gutil.host_dict(st))
        tree, _ = gutil.device_tree(ctx, ds.dev["keys"], st.n, 64, box)
        nn = tree.numNodes
        cen = ctx.alloc(4 * nn, np.float64)
        mp = ctx.alloc(8 * nn, np.float32)
        ctx.check(ctx.L.sx_gravity_upsweep(ctx.h, C.byref(ds.fields), C.byref(tree), 0.5, cen.ptr, mp.ptr), "upsweep")
        g = sx.SxGroups(firstBody=0, lastBody=st.n, numGroups=(st.n + 63) // 64)
        eg = C.c_double()
        assert ctx.L.sx_gravity_traverse(ctx.h, C.byref(g), C.byref(ds.fields), C.byref(tree), C.byref(box), cen.ptr,
                                         mp.ptr, 1.0, C.byref(eg)) == sx.SX_ERR_ARG  # periodic: the image walk only
        ctx.check(ctx.L.sx_gravity_traverse_pbc(ctx.h, C.byref(g), C.byref(ds.fields), C.byref(tree), C.byref(box),
                                                cen.ptr, mp.ptr, 1.0, 1, C.byref(eg)), "traverse_pbc")
        if exact:
            assert np.array_equal(cen.get().reshape(-1, 4), d["centers"])
            assert np.array_equal(mp.get().reshape(-1, 8), d["multipoles"])
        else:  # the fast upsweep's per-wave leaf sums (tests/test_gpu_gravity.py)
            from test_gpu_gravity import check_upsweep_fast
            check_upsweep_fast(cen.get().reshape(-1, 4), mp.get().reshape(-1, 8), d["centers"], d["multipoles"])
        acc = np.stack([ds.get("ax"), ds.get("ay"), ds.get("az")]).astype(np.float64)
    finally:
        ctx.set_exact(False)
    ref = d["shells1_acc"].astype(np.float64)
    rtol, afrac = (1e-6, 1e-7) if exact else (1e-5, 1e-6)
    # complete 16-target groups only: the reference pads the last group's target array with zeros
    # (traversal_cpu.hpp:190-197), which its shifted images carry to -(ix Lx, iy Ly, iz Lz) and into that group's box
    n = st.n - st.n % 16
    err = np.abs(acc - ref) - (rtol * np.abs(ref) + afrac * np.abs(ref).max())
    print("periodic walk", "exact" if exact else "fast", "max |a - a_ref| complete groups",
          f"{np.abs(acc - ref)[:, :n].max():.3g}", "last group", f"{np.abs(acc - ref)[:, n:].max():.3g}",
          "worst index", int(np.argmax(np.abs(acc - ref).max(0))), "of", st.n, "max|a|", f"{np.abs(ref).max():.3g}")
    assert err[:, :n].max() <= 0, err[:, :n].max()
    assert np.abs(acc - ref)[:, n:].max() <= 1e-3 * np.abs(ref).max()
    assert eg.value == pytest.approx(float(d["shells1_egrav"][0]), rel=1e-5)
    ctx.free_all()


def test_sim_periodic_gravity_uniform_medium(ctx):
    """a uniform lattice at rest with uniform temperature in its periodic box: no pressure gradient and, with the image
    walk + Ewald correction, no net gravity; the same medium in an open box falls inwards"""
    import pyoracle as po
    res = {}
    for bnd in (1, 0):
        st, obox = po.sedov_state(12)
        st.temp[:] = np.float64(st.temp.min())
        for k in ("vx", "vy", "vz"):
            st.arrays[k][:] = 0
        for k in ("x", "y", "z"):
            st.arrays[k + "_m1"][:] = 0
        box = sx.make_box(list(obox.lim), [bnd] * 3)
        sim = sx.Sim(ctx, st.n, box, params=sx.default_params(g=1.0))
        try:
            sim.set_state(st.arrays, st.minDt, st.minDt_m1)
            sim.step()
            assert sim.stats()["numFailed"] == 0
            f = sim.get(["ax", "ay", "az"])
            res[bnd] = np.sqrt(f["ax"].astype(float) ** 2 + f["ay"] ** 2 + f["az"] ** 2).max()
            assert np.isfinite(sim.conserved()["egrav"])
        finally:
            sim.close()
    print("uniform medium: max |a| periodic", f"{res[1]:.3g}", "open", f"{res[0]:.3g}")
    assert res[1] < 1e-2 * res[0], res


def test_sim_refuses_periodic_self_gravity_bdt(ctx):
    box = sx.make_box([-0.5, 0.5, -0.5, 0.5, -0.5, 0.5], [1, 1, 1])
    with pytest.raises(Exception):
        sx.Sim(ctx, 1000, box, params=sx.default_params(g=1.0, bdt=True))


def test_sim_refuses_mixed_or_noncubic_periodic_gravity(ctx):
    """self-gravity with periodic images needs a box periodic along every axis (the reference decides on boundaryX and
    would walk images along open axes) and a cube (the Ewald sum): refused at creation, not half-way through a step"""
    for lim, bnd in (([-0.5, 0.5] * 3, [1, 0, 1]), ([-0.5, 0.5] * 3, [0, 1, 1]), ([-0.5, 0.5, -0.5, 0.5, -1, 1], [1] * 3)):
        with pytest.raises(Exception):
            sx.Sim(ctx, 1000, sx.make_box(lim, bnd), params=sx.default_params(g=1.0))


def test_sim_periodic_gravity_crossing_particles_skin_off(ctx):
    """with periodic self-gravity every step syncs (no skin reuse step), so a particle that crossed a periodic
    face is in the leaf of its wrapped position when the multipoles are formed.  A medium drifting through the box
    (particles cross the faces every few steps) with the default skin gives the same accelerations and potential,
    bit for bit by id, and the same potential to rounding, as the same run with the skin off"""
    import pyoracle as po
    out = {}
    for skin in (0.08, 0.0):
        st, obox = po.sedov_state(12)
        st.temp[:] = np.float64(st.temp.min()) * (1 + 0.1 * np.sin(7 * st.x))
        # a uniform drift of 0.4 lattice spacings (1/12) per first step in x, 0.2 in y: relative velocities stay zero,
        # so the time-step grows by maxDtIncrease per step and the medium moves several spacings in six steps
        v = 0.4 / 12 / st.minDt
        st.arrays["vx"][:] = np.float32(v)
        st.arrays["vy"][:] = np.float32(0.5 * v)
        st.arrays["vz"][:] = 0
        for k in ("x", "y", "z"):
            st.arrays[k + "_m1"][:] = st.arrays["v" + k] * np.float32(st.minDt)
        sim = sx.Sim(ctx, st.n, sx.make_box(list(obox.lim), [1, 1, 1]), params=sx.default_params(g=1.0))
        try:
            sim.set_skin(skin, 24)
            sim.set_state(st.arrays, st.minDt, st.minDt_m1)
            rec = []
            for _ in range(6):
                sim.step()
                assert sim.stats()["numFailed"] == 0
                f = sim.get(["id", "ax", "ay", "az", "x"])
                o = np.argsort(f["id"])
                rec.append(({k: f[k][o] for k in ("ax", "ay", "az", "x")}, sim.conserved()["egrav"]))
            assert sim.skin_stats()["reuse_steps"] == 0
            out[skin] = rec
        finally:
            sim.close()
    x0 = out[0.0][0][0]["x"]
    assert np.any(np.abs(out[0.0][-1][0]["x"] - x0) > 0.5), "no particle crossed a periodic face"
    for (a, ea), (b, eb) in zip(out[0.08], out[0.0]):
        for k in ("ax", "ay", "az"):
            assert np.array_equal(a[k], b[k]), k
        assert abs(ea - eb) <= 1e-12 * abs(eb)  # the Ewald energy is summed with device atomics (order varies)
