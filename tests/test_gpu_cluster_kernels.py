"""Per-kernel parity of the PRODUCTION pair kernels: the LDS cluster kernels of sx_hydro_cluster.hip (polynomial W,
one-pass fused IAD + divv/curlv, folded momentum coefficients, split-K combine), which run whenever the neighbor lists
are the search's own cluster lists (sx_find_neighbors), i.e. in every bench / sx_sim step.

Each kernel is run IN ISOLATION through the C-ABI: its inputs are set to the reference's values (the previous
kernel's reference outputs), so a deviation is this kernel's own.  Reference: the fixture tests/golden/kernels.npz
(made from oracle/_ref, the reference's own CPU loops) and, for larger and non-trivial flows, the oracle (pinned
bit-for-bit to oracle/_ref) on Sedov / Noh states advanced by the oracle itself.

Tolerance, per element and scale-aware (SURVEY.md 8(c) tier 1), no global floor:
    |gpu - ref| <= RTOL * scale_i
  scale_i = the magnitude of the terms of particle i's float sum, exported by the oracle's J-loops
  (ox_set_scales: sum_j |term_j| for du, a (L1 over components), divv/curlv (dv), gradh, and the graddivv sum
  propagated through alphaloc for alpha); positive sums (xm, kx) use their value, the IAD matrix its diagonal
  (c_ij is the inverse of a sum of positive-semidefinite terms), prho/c (no sum) their value.
RTOL = 2e-5: float32 rounding of ~100-term sums in another order (the GPU's neighbor order is the search's stream
order, not the reference's DFS order) and the degree-6 polynomial W instead of the 20000-point table (relative
deviation < 2e-6, sx_kernel_poly.hpp).
The cluster kernels flush float denormals (-fgpu-flush-denormals-to-zero, sx_hydro_cluster.hip): a velocity-moment
product below FLT_MIN (velocity differences ~1e-30 in the quiescent Sedov outskirts) is dropped where the CPU keeps
it, so divv/curlv/dV also get the bound of those drops: norm_kxi * |c|max * 3 * nc * FLT_MIN.  Conversely the
reference's curlv = norm_kxi * sqrt(cv0*cv0 + ...) underflows in float when the cv are below ~3e-23 (squares under
the smallest denormal round to 0: curlv exactly 0 where the GPU's scaled norm keeps ~1e-19), so curlv also gets the
reference's own underflow uncertainty norm_kxi * sqrt(6 * 2^-149).
"""
import ctypes as C

import numpy as np
import pytest

import golden_util as gu
import gpu_util as gutil
import pyoracle as po
import sphexa_amd as sx

pytestmark = pytest.mark.gpu

RTOL = 2e-5
FLOAT_OUT = ["xm", "kx", "gradh", "prho", "c", "c11", "c12", "c13", "c22", "c23", "c33", "divv", "curlv", "alpha",
             "du", "ax", "ay", "az"]
GRADV = ["dV11", "dV12", "dV13", "dV22", "dV23", "dV33"]


@pytest.fixture(scope="module")
def ctx():
    c = sx.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def ora():
    return po.load_oracle()


def reference_chain(ora, st, box, nbr, params, minDt):
    """the oracle's VE kernels on st (in place) with the reference neighbor list; returns per-kernel snapshots of
    the outputs and the per-particle error scales"""
    st.minDt = minDt
    sc = ora.scales_on(st.n)
    try:
        ora.xmass(st, box, nbr, params=params)
        ora.ve_def_gradh(st, box, nbr, params=params)
        ora.eos(st, params=params)
        ora.iad_divv_curlv(st, box, nbr, params=params)
        ora.av_switches(st, box, nbr, params=params)
        dt = ora.momentum_energy(st, box, nbr, params=params)
    finally:
        ora.scales_off()
    ref = {k: st.arrays[k].copy() for k in FLOAT_OUT + (GRADV if params.avClean else []) + ["h", "nc"]}
    ref["minDtCourant"] = np.array([dt])
    return ref, {k: v.copy() for k, v in sc.items()}


def scale_of(k, ref, sc):
    if k in ("xm", "kx", "prho", "c"):
        return np.abs(ref[k].astype(np.float64))
    if k.startswith("c") and len(k) == 3:  # IAD matrix
        return np.maximum(np.maximum(np.abs(ref["c11"]), np.abs(ref["c22"])), np.abs(ref["c33"])).astype(np.float64)
    if k in ("divv", "curlv") or k.startswith("dV"):
        return sc["dv"]
    if k in ("ax", "ay", "az"):
        return sc["a"]
    if k == "du":
        return sc["du"]
    if k == "gradh":
        return sc["gradh"]
    if k == "alpha":
        return np.abs(ref["alpha"].astype(np.float64)) + sc["alpha"]
    raise KeyError(k)


FLT_MIN = float(np.finfo(np.float32).tiny)


def ftz_floor(ref):
    """bound of the flushed (denormal) velocity-moment products in divv/curlv/dV, see the module docstring"""
    K = po.load_oracle().K
    h = ref["h"].astype(np.float64)
    norm = K / (h ** 3 * ref["kx"].astype(np.float64))
    cmax = np.max(np.abs(np.stack([ref[k] for k in ("c11", "c12", "c13", "c22", "c23", "c33")])), axis=0)
    return norm * cmax * 3.0 * ref["nc"].astype(np.float64) * FLT_MIN * 2.0


def check_all(name, got, ref, sc):
    a = got.astype(np.float64)
    b = ref[name].astype(np.float64)
    s = scale_of(name, ref, sc)
    if name in ("divv", "curlv") or name.startswith("dV"):
        s = s + ftz_floor(ref) / RTOL
    if name == "curlv":
        K = po.load_oracle().K
        norm = K / (ref["h"].astype(np.float64) ** 3 * ref["kx"].astype(np.float64))
        s = s + norm * np.sqrt(6.0 * 2.0 ** -149) / RTOL
    err = np.abs(a - b)
    bad = err > RTOL * s
    assert not bad.any(), (name, int(bad.sum()), np.nonzero(bad)[0][:5], float(np.max(err / (s + 1e-300))))
    return float(np.max(err / (s + 1e-300)))


def run_cluster_kernels(ctx, st, box_sx, inputs, ref, sc, params, minDt, av_clean, view=None):
    """GPU: own search (cluster lists) with the reference h, then each kernel in isolation on reference inputs.
    view = (groupStart, groupEnd, active mask): the kernels run on that explicit-group view (a ve-bdt partial
    substep); inside it the reference's values, outside it the previous device values untouched"""
    n = st.n
    host = gutil.host_dict(st)
    for k in ("h", "nc"):
        host[k] = inputs[k]
    ds = sx.DeviceState(ctx, host, grad_v=av_clean)
    tree, _ = gutil.device_tree(ctx, ds.dev["keys"], n, 64, box_sx)
    p = sx.default_params(av_clean=av_clean)
    stats = sx.SxNbStats()
    L, h = ctx.L, ctx.h
    ctx.check(L.sx_find_neighbors(h, C.byref(ds.fields), C.byref(tree), C.byref(box_sx), C.byref(p), 0, n, 0,
                                  C.byref(stats)), "search")
    assert np.array_equal(ds.get("nc"), inputs["nc"])  # same neighbor sets as the reference
    g = sx.SxGroups(firstBody=0, lastBody=n, numGroups=(n + 63) // 64)
    act = np.ones(n, bool)
    if view is not None:
        gs, ge, act = view
        gsd, ged = ctx.upload(gs), ctx.upload(ge)
        g = sx.SxGroups(firstBody=0, lastBody=0, numGroups=gs.size, groupStart=gsd.ptr, groupEnd=ged.ptr)
    f = ds.fields
    worst = {}
    before = {}

    def setf(names, src):
        for k in names:
            ds.set(k, src[k])
        for k in names:
            before[k] = src[k]

    def check(name, got, ref, sc):
        """inside the view against the oracle; outside it the value the device held before the kernel"""
        if view is None:
            return check_all(name, got, ref, sc)
        prev = before[name] if name in before else host.get(name, np.zeros(n, got.dtype))
        assert np.array_equal(got[~act], np.asarray(prev)[~act].astype(got.dtype)), ("outside the view", name)
        return check_all(name, np.where(act, got, ref[name].astype(got.dtype)), ref, sc)

    ctx.check(L.sx_xmass_only(h, C.byref(g), C.byref(f), C.byref(p), C.byref(box_sx)), "xmass")
    worst["xm"] = check("xm", ds.get("xm"), ref, sc)
    setf(["xm"], ref)
    ctx.check(L.sx_ve_def_gradh(h, C.byref(g), C.byref(f), C.byref(p), C.byref(box_sx)), "gradh")
    for k in ("kx", "gradh"):
        worst[k] = check(k, ds.get(k), ref, sc)
    setf(["kx", "gradh"], ref)
    ctx.check(L.sx_eos(h, 0, n, 10.0, 5.0 / 3.0, f.temp, f.m, f.kx, f.xm, f.gradh, f.prho, f.c, None, None), "eos")
    for k in ("prho", "c"):  # computeEOS(first, last): every target, view or not
        worst[k] = check_all(k, ds.get(k), ref, sc)
    setf(["prho", "c"], ref)
    ctx.check(L.sx_iad_divv_curlv(h, C.byref(g), C.byref(f), C.byref(p), C.byref(box_sx)), "iad")
    for k in ["c11", "c12", "c13", "c22", "c23", "c33", "divv", "curlv"] + (GRADV if av_clean else []):
        worst[k] = check(k, ds.get(k), ref, sc)
    setf(["c11", "c12", "c13", "c22", "c23", "c33", "divv", "curlv"] + (GRADV if av_clean else []), ref)
    ctx.check(L.sx_av_switches(h, C.byref(g), C.byref(f), C.byref(p), C.byref(box_sx), float(minDt)), "av")
    worst["alpha"] = check("alpha", ds.get("alpha"), ref, sc)
    setf(["alpha"], ref)
    mdt = C.c_float()
    me = L.sx_momentum_energy_avclean if av_clean else L.sx_momentum_energy
    ctx.check(me(h, C.byref(g), None, C.byref(f), C.byref(p), C.byref(box_sx), C.byref(mdt)), "momentum")
    for k in ("du", "ax", "ay", "az"):
        worst[k] = check(k, ds.get(k), ref, sc)
    if view is None:
        assert mdt.value == pytest.approx(float(ref["minDtCourant"][0]), rel=1e-5)
    ctx.free_all()
    return worst


def test_cluster_kernels_fixture(ctx, ora):
    """kernels.npz (12^3 Sedov state, reference outputs from oracle/_ref)"""
    d = gu.load("kernels.npz")
    box = gu.box_from(d["box"])
    st = gu.state_from(d, "in_")
    st.h[:] = d["h_after_iter"]
    st.nc[:] = d["nc"]
    chk = st.copy()
    ref, sc = reference_chain(ora, chk, box, d["nbr"], ora.params(), st.minDt)
    for k in FLOAT_OUT:  # the oracle reproduces the fixture bit for bit (it is pinned to the reference)
        assert np.array_equal(ref[k], d[k].astype(ref[k].dtype)), k
    inputs = {"h": d["h_after_iter"], "nc": d["nc"]}
    run_cluster_kernels(ctx, st, gutil.box_to_sx(box), inputs, ref, sc, ora.params(), st.minDt, False)


def advanced_state(ora, ic, side, steps, params):
    st, box = (po.sedov_state if ic == "sedov" else po.noh_state)(side)
    for _ in range(steps):
        ora.step(st, box, params=params)
    gutil.sorted_state(st, box, ora)
    nbr, nc = ora.find_neighbors(st, box, iterate_h=True)
    st.nc[:] = nc
    return st, box, nbr


@pytest.mark.parametrize("ic,side,steps,av_clean", [("sedov", 30, 2, False), ("noh", 24, 3, False),
                                                     ("noh", 20, 3, True)])
def test_cluster_kernels_vs_oracle(ctx, ora, ic, side, steps, av_clean):
    """27k-particle Sedov and Noh states after a few oracle steps (non-zero velocities, shocks, AV active;
    several 256-particle clusters, unions of ~1200 records, the split-K momentum combine)"""
    params = ora.params(av_clean=av_clean)
    st, box, nbr = advanced_state(ora, ic, side, steps, params)
    chk = st.copy()
    ref, sc = reference_chain(ora, chk, box, nbr, params, st.minDt)
    inputs = {"h": st.h.copy(), "nc": st.nc.copy()}
    worst = run_cluster_kernels(ctx, st, gutil.box_to_sx(box), inputs, ref, sc, params, st.minDt, av_clean)
    print(ic, side, {k: f"{v:.2e}" for k, v in worst.items()})


@pytest.mark.parametrize("ic,side,steps,seed,av_clean", [("sedov", 24, 2, 1, False), ("noh", 20, 3, 2, True)])
def test_cluster_kernels_view_vs_oracle(ctx, ora, ic, side, steps, seed, av_clean):
    """the production kernels on a ve-bdt partial-substep view (a shuffled third of random-size explicit groups, as
    the rung-sorted activeRungs_ slices are): the view's targets within the per-kernel tolerance of the oracle, every
    other target untouched"""
    from test_gpu_group_views import make_view

    params = ora.params(av_clean=av_clean)
    st, box, nbr = advanced_state(ora, ic, side, steps, params)
    chk = st.copy()
    ref, sc = reference_chain(ora, chk, box, nbr, params, st.minDt)
    inputs = {"h": st.h.copy(), "nc": st.nc.copy()}
    view = make_view(st.n, seed)
    assert 0 < view[2].sum() < st.n
    run_cluster_kernels(ctx, st, gutil.box_to_sx(box), inputs, ref, sc, params, st.minDt, av_clean, view=view)


STD_OUT = ["rho", "p", "c", "c11", "c12", "c13", "c22", "c23", "c33", "du", "ax", "ay", "az"]


@pytest.mark.parametrize("ic,side,steps", [("sedov", 24, 2), ("noh", 22, 3)])
def test_cluster_kernels_std_vs_oracle(ctx, ora, ic, side, steps):
    """std propagator (HydroProp): density (xmass into rho), EOS_HydroStd, IAD with m/rho volumes and
    momentumEnergySTD as cluster kernels, each in isolation on the oracle's inputs"""
    params = ora.params(std=True)
    st, box, nbr = advanced_state(ora, ic, side, steps, params)
    chk = st.copy()
    sc = ora.scales_on(st.n)
    try:
        ora.density(chk, box, nbr, params=params)
        ora.eos_std(chk, params=params)
        ora.iad_std(chk, box, nbr, params=params)
        dt = ora.momentum_energy_std(chk, box, nbr, params=params)
    finally:
        ora.scales_off()
    ref = {k: chk.arrays[k].copy() for k in STD_OUT}
    sc = {k: v.copy() for k, v in sc.items()}
    n = st.n
    host = gutil.host_dict(st)
    ds = sx.DeviceState(ctx, host, std=True)
    box_sx = gutil.box_to_sx(box)
    tree, _ = gutil.device_tree(ctx, ds.dev["keys"], n, 64, box_sx)
    p = sx.default_params(std=True)
    L, h = ctx.L, ctx.h
    ctx.check(L.sx_find_neighbors(h, C.byref(ds.fields), C.byref(tree), C.byref(box_sx), C.byref(p), 0, n, 0, None),
              "search")
    assert np.array_equal(ds.get("nc"), st.nc)
    g = sx.SxGroups(firstBody=0, lastBody=n, numGroups=(n + 63) // 64)
    f = ds.fields

    def close(k, scale):
        a, b = ds.get(k).astype(np.float64), ref[k].astype(np.float64)
        err = np.abs(a - b)
        assert np.all(err <= RTOL * scale), (k, float(np.max(err / (scale + 1e-300))))

    ctx.check(L.sx_density_only(h, C.byref(g), C.byref(f), C.byref(p), C.byref(box_sx)), "density")
    close("rho", np.abs(ref["rho"]))
    ds.set("rho", ref["rho"])
    ctx.check(L.sx_eos_std(h, 0, n, 10.0, 5.0 / 3.0, f.temp, f.m, f.rho, f.p, f.c), "eos_std")
    close("p", np.abs(ref["p"]))
    close("c", np.abs(ref["c"]))
    ds.set("p", ref["p"])
    ds.set("c", ref["c"])
    ctx.check(L.sx_iad(h, C.byref(g), C.byref(f), C.byref(p), C.byref(box_sx)), "iad")
    diag = np.maximum(np.maximum(np.abs(ref["c11"]), np.abs(ref["c22"])), np.abs(ref["c33"])).astype(np.float64)
    for k in ("c11", "c12", "c13", "c22", "c23", "c33"):
        close(k, diag)
        ds.set(k, ref[k])
    mdt = C.c_float()
    ctx.check(L.sx_momentum_energy_std(h, C.byref(g), C.byref(f), C.byref(p), C.byref(box_sx), C.byref(mdt)), "me")
    close("du", sc["du"])
    for k in ("ax", "ay", "az"):
        close(k, sc["a"])
    assert mdt.value == pytest.approx(dt, rel=1e-5)
    ctx.free_all()


def test_mark_ramp_on_cluster_lists(ctx, ora):
    """computeMarkRamp (hydro_ve/additional_fields.cu:47-98, markRampJLoop additional_fields_kern.hpp:38-58) on the
    search's own cluster lists vs numpy over the reference neighbor list of the fixture (same sets, float sums in
    another order: 1e-5 relative); a Noh state has Atwood numbers across the whole ramp"""
    params = ora.params()
    st, box, nbr = advanced_state(ora, "noh", 20, 3, params)
    chk = st.copy()
    ref, _ = reference_chain(ora, chk, box, nbr, params, st.minDt)
    n = st.n
    rho = (ref["kx"].astype(np.float32) * st.m / ref["xm"]).astype(np.float32)
    cnt = np.minimum(st.nc.astype(np.int64) - 1, 150)
    nb = nbr.reshape(n, 150)
    want = np.zeros(n, np.float64)
    p = sx.default_params()
    for i in range(n):
        js = nb[i, :cnt[i]]
        at = np.abs(rho[i] - rho[js]) / (rho[i] + rho[js])
        want[i] = np.sum(np.where(at > p.Atmax, 1.0, np.where(at >= p.Atmin, p.ramp * (at - p.Atmin), 0.0))) / cnt[i]
    host = gutil.host_dict(st)
    host["xm"], host["kx"] = ref["xm"], ref["kx"]
    ds = sx.DeviceState(ctx, host)
    box_sx = gutil.box_to_sx(box)
    tree, _ = gutil.device_tree(ctx, ds.dev["keys"], n, 64, box_sx)
    ctx.check(ctx.L.sx_find_neighbors(ctx.h, C.byref(ds.fields), C.byref(tree), C.byref(box_sx), C.byref(p), 0, n, 0,
                                      None), "search")
    out = ctx.alloc(n, np.float32)
    g = sx.SxGroups(firstBody=0, lastBody=n, numGroups=(n + 63) // 64)
    ctx.check(ctx.L.sx_mark_ramp(ctx.h, C.byref(g), C.byref(ds.fields), C.byref(p), C.byref(box_sx), out.ptr), "ramp")
    got = out.get().astype(np.float64)
    assert np.max(want) > 0.5  # the ramp is exercised
    assert np.all(np.abs(got - want) <= 1e-5 * np.abs(want) + 1e-7), float(np.max(np.abs(got - want)))
    ctx.free_all()
