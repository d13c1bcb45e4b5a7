"""Group views of the pair kernels: the ve-bdt active rungs (main/src/propagator/ve_hydro_bdt.hpp:222-290).

HydroVeBdtProp passes each kernel a GroupView: on a substep, a slice of the rung-sorted groups (`activeRungs_`,
extracted groups with firstBody = lastBody = 0, sph/groups.hpp:33-58).  The reference's GPU kernels visit only the
view's groups, so every target outside them keeps its previous values -- which are what its active neighbours read
in the later kernels of the substep.  Momentum's Courant step goes per view group into groupDt[k] (min with the
previous value, momentum_energy_gpu.cu:98-104); updateSmoothingLengthGpu updates only the view's targets.

Checks, through the C-ABI with an explicit-group view (a shuffled third of random-size groups, firstBody = lastBody
= 0):
  * exact variant + the oracle's own neighbor list imported: every output of XMass, VeDefGradh, EOS (all targets,
    as the reference's computeEOS(first, last)), IAD + divv/curlv, AV switches and momentum/energy is bit-identical to
    the oracle run over all targets with the targets outside the view restored after each kernel -- i.e. inside the
    view the reference's values, outside it untouched; groupDt[k] bit-identical to the oracle's Courant minimum over
    group k; the h update only inside the view;
  * the search with the h-nc iteration (sx_xmass on the view): h and nc of the view's targets bit-identical to the
    oracle's iteration, the others untouched.
"""
import ctypes as C

import numpy as np
import pytest

import gpu_util as gutil
import pyoracle as po
import sphexa_amd as sx

pytestmark = pytest.mark.gpu

NGMAX = 150


@pytest.fixture(scope="module")
def ctx():
    c = sx.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def ora():
    return po.load_oracle()


def make_view(n, seed):
    """random-size groups (1..64 targets) tiling [0, n); every third one, in shuffled order"""
    rng = np.random.default_rng(seed)
    b = [0]
    while b[-1] < n:
        b.append(min(n, b[-1] + int(rng.integers(1, 65))))
    gs, ge = np.array(b[:-1], np.uint32), np.array(b[1:], np.uint32)
    sel = np.arange(gs.size)[seed % 3::3]
    rng.shuffle(sel)
    act = np.zeros(n, bool)
    for s, e in zip(gs[sel], ge[sel]):
        act[s:e] = True
    return gs[sel].copy(), ge[sel].copy(), act


def advanced(ora, ic, side, steps):
    st, box = (po.sedov_state if ic == "sedov" else po.noh_state)(side)
    for _ in range(steps):
        ora.step(st, box)
    gutil.sorted_state(st, box, ora)
    nbr, nc = ora.find_neighbors(st, box, iterate_h=True)
    st.nc[:] = nc
    return st, box, nbr


STAGES = [("xmass", ["xm"]), ("ve_def_gradh", ["kx", "gradh"]), ("eos", ["prho", "c"]),
          ("iad_divv_curlv", ["c11", "c12", "c13", "c22", "c23", "c33", "divv", "curlv"]), ("av_switches", ["alpha"]),
          ("momentum_energy", ["du", "ax", "ay", "az"])]


def oracle_view_chain(ora, st, box, nbr, act):
    """the reference semantics: each kernel over the view's targets only (computed for all, the others restored)"""
    outs = {}
    for name, fields in STAGES:
        keep = {k: st.arrays[k].copy() for k in fields}
        if name == "eos":
            ora.eos(st)  # computeEOS(first, last): every target
        else:
            getattr(ora, name)(st, box, nbr)
            for k in fields:
                st.arrays[k][~act] = keep[k][~act]
        outs[name] = {k: st.arrays[k].copy() for k in fields}
    return outs


@pytest.mark.parametrize("ic,side,steps,seed", [("sedov", 20, 2, 1), ("noh", 18, 3, 2)])
def test_view_kernels_exact_bitwise(ctx, ora, ic, side, steps, seed):
    st, obox, nbr = advanced(ora, ic, side, steps)
    n = st.n
    gs, ge, act = make_view(n, seed)
    ref = st.copy()
    outs = oracle_view_chain(ora, ref, obox, nbr, act)

    ctx.set_exact(True)
    try:
        box = gutil.box_to_sx(obox)
        ds = sx.DeviceState(ctx, gutil.host_dict(st))
        nb = ctx.upload(nbr)
        ctx.check(ctx.L.sx_import_neighbors(ctx.h, 0, n, NGMAX, nb.ptr), "import")
        gsd, ged = ctx.upload(gs), ctx.upload(ge)
        g = sx.SxGroups(firstBody=0, lastBody=0, numGroups=gs.size, groupStart=gsd.ptr, groupEnd=ged.ptr)
        p = sx.default_params()
        L, h, f = ctx.L, ctx.h, ds.fields
        groupDt0 = np.full(gs.size, 3.0e-3, np.float32)  # min with the previous value
        gdt = ctx.upload(groupDt0)
        calls = {
            "xmass": lambda: L.sx_xmass_only(h, C.byref(g), C.byref(f), C.byref(p), C.byref(box)),
            "ve_def_gradh": lambda: L.sx_ve_def_gradh(h, C.byref(g), C.byref(f), C.byref(p), C.byref(box)),
            "eos": lambda: L.sx_eos(h, 0, n, 10.0, 5.0 / 3.0, f.temp, f.m, f.kx, f.xm, f.gradh, f.prho, f.c, None,
                                    None),
            "iad_divv_curlv": lambda: L.sx_iad_divv_curlv(h, C.byref(g), C.byref(f), C.byref(p), C.byref(box)),
            "av_switches": lambda: L.sx_av_switches(h, C.byref(g), C.byref(f), C.byref(p), C.byref(box),
                                                    float(st.minDt)),
            "momentum_energy": lambda: L.sx_momentum_energy(h, C.byref(g), C.c_void_p(gdt.ptr), C.byref(f), C.byref(p),
                                                            C.byref(box), None),
        }
        for name, fields in STAGES:
            ctx.check(calls[name](), name)
            for k in fields:
                got = ds.get(k)
                assert np.array_equal(got, outs[name][k].astype(got.dtype)), (name, k)
        # per view group: min(previous, Courant minimum over the group's targets)
        want = np.empty(gs.size, np.float32)
        for k, (s, e) in enumerate(zip(gs, ge)):
            tmp = ref.copy()
            dt = ora.momentum_energy(tmp, obox, nbr[int(s) * NGMAX:int(e) * NGMAX], int(s), int(e))
            want[k] = min(groupDt0[k], np.float32(dt))
        assert np.array_equal(gdt.get(), want)
        # h update only inside the view
        h0 = ds.get("h")
        ctx.check(L.sx_update_h_groups(h, C.byref(g), 100, C.c_void_p(ds.dev["nc"].ptr), C.c_void_p(ds.dev["h"].ptr)),
                  "update_h")
        h1 = ds.get("h")
        tmp = ref.copy()
        tmp.h[:] = h0
        for s, e in zip(gs, ge):
            ora.update_h_range(tmp, 100, int(s), int(e))
        assert np.array_equal(h1, tmp.h) and np.array_equal(h1[~act], h0[~act])
    finally:
        ctx.set_exact(False)
        ctx.free_all()


@pytest.mark.parametrize("ic,side,steps,seed", [("sedov", 20, 1, 0), ("noh", 18, 2, 1)])
def test_view_search_h_iteration(ctx, ora, ic, side, steps, seed):
    """sx_xmass on a view: the h-nc iteration runs for the view's targets only"""
    st, obox, _ = advanced(ora, ic, side, steps)
    n = st.n
    st.h[:] = (st.h * np.float32(1.3)).astype(np.float32)  # off the converged h: the iteration runs
    gs, ge, act = make_view(n, seed)
    ref = st.copy()
    _, rnc = ora.find_neighbors(ref, obox, iterate_h=True)
    box = gutil.box_to_sx(obox)
    ds = sx.DeviceState(ctx, gutil.host_dict(st))
    tree, _ = gutil.device_tree(ctx, ds.dev["keys"], n, 64, box)
    gsd, ged = ctx.upload(gs), ctx.upload(ge)
    g = sx.SxGroups(firstBody=0, lastBody=0, numGroups=gs.size, groupStart=gsd.ptr, groupEnd=ged.ptr)
    p = sx.default_params()
    ctx.check(ctx.L.sx_xmass(ctx.h, C.byref(g), C.byref(ds.fields), C.byref(p), C.byref(box), C.byref(tree)), "xmass")
    h, nc = ds.get("h"), ds.get("nc")
    assert np.array_equal(h[act], ref.h[act]) and np.array_equal(nc[act], rnc[act])
    assert np.array_equal(h[~act], st.h[~act]) and np.array_equal(nc[~act], st.nc[~act])
    assert not np.array_equal(h[act], st.h[act])  # the iteration ran
    ctx.free_all()
