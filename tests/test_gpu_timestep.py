"""Block time-step seam (HydroVeBdtProp, main/src/propagator/ve_hydro_bdt.hpp) on the GPU, bit-exact against the
oracle's restatement (sph_oracle.c ox_positions_rungs / ox_drift_positions / ox_group_*_dt, which repeat the
reference's positions.hpp:54-88 formulas and ts_groups.cu:17-108):
  sx_positions_rungs     computePositionsGpu with dt_m1 per rung (positions_gpu.cu:110-179)
  sx_drift_positions     driftPositionsGpu (positions_gpu.cu:45-108)
  sx_group_divv_timestep groupDivvTimestepGpu, sx_group_acc_timestep groupAccTimestepGpu, sx_store_rung storeRungGpu
on spatial groups (sx_spatial_groups) and on the implicit fixed 64-groups, with rung arrays and without.
temp is bit-exact while u stays positive; energyUpdate's u < 0 guard (cooling) evaluates u_old*exp(x) with |x| up to
~50 when du is random, where an ulp of the device exp vs glibc's, amplified by |x| through the drift's two updates,
shows up: the test with such du holds temp to a relative 1e-13 instead."""
import ctypes as C

import numpy as np
import pytest

import gpu_util as gutil
import pyoracle as po
import sphexa_amd as sx

pytestmark = pytest.mark.gpu
P = C.c_void_p


@pytest.fixture(scope="module")
def ctx():
    c = sx.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def olib():
    lib = po.load_oracle().lib
    lib.ox_positions_rungs.argtypes = [C.POINTER(po.OxState), P, P, C.c_uint, C.c_float, P, P, C.c_double,
                                       C.POINTER(po.OxBox)]
    lib.ox_drift_positions.argtypes = [C.POINTER(po.OxState), P, P, C.c_uint, C.c_float, C.c_float, P, P,
                                       C.c_double]
    lib.ox_group_divv_dt.argtypes = [C.c_float, P, P, C.c_uint, P, P]
    lib.ox_group_acc_dt.argtypes = [C.c_float, P, P, C.c_uint, P, P, P, P]
    return lib


def moving_state(side, seed, periodic=True, cooling=False):
    st, obox = po.sedov_state(side)
    gutil.sorted_state(st, obox, po.load_oracle())  # SFC order first: the fields below are not permuted by it
    rng = np.random.default_rng(seed)
    n = st.n
    for k in ("vx", "vy", "vz", "ax", "ay", "az", "divv"):
        st.arrays[k][:] = rng.standard_normal(n).astype(np.float32) * (0.3 if k[0] == "v" else 20.0)
    for k in ("x_m1", "y_m1", "z_m1"):
        st.arrays[k][:] = rng.standard_normal(n).astype(np.float32) * 1e-6
    u = st.temp * po.ideal_gas_cv()
    scale = 10.0 if cooling else 0.1 * u / 1e-3  # |du dt| < u/10 keeps u > 0 unless cooling
    st.du[:] = rng.standard_normal(n) * scale
    st.du_m1[:] = (rng.standard_normal(n) * scale).astype(np.float32)
    if not periodic:
        obox = po.make_box(-0.5, 0.5, False)
    return st, obox


def groups_of(ctx, ora, st, obox, spatial):
    n = st.n
    if not spatial:
        starts = np.arange(0, n, 64, dtype=np.uint32)
        return starts, np.minimum(starts + 64, n).astype(np.uint32), None
    t = ora.octree(st.keys, 64)
    layout = np.concatenate([[0], np.cumsum(t["counts"])]).astype(np.uint32)
    g = ora.group_splits(0, n, st.x, st.y, st.z, t["leaves"], layout, obox, 2.0)
    return g[:-1].copy(), g[1:].copy(), g


@pytest.mark.parametrize("spatial,use_rung,periodic,cooling", [(True, True, True, False), (False, True, False, False),
                                                               (True, False, True, False), (True, True, True, True)])
def test_positions_drift_groupdt_bitexact(ctx, olib, spatial, use_rung, periodic, cooling):
    ora = po.load_oracle()
    st, obox = moving_state(20, 3, periodic, cooling)
    ttol = 1e-13 if cooling else 0.0
    gs, ge, bounds = groups_of(ctx, ora, st, obox, spatial)
    ng = gs.size
    rng = np.random.default_rng(4)
    rung = rng.integers(0, 4, st.n).astype(np.uint8) if use_rung else None
    dt_m1 = np.array([1e-4, 2e-4, 4e-4, 8e-4], np.float32)
    dt, dt_back = np.float32(1.7e-4), np.float32(0.6e-4)
    constCv = float(po.ideal_gas_cv())
    box = gutil.box_to_sx(obox)

    ds = sx.DeviceState(ctx, gutil.host_dict(st))
    if bounds is not None:
        db = ctx.upload(bounds)
        grp = sx.SxGroups(firstBody=0, lastBody=st.n, numGroups=ng, groupStart=db.ptr, groupEnd=db.ptr + 4)
    else:
        grp = sx.SxGroups(firstBody=0, lastBody=st.n, numGroups=ng)
    drung = ctx.upload(rung) if use_rung else None
    L, h = ctx.L, ctx.h

    # group time-steps
    gdt = ctx.upload(np.full(ng, 1e30, np.float32))
    ctx.check(L.sx_group_divv_timestep(h, np.float32(0.06), C.byref(grp), ds.dev["divv"].ptr, gdt.ptr), "divv dt")
    ctx.check(L.sx_group_acc_timestep(h, np.float32(0.2 * np.sqrt(0.005)), C.byref(grp), ds.dev["ax"].ptr,
                                      ds.dev["ay"].ptr, ds.dev["az"].ptr, gdt.ptr), "acc dt")
    ref_dt = np.full(ng, 1e30, np.float32)
    olib.ox_group_divv_dt(np.float32(0.06), gs.ctypes.data, ge.ctypes.data, ng, st.divv.ctypes.data,
                          ref_dt.ctypes.data)
    olib.ox_group_acc_dt(np.float32(0.2 * np.sqrt(0.005)), gs.ctypes.data, ge.ctypes.data, ng, st.ax.ctypes.data,
                         st.ay.ctypes.data, st.az.ctypes.data, ref_dt.ctypes.data)
    assert np.array_equal(gdt.get(), ref_dt)

    # store rungs: rung g % 4 for group g
    rg = ctx.upload(np.zeros(st.n, np.uint8))
    for r in range(4):
        if bounds is not None:
            sel = np.arange(r, ng, 4)
            sub = np.concatenate([gs[sel], ge[sel]]).astype(np.uint32)
            dsub = ctx.upload(sub)
            g2 = sx.SxGroups(firstBody=0, lastBody=st.n, numGroups=sel.size, groupStart=dsub.ptr,
                             groupEnd=dsub.ptr + 4 * sel.size)
            ctx.check(L.sx_store_rung(h, C.byref(g2), r, rg.ptr), "store rung")
    if bounds is not None:
        want = np.zeros(st.n, np.uint8)
        for g in range(ng):
            want[gs[g]:ge[g]] = g % 4
        assert np.array_equal(rg.get(), want)

    # drift of every group, then the rung-aware position update
    ctx.check(L.sx_drift_positions(h, C.byref(grp), dt, dt_back, dt_m1.ctypes.data,
                                   drung.ptr if use_rung else None, C.byref(ds.fields), 5.0 / 3.0, constCv), "drift")
    ref = st.copy()
    s = ref.struct()
    rp = rung.ctypes.data if use_rung else None
    olib.ox_drift_positions(C.byref(s), gs.ctypes.data, ge.ctypes.data, ng, dt, dt_back, dt_m1.ctypes.data, rp,
                            constCv)
    for k in ("x", "y", "z", "vx", "vy", "vz", "x_m1", "du_m1"):
        assert np.array_equal(ds.get(k), ref.arrays[k]), ("drift", k)
    assert np.allclose(ds.get("temp"), ref.temp, rtol=ttol, atol=0), "drift temp"
    ctx.check(L.sx_positions_rungs(h, C.byref(grp), dt, dt_m1.ctypes.data, drung.ptr if use_rung else None,
                                   C.byref(ds.fields), 5.0 / 3.0, constCv, C.byref(box)), "positions")
    olib.ox_positions_rungs(C.byref(s), gs.ctypes.data, ge.ctypes.data, ng, dt, dt_m1.ctypes.data, rp, constCv,
                            C.byref(obox))
    for k in ("x", "y", "z", "vx", "vy", "vz", "x_m1", "y_m1", "z_m1", "du_m1"):
        assert np.array_equal(ds.get(k), ref.arrays[k]), ("positions", k)
    assert np.allclose(ds.get("temp"), ref.temp, rtol=ttol, atol=0), "positions temp"
    ctx.free_all()
