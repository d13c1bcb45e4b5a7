"""Conserved quantities on the GPU (sx_conserved_quantities / sx_sim_conserved) against the numpy restatement of
localConservedQuantities (oracle/pyoracle.py, conserved_quantities.hpp:49-101): double sums, relative 1e-12
(only the summation order differs)."""
import ctypes as C

import numpy as np
import pytest

import gpu_util as gutil
import pyoracle as po
import sphexa_amd as sx

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = sx.Context(0)
    yield c
    c.close()


def test_conserved_quantities_random(ctx):
    rng = np.random.default_rng(7)
    n = 100003
    st = po.HostState(n)
    st.x[:], st.y[:], st.z[:] = rng.uniform(-1, 1, (3, n))
    for k in ("vx", "vy", "vz"):
        st.arrays[k][:] = rng.normal(0, 1, n).astype(np.float32)
    st.m[:] = rng.uniform(0.5, 1.5, n).astype(np.float32)
    st.temp[:] = rng.uniform(1e-3, 1e-2, n)
    st.nc[:] = rng.integers(50, 150, n).astype(np.uint32)
    ds = sx.DeviceState(ctx, gutil.host_dict(st))
    out = (C.c_double * 9)()
    first, last = 17, n - 5
    ctx.check(ctx.L.sx_conserved_quantities(ctx.h, C.byref(ds.fields), first, last, 10.0, 5.0 / 3.0, out), "cq")
    ek, ei, lin, ang, nc = po.conserved_quantities(st, first, last)
    got = list(out)
    assert got[0] == pytest.approx(ek, rel=1e-12) and got[1] == pytest.approx(ei, rel=1e-12)
    scale = float(np.sum(st.m[first:last]) * 3)
    assert np.allclose(got[2:5], lin, rtol=0, atol=1e-12 * scale)
    assert np.allclose(got[5:8], ang, rtol=0, atol=1e-12 * scale)
    assert got[8] == nc
    ctx.free_all()


def test_sim_conserved_energy(ctx):
    """sx_sim_conserved after Sedov steps: matches the numpy sums of the downloaded state; total energy of the
    n=30 lattice drifts by < 1e-5 over 5 steps"""
    st, obox = po.sedov_state(30)
    sim = sx.Sim(ctx, st.n, gutil.box_to_sx(obox))
    sim.set_state(st.arrays, st.minDt, st.minDt_m1)
    e0 = None
    for s in range(5):
        sim.step()
        c = sim.conserved()
        got = sim.get(["x", "y", "z", "vx", "vy", "vz", "m", "temp", "nc"])
        hs = po.HostState(st.n)
        for k, v in got.items():
            hs.arrays[k][:] = v
        ek, ei, lin, ang, nc = po.conserved_quantities(hs)
        assert c["ecin"] == pytest.approx(ek, rel=1e-12) and c["eint"] == pytest.approx(ei, rel=1e-12)
        assert c["totalNeighbors"] == nc and c["egrav"] == 0.0
        assert c["etot"] == pytest.approx(ek + ei, rel=1e-12)
        e0 = c["etot"] if e0 is None else e0
    assert abs(c["etot"] - e0) < 1e-5 * e0
    sim.close()


@pytest.mark.parametrize("suffix", ["npz", "h5"])
def test_checkpoint_restart_bitwise(ctx, tmp_path, suffix):
    """save after 2 Sedov steps, continue 2 steps; a new simulation restarted from the file reproduces those 2
    steps bit for bit (the step is deterministic: atomics only take minima / ORs); .h5 = the reference's H5Part
    layout (sphexa_amd.h5part, pinned to the reference's reader/writer in tests/test_h5part.py)"""
    st, obox = po.sedov_state(20)
    box = gutil.box_to_sx(obox)
    a = sx.Sim(ctx, st.n, box)
    a.set_state(st.arrays, st.minDt, st.minDt_m1)
    a.step()
    a.step()
    ck = str(tmp_path / f"restart.{suffix}")
    a.save_checkpoint(ck)
    a.step()
    a.step()
    names = ["id", "x", "y", "z", "vx", "vy", "vz", "temp", "h", "alpha", "du_m1"]
    ga = a.get(names)
    b = sx.Sim(ctx, st.n, box)
    b.load_checkpoint(ck)
    b.step()
    b.step()
    gb = b.get(names)
    oa, ob = np.argsort(ga["id"]), np.argsort(gb["id"])
    for k in names:
        assert np.array_equal(ga[k][oa], gb[k][ob]), k
    assert a.scalars() == b.scalars()  # incl. ttot: the restart continues the file's time
    d = b._read_checkpoint(ck, -1)  # the reference's restart attributes (particles_data.hpp:170-190)
    assert all(n in d for n in sx.ATTRIBUTE_NAMES)
    assert int(d["iteration"]) == 2 and int(d["numParticlesGlobal"]) == st.n
    assert b.iteration == 4
    a.close()
    b.close()


@pytest.mark.parametrize("suffix", ["npz", "h5"])
def test_ve_bdt_checkpoint_restart_bitwise(ctx, tmp_path, suffix):
    """ve-bdt (propagator 2) restart: the file holds the rung of every particle (ConservedFields,
    ve_hydro_bdt.hpp:94) and the Timestep's numRungs and dt_m1 under "ts::" (HydroVeBdtProp::save/load, :153-168);
    restarting from a hierarchy boundary reproduces the uninterrupted run's next hierarchy bit for bit, and a save
    inside a hierarchy is refused (the reference writes files only when isSynced(), sphexa.cpp:165)"""
    st, obox = po.sedov_state(20)
    box = gutil.box_to_sx(obox)
    params = sx.default_params(bdt=True)
    a = sx.Sim(ctx, st.n, box, params=params)
    a.set_state(st.arrays, st.minDt, st.minDt_m1)
    ck = str(tmp_path / f"restart_bdt.{suffix}")
    seen_multi, saved, refused = False, False, False
    for _ in range(60):
        a.step()
        ts = a.timestep()
        seen_multi |= ts["numRungs"] > 1
        if not sx.Sim._hierarchy_boundary(ts):
            if not refused:
                with pytest.raises(ValueError):
                    a.save_checkpoint(str(tmp_path / f"mid.{suffix}"))
                refused = True
        elif seen_multi:
            a.save_checkpoint(ck)
            saved = True
            break
    assert saved and refused, "no multi-rung hierarchy formed"
    d = a._read_checkpoint(ck, -1)
    num_rungs = int(d["ts::numRungs"])
    assert num_rungs > 1 and np.asarray(d["ts::dt_m1"]).dtype == np.float32 and d["rung"].max() > 0
    substeps = 2 * (1 << num_rungs) + 1  # past the end of the next hierarchy, into the one after
    for _ in range(substeps):
        a.step()
    names = ["id", "x", "y", "z", "vx", "vy", "vz", "temp", "h", "alpha", "du_m1", "rung"]
    ga = a.get(names)
    b = sx.Sim(ctx, st.n, box, params=params)
    b.load_checkpoint(ck)
    for _ in range(substeps):
        b.step()
    gb = b.get(names)
    oa, ob = np.argsort(ga["id"]), np.argsort(gb["id"])
    for k in names:
        assert np.array_equal(ga[k][oa], gb[k][ob]), k
    assert a.scalars() == b.scalars() and a.timestep() == b.timestep()
    a.close()
    b.close()
