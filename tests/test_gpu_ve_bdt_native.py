"""The native ve-bdt propagator: sx_sim with propagator 2 (sph-exa_amd/csrc/sx_bdt.cpp), HydroVeBdtProp
(main/src/propagator/ve_hydro_bdt.hpp:51-378) in C++ on sx_sim's domain.

* One rank, exact and production kernels: every substep (full syncs, partial syncs, rung re-sorting, drift of the
  inactive rungs) leaves the conserved fields, rungs, nc and the Timestep bit-identical to the seam driver
  sphexa_amd.ve_bdt.HydroVeBdtProp, which test_gpu_ve_bdt.py pins bit for bit to the CPU oracle (exact kernels).
* avClean (HydroVeBdtProp<true>): the velocity-gradient correction over two hierarchies conserves energy.
  The bitwise cases include self-gravity on the active rungs (MultipoleHolder::traverse(gravGroup), :272-286; Noh
  with G = 1 in its open box) and avClean (HydroVeBdtProp<true>).
* Self-gravity with one rung (Evrard): ve-bdt follows the VE propagator step for step.
* 2 and 3 ranks on one GPU (host-staged transport): one rung hierarchy on every rank (rungTimestep is min-reduced),
  the merged positions after the first substep close to the single-rank run, energy conserved.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import gpu_util as gutil
import pyoracle as po
import sphexa_amd as sx
from sphexa_amd.ve_bdt import HydroVeBdtProp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONS = ["x", "y", "z", "h", "m", "temp", "vx", "vy", "vz", "x_m1", "y_m1", "z_m1", "du_m1", "alpha", "id"]


@pytest.fixture(scope="module")
def ctx():
    c = sx.Context(0)
    yield c
    c.close()


def initial(ic, side, ora):
    st, box = {"sedov": po.sedov_state, "noh": po.noh_state, "evrard": po.evrard_state}[ic](side)
    po.converge_h(ora, st, box)
    return st, box


def energy(g):
    v2 = sum(g[k].astype(np.float64) ** 2 for k in ("vx", "vy", "vz"))
    return np.sum(0.5 * g["m"] * v2) + np.sum(g["m"] * np.float64(po.ideal_gas_cv()) * g["temp"])


@pytest.mark.parametrize("ic,exact,opts", [("sedov", True, {}), ("sedov", False, {}), ("noh", True, {}),
                                           ("noh", False, {}), ("noh", False, {"g": 1.0}), ("noh", True, {"g": 1.0}),
                                           ("sedov", False, {"av_clean": True})])
def test_native_bdt_bitwise_seam_driver(ctx, ic, exact, opts):
    ora = po.load_oracle()
    st, obox = initial(ic, 14, ora)
    host = {k: st.arrays[k].copy() for k in CONS}
    box = gutil.box_to_sx(obox)
    ctx.set_exact(exact)
    params = sx.default_params(bdt=True, **opts)
    sim = sx.Sim(ctx, st.n + 64, box, params=params)
    try:
        prop = HydroVeBdtProp(ctx, host, box, st.minDt, params=sx.default_params(bdt=True, **opts))
        sim.set_state(host, st.minDt, st.minDt)
        partial, rungs = 0, 1
        for s in range(10):
            partial += not prop.is_synced()
            prop.step()
            sim.step()
            got = sim.get(CONS + ["rung", "nc"])
            for k in CONS + ["rung", "nc"]:
                ref = prop.get(k)
                assert np.array_equal(got[k], ref), (s, k, int(np.sum(got[k] != ref)))
            ts, pt = sim.timestep(), prop.ts
            assert ts["numRungs"] == pt.numRungs and ts["substep"] == pt.substep, (s, ts)
            assert ts["rungRanges"] == list(pt.rungRanges), s
            assert np.float32(ts["nextDt"]) == np.float32(pt.nextDt), s
            assert np.array_equal(np.float32(ts["dt_m1"]), np.float32(pt.dt_m1[:])), s
            assert np.array_equal(np.float32(ts["dt_drift"]), np.float32(pt.dt_drift[:])), s
            sc = sim.scalars()
            assert sc["minDt"] == prop.min_dt and sc["ttot"] == pytest.approx(prop.ttot, rel=1e-12)
            if "g" in opts:
                assert sc["egrav"] == prop.egrav and prop.egrav < 0, s
            rungs = max(rungs, ts["numRungs"])
        assert partial > 0 and rungs >= 2, "no partial substep ran: the hierarchy had a single rung"
    finally:
        sim.close()
        ctx.set_exact(False)
        ctx.free_all()


def test_native_bdt_avclean_conserves_energy(ctx):
    ora = po.load_oracle()
    st, obox = initial("sedov", 16, ora)
    host = {k: st.arrays[k].copy() for k in CONS}
    e0 = po.total_energy(st)
    sim = sx.Sim(ctx, st.n + 64, gutil.box_to_sx(obox), params=sx.default_params(bdt=True, av_clean=True))
    try:
        sim.set_state(host, st.minDt, st.minDt)
        rungs = 1
        for s in range(12):
            sim.step()
            rungs = max(rungs, sim.timestep()["numRungs"])
            e = energy(sim.get(["vx", "vy", "vz", "m", "temp"]))
            assert abs(e / e0 - 1) < 1e-6, (s, e / e0 - 1)
        assert rungs >= 2
        f = sim.get(["dV11", "dV22", "dV33"])
        assert all(np.all(np.isfinite(v)) for v in f.values()) and np.any(f["dV11"] != 0)
    finally:
        sim.close()
        ctx.free_all()


def test_native_bdt_single_rung_follows_ve(ctx):
    """Evrard with self-gravity keeps one rung (dt grows by maxDtIncrease each step): every substep starts a hierarchy,
    gravity acts on all targets, and the ve-bdt run follows the VE propagator (which keeps dt in double in the
    position update where ve-bdt passes float, computePositionsGpu's signature: agreement to float rounding)"""
    ora = po.load_oracle()
    st, obox = initial("evrard", 20, ora)
    host = {k: st.arrays[k].copy() for k in CONS}
    runs = {}
    for bdt in (False, True):
        sim = sx.Sim(ctx, st.n + 64, gutil.box_to_sx(obox), params=sx.default_params(bdt=bdt, g=1.0))
        try:
            sim.set_state(host, st.minDt, st.minDt)
            out = []
            for s in range(6):
                sim.step()
                if bdt:
                    assert sim.timestep()["numRungs"] == 1 and sim.timestep()["substep"] == 1
                out.append((sim.get(CONS), sim.conserved()))
            runs[bdt] = out
        finally:
            sim.close()
    for s in range(6):
        (a, ca), (b, cb) = runs[False][s], runs[True][s]
        oa, ob = np.argsort(a["id"]), np.argsort(b["id"])
        for k in ("x", "y", "z", "vx", "vy", "vz", "temp", "h"):
            x, y = a[k][oa].astype(np.float64), b[k][ob].astype(np.float64)
            assert np.all(np.abs(x - y) <= 1e-6 * np.abs(x) + 1e-6 * np.max(np.abs(x))), (s, k)
        assert cb["egrav"] == pytest.approx(ca["egrav"], rel=1e-6) and cb["egrav"] < 0
    ctx.free_all()


def run_ranks(tmp_path, nproc, side, steps, port, ic="sedov", g=0.0):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", str(nproc), "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "tests", "dist_worker.py"), "--out",
           str(tmp_path), "--side", str(side), "--steps", str(steps), "--ic", ic, "--g", str(g), "--bdt"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    why = "\n".join(line for line in r.stderr.splitlines() if "sx_sim_step" in line or "Error" in line)
    assert r.returncode == 0, why + r.stdout[-2000:] + r.stderr[-2000:]
    return [dict(np.load(os.path.join(tmp_path, f"rank{q}.npz"))) for q in range(nproc)]


@pytest.mark.parametrize("nproc,port,ic,g", [(2, 29651, "sedov", 0.0), (3, 29652, "sedov", 0.0),
                                             (2, 29653, "noh", 1.0)])
def test_native_bdt_multirank(ctx, tmp_path, nproc, port, ic, g):
    """with G = 1 (Noh's open box) the inactive rungs' gravity stays untouched on every rank (the multi-rank
    traversal takes the active view as a target mask)"""
    side, steps = 16, 6
    ranks = run_ranks(tmp_path, nproc, side, steps, port, ic, g)
    # single rank, same IC (the Sedov workers start from the unconverged lattice h, the Noh ones from converged h)
    st, obox = initial("noh", side, po.load_oracle()) if ic == "noh" else po.sedov_state(side)
    e0 = po.total_energy(st)
    sim = sx.Sim(ctx, st.n + 64, gutil.box_to_sx(obox), params=sx.default_params(bdt=True, g=g))
    try:
        sim.set_state({k: st.arrays[k] for k in CONS}, st.minDt, st.minDt_m1)
        for s in range(steps):
            sim.step()
            one = sim.get(CONS)
            tss = {tuple(d[f"s{s}_ts"][:2]) for d in ranks}
            assert len(tss) == 1, (s, tss)  # one hierarchy: numRungs and substep agree on every rank
            got = {k: np.concatenate([d[f"s{s}_{k}"] for d in ranks]) for k in ["id"] + CONS[:-1] + ["rung"]}
            o = np.argsort(got["id"])
            assert np.array_equal(got["id"][o], np.arange(st.n))
            e = energy({k: got[k] for k in ("vx", "vy", "vz", "m", "temp")})
            assert g != 0.0 or abs(e / e0 - 1) < 1e-6, (s, e / e0 - 1)
            if s == 0:
                # the first substep is a full sync on both sides; its dt is the global minimum either way, but the
                # rank-local spatial groups (and the rank-local 40 % fractile of rungTimestep) may put a particle
                # on another rung, i.e. drifted instead of advanced: positions agree to O(a dt^2), far below h
                oi = np.argsort(one["id"])
                hmax = float(np.max(one["h"]))
                for k in ("x", "y", "z"):
                    d = np.abs(got[k][o].astype(np.float64) - one[k][oi].astype(np.float64))
                    assert np.max(d) < 1e-3 * hmax, (k, np.max(d), hmax)
        assert any(ranks[0][f"s{s}_ts"][0] > 1 for s in range(steps)), "the hierarchy had a single rung"
    finally:
        sim.close()
        ctx.free_all()
