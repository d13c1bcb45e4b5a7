"""BASELINE configs 3, 4 and 5 at full size, run un-reseeded to their configured lengths on one GPU.

test_gpu_fullsize.py checks the full-size problems over 2-3 steps; here they run as long as BASELINE.json configures
them (missing #1: shock formation at 14M particles, the redo-list search, large unions and AV's second
launch over a whole run, and the Evrard collapse over 100 steps):
  * Noh -n 300 -s 100 (config 3, 14.1M particles) and Evrard -n 300 -s 100 with self-gravity (config 5, 14.1M) against
    the reference's own CPU run of the same IC at the same size (oracle/gen_trajectory.py --fast noh300 evrard300 ->
    tests/golden/traj_noh300.npz, traj_evrard300.npz): the time of every step within 1e-3, the energy of every step
    (Evrard: kinetic + internal + the step's potential) within 1e-5 of the reference's energy, the binned radial
    profiles of rho, p, |v|, u (oracle/trajectory.py) within 1 % at the profile steps; Noh also the reference's
    analytic check, the density L1 against nohRho (compare_noh.py:49-61,141-153), within 2 % of the reference run's;
  * Sedov -n 400 (config 4's workload, 64M particles, on one GPU) against the reference's own CPU run for 30 steps
    (traj_sedov400.npz: a full skin rebuild falls inside them), and over the configured 200 steps, which the
    reference cannot run in test time, through size-independent properties: the energy drift within 1.5x the reference's own n=50
    budget over 200 steps, and the density L1 against the reference's analytic solution (self-similar rescale to the
    fixture's time, as the config-2 test) below the n=200 run's 0.032 (test_gpu_trajectory.py, round 4): resolution
    convergence;
  * every step: no search/h failure, maxNeighbors <= ngmax; at the end ids a permutation, h and temp finite.
"""
import numpy as np
import pytest

import golden_util as gu
import pyoracle as po
import sphexa_amd as sx
import trajectory as tj

pytestmark = pytest.mark.gpu


def _step_checked(sim, case, s):
    st = sim.stats()
    assert st["numFailed"] == 0 and st["maxNeighbors"] <= 150, (case, s, st)


def _final_checks(sim, n):
    f = sim.get(["id", "h", "temp"])
    assert np.array_equal(np.sort(f["id"]), np.arange(n, dtype=np.uint64))
    assert np.all(np.isfinite(f["h"])) and np.all(f["h"] > 0) and np.all(np.isfinite(f["temp"]))


def _run_vs_reference(case):
    fname, init, side, steps, prof_steps, rmax, nbins = tj.CASES[case]
    kw = tj.CASE_PARAMS.get(case, {})
    grav = kw.get("g", 0.0) != 0.0
    fx = gu.load(fname)
    st, obox = getattr(po, init + "_state")(side)
    n = st.n
    ctx = sx.Context(0)
    sim = sx.Sim(ctx, n, sx.make_box(list(obox.lim), list(obox.bnd)), params=sx.default_params(**kw))
    ttot, etot, egrav, prof = [0.0], [tj.energies(st.arrays)[0]], [np.nan], {}
    try:
        sim.set_state(st.arrays, st.minDt, st.minDt_m1)
        del st
        for s in range(1, steps + 1):
            sim.step()
            _step_checked(sim, case, s)
            c = sim.conserved()
            ttot.append(sim.scalars()["ttot"])
            etot.append(c["ecin"] + c["eint"])
            egrav.append(c["egrav"] if grav else np.nan)
            if s in prof_steps:
                prof[s] = tj.profiles(sim.get(tj.FIELDS), rmax, nbins)[1]
        final = sim.get(tj.FIELDS)
        _final_checks(sim, n)
        skin = sim.skin_stats()
    finally:
        sim.close()
        ctx.close()
    t_ref, e_ref = fx["series_ttot"], fx["series_etot"]
    dt_rel = np.abs(np.array(ttot[1:]) / t_ref[1:] - 1)
    if grav:  # the potential of step s is computed inside step s, for both runs
        tot_ref = e_ref[1:] + fx["series_egrav"][1:]
        tot = np.array(etot[1:]) + np.array(egrav[1:])
        de = np.abs(tot - tot_ref) / abs(tot_ref[0])
        print(case, "reference etot (incl. egrav) drift", f"{tot_ref[-1] / tot_ref[0] - 1:.3g}",
              "GPU", f"{tot[-1] / tot[0] - 1:.3g}")
    else:
        de = np.abs(np.array(etot) - e_ref) / e_ref[0]
    l1 = {s: {k: tj.profile_l1(prof[s][k], fx[f"s{s}_{k}"], fx[f"s{s}_count"]) for k in ("rho", "p", "vel", "u")}
          for s in prof_steps}
    print(case, "time rel max", f"{dt_rel.max():.2g}", "energy vs ref max", f"{de.max():.2g}",
          {s: {k: f"{v:.2g}" for k, v in d.items()} for s, d in l1.items()})
    assert dt_rel.max() < 1e-3, dt_rel.max()
    assert de.max() < 1e-5, (de.max(), int(np.argmax(de)))
    for s, d in l1.items():
        for k, v in d.items():
            assert v <= 0.01, (case, s, k, v)
    return fx, final, ttot[-1], skin


def test_noh_n300_100_steps_vs_reference():
    fx, final, t, _ = _run_vs_reference("noh300")
    for key, rho0 in (("ref_l1_noh_density_attr", tj.NOH_RHO0_ATTR), ("ref_l1_noh_density_ic", tj.NOH_RHO0_IC)):
        l1, ref = tj.noh_l1(final, t, rho0), float(fx[key][0])
        print(f"Noh -n 300 -s 100 density L1 vs nohRho (rho0 = {rho0:.4g}) at t = {t:.6g}: GPU {l1:.4f}, "
              f"reference {ref:.4f}")
        assert abs(l1 / ref - 1) <= 0.02, (key, l1, ref)


def test_evrard_n300_gravity_100_steps_vs_reference():
    _run_vs_reference("evrard300")


def test_sedov_n400_30_steps_vs_reference():
    """the metric's own workload (Sedov -n 400, 64M particles) against the reference's CPU run of the same lattice
    (tests/golden/traj_sedov400.npz, oracle/gen_trajectory.py --fast sedov400): 30 steps un-reseeded with the default
    skin lists, so that the forced full sync + rebuild of every skin after max_reuse = 24 filter-served steps falls
    inside the compared window; time, energy of every step, binned profiles at steps 10/20/30, and the density L1 against
    the reference's analytic solution within 2 % of the reference run's"""
    fx, final, t, skin = _run_vs_reference("sedov400")
    assert skin["builds"] >= 2 and skin["reuse_steps"] >= 24, skin
    rho, _ = tj.eos_rho_p(final)
    l1 = tj.analytic_l1(tj.radii(final), rho.astype(np.float64), fx["sol"][:, 0], fx["sol"][:, 1])
    ref = float(fx["ref_l1_density_subsampled"][0])
    print(f"Sedov -n 400 -s 30: t = {t:.6g}, density L1 vs analytic GPU {l1:.4f}, reference {ref:.4f}; skin {skin}")
    assert abs(l1 / ref - 1) <= 0.02, (l1, ref)


def test_sedov_n400_200_steps_full_size():
    side, steps = 400, 200
    n = side ** 3
    fx = gu.load(tj.CASES["sedov"][0])
    ctx = sx.Context(0)
    sim = sx.Sim(ctx, n, sx.make_box([-0.5, 0.5, -0.5, 0.5, -0.5, 0.5], [1, 1, 1]))
    try:
        sim.init_sedov(side)
        e0 = sim.conserved()["etot"]
        emax = 0.0
        for s in range(1, steps + 1):
            sim.step()
            _step_checked(sim, "sedov400", s)
            if s % 10 == 0:
                emax = max(emax, abs(sim.conserved()["etot"] / e0 - 1))
        _final_checks(sim, n)
        f = sim.get(tj.FIELDS)
        t = sim.scalars()["ttot"]
    finally:
        sim.close()
        ctx.close()
    ref_budget = float(np.max(np.abs(fx["series_etot"] / fx["series_etot"][0] - 1)))
    rho, _ = tj.eos_rho_p(f)
    l1 = tj.analytic_l1(tj.radii(f) * (float(fx["sol_time"][0]) / t) ** 0.4, rho.astype(np.float64), fx["sol"][:, 0],
                        fx["sol"][:, 1])
    print(f"Sedov -n 400 -s 200: t = {t:.6g}, energy drift max {emax:.3g} (reference n=50 budget {ref_budget:.3g}), "
          f"density L1 vs analytic {l1:.4f} (n=200: 0.032)")
    assert emax <= 1.5 * ref_budget, (emax, ref_budget)
    assert l1 < 0.032, l1
