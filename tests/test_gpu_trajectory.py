"""Trajectory parity: whole GPU runs at the configured step counts, un-reseeded, against the reference's own runs.

The per-step tests (test_gpu_parity.py, gpu_util.shadow_steps) hand the oracle the GPU's state before every step, so
they pin the step map but not what accumulates over a run.  Here the GPU runs alone from the IC for the configured
number of steps, and the run is compared with the reference CPU path's run of the same IC (oracle/_ref; fixtures
tests/golden/traj_*.npz made by oracle/gen_trajectory.py):
  * Sedov -n 50 -s 200 (the reference CI's case, .jenkins/reframe_ci.py:286) and the Noh lattice -n 30 -s 100;
  * binned radial profiles of rho, p, |v|, u (oracle/trajectory.py) at three steps of each run: particle-weighted
    relative L1 distance <= 1 % (SURVEY 8(c) tier 3);
  * the time of every step (the integrated dt series) within 1e-3 relative, and the total energy of every step within
    1e-5 of the initial energy of the reference's energy at that step (the reference itself drifts by -1.2e-3 on Sedov
    and +1e-4 on Noh over these runs: the test pins the GPU to the reference's budget, not to exact conservation) --
    at the steps both runs take with the same dt; a dt limiter that triggers one step apart leaves a transient
    excursion at the step between (at most 3 such steps, 5e-5), and the final energy within 1e-5;
  * Sedov: the density L1 against the reference's analytic solution (main/src/analytical_solutions/sedov_solution, at
    the final time; computeL1Error of compare_solutions.py:85-89) within +-0.01 of the reference run's own L1 (the CI
    band's width, reframe_ci.py:350-351).  The reference CI records 0.138 for this case; this revision's reference
    CPU path gives 0.336 with the VE propagator (t = 0.1155 after 200 steps) and 0.161 with the std propagator
    (t = 0.0679), both measured here with the reference's own solver (oracle/gen_trajectory.py).  Neither reproduces
    the CI value, so it is unpinned and each band is centred on the reference run of the same propagator;
  * Noh: the density L1 against nohRho (compare_noh.py:49-61,141-153) within 2 % of the reference run's.
Full size: Sedov -n 200 -s 200 (config 2, 8M particles) as a property run: no search/h error, ids a permutation,
energy within the reference's n=50 budget, the analytic density L1 below the n=50 value (resolution convergence).
"""
import numpy as np
import pytest

import golden_util as gu
import pyoracle as po
import sphexa_amd as sx
import trajectory as tj

pytestmark = pytest.mark.gpu


def _run(case):
    fname, init, side, steps, prof_steps, rmax, nbins = tj.CASES[case]
    kw = tj.CASE_PARAMS.get(case, {})
    std = bool(kw.get("std", False))
    fields = tj.FIELDS_STD if std else tj.FIELDS
    fx = gu.load(fname)
    st, obox = getattr(po, init + "_state")(side)
    ctx = sx.Context(0)
    sim = sx.Sim(ctx, st.n, sx.make_box(list(obox.lim), list(obox.bnd)), params=sx.default_params(**kw))
    got = {"ttot": [0.0], "etot": [tj.energies(st.arrays)[0]]}
    prof = {}
    try:
        sim.set_state(st.arrays, st.minDt, st.minDt_m1)
        for s in range(1, steps + 1):
            sim.step()
            assert sim.stats()["numFailed"] == 0, (case, s)
            f = sim.get(fields)
            got["ttot"].append(sim.scalars()["ttot"])
            got["etot"].append(tj.energies(f)[0])
            if s in prof_steps:
                prof[s] = tj.profiles(f, rmax, nbins, std=std)[1]
        final = f
        ids = np.sort(sim.get(["id"])["id"])
        assert np.array_equal(ids, np.arange(st.n, dtype=np.uint64))
    finally:
        sim.close()
        ctx.close()
    return fx, got, prof, final


def _check(case, fx, got, prof):
    _, _, _, steps, prof_steps, _, _ = tj.CASES[case]
    t_ref = fx["series_ttot"]
    t_got = np.array(got["ttot"])
    dt_rel = np.abs(t_got[1:] / t_ref[1:] - 1)
    e_ref = fx["series_etot"]
    e_got = np.array(got["etot"])
    de = np.abs(e_got - e_ref) / e_ref[0]
    l1 = {s: {k: tj.profile_l1(prof[s][k], fx[f"s{s}_{k}"], fx[f"s{s}_count"]) for k in ("rho", "p", "vel", "u")}
          for s in prof_steps}
    print(case, "time rel max", f"{dt_rel.max():.2g}", "energy vs ref max", f"{de.max():.2g}",
          "(ref drift", f"{e_ref[-1] / e_ref[0] - 1:.3g})",
          {s: {k: f"{v:.2g}" for k, v in d.items()} for s, d in l1.items()})
    assert dt_rel.max() < 1e-3, dt_rel.max()
    # energy step by step where both runs took the same step (dt within 2 %): a time-step limiter that triggers one step
    # apart (rounding-level state differences decide which step crosses its threshold; Sedov step 187 with skin
    # lists: the reference's dt drops 10 % there, this run's one step later) gives the one step between a transient
    # excursion of the step-indexed energy, so such steps (at most 3) get 5e-5, and the run must end within 1e-5
    same = np.abs(np.diff(t_got) / np.diff(t_ref) - 1) < 0.02
    de_s = de[1:]
    print(case, "steps with the reference's dt", int(same.sum()), "of", same.size,
          "energy max there", f"{de_s[same].max():.2g}", "elsewhere", f"{de_s[~same].max() if (~same).any() else 0:.2g}")
    assert de_s[same].max() < 1e-5, (de_s[same].max(), int(np.argmax(np.where(same, de_s, 0))) + 1)
    assert (~same).sum() <= 3 and de.max() < 5e-5 and de[-1] < 1e-5, (int((~same).sum()), de.max(), de[-1])
    for s, d in l1.items():
        for k, v in d.items():
            assert v <= 0.01, (case, s, k, v)


def test_sedov_n50_200_steps_vs_reference():
    fx, got, prof, final = _run("sedov")
    _check("sedov", fx, got, prof)
    sol = fx["sol"]
    rho, _ = tj.eos_rho_p(final)
    l1 = tj.analytic_l1(tj.radii(final), rho.astype(np.float64), sol[:, 0], sol[:, 1])
    ref = float(fx["ref_l1_density_subsampled"][0])
    print(f"Sedov -n 50 -s 200 density L1 vs analytic: GPU {l1:.4f}, reference {ref:.4f} "
          f"(t = {got['ttot'][-1]:.6g} vs {float(fx['sol_time'][0]):.6g})")
    assert abs(l1 - ref) <= 0.01, (l1, ref)


def test_noh_n30_100_steps_vs_reference():
    fx, got, prof, final = _run("noh")
    _check("noh", fx, got, prof)
    # the reference's Noh check (compare_noh.py:141-153): density L1 against nohRho at the final time, with the
    # reference's rho0 attribute and with the IC's own density; within 2 % of the reference run's values
    t = got["ttot"][-1]
    for key, rho0 in (("ref_l1_noh_density_attr", tj.NOH_RHO0_ATTR), ("ref_l1_noh_density_ic", tj.NOH_RHO0_IC)):
        l1, ref = tj.noh_l1(final, t, rho0), float(fx[key][0])
        print(f"Noh -n 30 -s 100 density L1 vs nohRho (rho0 = {rho0:.4g}): GPU {l1:.4f}, reference {ref:.4f}")
        assert abs(l1 / ref - 1) <= 0.02, (key, l1, ref)


def test_sedov_n50_std_200_steps_vs_reference():
    """the std propagator (HydroProp) over the CI's Sedov case against the reference's std run, and its analytic
    density L1 (0.161 at t = 0.0679 for the reference; the VE run's is 0.336 at t = 0.1155; the CI's 0.138 is
    reproduced by neither)"""
    fx, got, prof, final = _run("sedov_std")
    _check("sedov_std", fx, got, prof)
    rho, _ = tj.eos_rho_p(final, std=True)
    l1 = tj.analytic_l1(tj.radii(final), rho.astype(np.float64), fx["sol"][:, 0], fx["sol"][:, 1])
    ref = float(fx["ref_l1_density_subsampled"][0])
    print(f"Sedov std -n 50 -s 200 density L1 vs analytic: GPU {l1:.4f}, reference {ref:.4f}")
    assert abs(l1 - ref) <= 0.01, (l1, ref)


def test_sedov_n200_200_steps_full_size():
    """config 2 (Sedov -n 200 -s 200, 8M particles) run to its configured length on one GPU"""
    side, steps = 200, 200
    n = side ** 3
    fx = gu.load(tj.CASES["sedov"][0])
    ctx = sx.Context(0)
    sim = sx.Sim(ctx, n, sx.make_box([-0.5, 0.5, -0.5, 0.5, -0.5, 0.5], [1, 1, 1]))
    try:
        sim.init_sedov(side)
        e0 = sim.conserved()["etot"]
        emax = 0.0
        for s in range(steps):
            sim.step()
            st = sim.stats()
            assert st["numFailed"] == 0 and st["maxNeighbors"] <= 150, (s, st)
            if s % 20 == 19:
                emax = max(emax, abs(sim.conserved()["etot"] / e0 - 1))
        f = sim.get(tj.FIELDS + ["id", "h"])
        t = sim.scalars()["ttot"]
    finally:
        sim.close()
        ctx.close()
    assert np.array_equal(np.sort(f["id"]), np.arange(n, dtype=np.uint64))
    assert np.all(np.isfinite(f["h"])) and np.all(f["h"] > 0) and np.all(np.isfinite(f["temp"]))
    ref_budget = float(np.max(np.abs(fx["series_etot"] / fx["series_etot"][0] - 1)))
    rho, _ = tj.eos_rho_p(f)
    # the n=200 run ends at a time of its own: the blast (p0 = 0) is self-similar, rho(r, t) = rho_sol(r (t_sol /
    # t)^(2/5), t_sol) with the shock radius ~ t^(2/5), so the reference solver's profile at the fixture's time serves
    l1 = tj.analytic_l1(tj.radii(f) * (float(fx["sol_time"][0]) / t) ** 0.4, rho.astype(np.float64), fx["sol"][:, 0],
                        fx["sol"][:, 1])
    l1_50 = float(fx["ref_l1_density_subsampled"][0])
    print(f"Sedov -n 200 -s 200: t = {t:.6g}, energy drift max {emax:.3g} (reference n=50 budget {ref_budget:.3g}), "
          f"density L1 vs analytic {l1:.4f} (n=50: {l1_50:.4f})")
    assert emax <= 1.5 * ref_budget, (emax, ref_budget)
    assert l1 < l1_50, (l1, l1_50)
